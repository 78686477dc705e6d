# round 5: the context stream at the highest priority (EDGPU_STREAM_PRIORITY=1) against the default,
# alternating on one box, interleaved and descriptor lines.  Logs under gpurun_out/$1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05zm}
O=gpurun_out/$TAG
mkdir -p $O
for rep in 1 2 3; do
  for v in base prio; do
    for ing in tcp desc; do
      n=${v}_${ing}_$rep
      if [ $v = prio ]; then export EDGPU_STREAM_PRIORITY=1; else unset EDGPU_STREAM_PRIORITY; fi
      timeout -k 10 200 python bench.py --no-cpu-baseline --ingest $ing > $O/$n.json 2> $O/$n.err || exit $?
      python -c "
import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1])
print('$n', d['ms_per_step'], 'ingest', d['ingest']['avg_ms'], 'fanout', d['roofline']['avg_kernel_ms'])"
    done
  done
done
