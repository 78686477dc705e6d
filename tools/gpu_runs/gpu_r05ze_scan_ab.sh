# round 5: A/B of the tree against easydarwin_amd/ab/libedgpu_prev.so (the previous commit, built by
# hand), alternating on one box, descriptor and interleaved lines: first k_ingest's one-pass sender
# scans (r05ze), then the first round's descriptors and headers loaded with the session's tables
# (r05zg, after the GPU suite).  Logs under gpurun_out/$1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05ze}
O=gpurun_out/$TAG
mkdir -p $O
if [ "${SUITE:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu -x tests > $O/gputests.log 2>&1; rc=$?
  tail -2 $O/gputests.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2 3; do
  for v in new prev; do
    for ing in desc tcp; do
      n=${v}_${ing}_$rep
      if [ $v = prev ]; then export EDGPU_LIB=$GRAFT_REPO_ROOT/easydarwin_amd/ab/libedgpu_prev.so; else unset EDGPU_LIB; fi
      timeout -k 10 200 python bench.py --no-cpu-baseline --ingest $ing > $O/$n.json 2> $O/$n.err || exit $?
      python -c "
import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1])
print('$n', d['ms_per_step'], 'ingest', d['ingest']['avg_ms'], 'fanout', d['roofline']['avg_kernel_ms'])"
    done
  done
done
