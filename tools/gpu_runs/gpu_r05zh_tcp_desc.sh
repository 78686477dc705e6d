# round 5: the interleaved ingest with a descriptor and source address for every frame from
# k_tcp_finish (the tree's default) against k_ingest finding the recorded chunks' frames itself
# (EDGPU_TCP_DIRECT=1, rounds 3-4), alternating on one box; the GPU suite first.  Logs under
# gpurun_out/$1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05zh}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu -x tests > $O/gputests.log 2>&1; rc=$?
tail -2 $O/gputests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in desc direct; do
    n=${v}_$rep
    if [ $v = direct ]; then export EDGPU_TCP_DIRECT=1; else unset EDGPU_TCP_DIRECT; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --ingest tcp > $O/$n.json 2> $O/$n.err || exit $?
    python -c "
import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1])
print('$n', d['ms_per_step'], 'ingest', d['ingest']['avg_ms'], d['ingest']['frac'], 'fanout', d['roofline']['avg_kernel_ms'])"
  done
done
unset EDGPU_TCP_DIRECT
bash tools/profile.sh $TAG/prof_tcp "--ingest tcp" > $O/prof.log 2>&1
exit $?
