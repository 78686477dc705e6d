# round 5: join-burst ticks take the 32-packet-chunk fan-out kernel.  GPU suite, the C4 burst and
# its trace + PMC passes (profiles/pmc_c4.json for the new kernel), the default line.  Logs under
# gpurun_out/$1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05zj}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu -x tests > $O/gputests.log 2>&1; rc=$?
tail -2 $O/gputests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python tools/bench_c4.py > $O/c4_$i.json 2> $O/c4_$i.err || exit $?
  python -c "
import json; d=json.load(open('$O/c4_$i.json')); r=d['roofline']; print('c4', r['kernel'], r['frac'], d['burst_ms'])"
done
bash tools/profile_c4.sh $TAG/prof_c4 > $O/prof_c4.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || exit $?
python -c "
import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); print('c2', d['value']/1e9, d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic'])"
