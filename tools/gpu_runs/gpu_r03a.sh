# round 3, run a: baseline of the round-2 tree (GPU suite, smoke, default bench line)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest.log | tail -3; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic_source'], d['cpu_baseline']['value'])"
echo ALL_OK
