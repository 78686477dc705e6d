# round 3, final run 5: the committed tree's GPU suite, smoke() and the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03_final5
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "FAIL|ERROR" $O/gputests.log | head -20; tail -1 $O/gputests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rs=$?
echo "smoke rc=$rs"; tail -2 $O/smoke.log
[ $rs -ne 0 ] && exit $rs
timeout -k 10 500 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rb=$?
echo "bench rc=$rb"; head -c 400 $O/bench_default.json; echo
exit $rb
