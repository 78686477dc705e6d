# round 3, final run 3 (the tree after the overlapped deframe): the full GPU suite, smoke(), the default bench line
# with its CPU baseline, the RTSP-interleaved line, and that line's kernel trace + PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03_final3
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "FAIL|ERROR" $O/gputests.log | head -20; tail -1 $O/gputests.log
[ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rs=$?
echo "smoke rc=$rs"; tail -3 $O/smoke.log
[ $rs -ne 0 ] && exit $rs
timeout -k 10 500 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rb=$?
echo "bench rc=$rb"; cat $O/bench_default.json
[ $rb -ne 0 ] && exit $rb
timeout -k 10 300 python bench.py --ingest tcp --no-cpu-baseline > $O/bench_tcp.json 2> $O/bench_tcp.err; rt=$?
echo "bench tcp rc=$rt"; cat $O/bench_tcp.json
[ $rt -ne 0 ] && exit $rt
bash tools/profile.sh r03_final3/prof_tcp "--ingest tcp"; rp=$?
echo "profile rc=$rp"
exit $(( rc || rp ))
