# round 3, final run 6 (the committed tree after the gather-parts option): the full GPU suite and
# smoke(), then two rounds of the module threaded / prestaged soak
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03_final6
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "FAIL|ERROR" $O/gputests.log | head -20; tail -1 $O/gputests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rs=$?
echo "smoke rc=$rs"; tail -2 $O/smoke.log
[ $rs -ne 0 ] && exit $rs
T="tests/test_gpu_qtss_module.py::test_module_threaded_default_mode_matches_reference tests/test_gpu_random.py::test_module_streams_batches_ahead_of_the_tick"
for k in 1 2; do
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $T > $O/soak_$k.log 2>&1; r=$?
  echo "soak $k rc=$r $(tail -1 $O/soak_$k.log)"
  [ $r -ne 0 ] && exit $r
done
exit 0
