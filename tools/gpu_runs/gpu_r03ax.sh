# round 3, run ax: soak of the module's threaded default mode and the prestaged heavy trace (the
# adapter's stager thread beside the pushers and the tick), four rounds in one pytest process each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ax
mkdir -p $O
T="tests/test_gpu_qtss_module.py::test_module_threaded_default_mode_matches_reference tests/test_gpu_random.py::test_module_streams_batches_ahead_of_the_tick"
for k in 1 2 3 4; do
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $T > $O/soak_$k.log 2>&1; rc=$?
  echo "round $k rc=$rc $(tail -1 $O/soak_$k.log)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
