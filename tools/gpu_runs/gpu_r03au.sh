# round 3, run au: the stager waits while no batch is armed: module / adapter / prestage tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03au
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qtss_module.py tests/test_gpu_adapter.py "tests/test_gpu_random.py::test_module_streams_batches_ahead_of_the_tick" tests/test_gpu_lifecycle.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAIL|ERROR" $O/tests.log | head -20; tail -1 $O/tests.log
exit $rc
