# round 3, run aq: edgpu_ingest_prestage's API contract test and the engine API suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03aq
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine_api.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAIL|ERROR|Error" $O/tests.log | head -20; tail -1 $O/tests.log
exit $rc
