# round 2, run z14: the per-tick kernel-choice test
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z14
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine_api.py -m gpu -v --timeout 120 --timeout-method thread > $O/test.log 2>&1; rc=$?
tail -15 $O/test.log; exit $rc
