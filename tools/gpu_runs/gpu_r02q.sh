set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02q
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "random" > gpurun_out/r02q/gputest.log 2>&1; rc=$?
echo "rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r02q/gputest.log | tail -30; exit $rc
