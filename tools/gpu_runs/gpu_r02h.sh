# round 2, run h: full GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/gputest.log | tail -15
exit $rc
