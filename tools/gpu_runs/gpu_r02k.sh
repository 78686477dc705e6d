set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "qtss_module or adapter" > $O/gputest.log 2>&1; rc=$?
echo "rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest.log | tail -8; exit $rc
