# round 2, run f: full GPU suite (readback refactor, transmit times, egress fix) + bisect round 2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02f
mkdir -p $O
fatal() { [ $1 -ge 124 ]; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest.log | tail -12; fatal $rc && exit 1
VARIANTS="B Bi D F" RUNS=40 timeout -k 10 600 bash tools/fpi_bisect.sh > $O/bisect.jsonl 2>&1; rc=$?; cat $O/bisect.jsonl; fatal $rc && exit 1
echo ALL_OK
