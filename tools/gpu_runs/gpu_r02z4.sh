# round 2, run z4: the QTSS module with UDP pushers (socket pairs, loopback datagrams, receiver
# reports) -- module tests on the golden + random traces
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z4
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "module" > $O/gputest.log 2>&1; rc=$?
echo "module tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/gputest.log | tail -25; exit $rc
