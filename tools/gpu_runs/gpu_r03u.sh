# round 3, run u: the long-session interleave test (global chunk / read lookups, unrecorded
# chunks), then a kernel trace of the --ingest tcp line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_interleave.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAIL|Error|assert|passed|failed" $O/tests.log | tail -15
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_tcp -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --ingest tcp > $O/kt_tcp.json 2> $O/kt_tcp.err
