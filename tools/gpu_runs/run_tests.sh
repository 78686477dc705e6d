# GPU test run: gpurun -- 'bash tools/gpu_runs/run_tests.sh TAG [pytest selection...]'
# Runs the selected GPU tests (default: the whole GPU suite) and smoke() under time limits, in
# one process each; logs under gpurun_out/TAG.  PYTEST_X=1 stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
SEL=${*:-tests}
X=""; [ "${PYTEST_X:-0}" = "1" ] && X="-x"
timeout -k 10 1000 python -u -m pytest -v $X --timeout 300 --timeout-method thread -m gpu $SEL > $O/gputests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "FAIL|ERROR" $O/gputests.log | head -30; tail -1 $O/gputests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rs=$?
echo "smoke rc=$rs"; tail -2 $O/smoke.log
exit $rs
