# round 4, final call on the committed tree: the full GPU suite and smoke(), every bench line (the
# default one with its CPU baseline), the module beside the reference module at 100- and 20-ms ticks,
# the module at C2's real rate on its own ticker, the socket egress, and rocprofv3 kernel trace +
# PMC passes of the default line.  Logs under gpurun_out/$1 (default r04_final).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r04_final}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "FAIL|ERROR" $O/gputests.log | head -20; tail -1 $O/gputests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rs=$?
echo "smoke rc=$rs"; tail -2 $O/smoke.log
[ $rs -ne 0 ] && exit $rs
run() {   # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err; local r=$?
  echo "$n rc=$r"; head -c 700 $O/$n.json; echo
  return $r
}
run bench_default 500 python bench.py && \
run bench_tcp 400 python bench.py --no-cpu-baseline --ingest tcp && \
run bench_module_t100 300 python tools/bench_module.py --tick-ms 100 && \
EDGPU_QTSS_TICK_MSEC=20 run bench_module_t20 300 python tools/bench_module.py --tick-ms 20 && \
run bench_module_realtime 300 python tools/bench_module.py --realtime --tick-ms 20 --seconds 5 && \
run bench_egress 300 python tools/bench_egress.py && \
bash tools/profile.sh $TAG/prof_desc ""
exit $?
