# round 5, a full call on the committed tree: the GPU suite and smoke(), the default line (with its
# CPU baseline), the interleaved line, the C4 burst, the module beside the reference module at 100-
# and 20-ms ticks and at the real rate, the socket egress, and rocprofv3 kernel trace + PMC passes
# of the default line.  Logs under gpurun_out/$1 (default r05_final).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05_final}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v -rs --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu tests > $O/gputests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "FAILED|ERROR|Timeout" $O/gputests.log | head -20; tail -1 $O/gputests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rs=$?
echo "smoke rc=$rs"; tail -2 $O/smoke.log
[ $rs -ne 0 ] && exit $rs
run() {   # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err; local r=$?
  echo "$n rc=$r"; head -c 500 $O/$n.json; echo
  return $r
}
run bench_default 400 python bench.py && \
run bench_tcp 200 python bench.py --no-cpu-baseline --ingest tcp && \
run bench_c4 200 python tools/bench_c4.py && \
run bench_module_t100 400 python tools/bench_module.py --tick-ms 100 && \
EDGPU_QTSS_TICK_MSEC=20 run bench_module_t20 400 python tools/bench_module.py --tick-ms 20 && \
run bench_module_realtime 300 python tools/bench_module.py --realtime --tick-ms 20 --seconds 5 && \
run bench_egress 300 python tools/bench_egress.py && \
bash tools/profile.sh $TAG/prof_desc ""
exit $?
