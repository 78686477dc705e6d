# round 4 bench run: the default bench line (C2 CPU baseline on the process's affinity cores), the
# interleaved-ingest line, the module through the fake server next to the REFERENCE module at 100-ms
# and 20-ms ticks (with the latency the tick adds), the socket egress, and rocprofv3 kernel trace +
# PMC passes of the default line.  Logs under gpurun_out/$1 (default r04_bench).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r04_bench}
O=gpurun_out/$TAG
mkdir -p $O
run() {   # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err; local r=$?
  echo "$n rc=$r"; head -c 900 $O/$n.json; echo
  return $r
}
run bench_default 500 python bench.py && \
run bench_tcp 400 python bench.py --no-cpu-baseline --ingest tcp && \
run bench_module_t100 300 python tools/bench_module.py --tick-ms 100 && \
EDGPU_QTSS_TICK_MSEC=20 run bench_module_t20 300 python tools/bench_module.py --tick-ms 20 && \
run bench_egress 300 python tools/bench_egress.py && \
bash tools/profile.sh $TAG/prof_desc ""
exit $?
