# round 6, the final measurements on the committed tree (the GPU suite runs in its own call):
# smoke(), the default line (with its CPU baseline), the interleaved line, the 100- and 20-ms tick
# lines with their rocprofv3 kernel traces and a PMC pass of the 100-ms line, the C4 burst, the
# module at 100-ms ticks beside the reference module, the realtime session sweep, and the 2-rank
# replica rehearsal.  Logs under gpurun_out/$1 (default r06_final).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r06_final}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rs=$?
echo "smoke rc=$rs"; tail -2 $O/smoke.log
[ $rs -ne 0 ] && exit $rs
run() {   # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err; local r=$?
  echo "$n rc=$r"; head -c 400 $O/$n.json; echo
  return $r
}
run bench_default 400 python bench.py && \
run bench_tcp 200 python bench.py --no-cpu-baseline --ingest tcp && \
bash tools/tick_sweep.sh $TAG/ticks && \
bash tools/profile.sh $TAG/prof_t100 "--tick-ms 100 --steps 100 --warmup 30" && \
run bench_c4 200 python tools/bench_c4.py && \
run bench_module_t100 400 python tools/bench_module.py --tick-ms 100 && \
run bench_module_sweep 700 python tools/bench_module.py --realtime-sweep --seconds 6 && \
EDGPU_BENCH_BACKEND=gloo run bench_rank2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline
exit $?
