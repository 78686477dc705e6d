# round 5: the bench lines the final call does not run, on the round-5 tree (rewriting, C3's
# per-GPU shape, pinned host ingest, C5, the module with concurrent pushes), and the
# N-rank bench path rehearsed over gloo with 2 and 4 ranks sharing the one GPU.
# Logs under gpurun_out/$1 (default r05_lines).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05_lines}
O=gpurun_out/$TAG
mkdir -p $O
run() {   # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err; local r=$?
  echo "$n rc=$r"; tail -c 700 $O/$n.json; echo
  return $r
}
run bench_rewrite 300 python bench.py --no-cpu-baseline --rewrite && \
run bench_c3 300 python bench.py --no-cpu-baseline --subs 64 && \
run bench_host 300 python bench.py --no-cpu-baseline --ingest host && \
run bench_c5 300 python tools/bench_c5.py && \
run bench_module_conc 300 python tools/bench_module.py --no-reference --concurrent-push && \
EDGPU_BENCH_BACKEND=gloo run rank2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline && \
EDGPU_BENCH_BACKEND=gloo run rank4 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 4 --steps 5 --warmup 2 --no-cpu-baseline
exit $?
