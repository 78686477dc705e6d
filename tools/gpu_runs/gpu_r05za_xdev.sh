# round 5: bench.py's N-rank path with the cross-device session-image check, rehearsed over gloo
# with 2 and 4 ranks sharing the one GPU (the driver's 8-GPU run uses RCCL between devices), and
# the N=1 line.  Logs under gpurun_out/$1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05za}
O=gpurun_out/$TAG
mkdir -p $O
run() {   # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err; local r=$?
  echo "$n rc=$r"; python -c "
import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1])
print(d['value']/1e9, 'G', d['ms_per_step'], d['n_gpus'], d.get('cross_device'))"
  return $r
}
EDGPU_BENCH_BACKEND=gloo run rank2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline && \
EDGPU_BENCH_BACKEND=gloo run rank4 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 4 --steps 5 --warmup 2 --no-cpu-baseline && \
run n1 300 python bench.py --no-cpu-baseline
exit $?
