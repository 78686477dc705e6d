# round 3, run as: rehearsal (after the timing-level change) of the driver's N-rank bench path on the one-GPU box -- 2 and 4
# ranks over gloo sharing the card (EDGPU_BENCH_BACKEND=gloo), checking the rank-0 line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03as
mkdir -p $O
for n in 2 4; do
  EDGPU_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 5 --warmup 2 > $O/rank$n.json 2> $O/rank$n.err; r=$?
  echo "n=$n rc=$r $(python -c "import json;d=json.loads(open('$O/rank$n.json').read().strip().splitlines()[-1]);print(d['n_gpus'], d['value'], d['ms_per_step'], d['config'].get('parallelism'), d['cpu_baseline'])")"
  [ $r -ne 0 ] && exit $r
done
EDGPU_BENCH_FORCE_PG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --steps 5 --warmup 2 > $O/rccl1.json 2> $O/rccl1.err; r=$?
echo "rccl world 1 rc=$r $(tail -1 $O/rccl1.json | head -c 300)"
exit $r
