# round 2, run z23: rehearsal of bench.py's N-rank path on one GPU (gloo, 2 and 4 ranks sharing
# the card): owned_sessions sharding, barrier + max-over-ranks timing, rank-0 JSON line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z23
mkdir -p $O
export EDGPU_BENCH_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2951$n bench.py --gpus $n --steps 4 --warmup 1 > $O/n$n.json 2> $O/n$n.err || { echo "N=$n FAIL"; tail -20 $O/n$n.err; exit 1; }
  cut -c1-400 $O/n$n.json
done
echo ALL_OK
