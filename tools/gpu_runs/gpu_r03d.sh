# round 3, run d: two engine processes on one GPU (sharding, session-image exchange), the UDP
# overload ordering test, and bench.py's RCCL code path at world size 1 under torchrun
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multiprocess.py \
  "tests/test_gpu_egress.py::test_udp_overload_loses_datagrams_without_reordering" > $O/mp.log 2>&1; rc=$?
echo "multiprocess tests rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed|Error" $O/mp.log | tail -30
[ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
EDGPU_BENCH_FORCE_PG=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline \
  > $O/bench_rccl_world1.json 2> $O/bench_rccl_world1.err; rc2=$?
echo "rccl world-1 bench rc=$rc2"; tail -3 $O/bench_rccl_world1.err; cat $O/bench_rccl_world1.json | head -c 600; echo
exit $(( rc || rc2 ))
