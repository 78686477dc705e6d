#!/bin/bash
# Mailbox control words in POSIX shared memory (images stay in the owner's HBM): the replica
# goldens through the mailbox, the two-process IPC tests, then the 2-rank bench rehearsal.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zb
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_replica.py tests/test_gpu_multiprocess.py > $O/tests.log 2>&1 || exit $?
for rep in 1 2; do
EDGPU_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline \
    > $O/bench_rank2_$rep.json 2> $O/bench_rank2_$rep.err || exit $?
done
