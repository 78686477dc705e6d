#!/bin/bash
# Round 6 final tree, the other lines: two ranks sharing the box's GPU with replica sessions fed
# through peer mailboxes, the C4 burst, the module at 100-ms ticks beside the reference module.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06zn_lines
mkdir -p $O
EDGPU_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline \
    > $O/bench_rank2.json 2> $O/bench_rank2.err || exit $?
timeout -k 10 200 python tools/bench_c4.py > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
timeout -k 10 400 python tools/bench_module.py --tick-ms 100 > $O/bench_module_t100.json 2> $O/bench_module_t100.err || exit $?
echo done
