#!/bin/bash
# The two product fan-out kernels at 20 / 100 / 1000-ms ticks (EDGPU_FANOUT=0: k_fanout4<1024,32>,
# the patching kernel; 1: k_fanout6<1024,16>, the plain default), two runs each, interleaved.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06z
mkdir -p $O
cd $R
for T in 20 100 1000; do
  S=$((10000 / T)); W=$((3000 / T))
  A="--tick-ms $T --steps $S --warmup $W --no-cpu-baseline"
  for rep in 1 2; do
    for v in 0 1; do
      EDGPU_FANOUT=$v timeout -k 10 300 python bench.py $A > $O/bench_v${v}_t${T}_$rep.json 2> $O/bench_v${v}_t${T}_$rep.err || exit $?
    done
  done
done
