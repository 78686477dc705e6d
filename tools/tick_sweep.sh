#!/bin/bash
# Small-tick lines, run on the GPU box through gpurun:
#   bench.py at 100-ms and 20-ms ticks (the same 10-s-of-traffic window as C2's 10 x 1-s steps),
#   each with a rocprofv3 kernel-trace summary.  Usage: tools/tick_sweep.sh <out tag>
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-ticks}
mkdir -p $OUT
for T in 100 20; do
    S=$((10000 / T)); W=$((3000 / T))
    ARGS="--tick-ms $T --steps $S --warmup $W --no-cpu-baseline"
    timeout -k 10 300 python3 $R/bench.py $ARGS > $OUT/bench_t$T.json 2> $OUT/bench_t$T.err
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/kt$T -o kt -- python3 $R/bench.py $ARGS > $OUT/kt_bench_t$T.json 2> $OUT/kt_bench_t$T.err
done
echo done
