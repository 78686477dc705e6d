#!/bin/bash
# A/B the fan-out variants on the C2 bench (GPU box).  Usage: tools/ab_fanout.sh <out-tag> <variants...>
# BENCH_EXTRA: extra bench.py flags (e.g. "--rewrite"); TAGSUF: suffix of the output files.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
mkdir -p $R/gpurun_out/$TAG
for v in "$@"; do
  EDGPU_FANOUT=$v timeout -k 10 300 python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline $BENCH_EXTRA > $R/gpurun_out/$TAG/v$v$TAGSUF.json 2> $R/gpurun_out/$TAG/v$v$TAGSUF.err || exit 1
done
