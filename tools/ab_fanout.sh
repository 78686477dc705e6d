#!/bin/bash
# A/B the fan-out variants on the C2 bench (GPU box).  Usage: tools/ab_fanout.sh <out-tag> <variants...>
# BENCH_EXTRA: extra bench.py flags (e.g. "--rewrite"); TAGSUF: suffix of the output files.
R=${GRAFT_REPO_ROOT:-$(pwd)}
# the measurement build (every variant, EDGPU_ABLATE): make -C easydarwin_amd/csrc ab
export EDGPU_LIB=$R/easydarwin_amd/ab/libedgpu_ab.so
[ -e $EDGPU_LIB ] || { echo "build $EDGPU_LIB first"; exit 2; }
TAG=$1; shift
mkdir -p $R/gpurun_out/$TAG
k=0
for v in "$@"; do
  k=$((k+1))                                    # a variant listed twice keeps both runs (vN.json, vN_rK.json)
  f=v$v$TAGSUF; [ -e $R/gpurun_out/$TAG/$f.json ] && f=v$v${TAGSUF}_r$k
  EDGPU_FANOUT=$v timeout -k 10 300 python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline $BENCH_EXTRA > $R/gpurun_out/$TAG/$f.json 2> $R/gpurun_out/$TAG/$f.err || exit 1
done
