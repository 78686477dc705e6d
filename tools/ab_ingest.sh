#!/bin/bash
# Ingest A/B (GPU box): each argument is "MODE:ABLATE" -- EDGPU_INGEST copy mode (0 in-kernel,
# 1 separate copy kernel) and EDGPU_ABLATE bits (16: no block-total atomics).  Timing only.
R=${GRAFT_REPO_ROOT:-$(pwd)}
# the measurement build (every variant, EDGPU_ABLATE): make -C easydarwin_amd/csrc ab
export EDGPU_LIB=$R/easydarwin_amd/ab/libedgpu_ab.so
[ -e $EDGPU_LIB ] || { echo "build $EDGPU_LIB first"; exit 2; }
TAG=$1; shift
mkdir -p $R/gpurun_out/$TAG
for ma in "$@"; do
  m=${ma%%:*}; a=${ma##*:}
  EDGPU_INGEST=$m EDGPU_ABLATE=$a timeout -k 10 300 python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline > $R/gpurun_out/$TAG/m${m}a$a.json 2> $R/gpurun_out/$TAG/m${m}a$a.err || exit 1
done
