#!/bin/bash
# Ablation timing (GPU box): fan-out variant $2 with EDGPU_ABLATE = each of ${ABL:-0 1 2 3}:
# 1 no descriptors, 2 no arena stores, 4 no chunk-word loads (stores write whatever the
# registers hold).  Outputs are wrong except at 0: timing only.
R=${GRAFT_REPO_ROOT:-$(pwd)}
# the measurement build (every variant, EDGPU_ABLATE): make -C easydarwin_amd/csrc ab
export EDGPU_LIB=$R/easydarwin_amd/ab/libedgpu_ab.so
[ -e $EDGPU_LIB ] || { echo "build $EDGPU_LIB first"; exit 2; }
TAG=$1; V=$2
mkdir -p $R/gpurun_out/$TAG
for a in ${ABL:-0 1 2 3}; do
  EDGPU_FANOUT=$V EDGPU_ABLATE=$a timeout -k 10 300 python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline --ablation-study > $R/gpurun_out/$TAG/a$a.json 2> $R/gpurun_out/$TAG/a$a.err || exit 1
  python3 -c "import json; d=json.load(open('$R/gpurun_out/$TAG/a$a.json')); print('ablate=$a', d['roofline']['avg_kernel_ms'], d['ms_per_step'])"
done
