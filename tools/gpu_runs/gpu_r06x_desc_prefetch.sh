#!/bin/bash
# k_ingest: the first round's descriptors loaded beside the session / sender records.  Parity
# subset, then 20 / 100 / 1000-ms lines A/B against HEAD's library (ab/libedgpu_base.so).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06x
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_passes.py tests/test_gpu_ring_growth.py > $O/tests.log 2>&1 || exit $?
for T in 20 100 1000; do
  S=$((10000 / T)); W=$((3000 / T))
  A="--tick-ms $T --steps $S --warmup $W --no-cpu-baseline"
  for rep in 1 2; do
    for v in base new; do
      L=""; [ $v = base ] && L="EDGPU_LIB=easydarwin_amd/ab/libedgpu_base.so"
      env $L timeout -k 10 300 python bench.py $A > $O/bench_${v}_t${T}_$rep.json 2> $O/bench_${v}_t${T}_$rep.err || exit $?
    done
  done
done
