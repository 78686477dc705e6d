#!/bin/bash
# k_plan_final: work-item reservations aggregated per block and its independent loads hoisted
# sender): parity subset, then the 20- and 100-ms tick lines A/B against the previous library
# (easydarwin_amd/ab/libedgpu_base.so), each with a kernel trace.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06w
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_passes.py tests/test_gpu_scale.py > $O/tests.log 2>&1 || exit $?
for T in 20 100; do
  S=$((10000 / T)); W=$((3000 / T))
  A="--tick-ms $T --steps $S --warmup $W --no-cpu-baseline"
  for v in base new; do
    L=""; [ $v = base ] && L="EDGPU_LIB=easydarwin_amd/ab/libedgpu_base.so"
    env $L timeout -k 10 300 python bench.py $A > $O/bench_${v}_t$T.json 2> $O/bench_${v}_t$T.err || exit $?
  done
  for v in base new; do
    if [ $v = base ]; then export EDGPU_LIB=easydarwin_amd/ab/libedgpu_base.so; else unset EDGPU_LIB; fi
    timeout -s KILL 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_${v}_t$T -o kt -- python3 bench.py $A > /dev/null 2> $O/kt_${v}_t$T.err || exit $?
  done
  unset EDGPU_LIB
done
