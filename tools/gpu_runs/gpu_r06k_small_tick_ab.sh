mkdir -p gpurun_out/r06k
for V in 40 42 59; do for T in 20 100; do S=$((10000 / T)); W=$((3000 / T)); EDGPU_LIB=easydarwin_amd/ab/libedgpu_ab.so EDGPU_FANOUT=$V timeout -k 10 200 python3 bench.py --tick-ms $T --steps $S --warmup $W --no-cpu-baseline > gpurun_out/r06k/v${V}_t$T.json 2> gpurun_out/r06k/v${V}_t$T.err || exit 1; done; done
timeout -k 10 700 python3 tools/bench_module.py --realtime-sweep --seconds 6 --sweep 1024,2048,4096 --no-reference > gpurun_out/r06k/sweep.json 2> gpurun_out/r06k/sweep.err
