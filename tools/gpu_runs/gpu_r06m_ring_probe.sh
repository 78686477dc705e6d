# Is the small-tick ingest latency the rings' spread over HBM (TLB)?  20-ms ticks with the default
# 16-MiB video rings, the same without growth, and 2-MiB rings without growth; the measurement
# build prints k_ingest's phase times (EDGPU_FAN_TAIL).
mkdir -p gpurun_out/r06m
for cfg in "16" "16 --no-ring-growth" "2 --no-ring-growth"; do
  tag=$(echo $cfg | tr -d ' -')
  EDGPU_LIB=easydarwin_amd/ab/libedgpu_ab.so EDGPU_FAN_TAIL=1 timeout -k 10 200 python3 bench.py --tick-ms 20 --steps 500 \
      --warmup 150 --no-cpu-baseline --ring-mb $cfg > gpurun_out/r06m/r$tag.json 2> gpurun_out/r06m/r$tag.err || exit 1
done
