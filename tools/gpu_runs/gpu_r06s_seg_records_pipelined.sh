#!/bin/bash
# Segmented deframe walk with header records (k_tcp_walk_seg writes each frame's first 32 B;
# k_ingest reads them): parity tests, then the interleaved C2 line A/B with traces and FETCH_SIZE.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06s_rec2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $R
T="tests/test_gpu_interleave.py tests/test_gpu_random.py tests/test_gpu_ring_growth.py tests/test_gpu_engine_api.py tests/test_gpu_passes.py"
B="--steps 10 --warmup 3 --no-cpu-baseline --ingest tcp"
EDGPU_TCP_WALK=seg EDGPU_TCP_SEG=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $T > $O/tests_seg4.log 2>&1 && \
EDGPU_TCP_WALK=seg EDGPU_TCP_SEG=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_interleave.py tests/test_gpu_random.py > $O/tests_seg3.log 2>&1 && \
for m in parallel seg4 seg8; do
  case $m in parallel) W=parallel; S=4;; seg4) W=seg; S=4;; seg8) W=seg; S=8;; esac
  EDGPU_TCP_WALK=$W EDGPU_TCP_SEG=$S timeout -k 10 200 python bench.py $B > $O/bench_$m.json 2> $O/bench_$m.err || exit $?
  EDGPU_TCP_WALK=$W EDGPU_TCP_SEG=$S timeout -s KILL 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_$m -o kt -- python3 bench.py $B > $O/kt_$m.json 2> $O/kt_$m.err || exit $?
  EDGPU_TCP_WALK=$W EDGPU_TCP_SEG=$S timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -T --output-format csv --kernel-include-regex 'k_ingest|k_tcp' -d $O/fetch_$m -o f -- python3 bench.py $B > $O/fetch_$m.json 2> $O/fetch_$m.err || exit $?
done
