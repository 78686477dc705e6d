#!/bin/bash
# Serial deframe walk (EDGPU_TCP_WALK=serial, k_tcp_chain): the deframe / interleaved parity tests
# under it, then the interleaved C2 line A/B (parallel vs serial) with kernel traces and FETCH_SIZE.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06p_serial
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $R
T="tests/test_gpu_interleave.py tests/test_gpu_random.py tests/test_gpu_ring_growth.py tests/test_gpu_engine_api.py tests/test_gpu_passes.py"
B="--steps 10 --warmup 3 --no-cpu-baseline --ingest tcp"
EDGPU_TCP_WALK=serial timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $T > $O/tests_serial.log 2>&1 && \
for m in parallel serial; do
  EDGPU_TCP_WALK=$m timeout -k 10 200 python bench.py $B > $O/bench_$m.json 2> $O/bench_$m.err || exit $?
  EDGPU_TCP_WALK=$m timeout -s KILL 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_$m -o kt -- python3 bench.py $B > $O/kt_$m.json 2> $O/kt_$m.err || exit $?
  EDGPU_TCP_WALK=$m timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -T --output-format csv --kernel-include-regex 'k_ingest|k_tcp' -d $O/fetch_$m -o f -- python3 bench.py $B > $O/fetch_$m.json 2> $O/fetch_$m.err || exit $?
done
