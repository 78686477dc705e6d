#!/bin/bash
# The speculative copy on interleaved batches (frame lengths from the walk's records, channels
# recorded by the walk): parity (every golden forced through it, the stress trace, the interleave
# tests), then the interleaved C2 line alternating with the header-first library, and its PMC.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_interleave.py tests/test_spec_stress.py tests/test_gpu_random.py > $O/tests.log 2>&1 || exit $?
for rep in 1 2 3; do
  for v in base spec; do
    L=easydarwin_amd/libedgpu.so; [ $v != spec ] && L=easydarwin_amd/ab/libedgpu_$v.so
    EDGPU_LIB=$L timeout -k 10 200 python bench.py --ingest tcp --steps 20 --warmup 3 --no-cpu-baseline > $O/tcp_${v}_$rep.json 2> $O/tcp_${v}_$rep.err || exit $?
  done
done
bash tools/profile.sh r06zp/prof_tcp "--ingest tcp" > $O/prof_tcp.log 2>&1 || exit $?
echo done
