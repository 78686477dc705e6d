#!/bin/bash
# k_ingest slot copy with non-temporal loads / stores (EDGPU_INGEST_NT 1 / 2 / 3) against the
# shipped library: parity subset on the nt-everything build, then the descriptor and interleaved
# C2 lines alternating, then one FETCH_SIZE pass per variant and line (k_ingest's re-read of
# each packet's first line is what the policy is for).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zf
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $R
EDGPU_LIB=easydarwin_amd/ab/libedgpu_ntls.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_adapter.py > $O/tests.log 2>&1 || exit $?
A="--steps 20 --warmup 3 --no-cpu-baseline"
for rep in 1 2; do
  for v in base ntl nts ntls; do
    L=easydarwin_amd/libedgpu.so; [ $v != base ] && L=easydarwin_amd/ab/libedgpu_$v.so
    EDGPU_LIB=$L timeout -k 10 200 python bench.py $A > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit $?
    EDGPU_LIB=$L timeout -k 10 200 python bench.py $A --ingest tcp > $O/tcp_${v}_$rep.json 2> $O/tcp_${v}_$rep.err || exit $?
  done
done
for v in base ntl nts ntls; do
  L=$R/easydarwin_amd/libedgpu.so; [ $v != base ] && L=$R/easydarwin_amd/ab/libedgpu_$v.so
  for line in desc tcp; do
    X=""; [ $line = tcp ] && X="--ingest tcp"
    EDGPU_LIB=$L timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -T --output-format csv --kernel-include-regex 'k_fanout|k_ingest|k_tcp' -d $O/fetch_${v}_$line -o fetch -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline $X > $O/fetch_${v}_$line.json 2> $O/fetch_${v}_$line.err || exit $?
  done
done
echo done
