#!/bin/bash
# k_ingest's speculative copy (SPEC: descriptor batches copy first, header words from the copy's
# registers) as the default: the whole GPU suite on it, then the descriptor C2 line and the 100-ms
# line alternating with the previous library (ab/libedgpu_base.so) and with non-temporal copy
# policies (nts / ntls), then one FETCH_SIZE pass per library.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zg
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $R
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1 || exit $?
A="--steps 20 --warmup 3 --no-cpu-baseline"
for rep in 1 2; do
  for v in base spec nts ntls; do
    L=easydarwin_amd/libedgpu.so; [ $v != spec ] && L=easydarwin_amd/ab/libedgpu_$v.so
    EDGPU_LIB=$L timeout -k 10 200 python bench.py $A > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit $?
    EDGPU_LIB=$L timeout -k 10 200 python bench.py --tick-ms 100 --steps 100 --warmup 30 --no-cpu-baseline > $O/t100_${v}_$rep.json 2> $O/t100_${v}_$rep.err || exit $?
  done
done
for v in base spec nts ntls; do
  L=$R/easydarwin_amd/libedgpu.so; [ $v != spec ] && L=$R/easydarwin_amd/ab/libedgpu_$v.so
  EDGPU_LIB=$L timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -T --output-format csv --kernel-include-regex 'k_fanout|k_ingest' -d $O/fetch_$v -o fetch -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/fetch_$v.json 2> $O/fetch_$v.err || exit $?
  EDGPU_LIB=$L timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -T --output-format csv --kernel-include-regex 'k_fanout|k_ingest' -d $O/write_$v -o write -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/write_$v.json 2> $O/write_$v.err || exit $?
done
echo done
