#!/bin/bash
# The speculative ingest with its spills cut (header words and arrival reloaded from LDS after the
# second copy, 32-bit segment counters): the whole GPU suite; the 1000-, 100- and 20-ms lines
# alternating with the header-first library (base) and with the speculative copy only from 128
# packets per segment (min128); the PMC passes of the 1000- and 100-ms lines.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zl
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $R
timeout -k 10 700 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1 || exit $?
for rep in 1 2 3; do
  for v in base spec min128; do
    L=easydarwin_amd/libedgpu.so; [ $v != spec ] && L=easydarwin_amd/ab/libedgpu_$v.so
    EDGPU_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit $?
    EDGPU_LIB=$L timeout -k 10 200 python bench.py --tick-ms 100 --steps 100 --warmup 30 --no-cpu-baseline > $O/t100_${v}_$rep.json 2> $O/t100_${v}_$rep.err || exit $?
    EDGPU_LIB=$L timeout -k 10 200 python bench.py --tick-ms 20 --steps 500 --warmup 150 --no-cpu-baseline > $O/t20_${v}_$rep.json 2> $O/t20_${v}_$rep.err || exit $?
  done
done
bash tools/profile.sh r06zl/prof_desc > $O/prof_desc.log 2>&1 || exit $?
bash tools/profile.sh r06zl/prof_t100 "--tick-ms 100 --steps 100 --warmup 30" > $O/prof_t100.log 2>&1 || exit $?
echo done
