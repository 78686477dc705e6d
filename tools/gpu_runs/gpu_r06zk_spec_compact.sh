#!/bin/bash
# k_ingest's speculative copy with compaction on refusals (the write high-water mark vclob): the
# whole GPU suite, then the C2 descriptor line and the 100-ms line alternating with the
# header-first library (ab/libedgpu_base.so), then the FETCH_SIZE / WRITE_SIZE passes of the new one.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zk
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $R
timeout -k 10 700 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1 || exit $?
A="--steps 20 --warmup 3 --no-cpu-baseline"
for rep in 1 2 3; do
  for v in base spec; do
    L=easydarwin_amd/libedgpu.so; [ $v != spec ] && L=easydarwin_amd/ab/libedgpu_$v.so
    EDGPU_LIB=$L timeout -k 10 200 python bench.py $A > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit $?
    EDGPU_LIB=$L timeout -k 10 200 python bench.py --tick-ms 100 --steps 100 --warmup 30 --no-cpu-baseline > $O/t100_${v}_$rep.json 2> $O/t100_${v}_$rep.err || exit $?
  done
done
bash tools/profile.sh r06zk/prof_desc > $O/prof_desc.log 2>&1 || exit $?
bash tools/profile.sh r06zk/prof_t100 "--tick-ms 100 --steps 100 --warmup 30" > $O/prof_t100.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
echo done
