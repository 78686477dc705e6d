# round 5: the RTSP-interleaved ingest chain's counters (verdict item 6): kernel trace + FETCH / WRITE
# passes of bench.py --ingest tcp, then SQ and TCC passes on k_tcp_* / k_ingest, with the deframe
# overlapping the previous fan-out (the default) and alone (EDGPU_DEFRAME_SERIAL=1).
# Logs under gpurun_out/$1 (default r05k).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05k}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
B="--steps 5 --warmup 2 --no-cpu-baseline --ingest tcp"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU"
bash tools/profile.sh $TAG/prof_tcp "--ingest tcp" || exit $?
for mode in overlap serial; do
  S=0; [ $mode = serial ] && S=1
  EDGPU_DEFRAME_SERIAL=$S timeout -k 10 120 python3 bench.py $B > $O/bench_$mode.json 2> $O/bench_$mode.err || exit $?
  echo "$mode: $(head -c 300 $O/bench_$mode.json)"
  EDGPU_DEFRAME_SERIAL=$S timeout -s KILL 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_$mode -o kt -- python3 bench.py $B > /dev/null 2> $O/kt_$mode.err || exit $?
  EDGPU_DEFRAME_SERIAL=$S timeout -s KILL 120 rocprofv3 --pmc $SQ -T --output-format csv --kernel-include-regex 'k_ingest|k_tcp' -d $O/sq_$mode -o sq -- python3 bench.py $B > /dev/null 2> $O/sq_$mode.err || exit $?
  EDGPU_DEFRAME_SERIAL=$S timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T --output-format csv --kernel-include-regex 'k_ingest|k_tcp' -d $O/tcc_$mode -o tcc -- python3 bench.py $B > /dev/null 2> $O/tcc_$mode.err || exit $?
done
echo done
