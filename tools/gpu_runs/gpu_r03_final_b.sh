# round 3, final run B: the other bench lines (RTSP-interleaved push with its CPU baseline,
# every sub-stream rewriting, C3's per-GPU shape, pinned host ingest, C5, the C4 burst, the
# QTSS module, socket egress)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03_final
mkdir -p $O
run() {   # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err; local r=$?
  echo "$n rc=$r"; head -c 600 $O/$n.json; echo
  return $r
}
run bench_tcp 500 python bench.py --ingest tcp && \
run bench_rewrite 300 python bench.py --no-cpu-baseline --rewrite && \
run bench_c3 300 python bench.py --no-cpu-baseline --subs 64 && \
run bench_host 300 python bench.py --no-cpu-baseline --ingest host && \
run bench_c5 300 python tools/bench_c5.py && \
run bench_c4 300 python tools/bench_c4.py && \
run bench_module 300 python tools/bench_module.py && \
run bench_egress 300 python tools/bench_egress.py
