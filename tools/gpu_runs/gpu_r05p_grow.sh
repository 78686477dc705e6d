# round 5: ring growth spread over ticks by a per-call time budget -- the growth tests, the module
# suites, and the per-tick trace of a 15-s C2 module run (the growth burst at ~8 s of stream).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05p}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_ring_growth.py tests/test_gpu_qtss_module.py tests/test_gpu_isolation.py tests/test_gpu_replica.py \
    -q -x --timeout 150 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
EDGPU_BENCH_TRACE=1 EDGPU_QTSS_WRITE_THREADS=16 EDGPU_QTSS_ARENA_MB=4096 EDGPU_QTSS_MAX_OUT_PACKETS=4194304 \
  timeout -k 10 200 $R/tools/qtss_replay $R/easydarwin_amd/libQTSSReflectorModule.so --bench 1024 16 15 100 8 > $O/trace.json 2> $O/trace.err || exit 1
python3 - $O/trace.err <<'PY'
import re, sys
rows = [(int(re.search(r"tick (\d+):", l).group(1)), float(re.search(r"tick ([\d.]+) ms", l).group(1))) for l in open(sys.argv[1]) if l.startswith("bench tick")]
big = sorted(rows, key=lambda r: -r[1])[:8]
print("slowest ticks", big, "median", sorted(r[1] for r in rows)[len(rows) // 2])
PY
