# round 5: sender rings from a pool -- the full GPU suite, then the growth trace of a 15-s C2 module run.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05r}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf --timeout 150 --timeout-method thread -p no:cacheprovider > $O/gputests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "FAILED|Timeout" $O/gputests.log | head -20; tail -1 $O/gputests.log
[ $rc -ne 0 ] && exit $rc
EDGPU_DEBUG_GROW=1 EDGPU_BENCH_TRACE=1 EDGPU_QTSS_WRITE_THREADS=16 EDGPU_QTSS_ARENA_MB=4096 EDGPU_QTSS_MAX_OUT_PACKETS=4194304 \
  timeout -k 10 200 $R/tools/qtss_replay $R/easydarwin_amd/libQTSSReflectorModule.so --bench 1024 16 15 100 8 > $O/trace.json 2> $O/trace.err || exit 1
python3 - $O/trace.err <<'PY'
import re, sys
rows = [(int(re.search(r"tick (\d+):", l).group(1)), float(re.search(r"tick ([\d.]+) ms", l).group(1))) for l in open(sys.argv[1]) if l.startswith("bench tick")]
big = sorted(rows, key=lambda r: -r[1])[:8]
print("slowest ticks", big, "median", sorted(r[1] for r in rows)[len(rows) // 2])
g = [l.strip() for l in open(sys.argv[1]) if "ring growth" in l]
print(len(g), "growth calls;", g[:4])
PY
