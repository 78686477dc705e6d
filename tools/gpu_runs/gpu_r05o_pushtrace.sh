# round 5: the drop-in's per-tick push and tick times over a 15-s C2 run (8 pusher threads), to see
# how the push path changes once the stream passes the reference's 10-s packet age.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05o}
mkdir -p $O
for ps in 1 0; do
  EDGPU_PUSH_STREAMING=$ps EDGPU_BENCH_TRACE=1 EDGPU_QTSS_WRITE_THREADS=16 EDGPU_QTSS_ARENA_MB=4096 EDGPU_QTSS_MAX_OUT_PACKETS=4194304 \
    timeout -k 10 200 $R/tools/qtss_replay $R/easydarwin_amd/libQTSSReflectorModule.so --bench 1024 16 15 100 8 > $O/trace_ps$ps.json 2> $O/trace_ps$ps.err || exit 1
  python3 - $O/trace_ps$ps.err <<'PY'
import re, sys
rows = [tuple(float(x) for x in re.findall(r"push ([\d.]+) ms \((\d+) frames\), tick ([\d.]+)", l)[0]) for l in open(sys.argv[1]) if l.startswith("bench tick")]
for a in range(0, len(rows), 15):
    seg = rows[a:a + 15]
    print(sys.argv[1][-12:], a, "push ms %.2f" % (sum(r[0] for r in seg) / len(seg)), "frames %.0f" % (sum(r[1] for r in seg) / len(seg)), "tick ms %.2f" % (sum(r[2] for r in seg) / len(seg)))
PY
done
