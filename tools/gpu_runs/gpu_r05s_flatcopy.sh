# round 5: the flat slot copy with loads first (k_ingest_copy2, EDGPU_INGEST=2) against the naive flat
# copy (1) and the fused k_ingest (0), measurement build, descriptor ingest; kernel traces.
set -o pipefail
R=$GRAFT_REPO_ROOT
export EDGPU_LIB=$R/easydarwin_amd/ab/libedgpu_ab.so TMPDIR=/tmp
O=$R/gpurun_out/${1:-r05s}
mkdir -p $O
for m in 0 1 2; do
  EDGPU_INGEST=$m timeout -s KILL 150 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt$m -o kt -- python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/b$m.json 2> $O/b$m.err || exit 1
  python3 - $O/kt$m/kt_kernel_trace.csv $O/b$m.json <<'PY'
import csv, sys, json, statistics
rows = list(csv.DictReader(open(sys.argv[1])))
d = {}
for r in rows:
    k = r["Kernel_Name"].split("(")[0]
    if k.startswith("k_ingest"):
        d.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
b = json.load(open(sys.argv[2]))
print(sys.argv[2][-7:], {k: round(statistics.median(v[-8:]), 1) for k, v in d.items()}, b["ms_per_step"], b["kernel_ms"]["ingest"])
PY
done
