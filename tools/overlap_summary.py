"""Summarises a rocprofv3 --kernel-trace --memory-copy-trace run of `bench.py --ingest host`:
for each large host->device copy (an ingest batch's blob), how much of it ran while an engine
kernel was running (the previous tick's fan-out / ingest), i.e. the PCIe overlap that the
pinned, double-buffered staging buys (docs/PARITY.md §4.12).
Usage: python tools/overlap_summary.py <trace dir> <out.json>"""
import csv
import glob
import json
import sys

d, out = sys.argv[1], sys.argv[2]
kern = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
        for r in csv.DictReader(open(glob.glob(d + "/*kernel_trace.csv")[0]))
        if r["Kernel_Name"].startswith(("k_", "void k_"))]
copies = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
          for r in csv.DictReader(open(glob.glob(d + "/*memory_copy_trace.csv")[0]))
          if r["Direction"].endswith("HOST_TO_DEVICE")]
big = [c for c in copies if c[1] - c[0] > 1_000_000]          # > 1 ms: a batch blob
kern.sort()
rows = []
for a, b in big:
    ov, names = 0, set()
    for s, e, n in kern:
        if e <= a or s >= b:
            continue
        ov += min(b, e) - max(a, s)
        names.add(n.split("<")[0].replace("void ", ""))
    rows.append({"copy_ms": round((b - a) / 1e6, 3), "overlapped_ms": round(ov / 1e6, 3),
                 "kernels": sorted(names)})
res = {"trace": d, "batch_copies": len(rows),
       "mean_copy_ms": round(sum(r["copy_ms"] for r in rows) / max(len(rows), 1), 3),
       "mean_overlapped_ms": round(sum(r["overlapped_ms"] for r in rows) / max(len(rows), 1), 3),
       "copies": rows}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "copies"}))
