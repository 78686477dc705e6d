"""Per-launch HBM traffic of tools/bench_c5.py's fan-out kernel from two rocprofv3 PMC passes
(FETCH_SIZE, WRITE_SIZE; gfx950: KiB, FETCH_SIZE doubled as in tools/summarize_profile.py), the
warm-up launch dropped.  Writes profiles/pmc_c5.json, which bench_c5.py reads for its roofline's
`traffic` when kernel and workload match.
Usage: python tools/summarize_pmc_c5.py gpurun_out/<run> <tag>   (<run>/fetch, <run>/write, <run>/c5.json)
"""
import csv
import json
import os
import statistics
import sys

run, tag = sys.argv[1], sys.argv[2]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path, name):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == name and r["Kernel_Name"].startswith("k_fanout")]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [float(r["Counter_Value"]) for r in rows][1:]          # the warm-up launch dropped


fetch = per_launch(os.path.join(run, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
write = per_launch(os.path.join(run, "write", "write_counter_collection.csv"), "WRITE_SIZE")
bench = json.load(open(os.path.join(run, "c5.json")))
fk, wk = statistics.mean(fetch), statistics.mean(write)
res = {"tag": tag, "bench_kernel": bench["fanout_kernel"], "workload": bench["workload"],
       "FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk, "launches": len(write),
       "hbm_bytes_per_launch": (2 * fk + wk) * 1024,
       "alg_bytes_per_launch": bench["roofline"]["alg_bytes_per_launch"]}
res["traffic_over_alg"] = round(res["hbm_bytes_per_launch"] / res["alg_bytes_per_launch"], 4)
json.dump(res, open(os.path.join(ROOT, "profiles", "pmc_c5.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
