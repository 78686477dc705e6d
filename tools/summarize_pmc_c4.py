"""HBM traffic of tools/bench_c4.py's burst fan-out from two rocprofv3 PMC passes (FETCH_SIZE,
WRITE_SIZE; gfx950: KiB, FETCH_SIZE doubled as in tools/summarize_profile.py): the last
`contexts` k_fanout dispatches of the run are the burst (the warm-up ticks' launches before them
serve no subscriber).  Writes profiles/pmc_c4.json, which bench_c4.py reads for its roofline's
`traffic` when kernel, layout and joins match; also the burst kernels' rocprofv3 durations.
Usage: python tools/summarize_pmc_c4.py gpurun_out/<run> <tag>   (<run>/fetch, <run>/write, <run>/kt, <run>/c4.json)
"""
import csv
import json
import os
import sys

run, tag = sys.argv[1], sys.argv[2]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
bench = json.load(open(os.path.join(run, "c4.json")))
n = bench["contexts"]


def burst(path, name):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == name and r["Kernel_Name"].startswith("k_fanout")]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [float(r["Counter_Value"]) for r in rows][-n:]


fetch = burst(os.path.join(run, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
write = burst(os.path.join(run, "write", "write_counter_collection.csv"), "WRITE_SIZE")
trace = [r for r in csv.DictReader(open(os.path.join(run, "kt", "kt_kernel_trace.csv"))) if r["Kernel_Name"].startswith("k_fanout")]
trace.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in trace][-n:]
fk, wk = sum(fetch), sum(write)
res = {"tag": tag, "bench_kernel": bench["roofline"]["kernel"], "contexts": n, "joins": bench["joins"],
       "workload": bench["workload"], "FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk,
       "hbm_bytes_per_burst": (2 * fk + wk) * 1024, "alg_bytes_per_burst": bench["roofline"]["alg_bytes"],
       "burst_kernel_ms_rocprof": dur, "burst_kernel_ms_hip_events": bench["burst_fanout_kernel_ms"]}
res["traffic_over_alg"] = round(res["hbm_bytes_per_burst"] / res["alg_bytes_per_burst"], 4)
res["frac_rocprof"] = round(res["alg_bytes_per_burst"] / (sum(dur) / 1e3) / 1e9 / 8000.0, 4)
json.dump(res, open(os.path.join(ROOT, "profiles", "pmc_c4.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
