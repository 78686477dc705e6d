"""Summarise a tools/profile.sh run into profiles/: kernel stats (rocprofv3 --stats) and the
per-launch HBM traffic of k_fanout from the separate FETCH_SIZE / WRITE_SIZE passes.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in KiB;
FETCH_SIZE reports half the bytes of a wide coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane streaming stores.
Usage: python tools/summarize_profile.py gpurun_out/<run> <tag>
"""
import csv
import json
import os
import shutil
import statistics
import sys

run, tag = sys.argv[1], sys.argv[2]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(ROOT, "profiles")


def counters(path, name):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name:
            out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return out


fetch = counters(os.path.join(run, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
write = counters(os.path.join(run, "write", "write_counter_collection.csv"), "WRITE_SIZE")
stats = list(csv.DictReader(open(os.path.join(run, "kt", "kt_kernel_stats.csv"))))
bench = json.load(open(os.path.join(run, "kt_bench.json")))
avg_ns = {r["Name"]: float(r["AverageNs"]) for r in stats}
res = {"tag": tag, "kernels": {}}
for k in sorted(set(fetch) | set(write)):
    # skip the warmup launches: the bench runs warmup + steps launches, report the timed ones
    f = fetch.get(k, [])[-bench["steps"]:]
    w = write.get(k, [])[-bench["steps"]:]
    fk, wk = statistics.mean(f), statistics.mean(w)
    res["kernels"][k] = {"FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk,
                         "hbm_read_bytes": 2 * fk * 1024, "hbm_write_bytes": wk * 1024,
                         "hbm_bytes_per_launch": (2 * fk + wk) * 1024,
                         "avg_duration_ns_rocprof": avg_ns.get(k)}
# per-dispatch durations from the kernel trace: the timed launches are the last `steps`
trace = list(csv.DictReader(open(os.path.join(run, "kt", "kt_kernel_trace.csv"))))
for k in res["kernels"]:
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace if r["Kernel_Name"] == k]
    if d:
        res["kernels"][k]["avg_duration_ns_rocprof_timed"] = statistics.mean(d[-bench["steps"]:])
# the bench line's copy kernel (a run's first tick may take the join-burst kernel: every
# subscriber joins before it), matched on the truncated name rocprofv3 -T gives
want = bench["roofline"]["kernel"].split("<")[0]
fan_name = next((k for k in res["kernels"] if k == want), None) or \
    next((k for k in res["kernels"] if k.startswith("k_fanout")), None)
fan = res["kernels"].get(fan_name, {})
res["fanout_kernel"] = fan_name                              # rocprofv3 -T (truncated) name
res["bench_fanout_kernel"] = bench["roofline"]["kernel"]     # the engine's variant name (template args)
res["workload"] = {k: bench["config"].get(k) for k in ("sessions_per_gpu", "subs_per_session", "ingest", "tick_ms", "rewrite")}
if bench["config"].get("deframe_walk"):
    res["workload"]["deframe_walk"] = bench["config"]["deframe_walk"]
res["hbm_bytes_per_launch"] = fan.get("hbm_bytes_per_launch")
# the ingest side of a step: k_ingest (+ the RTSP-interleaved deframe kernels k_tcp_*)
ing = [k for k in res["kernels"] if k.startswith("k_ingest") or k.startswith("k_tcp")]
res["ingest_kernels"] = ing
res["ingest_hbm_bytes_per_launch"] = sum(res["kernels"][k]["hbm_bytes_per_launch"] for k in ing) if ing else None
res["ingest_alg_bytes_per_launch"] = bench.get("ingest", {}).get("alg_bytes_per_launch")
res["alg_bytes_per_launch"] = bench["roofline"]["alg_bytes_per_launch"]
res["bench_avg_kernel_ms"] = bench["roofline"]["avg_kernel_ms"]
res["rocprof_avg_kernel_ms"] = (avg_ns.get(fan_name) or 0) / 1e6          # all launches incl. warmup
res["rocprof_avg_kernel_ms_timed"] = fan.get("avg_duration_ns_rocprof_timed", 0) / 1e6   # the bench's timed steps
json.dump(res, open(os.path.join(prof, f"{tag}_pmc.json"), "w"), indent=1)
# the registry bench.py reads traffic from: one file per workload (ingest mode, subs, tick, rewrite)
wl = res["workload"]
key = f"{wl['ingest']}_s{wl['sessions_per_gpu']}x{wl['subs_per_session']}_t{wl['tick_ms']}" + \
      ("" if wl.get("rewrite", "identity").startswith("identity") else "_rw")
json.dump(res, open(os.path.join(prof, f"pmc_fanout_c2_{key}.json"), "w"), indent=1)
shutil.copy(os.path.join(run, "kt", "kt_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
shutil.copy(os.path.join(run, "kt_bench.json"), os.path.join(prof, f"{tag}_bench.json"))
print(json.dumps(res, indent=1))
