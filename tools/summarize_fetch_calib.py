"""Summarizes tools/gpu_runs/gpu_r06o_fetch_calib.sh: per access pattern of tools/fetch_calib.hip,
the duration (bytes per touched line at the full stream's rate) beside FETCH_SIZE and the raw TCC
request counters; then the same raw counters for the ingest kernels.

usage: python tools/summarize_fetch_calib.py gpurun_out/r06o_calib > profiles/r06o_fetch_calib.json
"""
import csv
import glob
import json
import sys

PATTERNS = ["stream", "l128_o0_16", "l128_o48_16", "l128_o40_48", "l64_o0_16", "l256_o0_16", "l128_o0_4"]
REPS = 2            # fetch_calib 4 2: a warm-up launch + 2 per pattern under rocprofv3


def per_dispatch(d):
    """{counter: [values in dispatch order]} and the kernel names in that order."""
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    by = {}
    for r in rows:
        by.setdefault(int(r["Dispatch_Id"]), {"kernel": r["Kernel_Name"]})[r["Counter_Name"]] = float(r["Counter_Value"])
    return [by[k] for k in sorted(by)]


def calib(d):
    disp = [x for x in per_dispatch(d) if "k_fill" not in x["kernel"]]
    out = {}
    for i, p in enumerate(PATTERNS):
        runs = disp[i * (REPS + 1) + 1:(i + 1) * (REPS + 1)]
        if not runs:
            continue
        keys = [k for k in runs[0] if k != "kernel"]
        out[p] = {k: sum(r[k] for r in runs) / len(runs) for k in keys}
    return out


def main(d):
    times = {j["pattern"]: j for j in map(json.loads, open(f"{d}/time.jsonl"))}
    stream_ms = times["stream"]["ms"]
    gib = times["stream"]["bytes_loaded"]
    fetch, raw, hit = calib(f"{d}/p_fetch"), calib(f"{d}/p_raw"), calib(f"{d}/p_hit")
    res = {"buffer_bytes": gib, "patterns": {}}
    for p, t in times.items():
        lines = t["lines_touched"]
        e = {"ms": t["ms"], "lines_touched": lines, "bytes_loaded": t["bytes_loaded"],
             # the stream moves 128 B per line at its rate: a pattern as slow moved as much
             "bytes_per_line_by_time": round(128.0 * t["ms"] / stream_ms * (gib / 128) / lines, 1)}
        if p in fetch:
            e["FETCH_SIZE_bytes"] = fetch[p]["FETCH_SIZE"] * 1024
            e["FETCH_SIZE_per_line"] = round(e["FETCH_SIZE_bytes"] / lines, 2)
        if p in raw:
            e.update({k: raw[p][k] for k in raw[p]})
            e["RDREQ_per_line"] = round(raw[p]["TCC_EA0_RDREQ_sum"] / lines, 3)
        if p in hit:
            e.update({k: hit[p][k] for k in hit[p]})
        res["patterns"][p] = e
    for tag in ("tcp_raw", "desc_raw"):
        disp = per_dispatch(f"{d}/{tag}")
        ks = {}
        for x in disp:
            k = x["kernel"].split("(")[0].split("<")[0]
            ks.setdefault(k, []).append(x)
        res[tag] = {k: {c: sum(r[c] for r in v) / len(v) for c in v[0] if c != "kernel"} for k, v in ks.items()}
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
