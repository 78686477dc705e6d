#!/usr/bin/env python3
"""The drop-in path's throughput: libQTSSReflectorModule.so in the fake QTSS server
(tools/qtss_replay --bench) at C2 scale, next to the reference reflector on the same host.

Module side: <sessions> RTSP-interleaved H.264 1080p 4 Mb/s pushers (synthetic FU-A packets,
GOP 60, 120-KB IDR) fed through QTSS_RTSPIncomingData_Role from <threads> pusher threads,
<subs> UDP players per session, manual ticks every <tick_ms> of virtual time; the QTSS_Write
sink counts.  Reported: relayed packets/s over push + tick wall time, per-tick module-lock
hold, engine ingest / fan-out / readback / QTSS_Write time, readback (PCIe) bytes per tick
against the fan-out arena bytes per tick (what a whole-arena readback would move).

Reference module: the REFERENCE QTSSReflectorModule (oracle/_ref/libQTSSReflectorModule_ref.so) in
the same fake server at the same load and tick, its senders reflected on as many threads as the
drop-in has write threads -- the like-for-like comparison (module_vs_reference_module).

Both modules run <seconds> (default 15) of stream and are timed only after <warm-ms> (default
10 s: the reference's queues reach their 10-s packet age and recycle packets through each
socket's free queue, ReflectorStream.cpp:112-114, 1713, 2039-2047).

Reference side: oracle/_ref/ref_harness --bench-steady (EasyDarwin's reflector compiled from its
sources, memcpy sinks) on the same C2 fleet -- all <sessions> x <subs> -- at the same tick, in its
steady state, sessions sharded over one process per core (bench.py c2_reference_steady); compared
on push + reflect (with_ingest_per_s), as the module's rate counts both.

Placement (--affinity): by default every run -- the fake server with its pusher threads and either
module, and the reference reflector's processes -- runs on the CPUs of the GPU's NUMA node, as a
server is deployed next to its GPU; `none` leaves them to the scheduler (the box allows both
sockets).

Prints one JSON object.  Needs a GPU (the module initialises an edgpu context).
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# RTP packets per second one --bench pusher sends (tools/qtss_replay.cpp run_bench): a 2-s GOP of a
# 120-KB IDR (87 FU-A fragments + SPS + PPS) and 59 P frames of 14,915 B (11 fragments each)
PKT_PER_SESSION_S = (87 + 2 + 59 * 11) / 2.0


def gpu_node_cpus() -> list:
    """The CPUs of the GPU's NUMA node this process may use (edgpu_device_local_cpus), asked in a
    child process so that this one never initialises the GPU (it only starts the runs)."""
    r = subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, sys.argv[1]); "
                        "from easydarwin_amd import edgpu; print(','.join(map(str, edgpu.device_local_cpus(0))))", ROOT],
                       capture_output=True, text=True, timeout=120)
    if r.returncode or not r.stdout.strip():
        raise SystemExit(f"edgpu_device_local_cpus failed: {r.stderr.strip()[-300:]}")
    return [int(c) for c in r.stdout.strip().split(",")]


def cpu_ranges(cpus: list) -> str:
    out, i = [], 0
    cpus = sorted(cpus)
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


def module_run(args) -> dict:
    env = dict(os.environ, EDGPU_BENCH_WARM_MS=str(args.warm_ms))
    # one tick carries every session's IDR at once (all GOPs start together): 1024 x 16 x ~150 KB
    env.setdefault("EDGPU_QTSS_ARENA_MB", str(args.arena_mb))
    env.setdefault("EDGPU_QTSS_MAX_OUT_PACKETS", str(args.max_out_packets))
    env.setdefault("EDGPU_QTSS_WRITE_THREADS", str(args.write_threads))
    if args.concurrent_push:
        env["EDGPU_BENCH_CONCURRENT_PUSH"] = "1"
    cmd = [os.path.join(ROOT, "tools", "qtss_replay"), args.module,
           "--bench", str(args.sessions), str(args.subs), str(args.seconds), str(args.tick_ms), str(args.threads)]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=args.timeout)
    if r.returncode:
        raise SystemExit(f"qtss_replay --bench failed ({r.returncode}): {r.stderr.strip()[-400:]}")
    return json.loads(r.stdout)


def realtime_runs(args) -> list:
    """The module on its own ticker at the stream's real rate (qtss_replay --bench with
    EDGPU_BENCH_REALTIME=1): every frame pushed at its time, the latency from RTSPIncomingData to
    QTSS_Write of every RTP packet; a fixed tick every <tick_ms> and reflect-on-arrival at 1 and
    2 ms (EDGPU_QTSS_REFLECT_ON_ARRIVAL)."""
    out = []
    for arrival in ("0", "2", "1"):
        env = dict(os.environ, EDGPU_BENCH_REALTIME="1", EDGPU_QTSS_TICK_MSEC=str(args.tick_ms),
                   EDGPU_QTSS_REFLECT_ON_ARRIVAL=arrival)
        env.setdefault("EDGPU_QTSS_ARENA_MB", str(args.arena_mb))
        env.setdefault("EDGPU_QTSS_MAX_OUT_PACKETS", str(args.max_out_packets))
        env.setdefault("EDGPU_QTSS_WRITE_THREADS", str(args.write_threads))
        cmd = [os.path.join(ROOT, "tools", "qtss_replay"), os.path.join(ROOT, "easydarwin_amd", "libQTSSReflectorModule.so"),
               "--bench", str(args.sessions), str(args.subs), str(args.seconds), str(args.tick_ms), str(args.threads)]
        r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=args.timeout)
        if r.returncode:
            raise SystemExit(f"qtss_replay --bench realtime failed ({r.returncode}): {r.stderr.strip()[-400:]}")
        out.append(json.loads([ln for ln in r.stdout.splitlines() if '"mode": "realtime"' in ln][-1]))
    return out


def realtime_one(module: str, sessions: int, args, env_extra: dict) -> dict:
    env = dict(os.environ, EDGPU_BENCH_REALTIME="1", **env_extra)
    env.setdefault("EDGPU_QTSS_ARENA_MB", str(args.arena_mb))
    env.setdefault("EDGPU_QTSS_MAX_OUT_PACKETS", str(args.max_out_packets))
    env.setdefault("EDGPU_QTSS_WRITE_THREADS", str(args.write_threads))
    cmd = [os.path.join(ROOT, "tools", "qtss_replay"), module,
           "--bench", str(sessions), str(args.subs), str(args.seconds), str(args.tick_ms), str(args.threads)]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=args.timeout)
    if r.returncode:
        raise SystemExit(f"qtss_replay --bench realtime ({module}, {sessions}) failed ({r.returncode}): "
                         f"{r.stderr.strip()[-400:]}")
    return json.loads([ln for ln in r.stdout.splitlines() if '"mode": "realtime"' in ln][-1])


def realtime_sweep(args) -> dict:
    """Sessions 1024 -> 8192 at their real rate, the drop-in on its default ticker (reflect on
    arrival, at most every 2 ms) beside the reference module on the server's task threads (its
    senders swept every EDGPU_REF_REFLECT_MSEC = 1 ms by as many threads as the drop-in has write
    threads, oracle/ref_module_host.cpp EDGPU_REFHOST_Ticker).  A fleet is held when the RTP write
    latency's p99 is <= the bound and at least 98 % of the offered packets are written."""
    rows = {"drop-in": [], "reference": []}
    refmod = os.path.join(ROOT, "oracle", "_ref", "libQTSSReflectorModule_ref.so")
    for n in args.sweep:
        d = realtime_one(args.module, n, args, {"EDGPU_QTSS_REFLECT_ON_ARRIVAL": "2"})
        rows["drop-in"].append(d)
        print(json.dumps({"progress": "drop-in", "sessions": n, "p99": d["latency_ms"]["p99"],
                          "relayed_per_s": d["relayed_per_s"]}), file=sys.stderr, flush=True)
        if not args.no_reference and os.path.exists(refmod):
            r = realtime_one(refmod, n, args, {"EDGPU_REF_TICK_THREADS": str(args.write_threads)})
            rows["reference"].append(r)
            print(json.dumps({"progress": "reference", "sessions": n, "p99": r["latency_ms"]["p99"],
                              "relayed_per_s": r["relayed_per_s"]}), file=sys.stderr, flush=True)

    def held(rs):
        best = None
        for d in rs:
            # the offered write rate: every RTP packet to every player (the drop-in's first run sets it)
            want = d["sessions"] * d["subs"] * PKT_PER_SESSION_S
            if d["latency_ms"]["p99"] <= args.p99_ms and d["relayed_per_s"] >= 0.98 * want:
                best = d["sessions"]
        return best
    return {"p99_bound_ms": args.p99_ms, "runs": rows,
            "capacity_sessions": {k: held(v) for k, v in rows.items()}}


def reference_module_run(args, threads: int | None = None) -> dict | None:
    """The REFERENCE QTSSReflectorModule (oracle/_ref/libQTSSReflectorModule_ref.so, compiled from its
    sources) in the same fake server, same load, same pusher threads (or `threads`); its senders reflect
    on as many threads as the drop-in has write threads (EDGPU_REF_TICK_THREADS: the server's task
    threads)."""
    so = os.path.join(ROOT, "oracle", "_ref", "libQTSSReflectorModule_ref.so")
    if not os.path.exists(so):
        return None
    env = dict(os.environ, EDGPU_REF_TICK_THREADS=str(int(os.environ.get("EDGPU_QTSS_WRITE_THREADS", args.write_threads))),
               EDGPU_BENCH_WARM_MS=str(args.warm_ms))
    if args.concurrent_push:
        env["EDGPU_BENCH_CONCURRENT_PUSH"] = "1"
    cmd = [os.path.join(ROOT, "tools", "qtss_replay"), so, "--bench", str(args.sessions), str(args.subs),
           str(args.seconds), str(args.tick_ms), str(threads or args.threads)]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=args.timeout)
    if r.returncode:
        raise SystemExit(f"qtss_replay --bench (reference module) failed ({r.returncode}): {r.stderr.strip()[-400:]}")
    line = [ln for ln in r.stdout.splitlines() if '"relayed_per_s"' in ln][-1]   # (the module prints debug lines)
    d = json.loads(line)
    d["reflect_threads"] = int(env["EDGPU_REF_TICK_THREADS"])
    return d


def reference_run(args) -> dict | None:
    sys.path.insert(0, ROOT)
    import bench
    procs_n, why = bench.baseline_cores()
    d = bench.c2_reference_steady(args.sessions, args.subs, args.tick_ms, procs_n)
    if d is None:
        return None
    return {"relayed_per_s": round(d["both_per_s"], 1), "reflect_per_s": round(d["reflect_per_s"], 1),
            "ingest_per_s": round(d["ingest_per_s"], 1), "cores": procs_n, "cores_note": why,
            "relayed_packets": d["relayed_packets"],
            # one process's PushPacket time per packet (each process pushes on one thread)
            "push_us_per_packet_per_process": round(1e6 * procs_n / max(d["ingest_per_s"], 1e-9), 4),
            "sample": f"oracle/_ref/ref_harness --bench-steady: the C2 fleet, {args.sessions} sessions x {args.subs} UDP "
                      f"subs, a {bench.C2_SECONDS}-s trace replayed {bench.C2_LOOPS} times at {args.tick_ms}-ms ticks, "
                      f"counted after {bench.C2_WARM_MS // 1000} s, sharded over {procs_n} processes at once "
                      f"(memcpy sinks); relayed_per_s counts push + reflect time, as the module's does"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, default=1024)
    ap.add_argument("--subs", type=int, default=16)
    ap.add_argument("--seconds", type=float, default=15.0)
    ap.add_argument("--warm-ms", type=int, default=10_000)
    ap.add_argument("--tick-ms", type=int, default=100)
    ap.add_argument("--threads", type=int, default=8)
    # QTSS_Write threads: the box's CPU share is 16 (the reference baseline runs 16 processes)
    ap.add_argument("--write-threads", type=int, default=16)
    ap.add_argument("--arena-mb", type=int, default=4096)
    ap.add_argument("--max-out-packets", type=int, default=4 << 20)
    ap.add_argument("--timeout", type=int, default=300)
    ap.add_argument("--no-reference", action="store_true")
    # another build of the module (A/Bs)
    ap.add_argument("--module", default=os.path.join(ROOT, "easydarwin_amd", "libQTSSReflectorModule.so"))
    # the pushers push the next tick's packets while a tick runs, as a server's RTSP threads do
    # (default: pushing and ticking alternate, the conservative measure)
    ap.add_argument("--concurrent-push", action="store_true")
    # the module on its own ticker at the streams' real rate: throughput = the offered load,
    # plus the latency it adds (fixed tick vs reflect-on-arrival)
    ap.add_argument("--realtime", action="store_true")
    # --realtime-sweep: sessions 1024 -> 8192 (or --sweep) at their real rate, the drop-in on its
    # default ticker and the reference module on the server's task threads; the largest fleet each
    # holds at p99 write latency <= --p99-ms
    ap.add_argument("--realtime-sweep", action="store_true")
    ap.add_argument("--sweep", type=lambda s: [int(x) for x in s.split(",")], default=[1024, 2048, 4096, 8192])
    ap.add_argument("--p99-ms", type=float, default=10.0)
    # gpu-node: every run (the fake server with its pusher threads and either module, and the
    # reference reflector's processes) on the CPUs of the GPU's NUMA node, as a server is deployed
    # next to its GPU; none: wherever the scheduler puts them (the box allows both sockets)
    ap.add_argument("--affinity", choices=["gpu-node", "none"], default="gpu-node")
    args = ap.parse_args()
    affinity = {"mode": args.affinity}
    if args.affinity == "gpu-node":
        cpus = gpu_node_cpus()
        os.sched_setaffinity(0, cpus)                  # inherited by every run started below
        affinity.update(cpus=cpu_ranges(cpus), n_cpus=len(cpus))
    if args.realtime_sweep:
        print(json.dumps({"workload": f"C2-shaped fleets at their real rate through the QTSS module: RTSP-interleaved "
                                      f"H.264 30-fps 4 Mb/s pushers x {args.subs} UDP players, {args.threads} pusher "
                                      f"threads, {args.seconds} s timed after 1 s", "affinity": affinity,
                          **realtime_sweep(args)}))
        return
    if args.realtime:
        print(json.dumps({"workload": f"C2 at its real rate through the QTSS module: {args.sessions} RTSP-interleaved "
                                      f"H.264 30-fps pushers x {args.subs} UDP players, {args.threads} pusher threads, "
                                      f"the module's own ticker", "affinity": affinity, "runs": realtime_runs(args)}))
        return
    out = {"workload": f"C2 through the QTSS module: {args.sessions} RTSP-interleaved H.264 pushers x {args.subs} "
                       f"UDP players, {args.tick_ms}-ms ticks, {args.threads} pusher threads "
                       f"({'concurrent with' if args.concurrent_push else 'alternating with'} the ticks)",
           "write_threads": int(os.environ.get("EDGPU_QTSS_WRITE_THREADS", args.write_threads)),
           "affinity": affinity,
           "module": module_run(args)}
    m = out["module"]
    pt = m["per_tick_bytes"]
    out["readback_vs_arena"] = round(pt["readback"] / pt["arena"], 4) if pt["arena"] else None
    # The latency the tick adds over the reference's reflect on arrival (ReflectorStream.cpp:573 signals
    # the sender's socket task, :603-618 / :1676-1714 reflect at once): a packet waits for the next
    # tick (uniform over the tick period) and then for the tick's own wall time before its write.
    wall = 1000.0 * m["tick_s"] / max(m["ticks_timed"], 1)
    out["added_latency_ms"] = {"mean": round(args.tick_ms / 2 + wall, 3), "max": round(args.tick_ms + wall, 3),
                               "tick_wall_ms": round(wall, 3), "lock_hold_max_ms": m["per_tick_ms"]["hold_max"]}
    if not args.no_reference:
        out["reference_module"] = reference_module_run(args)
        if out["reference_module"]:
            out["module_vs_reference_module"] = round(m["relayed_per_s"] / out["reference_module"]["relayed_per_s"], 2)
            # its push path on one pusher thread: every pushed packet's Task::Signal takes the process-wide
            # mutex of CommonUtilitiesLib/atomic.cpp (atomic_or), so pusher threads do not scale there
            one = reference_module_run(args, threads=1)
            out["reference_module_push_us_per_packet"] = {
                f"{args.threads}_threads": out["reference_module"]["push_us_per_packet"],
                "1_thread": one["push_us_per_packet"]}
        out["reference"] = reference_run(args)
        if out["reference"]:
            out["module_vs_reference"] = round(m["relayed_per_s"] / out["reference"]["relayed_per_s"], 2)
            if out["reference"].get("push_us_per_packet_per_process"):
                out["reference_module_push_vs_harness"] = round(
                    out["reference_module_push_us_per_packet"]["1_thread"]
                    / out["reference"]["push_us_per_packet_per_process"], 2) if out.get("reference_module") else None
    print(json.dumps(out))


if __name__ == "__main__":
    main()
