#!/usr/bin/env python3
"""Socket egress throughput on the C2 stream set: can one GPU's fan-out
leave through the kernel's UDP stack in real time?

C2 in real time is 1024 H.264 1080p30 4 Mb/s pushes x 16 UDP subscribers = ~6.2 M datagrams/s
and ~8.2 GB/s per GPU.  Each step here is one `--tick-ms` tick of that input: ingest + keyframe
index + fan-out on the GPU, then edgpu_egress_send: the tick's arena is copied to pinned host
memory (PCIe) and `--threads` workers sendmmsg every datagram to its subscriber's loopback
address.  Receivers are a few bound sockets with small receive buffers that are never read, so
the receive side costs little and drops (the sender still does the whole send path).  Reports
per-step device time, copy time, send time, and whether egress keeps up with real time.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import make_batch_on_device  # noqa: E402
from easydarwin_amd import edgpu  # noqa: E402
from easydarwin_amd.workload import H264Fleet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, default=1024)
    ap.add_argument("--subs", type=int, default=16)
    ap.add_argument("--tick-ms", type=int, default=100)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--receivers", type=int, default=64)
    ap.add_argument("--dedup", type=int, default=1,
                    help="1: copy each tick's distinct bytes once (identity UDP sub-streams share their "
                         "sender's region); 0: copy the whole write-many arena (round 1)")
    ap.add_argument("--gso", type=int, default=1,
                    help="1: runs of equal-length datagrams to one subscriber leave as one UDP GSO message; "
                         "0: one datagram per message")
    ap.add_argument("--reference", action="store_true",
                    help="also time the reference's own write path on this host: oracle/_ref/ref_harness "
                         "--bench-udp (a sendto() per subscriber datagram) on the same C2 fleet, sharded over "
                         "one process per leased core")
    args = ap.parse_args()
    os.environ["EDGPU_EGRESS_DEDUP"] = str(args.dedup)     # read by edgpu_egress_create
    os.environ["EDGPU_EGRESS_GSO"] = str(args.gso)
    dev = torch.device("cuda", 0)
    fleet = H264Fleet(np.arange(args.sessions), tick_ms=args.tick_ms)
    gen = torch.Generator(device=dev)
    gen.manual_seed(0xEA5D + 5)
    batches = [make_batch_on_device(fleet.next_batch(), dev, gen) for _ in range(args.warmup + args.steps)]
    torch.cuda.synchronize(dev)
    max_pk = max(b["n"] for b in batches)
    # subscribers join before the first packet, so a tick relays about one batch per subscriber
    max_out = max_pk * args.subs * 2 + 4096
    ctx = edgpu.Context(device=0, video_ring_packets=8192, video_ring_bytes=16 << 20, other_ring_packets=256,
                        other_ring_bytes=64 << 10, out_arena_bytes=max_out * 1456, max_out_packets=max_out,
                        max_batch_packets=max_pk + 1, max_batch_bytes=1 << 20)
    eg = edgpu.Egress(ctx, args.threads)
    rx = []
    for _ in range(args.receivers):
        r = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        r.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)
        r.bind(("127.0.0.1", 0))
        rx.append(r)
    for g in range(args.sessions):
        s = ctx.session_add(fleet.sdp())
        for k in range(args.subs):
            h = ctx.subscriber_add(s, edgpu.TRANSPORT_UDP)
            port = rx[h % len(rx)].getsockname()[1]
            eg.udp(h, 0, "127.0.0.1", port, port)
    rows = []
    for i, b in enumerate(batches):
        t0 = time.perf_counter()
        ctx.ingest_device(b["desc"].data_ptr(), b["n"], b["seg"].data_ptr(), b["sess"].data_ptr(), b["nseg"],
                          b["blob"].data_ptr(), b["bytes"])
        ctx.keyframe_index()
        r = ctx.fanout(b["t"])
        ctx.sync()
        t1 = time.perf_counter()
        st = eg.send(r)
        t2 = time.perf_counter()
        if i >= args.warmup:
            rows.append(dict(gpu_ms=(t1 - t0) * 1e3, copy_ms=st.copy_ms, send_ms=st.send_ms,
                             total_ms=(t2 - t0) * 1e3, datagrams=st.udp_datagrams, bytes=st.udp_bytes,
                             copied=st.copied_bytes, dropped=st.udp_dropped))
    tot = {k: float(np.mean([r[k] for r in rows])) for k in rows[0]}
    res = {
        "workload": f"C2 stream set ({args.sessions} x 4 Mb/s H.264 1080p30) x {args.subs} UDP subs, "
                    f"{args.tick_ms}-ms ticks, egress over loopback UDP with {args.threads} threads",
        "dedup": args.dedup,
        "gso": args.gso,
        "per_tick_mean": {k: round(v, 3) for k, v in tot.items()},
        "egress_datagrams_per_s": round(tot["datagrams"] / (tot["copy_ms"] + tot["send_ms"]) * 1e3, 1),
        "egress_GBps": round(tot["bytes"] / (tot["copy_ms"] + tot["send_ms"]) / 1e6, 3),
        "copy_GBps": round(tot["copied"] / tot["copy_ms"] / 1e6, 2) if tot["copy_ms"] else None,
        "real_time_factor": round(args.tick_ms / tot["total_ms"], 3),
        "note": "loopback receivers are never read (receive-side drops); send errors are ignored as "
                "RTPStream::Write's (void)SendTo does",
    }
    eg.close()
    ctx.close()
    if args.reference:
        res["reference"] = reference_udp(args)
        if res["reference"]:
            res["egress_vs_reference_sendto"] = round(res["egress_datagrams_per_s"]
                                                      / res["reference"]["sendto_datagrams_per_s"], 3)
    print(json.dumps(res), flush=True)


def reference_udp(args) -> dict | None:
    """EasyDarwin's reflector writing every UDP subscriber datagram with a sendto() of its own (the
    reference's RTPStream::Write -> UDPSocket::SendTo, Server.tproj/RTPStream.cpp:1084-1147), each
    process to one unread loopback socket: ref_harness --bench-udp over the same C2 fleet, one process
    per leased core at once.  sendto_datagrams_per_s counts the ticks' time (ReflectPackets and the
    sends); with_push_per_s adds PushPacket."""
    import tempfile
    import bench
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(exe):
        return None
    procs_n, why = bench.baseline_cores()
    with tempfile.TemporaryDirectory(dir=os.environ.get("EDGPU_BASELINE_TMP")) as td:
        paths = bench._fleet_shards(args.sessions, args.subs, 3000, args.tick_ms, procs_n, td)
        procs = [subprocess.Popen([exe, "--bench-udp", p, "1"], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                                  text=True) for p in paths]
        outs = [json.loads(pr.communicate()[0]) for pr in procs]
        if any(pr.returncode for pr in procs):
            return None
    pk = sum(o["relayed_packets"] for o in outs)
    return {"sendto_datagrams_per_s": round(pk / max(o["reflect_seconds"] for o in outs), 1),
            "with_push_per_s": round(pk / max(o["seconds"] for o in outs), 1),
            "datagrams": pk, "processes": procs_n, "cores_note": why,
            "sample": f"oracle/_ref/ref_harness --bench-udp: the C2 fleet ({args.sessions} x {args.subs} UDP subs), "
                      f"3 s of stream at {args.tick_ms}-ms ticks, sharded over {procs_n} processes at once, "
                      f"each sending to one unread 127.0.0.1 socket; time = the longest process's"}


if __name__ == "__main__":
    main()
