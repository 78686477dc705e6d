#!/usr/bin/env python3
"""C5 (BASELINE.json configs[4]) on one GPU: mixed H.264 / MPEG-4 / MJPEG video with AAC / G.711
audio, jittered packet sizes (uniform 20..2059 bytes, so some are clamped at 2060 by PushPacket),
pusher RTCP SRs, and half of each session's subscribers RTSP-interleaved (TCP), half UDP.

Same step as bench.py (ingest + keyframe index + fan-out per 1-s tick, inputs resident in HBM
before timing).  The packets come from the parity generator (easydarwin_amd/synth.py), the
one that also feeds the `mixed` golden scenario; bit-exactness for this mix is covered there.
Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from easydarwin_amd import edgpu  # noqa: E402
from easydarwin_amd.synth import SEED_BASE, TrackSpec, make_sdp, session_packets  # noqa: E402

VIDEO = [("H264/90000", 96), ("MP4V-ES/90000", 97), ("JPEG/90000", 26)]
AUDIO = [("MPEG4-GENERIC/48000/2", 98), ("PCMA/8000", 8), ("PCMU/8000", 0)]


def tracks_of(g: int):
    v, a = VIDEO[g % 3], AUDIO[(g // 3) % 3]
    return [TrackSpec("video", v[0], v[1], bitrate=2_000_000, gop=60, idr_bytes=40_000, jitter_sizes=True,
                      rtcp_every_ms=1000),
            TrackSpec("audio", a[0], a[1], rtcp_every_ms=1000)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, default=1024)
    ap.add_argument("--subs", type=int, default=16)
    ap.add_argument("--ticks", type=int, default=4, help="1-s ticks generated (the first is warm-up)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    t0 = time.time()
    per_tick = [[] for _ in range(args.ticks)]
    sdps = []
    for g in range(args.sessions):
        tr = tracks_of(g)
        sdps.append(make_sdp(tr))
        for t, ch, data in session_packets(tr, args.ticks * 1000, SEED_BASE + 5000 + g, t0=(g * 7) % 33):
            k = min(int(t) // 1000, args.ticks - 1)
            per_tick[k].append((g, ch, int(t), data))
    batches = []
    for k, pk in enumerate(per_tick):
        desc, seg_off, seg_sess, blob = edgpu.build_batch(pk)
        batches.append({
            "desc": torch.from_numpy(desc.view(np.uint8)).to(dev), "n": len(desc),
            "seg": torch.from_numpy(seg_off.view(np.int32)).to(dev), "nseg": len(seg_sess),
            "sess": torch.from_numpy(seg_sess.view(np.int32)).to(dev),
            "blob": torch.from_numpy(blob).to(dev), "bytes": int(blob.nbytes), "t": (k + 1) * 1000})
    torch.cuda.synchronize(dev)
    gen_s = time.time() - t0
    max_pk = max(b["n"] for b in batches)
    max_out = max_pk * args.subs * 3 + 4096
    ctx = edgpu.Context(device=0, video_ring_packets=8192, video_ring_bytes=16 << 20, other_ring_packets=2048,
                        other_ring_bytes=1 << 20, out_arena_bytes=max(b["bytes"] for b in batches) * args.subs * 3,
                        max_out_packets=max_out, max_batch_packets=max_pk + 1, max_batch_bytes=1 << 20)
    for g in range(args.sessions):
        s = ctx.session_add(sdps[g])
        ctx.subscribers_add([s] * args.subs, [k & 1 for k in range(args.subs)])   # UDP, TCP alternating

    def step(b):
        ctx.ingest_device(b["desc"].data_ptr(), b["n"], b["seg"].data_ptr(), b["sess"].data_ptr(), b["nseg"],
                          b["blob"].data_ptr(), b["bytes"])
        ctx.keyframe_index()
        ctx.fanout(b["t"])

    step(batches[0])                                   # warm-up: subscribers start at the key / window
    ctx.sync()
    if ctx.stats().status:
        raise SystemExit(f"engine status {ctx.stats().status}")
    ctx.kernel_times(0), ctx.kernel_times(2)
    c0 = ctx.counters()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    for b in batches[1:]:
        step(b)
    ctx.sync()
    dt = time.perf_counter() - t1
    st = ctx.stats()
    if st.status:
        raise SystemExit(f"engine status {st.status}")
    c1 = ctx.counters()
    k_fan, k_ing = ctx.kernel_times(0), ctx.kernel_times(2)
    relayed = c1["relayed_packets"] - c0["relayed_packets"]
    alg = (c1["relayed_bytes"] - c0["relayed_bytes"]) + (c1["fanout_in_bytes"] - c0["fanout_in_bytes"]) + 16 * relayed
    launches = c1["fanout_launches"] - c0["fanout_launches"]
    fan_ms = float(np.mean(k_fan))
    res = {
        "workload": f"C5: {args.sessions} mixed sessions/GPU (H.264 / MPEG-4 / MJPEG 2 Mb/s video, jittered packet "
                    f"sizes 20..2059 B, AAC / PCMA / PCMU audio, pusher SRs) x {args.subs} subscribers "
                    f"(half RTSP-interleaved TCP, half UDP), 1-s ticks",
        "relayed_packets_per_s": round(relayed / dt, 1),
        "ms_per_step": round(dt / (len(batches) - 1) * 1e3, 4),
        "fanout_kernel": ctx.fanout_kernel(),
        "fanout_ms": round(fan_ms, 4), "ingest_ms": round(float(np.mean(k_ing)), 4),
        "fanout_achieved_GBps": round(alg / max(launches, 1) / (fan_ms / 1e3) / 1e9, 1),
        # the copy kernel against HBM (bench.py's roofline block; PMC traffic: tools/profile.sh)
        "roofline": {"bound": "hbm", "kernel": ctx.fanout_kernel(),
                     "alg_bytes_per_launch": int(alg / max(launches, 1)),
                     "achieved": round(alg / max(launches, 1) / (fan_ms / 1e3) / 1e9, 1), "peak": 8000.0,
                     "unit": "GB/s", "frac": round(alg / max(launches, 1) / (fan_ms / 1e3) / 1e9 / 8000.0, 4),
                     "traffic": None, "traffic_source": None},
        "ingested_packets_per_tick": int(np.mean([b["n"] for b in batches[1:]])),
        "relayed_packets_per_tick": int(relayed / (len(batches) - 1)),
        "generation_s": round(gen_s, 1),
        "data": "synthetic (easydarwin_amd/synth.py, the generator behind the `mixed` golden scenario)",
    }
    # HBM traffic per launch from the committed PMC passes of this kernel and workload
    # (tools/summarize_pmc_c5.py -> profiles/pmc_c5.json)
    pmc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_c5.json")
    if os.path.exists(pmc):
        pj = json.load(open(pmc))
        if pj.get("bench_kernel") == res["fanout_kernel"] and pj.get("workload") == res["workload"]:
            res["roofline"]["traffic"] = pj["hbm_bytes_per_launch"]
            res["roofline"]["traffic_source"] = f"profiles/pmc_c5.json ({pj['tag']}: rocprofv3 FETCH_SIZE/WRITE_SIZE passes)"
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
