#!/usr/bin/env python3
"""C4 keyframe fast-start burst (BASELINE.json configs[3]) on one GPU.

The C2 stream set (1024 H.264 1080p30 4 Mb/s pushers) runs for a few ticks; then 10,000
subscribers join at once, uniformly over the sessions.  A subscriber's egress GPU is
hash(subID) % 8, so 7/8 of them land on a GPU that does not own their stream: they join a
*replica session* there, fed by a full session image (key pointer -> newest) exported by the
owner, moved once per (session, destination), and imported (edgpu_session_export /
edgpu_memcpy_peer / edgpu_session_import).  Every joiner then receives its GOP replay in the
next fan-out.

On this one-GPU box the "remote" GPU is a second engine context on the same device, so the
peer copy is a device-local copy (the kernels and the image bytes are those of a real
cross-GPU join; the xGMI transfer time is not measured here -- at ~50 GB/s per xGMI link
direction it is bytes / 50e9 s, reported as an estimate).

Timed: image export + copy + import, the burst of joins (edgpu_subscribers_add), and the
burst fan-out, bracketed by device synchronisation.  By default the GPU's owned sessions and its
replica sessions live in one context, as a rank keeps them (replica.DistReplicaLink), so the
burst is one fan-out launch; --contexts 2 keeps owner and replica in two contexts (two launches,
the owner's ~1/8 of the burst alone in its own).  One JSON line out.
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

from bench import make_batch_on_device  # noqa: E402
from easydarwin_amd import edgpu  # noqa: E402
from easydarwin_amd.workload import H264Fleet, fnv1a64  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, default=1024)
    ap.add_argument("--joins", type=int, default=10_000)
    ap.add_argument("--gpus", type=int, default=8, help="egress GPU = hash(subID) % gpus")
    ap.add_argument("--warm-ticks", type=int, default=3)
    ap.add_argument("--contexts", type=int, choices=(1, 2), default=1,
                    help="1: owned + replica sessions in one context (a rank's layout); 2: apart")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    fleet = H264Fleet(np.arange(args.sessions), tick_ms=1000)
    gen = torch.Generator(device=dev)
    gen.manual_seed(0xEA5D + 3)
    batches = [make_batch_on_device(fleet.next_batch(), dev, gen) for _ in range(args.warm_ticks)]
    torch.cuda.synchronize(dev)
    max_pk = max(b["n"] for b in batches)
    cfg = dict(video_ring_packets=8192, video_ring_bytes=16 << 20, other_ring_packets=256,
               other_ring_bytes=64 << 10, out_arena_bytes=min(args.joins * (1 << 20) * 3 // 2, 24 << 30),
               max_out_packets=args.joins * 1200, max_batch_packets=max_pk + 1, max_batch_bytes=1 << 20)
    merged = args.contexts == 1
    owner = edgpu.Context(device=0, **cfg)
    # one process per GPU serves its own shard and its replicas from one context (DistReplicaLink
    # keeps replica sessions in the rank's one context), so the owner's and the replicas' joiners
    # are one fan-out launch; --contexts 2 keeps them apart (two launches)
    replica = owner if merged else edgpu.Context(device=0, **cfg)
    sdp = fleet.sdp()
    osess = [owner.session_add(sdp) for _ in range(args.sessions)]
    rsess = [replica.session_add(sdp) for _ in range(args.sessions)]
    for b in batches:
        owner.ingest_device(b["desc"].data_ptr(), b["n"], b["seg"].data_ptr(), b["sess"].data_ptr(), b["nseg"],
                            b["blob"].data_ptr(), b["bytes"])
        owner.keyframe_index()
        owner.fanout(b["t"])
    owner.sync()
    now = batches[-1]["t"]

    subs = np.arange(args.joins)
    sess_of = subs % args.sessions
    remote = np.array([fnv1a64(f"sub{int(k)}") % args.gpus != 0 for k in subs])
    need = np.unique(sess_of[remote])                               # sessions needing a replica
    ctxs = [owner] if merged else [owner, replica]
    c0 = [c.counters() for c in ctxs]
    # the joiners' engine sessions (host bookkeeping of the bench, outside the timed region)
    osess_a, rsess_a = np.asarray(osess, dtype=np.uint32), np.asarray(rsess, dtype=np.uint32)
    own_need, rep_need = osess_a[need], rsess_a[need]
    join_sess = np.where(remote, rsess_a[sess_of], osess_a[sess_of])   # every joiner, in sub-id order
    own_join, rep_join = osess_a[sess_of[~remote]], rsess_a[sess_of[remote]]

    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    offs, _heads = owner.session_export(own_need, now)                              # size query
    total = int(offs[-1])
    src = owner.device_alloc(total)
    dst = replica.device_alloc(total)
    t1 = time.perf_counter()
    owner.session_export(own_need, now, src.ptr, src.nbytes)
    replica.memcpy_peer(dst.ptr, 0, src.ptr, total)
    replica.session_import(dst.ptr, offs, rep_need)
    t2 = time.perf_counter()
    if merged:
        owner.subscribers_add(join_sess, edgpu.TRANSPORT_UDP)
    else:
        owner.subscribers_add(own_join, edgpu.TRANSPORT_UDP)
        replica.subscribers_add(rep_join, edgpu.TRANSPORT_UDP)
    t3 = time.perf_counter()
    for c in ctxs:
        c.fanout(now)
    for c in ctxs:
        c.sync()
    torch.cuda.synchronize(dev)
    t4 = time.perf_counter()

    for c in ctxs:
        if c.stats().status:
            raise SystemExit(f"engine status {c.stats().status}")
    copy_ms = [c.kernel_times(0)[-1] for c in ctxs]                 # the fan-out copy kernel(s)
    tick_ms = [c.kernel_times(1)[-1] for c in ctxs]                 # plan + copy
    c1 = [c.counters() for c in ctxs]
    d = {k: sum(b[k] - a[k] for a, b in zip(c0, c1)) for k in ("relayed_packets", "relayed_bytes", "fanout_in_bytes")}
    relayed, rbytes = d["relayed_packets"], d["relayed_bytes"]
    # the burst's copy kernel(s) against HBM: B = out + in + 16 per packet
    alg = rbytes + d["fanout_in_bytes"] + 16 * relayed
    kms = sum(copy_ms)
    kernel = owner.fanout_kernel()
    traffic, tsrc = None, None
    pmc = os.path.join(ROOT, "profiles", "pmc_c4.json")
    if os.path.exists(pmc):
        pj = json.load(open(pmc))
        if pj.get("bench_kernel") == kernel and pj.get("contexts") == args.contexts and pj.get("joins") == args.joins:
            traffic, tsrc = pj.get("hbm_bytes_per_burst"), f"profiles/{pj.get('tag')} (rocprofv3 FETCH_SIZE/WRITE_SIZE passes)"
    res = {
        "workload": f"C4: {args.joins} joins over {args.sessions} C2 sessions after {args.warm_ticks} s, "
                    f"egress GPU = hash(subID) % {args.gpus}; remote joins served by replica sessions",
        "contexts": args.contexts,
        "layout": ("one context: the GPU's owned sessions and its replica sessions together, one fan-out launch "
                   "(as a rank's DistReplicaLink keeps them)" if merged else
                   "two contexts: owner and replica apart, one launch each"),
        "joins": args.joins, "remote_joins": int(remote.sum()), "replica_sessions": int(len(need)),
        "image_bytes": total, "image_bytes_per_session": round(total / max(len(need), 1)),
        "burst_ms": round((t4 - t1) * 1e3, 3),
        "image_export_copy_import_ms": round((t2 - t1) * 1e3, 3),
        "join_calls_ms": round((t3 - t2) * 1e3, 3),
        "burst_fanout_ms": round((t4 - t3) * 1e3, 3),
        "burst_fanout_kernel_ms": [round(x, 4) for x in copy_ms],
        "burst_tick_ms": [round(x, 4) for x in tick_ms],
        "relayed_packets": int(relayed), "relayed_bytes": int(rbytes),
        "roofline": {"bound": "hbm", "kernel": kernel, "alg_bytes": int(alg),
                     "achieved": round(alg / (kms / 1e3) / 1e9, 1) if kms else None, "peak": 8000.0, "unit": "GB/s",
                     "frac": round(alg / (kms / 1e3) / 1e9 / 8000.0, 4) if kms else None, "traffic": traffic,
                     "traffic_source": tsrc},
        "relayed_packets_per_join": round(relayed / args.joins, 1),
        "xgmi_estimate_ms_one_link": round(total / 50e9 * 1e3, 3),
        "note": "one GPU: the image comes from the same device, so its copy is device-local",
    }
    print(json.dumps(res), flush=True)
    src.free()
    dst.free()
    owner.close()
    if not merged:
        replica.close()


if __name__ == "__main__":
    main()
