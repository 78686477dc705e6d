#!/usr/bin/env python3
"""Relay benchmark: relayed RTP packets/s (whole node) + achieved HBM GB/s, 1080p H.264 fan-out.

One *step* = one pass of the hot path over one batch (one 1-s tick of synthetic input):
``edgpu_ingest`` + ``edgpu_keyframe_index`` + ``edgpu_fanout`` for every session of this
rank.  At N=1 the workload is BASELINE.json configs[1] (C2: 1024 H.264 1080p30 4 Mb/s
streams x 16 UDP subscribers on one MI355X).  With N ranks the global session set is
N x 1024 streams sharded by FNV-1a(stream ID) with no collective on the data path (weak
scaling); ``--subs 64`` gives the C3 per-GPU shape.

All W+K input batches are generated and made resident in HBM before timing.  Launch::

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from easydarwin_amd import edgpu  # noqa: E402
from easydarwin_amd.dist import reduce_run  # noqa: E402
from easydarwin_amd.workload import H264Fleet, owned_sessions  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md, chip table)
C2_SECONDS = 5                 # stream seconds of the CPU baseline's C2 trace (2.6 GB of packets) ...
C2_LOOPS = 4                   # ... replayed back to back on the same sessions: 20 s of stream, of which
C2_WARM_MS = 10_000            # the window after the reference's 10-s packet age counts (steady state)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def make_batch_on_device(b: dict, dev: torch.device, gen: torch.Generator):
    """Materialise one batch in HBM: random payload bytes + the synthetic RTP/FU headers."""
    n = b["n"]
    slot_bytes = b["slot_bytes"]
    slot_off = np.concatenate([[0], np.cumsum(slot_bytes)[:-1]])
    total = int(slot_bytes.sum())
    blob = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=gen)
    words = blob.view(-1, 16)
    widx = torch.from_numpy(slot_off // 16).to(dev)
    words[widx] = torch.from_numpy(b["hdr"]).to(dev)
    # bytes 16..17 of the slot: packet bytes 12..13 (FU indicator/header or NAL bytes)
    fu_pos = torch.from_numpy(slot_off + 16).to(dev)
    blob[fu_pos] = torch.from_numpy(np.ascontiguousarray(b["fu"][:, 0])).to(dev)
    blob[fu_pos + 1] = torch.from_numpy(np.ascontiguousarray(b["fu"][:, 1])).to(dev)
    desc = np.zeros(n, dtype=edgpu.PKT_DTYPE)
    desc["slot"] = slot_off // 16
    desc["len"] = b["len"]
    desc["channel"] = b["channel"]
    desc["arrival_ms"] = b["arrival"]
    d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
    d_seg = torch.from_numpy(b["seg_off"].astype(np.uint32).view(np.int32)).to(dev)
    nseg = len(b["seg_off"]) - 1
    d_sess = torch.arange(nseg, dtype=torch.int32, device=dev)
    return {"desc": d_desc, "seg": d_seg, "sess": d_sess, "blob": blob, "n": n, "nseg": nseg,
            "bytes": total, "t": b["t_end"], "in_bytes": int(b["len"].astype(np.int64).sum())}


def make_tcp_on_device(bt: dict, b: dict, dev: torch.device, read_bytes: int = 65536):
    """The same batch as the pushers' RTSP connections carry it: per session, its packets as
    '$' ch BE16(len) frames back to back in HBM, cut into `read_bytes` TCP reads (a read's
    arrival is that of the frame holding its last byte).  Built once, outside the timing."""
    flen = b["len"].astype(np.int64) + 4
    raw_off = np.concatenate([[0], np.cumsum(flen)[:-1]])
    slot_off = bt["desc"].cpu().numpy().view(edgpu.PKT_DTYPE)["slot"].astype(np.int64) * 16
    total = int(flen.sum())
    # gather: raw[raw_off_i + k] = slot bytes [slot_off_i + k] (the slot = 4-B prefix + packet)
    delta = torch.from_numpy(slot_off - raw_off).to(dev)
    idx = torch.repeat_interleave(delta, torch.from_numpy(flen).to(dev)) + torch.arange(total, device=dev)
    raw = bt["blob"][idx]
    del idx
    hdr = np.stack([np.full(len(flen), 0x24, np.uint8), b["channel"].astype(np.uint8),
                    (b["len"] >> 8).astype(np.uint8), (b["len"] & 0xFF).astype(np.uint8)], axis=1)
    pos = torch.from_numpy(raw_off).to(dev)
    hd = torch.from_numpy(hdr).to(dev)
    for k in range(4):
        raw[pos + k] = hd[:, k]
    seg = b["seg_off"].astype(np.int64)
    rows = []
    frame_end = raw_off + flen
    for s in range(len(seg) - 1):
        lo = int(raw_off[seg[s]]) if seg[s + 1] > seg[s] else 0
        hi = int(frame_end[seg[s + 1] - 1]) if seg[s + 1] > seg[s] else 0
        for o in range(lo, hi, read_bytes):
            ln = min(read_bytes, hi - o)
            last = int(np.searchsorted(frame_end, o + ln, side="left"))
            rows.append((s, ln, o, int(b["arrival"][min(last, len(flen) - 1)])))
    return {"raw": raw, "reads": np.array(rows, dtype=edgpu.TCP_READ_DTYPE), "raw_bytes": total}


def make_pinned(ctx: edgpu.Context, bt: dict):
    """The batch in pinned host memory (edgpu_host_alloc), as a host socket reader would have
    written it: descriptors, segments, sessions and the slot blob."""
    parts = {}
    for k in ("desc", "seg", "sess", "blob"):
        a = bt[k].cpu().numpy().view(np.uint8).ravel()
        hb = ctx.host_alloc(a.nbytes)
        hb.array[:] = a
        parts[k] = hb
    return parts


def run_step(ctx: edgpu.Context, bt: dict, link=None):
    if "pinned" in bt:
        p = bt["pinned"]
        ctx.ingest_pinned(p["desc"].ptr, bt["n"], p["seg"].ptr, p["sess"].ptr, bt["nseg"], p["blob"].ptr, bt["bytes"])
    elif "tcp" in bt:
        ctx.ingest_interleaved(bt["tcp"]["reads"], bt["tcp"]["raw_bytes"], device_ptr=bt["tcp"]["raw"].data_ptr())
    else:
        ctx.ingest_device(bt["desc"].data_ptr(), bt["n"], bt["seg"].data_ptr(), bt["sess"].data_ptr(),
                          bt["nseg"], bt["blob"].data_ptr(), bt["bytes"])
    ctx.keyframe_index()
    if link is not None:                # N > 1: this rank's images to its replicas' ranks, and back
        link.sync(bt["t"])
    ctx.fanout(bt["t"])


def replica_preflight(ctx, world: int, rank: int) -> dict:
    """N > 1, before the steady state: can this node's processes map each other's HBM (IPC handles,
    HSA dmabuf)?  Every rank exports a small buffer, opens the next rank's, writes / reads a word
    there and pulls it with a peer DMA copy (the mailboxes' exact mechanisms); failures are caught
    locally so every rank reaches every collective.  All ranks get the
    same verdict (the replicas run only if every rank passed)."""
    import numpy as np
    import torch.distributed as tdist
    mine, err, buf, loc = None, None, None, None
    try:
        buf = ctx.device_alloc(4096)
        loc = ctx.device_alloc(4096)
        ctx.copy_to_device(buf.ptr, np.zeros(16, np.uint8))
        mine = (ctx.ipc_export(buf.ptr), ctx.device)
    except Exception as e:                            # noqa: BLE001 -- reported in the line
        err = f"export: {type(e).__name__}: {e}"
    hs = [None] * world
    tdist.all_gather_object(hs, mine)
    nxt = hs[(rank + 1) % world]
    if err is None and nxt is not None:
        try:
            p = ctx.ipc_open(nxt[0])
            off = 8 * rank % 4096
            ctx.copy_to_device(p + off, np.array([rank + 1], np.uint64))
            ok = int(ctx.copy_to_host(p + off, 8).view(np.uint64)[0]) == rank + 1
            ctx.memcpy_peer(loc.ptr, nxt[1], p + off, 8)          # a peer DMA pull, as the replicas do
            ok = ok and int(ctx.copy_to_host(loc.ptr, 8).view(np.uint64)[0]) == rank + 1
            ctx.ipc_close(p)
            if not ok:
                err = "peer word read back wrong"
        except Exception as e:                        # noqa: BLE001
            err = f"open: {type(e).__name__}: {e}"
    elif err is None:
        err = "next rank exported no handle"
    res = [None] * world
    tdist.all_gather_object(res, err)
    tdist.barrier()
    for b in (buf, loc):
        if b is not None:
            b.free()
    errs = [e for e in res if e]
    return {"ok": not errs, "error": errs[0] if errs else None}


def replica_check(ctx, link, gids, world: int) -> dict:
    """After the timing: every replica's GOP (the CKeyFrameCache image, key packet -> newest) equals
    its owner's byte for byte (sha256, gathered)."""
    import hashlib
    import torch.distributed as tdist

    def digest(s):
        return hashlib.sha256(ctx.gop_copy(s, 0)[0]).hexdigest()
    mine = {int(g): digest(si) for si, g in enumerate(gids) if int(g) in link.wanted_by_others}
    every = [None] * world
    tdist.all_gather_object(every, mine)
    owners = {g: d for m in every for g, d in m.items()}
    ok = all(digest(s) == owners[g] for g, s in link.replica_of.items())
    res = [None] * world
    tdist.all_gather_object(res, ok)
    return {"ok": all(res), "check": "each replica's GOP image (key packet -> newest) equals its owner's (sha256)"}


def run_bounded(fn, seconds: float):
    """fn() on a thread of its own, waited for at most `seconds`: (result, hung).  An exception is
    a failed result; a hang leaves the thread behind (the caller then ends the process)."""
    import threading
    out = {}

    def work():
        try:
            out["v"] = fn()
        except Exception as e:                        # noqa: BLE001 -- reported in the line
            out["v"] = {"ok": False, "error": f"{type(e).__name__}: {e}"}
    th = threading.Thread(target=work, daemon=True)
    th.start()
    th.join(seconds)
    if th.is_alive():
        return {"ok": False, "error": f"timed out after {seconds:.0f} s"}, True
    return out["v"], False


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _sample_trace(args, n_sess=64, dur=3000, tick=100):
    """The CPU baseline's bounded sample of the bench workload: n_sess H.264 1080p 4 Mb/s
    sessions x subs UDP subscribers x dur ms at `tick`-ms ticks."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from easydarwin_amd.synth import TrackSpec, make_sdp, session_packets
    from easydarwin_amd.trace import Trace, UDP
    from scenarios import _assemble
    tracks = [TrackSpec("video", "H264/90000", 96, bitrate=4_000_000, gop=60, idr_bytes=120_000)]
    tr = Trace()
    per = []
    for s in range(n_sess):
        tr.add_session(make_sdp(tracks))
        per.append(session_packets(tracks, dur, 0xEA5D + 1 + s, t0=(s * 7) % 33))
    joins = [(0, s, s * args.subs + k, UDP) for s in range(n_sess) for k in range(args.subs)]
    _assemble(tr, per, tick, dur, joins)
    return tr


def _shard(tr, k: int, n: int):
    """Sessions s with s % n == k (renumbered), their events, and every TICK."""
    from easydarwin_amd.trace import BLOCK, JOIN, PKT, Trace
    keep = {s: i for i, s in enumerate(range(k, len(tr.sdps), n))}
    out = Trace(sdps=[tr.sdps[s] for s in keep])
    for ev in tr.events:
        if ev[0] in (PKT, JOIN):
            if ev[2] in keep:
                out.events.append((ev[0], ev[1], keep[ev[2]]) + tuple(ev[3:]))
        elif ev[0] != BLOCK:
            out.events.append(ev)
    return out


def baseline_cores() -> tuple[int, str]:
    """The host cores the CPU baseline runs on: the process's affinity mask, capped by the CPU share
    the GPU box leases to a one-GPU job (it exports OMP_NUM_THREADS = that share); the reason is
    stated in the line when fewer than the CPU's cores are used."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    n = min(aff, share) if share > 0 else aff
    why = (f"affinity mask {aff} CPUs of {os.cpu_count()}; the box leases {share} CPUs to a one-GPU job "
           f"(OMP_NUM_THREADS={share}), so {n} processes" if n < (os.cpu_count() or n) else
           f"every CPU of the host ({n})")
    return n, why


def _fleet_shards(n_sess: int, subs: int, dur_ms: int, tick_ms: int, nshards: int, td: str) -> list[str]:
    """The bench workload itself as reference-harness traces: the C2 fleet (easydarwin_amd/workload.py
    H264Fleet, the same generator as the GPU steps) for `dur_ms` at `tick_ms`-ms ticks, every session
    with `subs` UDP subscribers joined at t = 0, sessions s = k mod nshards in shard k (renumbered
    s // nshards).  Packets carry the synthetic RTP / FU-A headers; the rest of each payload is zero
    (the reflector only moves it).  Written vectorised (trace.py format, version 1)."""
    import struct as st
    from easydarwin_amd.workload import H264Fleet
    fleet = H264Fleet(np.arange(n_sess), tick_ms=tick_ms)
    sdp = fleet.sdp().encode()
    files = []
    for k in range(nshards):
        mine = len(range(k, n_sess, nshards))
        f = open(os.path.join(td, f"c2_{k}.edtr"), "wb")
        f.write(b"EDTR" + st.pack("<II", 1, mine) + (st.pack("<I", len(sdp)) + sdp) * mine)
        files.append(f)
    rec = np.dtype([("type", "u1"), ("t", "<i8"), ("session", "<u4"), ("channel", "u1"), ("len", "<u4")])
    for tick in range(0, dur_ms + 1, tick_ms):
        b = fleet.next_batch() if tick < dur_ms else None
        if tick == 0:                                 # players join before the first tick
            for k in range(nshards):
                mine = len(range(k, n_sess, nshards))
                j = np.zeros(mine * subs, dtype=[("type", "u1"), ("t", "<i8"), ("session", "<u4"), ("sub", "<u4"),
                                                  ("tr", "u1"), ("ua", "u1")])
                j["type"] = 2
                j["session"] = np.repeat(np.arange(mine), subs)
                j["sub"] = np.arange(mine * subs)
                files[k].write(j.tobytes())
        tick_rec = st.pack("<Bq", 3, tick)
        if tick > 0 and prev is not None:
            sess = np.repeat(np.arange(n_sess), np.diff(prev["seg_off"].astype(np.int64)))
            order = np.argsort(prev["arrival"], kind="stable")   # arrival order across sessions
            ln = prev["len"].astype(np.int64)
            for k in range(nshards):
                sel = order[(sess[order] % nshards) == k]
                n = len(sel)
                if n == 0:                            # (short ticks: a shard may push nothing in one)
                    continue
                hdr = np.zeros(n, dtype=rec)
                hdr["type"] = 1
                hdr["t"] = prev["arrival"][sel]
                hdr["session"] = sess[sel] // nshards
                hdr["len"] = ln[sel]
                size = 18 + ln[sel]
                off = np.concatenate([[0], np.cumsum(size)[:-1]])
                out = np.zeros(int(size.sum()), dtype=np.uint8)
                out[off[:, None] + np.arange(18)] = hdr.view(np.uint8).reshape(n, 18)
                out[off[:, None] + 18 + np.arange(12)] = prev["hdr"][sel, 4:16]
                out[off[:, None] + 30 + np.arange(2)] = prev["fu"][sel]
                files[k].write(out.tobytes())
        if tick > 0:
            for f in files:
                f.write(tick_rec)
        prev = b
    for f in files:
        f.write(b"\x00")
        f.close()
    return [f.name for f in files]


def _parallel_bench(exe: str, mode: str, paths: list[str], target_s: float, extra=()):
    """Every shard replayed by its own process at once, each repeating its replay to about
    `target_s` seconds: (relayed packets, relayed bytes, longest process seconds, repeats)."""
    probe = json.loads(subprocess.run([exe, mode, paths[0], *extra, "1"], capture_output=True, text=True,
                                      check=True).stdout)
    rep = int(max(1, min(2000, target_s / max(probe["seconds"], 1e-4))))
    procs = [subprocess.Popen([exe, mode, p, *extra, str(rep)], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                              text=True) for p in paths]
    outs = [json.loads(pr.communicate()[0]) for pr in procs]
    if any(pr.returncode for pr in procs):
        return None
    return (sum(o["relayed_packets"] for o in outs), sum(o["relayed_bytes"] for o in outs),
            max(o["seconds"] for o in outs), rep)


def _parallel_steady(exe: str, paths: list[str], loops: int = C2_LOOPS, warm_ms: int = C2_WARM_MS):
    """Every shard replayed by its own process at once in the harness's steady-state mode
    (ref_harness --bench-steady): `loops` back-to-back replays on the same sessions, counted from
    virtual time warm_ms.  Returns the per-process results, or None."""
    procs = [subprocess.Popen([exe, "--bench-steady", p, str(loops), str(warm_ms)], stdout=subprocess.PIPE,
                              stderr=subprocess.DEVNULL, text=True) for p in paths]
    outs = [pr.communicate()[0] for pr in procs]
    if any(pr.returncode for pr in procs):
        return None
    return [json.loads(o) for o in outs]


def _reference_replay(args, tick: int, procs_n: int, mode: str = "--bench"):
    """The cache-resident extra line (round 3's sample): 64 sessions x 3 s at `tick`-ms ticks,
    sharded over procs_n processes: (relayed packets, relayed bytes, longest seconds, repeats)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    tr = _sample_trace(args, tick=tick)
    with tempfile.TemporaryDirectory() as td:
        paths = []
        for k in range(procs_n):
            p = os.path.join(td, f"s{k}.edtr")
            _shard(tr, k, procs_n).write(p)
            paths.append(p)
        return _parallel_bench(exe, mode, paths, 1.5)


def _steady_summary(outs: list[dict]) -> dict:
    """Aggregate of the processes of one --bench-steady run (all ran at once): the reflect loop's
    rate is the sum of each process's relayed packets over its own reflect time, the ingest's the
    sum of its pushes over its PushPacket time."""
    return {"reflect_per_s": sum(o["relayed_packets"] / max(o["reflect_seconds"], 1e-9) for o in outs),
            "reflect_GBps": sum(o["relayed_bytes"] / max(o["reflect_seconds"], 1e-9) for o in outs) / 1e9,
            "ingest_per_s": sum(o["pushed_packets"] / max(o["push_seconds"], 1e-9) for o in outs),
            "relayed_packets": sum(o["relayed_packets"] for o in outs),
            "pushed_packets": sum(o["pushed_packets"] for o in outs),
            "reflect_seconds_max": max(o["reflect_seconds"] for o in outs),
            "push_seconds_max": max(o["push_seconds"] for o in outs),
            "both_per_s": sum(o["relayed_packets"] / max(o["reflect_seconds"] + o["push_seconds"], 1e-9) for o in outs)}


def c2_reference_steady(sessions: int, subs: int, tick_ms: int, procs_n: int) -> dict | None:
    """EasyDarwin's reflector (ref_harness --bench-steady) on the C2 fleet at `tick_ms` ticks, in its
    steady state, sessions sharded over procs_n processes running at once (also tools/bench_module.py's
    reference)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(exe):
        return None
    with tempfile.TemporaryDirectory(dir=os.environ.get("EDGPU_BASELINE_TMP")) as td:
        t0 = time.time()
        paths = _fleet_shards(sessions, subs, C2_SECONDS * 1000, tick_ms, procs_n, td)
        gen_s = time.time() - t0
        trace_gb = sum(os.path.getsize(p) for p in paths) / 1e9
        outs = _parallel_steady(exe, paths)
    if outs is None:
        return None
    d = _steady_summary(outs)
    d.update(gen_s=gen_s, trace_gb=trace_gb, procs=procs_n, tick_ms=tick_ms)
    return d


def cpu_baseline_reference(args) -> dict | None:
    """The REFERENCE reflector itself (oracle/_ref/ref_harness: EasyDarwin's ReflectorStream /
    ReflectorSender / RTPSessionOutput compiled from its sources, fake QTSS server, memcpy sinks) on
    the bench's own C2 workload -- all args.sessions sessions x args.subs UDP players, sessions sharded
    over one process per leased core, all running at once -- in its STEADY STATE (--bench-steady): the
    C2_SECONDS-s trace replayed C2_LOOPS times back to back on the same sessions and players, only
    what happens after C2_WARM_MS counted (the reference's queues have reached their 10-s packet age,
    ReflectorStream.cpp:112-114, and recycle packets through each socket's free queue, :1713,
    2039-2047), at 100-ms ticks (the reflector's own wakeup scale, RS.cpp:1125-1131).  value = the
    reflect loop's rate (ReflectPackets alone); the ingest (PushPacket) is timed apart
    and reported beside it.  Extra lines: the same at the GPU step's 1000-ms tick, a real sendto() per
    subscriber packet, and the clean-room restatement."""
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(exe):
        return None
    procs_n, why = baseline_cores()
    dur = C2_SECONDS * 1000
    with tempfile.TemporaryDirectory(dir=os.environ.get("EDGPU_BASELINE_TMP")) as td:
        t0 = time.time()
        paths = _fleet_shards(args.sessions, args.subs, dur, 100, procs_n, td)
        gen_s = time.time() - t0
        trace_gb = sum(os.path.getsize(p) for p in paths) / 1e9
        s100 = _parallel_steady(exe, paths)
        rudp = _parallel_bench(exe, "--bench-udp", paths, 3.0)
        port = os.path.join(ROOT, "oracle", "relay_model")
        rport = _parallel_bench(port, "--bench", paths, 5.0, extra=("1",)) if os.path.exists(port) else None
        for p in paths:
            os.remove(p)
        paths1 = _fleet_shards(args.sessions, args.subs, dur, 1000, procs_n, td)
        s1000 = _parallel_steady(exe, paths1)
    if s100 is None:
        return None
    d = _steady_summary(s100)
    out = {"value": round(d["reflect_per_s"], 1), "unit": "relayed RTP packets/s", "cores": procs_n, "kind": "reference",
           "cpu_model": cpu_model(), "cores_note": why, "GBps": round(d["reflect_GBps"], 3), "tick_ms": 100,
           "ingest_per_s": round(d["ingest_per_s"], 1), "with_ingest_per_s": round(d["both_per_s"], 1),
           "sample": f"EasyDarwin's reflector (oracle/_ref/ref_harness --bench-steady, compiled from the reference "
                     f"sources) on the bench's C2 workload itself: {args.sessions} H.264 1080p 4 Mb/s sessions x "
                     f"{args.subs} UDP subs, a {C2_SECONDS}-s trace ({trace_gb:.2f} GB, generated in {gen_s:.0f} s) "
                     f"replayed {C2_LOOPS} times back to back on the same sessions at 100-ms ticks, counted after "
                     f"{C2_WARM_MS // 1000} s of stream (steady state: packets recycled through each socket's free "
                     f"queue), sessions sharded over {procs_n} processes at once; value = ReflectPackets alone "
                     f"({d['relayed_packets']} relayed packets), PushPacket timed apart (ingest_per_s; "
                     f"with_ingest_per_s: both) (memcpy sinks)"}
    if s1000 is not None:
        d1 = _steady_summary(s1000)
        out["tick_1000ms"] = {"value": round(d1["reflect_per_s"], 1), "GBps": round(d1["reflect_GBps"], 3),
                              "ingest_per_s": round(d1["ingest_per_s"], 1), "relayed_packets": d1["relayed_packets"]}
    if rudp is not None:            # the full write path: one sendto() per subscriber packet
        pku, byu, secsu, repu = rudp
        out["with_udp_sockets"] = {"value": round(pku / secsu, 1), "unit": "datagrams/s",
                                   "GBps": round(byu / secsu / 1e9, 3), "relayed_packets": pku,
                                   "seconds": round(secsu, 3), "repeat": repu, "tick_ms": 100,
                                   "sink": "one unread 127.0.0.1 UDP socket per process"}
    if rport is not None:          # the clean-room restatement on the same shards
        pkp, byp, secsp, repp = rport
        out["restatement"] = {"value": round(pkp / secsp, 1), "cores": procs_n, "kind": "port",
                              "sample": f"oracle/relay_model --bench, one thread per process, the same shards, "
                                        f"{repp} replays each"}
    return out


def cpu_baseline(args) -> dict | None:
    """The CPU restatement (oracle/relay_model --bench, memcpy sinks) on the same C2 workload,
    one process per leased core."""
    exe = os.path.join(ROOT, "oracle", "relay_model")
    if not os.path.exists(exe):
        try:
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        except Exception:
            return None
    if not os.path.exists(exe):
        return None
    procs_n, why = baseline_cores()
    with tempfile.TemporaryDirectory(dir=os.environ.get("EDGPU_BASELINE_TMP")) as td:
        paths = _fleet_shards(args.sessions, args.subs, C2_SECONDS * 1000, 100, procs_n, td)
        r = _parallel_bench(exe, "--bench", paths, 5.0, extra=("1",))
    if r is None:
        return None
    pk, by, secs, rep = r
    return {"value": round(pk / secs, 1), "unit": "relayed RTP packets/s", "cores": procs_n, "kind": "port",
            "cpu_model": cpu_model(), "cores_note": why, "GBps": round(by / secs / 1e9, 3),
            "sample": f"oracle/relay_model --bench (one thread per process) on the C2 workload: {args.sessions} sessions x "
                      f"{args.subs} UDP subs x {C2_SECONDS} s at 100-ms ticks, sharded over {procs_n} processes, "
                      f"{rep} replays each; {pk} relayed packets in {secs:.2f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)   # C2: a 10-s window of 1-s batches
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--sessions", type=int, default=1024, help="sessions per GPU")
    ap.add_argument("--subs", type=int, default=16, help="UDP subscribers per session")
    ap.add_argument("--tick-ms", type=int, default=1000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ingest", choices=["desc", "tcp", "host"], default="desc",
                    help="desc: packets handed over as descriptors + slots in HBM (edgpu_ingest, the "
                         "reflector's per-packet PushPacket boundary); tcp: the pushers' RTSP-interleaved TCP "
                         "reads in HBM, deframed on the GPU (edgpu_ingest_interleaved); host: the batches in "
                         "pinned host memory, copied over PCIe on the copy stream beside the previous fan-out "
                         "(EDGPU_PTR_PINNED) -- a separate line, PCIe-bound")
    ap.add_argument("--rewrite-same-ssrc", action="store_true",
                    help="diagnostic: every subscriber's SSRC overridden with its stream's own SSRC, so the "
                         "copy kernel takes its patch path while the bytes stay the identity's")
    ap.add_argument("--rewrite", action="store_true",
                    help="per-output rewrite stage on every subscriber (seq/ts deltas + SSRC override, "
                         "edgpu_subscriber_rewrite); the reference's parity mode is the identity (default)")
    ap.add_argument("--timing-steps", type=int, default=3,
                    help="steps after the timed region that record every timing event (the ingest, "
                         "keyframe and plan durations of the line)")
    ap.add_argument("--all-timing-events", action="store_true",
                    help="record every timing event inside the timed steps too (the ingest / keyframe / "
                         "plan durations then come from them; each event costs the step 4-8 us)")
    ap.add_argument("--replicas", type=int, default=64,
                    help="N > 1: sessions of the next rank each rank replicates in the steady state (BASELINE "
                         "C4: subscribers whose egress GPU is not the stream's owner), fed every step through "
                         "peer mailboxes (xGMI, no collective); 0: none")
    ap.add_argument("--replica-subs", type=int, default=1, help="UDP subscribers per replica session")
    ap.add_argument("--ring-mb", type=int, default=16,
                    help="diagnostic: initial video ring MiB per sender (default 16; recorded in the line)")
    ap.add_argument("--no-ring-growth", action="store_true", help="diagnostic: rings keep their initial sizes")
    ap.add_argument("--ablation-study", action="store_true",
                    help="allow EDGPU_ABLATE (timing experiments that skip work): the line is then not a "
                         "valid measurement and says so")
    args = ap.parse_args()

    # Engine switches that change what is measured are recorded in the line; EDGPU_ABLATE skips
    # work inside the timed region, so a bench under it is refused unless it is an ablation study.
    knobs = {k: os.environ[k] for k in ("EDGPU_TCP_WALK", "EDGPU_TCP_SEG", "EDGPU_FANOUT", "EDGPU_INGEST_DEPTH", "EDGPU_INGEST", "EDGPU_INGEST_TCP", "EDGPU_INGEST_THREADS", "EDGPU_ABLATE",
                                        "EDGPU_POISON", "EDGPU_LIB") if k in os.environ}
    if "EDGPU_ABLATE" in knobs and not args.ablation_study:
        raise SystemExit("EDGPU_ABLATE is set: ablations skip work in the timed region (use --ablation-study)")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    dist = None
    # EDGPU_BENCH_BACKEND=gloo: a rehearsal of the N-rank path with several ranks sharing the GPUs
    # there are (rank r on GPU r % count, host-side reductions); the driver's runs use RCCL
    backend = os.environ.get("EDGPU_BENCH_BACKEND", "nccl")
    if backend not in ("nccl", "gloo"):
        raise SystemExit(f"EDGPU_BENCH_BACKEND={backend}: nccl or gloo")
    if backend == "gloo":
        local = local % max(torch.cuda.device_count(), 1)
    # EDGPU_BENCH_FORCE_PG=1: the process group (RCCL, barriers, the device-side reduction) even at
    # world size 1 -- the driver's N-rank code path exercised on a one-GPU box
    force_pg = os.environ.get("EDGPU_BENCH_FORCE_PG") == "1"
    if world > 1 or force_pg:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)

    if rank == 0:
        log(f"[bench] C3 (BASELINE configs[2], 8192 streams x 64 subscribers over 8 GPUs): "
            f"python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 "
            f"bench.py --gpus 8 --subs 64   (this run: --subs {args.subs}, {world} rank(s))")
    # every rank owns exactly args.sessions streams of the hash-sharded population (weak scaling)
    gids = owned_sessions(args.sessions, rank, world) if world > 1 else np.arange(args.sessions)
    fleet = H264Fleet(gids, tick_ms=args.tick_ms)
    steps, warm = args.steps, args.warmup
    extra = 0 if args.all_timing_events else args.timing_steps
    log(f"[bench] rank {rank}/{world}: {len(gids)} sessions x {args.subs} subs, generating {steps + warm + extra} batches")
    t_gen = time.time()
    gen = torch.Generator(device=dev)
    gen.manual_seed(0xEA5D + rank)
    batches = []
    for _ in range(steps + warm + extra):
        b = fleet.next_batch()
        bt = make_batch_on_device(b, dev, gen)
        if args.ingest == "tcp":
            bt["tcp"] = make_tcp_on_device(bt, b, dev)
            bt.pop("blob")
            bt["raw_bytes"] = bt["tcp"]["raw_bytes"]
        batches.append(bt)
    torch.cuda.synchronize(dev)
    log(f"[bench] generated in {time.time() - t_gen:.1f}s; max batch {max(b['n'] for b in batches)} pkts, "
        f"{max(b['bytes'] for b in batches) / 2**20:.0f} MiB")

    # Output capacity per tick: every subscriber gets at most the packets of one batch (the
    # first fan-out replays key pointer -> newest, which lies inside batch 0 at that point).
    max_pk = max(b["n"] for b in batches)
    max_out = int(max(b["n"] for b in batches) * args.subs * 1.05) + 1024
    max_arena = int(max(b["bytes"] for b in batches) * args.subs * 1.05) // 16 * 16 + (1 << 20)
    ring_cfg = {"ring_growth": edgpu.FALSE} if args.no_ring_growth else {}
    ctx = edgpu.Context(device=local, video_ring_packets=8192, video_ring_bytes=args.ring_mb << 20, **ring_cfg,
                        other_ring_packets=256, other_ring_bytes=64 << 10,
                        out_arena_bytes=max_arena, max_out_packets=max_out,
                        max_batch_packets=max_pk + 1,
                        max_batch_bytes=(max(b["bytes"] for b in batches) + (1 << 20)) if args.ingest in ("tcp", "host")
                        else 1 << 20)
    if args.ingest == "host":
        for bt in batches:
            bt["pinned"] = make_pinned(ctx, bt)
            bt.pop("blob")
        torch.cuda.empty_cache()
    for si, _ in enumerate(gids):
        s = ctx.session_add(fleet.sdp())
        for _k in range(args.subs):
            h = ctx.subscriber_add(s, edgpu.TRANSPORT_UDP)
            if args.rewrite_same_ssrc:      # the patch path runs, the bytes stay the identity's
                ctx.subscriber_rewrite(h, 0, ssrc=int(fleet.ssrc[si]))
            elif args.rewrite:
                ctx.subscriber_rewrite(h, 0, seq_delta=h * 7919 + 1, ts_delta=h * 0x9E3779B1, ssrc=0x5EED0000 + h)
    # N > 1: BASELINE C4's steady state inside the timed steps -- each rank replicates the first
    # --replicas sessions of the next rank (subscribers whose egress GPU is not the owner's), joined
    # here (the collective: mailbox handles) and fed every step through peer mailboxes (no collective)
    link, rep = None, None
    if dist and world > 1 and args.replicas > 0:
        pre = replica_preflight(ctx, world, rank)
        rep = {"preflight": pre}
        if pre["ok"]:
            from easydarwin_amd.replica import DistReplicaLink
            link = DistReplicaLink(ctx, world, rank, lockstep=False)
            for si, g in enumerate(gids):
                link.own(int(g), si)
            for g in owned_sessions(args.sessions, (rank + 1) % world, world)[:args.replicas]:
                rs = link.want(int(g), fleet.sdp())
                for _k in range(args.replica_subs):
                    ctx.subscriber_add(rs, edgpu.TRANSPORT_UDP)
            link.connect()

    for i in range(warm):
        run_step(ctx, batches[i], link)
    ctx.sync()
    st = ctx.stats()
    if st.status != 0:
        raise SystemExit(f"engine status {st.status} after warmup")
    ctx.kernel_times(0), ctx.kernel_times(1), ctx.kernel_times(2), ctx.kernel_times(3)
    c0 = ctx.counters()
    # The timed steps record only the fan-out copy kernel's event pair (the roofline's duration):
    # every event is a marker the stream waits on, 4-8 us of idle GPU each
    # (profiles/r03ak_timing_events_ab/).  The ingest / keyframe / plan durations come from
    # `extra` steps after the timed region, with every event recorded.
    ctx.set_timing(ctx.TIMING_ALL if args.all_timing_events else ctx.TIMING_FANOUT)

    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    x0 = (link.sync_s, link.bytes_sent, sum(mb.wait_s for mb, _ in list(link.out.values()) + list(link.inbox.values()))) \
        if link else None
    t0 = time.perf_counter()
    for i in range(warm, warm + steps):
        run_step(ctx, batches[i], link)
    ctx.sync()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    x1 = (link.sync_s, link.bytes_sent, sum(mb.wait_s for mb, _ in list(link.out.values()) + list(link.inbox.values()))) \
        if link else None

    c1 = ctx.counters()
    st = ctx.stats()
    if st.status != 0:
        raise SystemExit(f"engine status {st.status}")
    k_fan = ctx.kernel_times(0)
    if extra:
        ctx.set_timing(ctx.TIMING_ALL)
        for i in range(warm + steps, warm + steps + extra):
            run_step(ctx, batches[i], link)
        ctx.sync()
        if ctx.stats().status != 0:
            raise SystemExit("engine status after the timing steps")
        ctx.kernel_times(0)
    k_tick = ctx.kernel_times(1)
    k_ing = ctx.kernel_times(2)
    k_key = ctx.kernel_times(3)
    relayed = c1["relayed_packets"] - c0["relayed_packets"]
    out_bytes = c1["relayed_bytes"] - c0["relayed_bytes"]
    in_bytes = c1["fanout_in_bytes"] - c0["fanout_in_bytes"]
    launches = c1["fanout_launches"] - c0["fanout_launches"]
    alg_bytes = out_bytes + in_bytes + 16 * relayed      # SURVEY.md §8.d per-launch definition
    per_step = {"kernel_launches": round((c1["kernel_launches"] - c0["kernel_launches"]) / steps, 2),
                "host_syncs": round((c1["host_syncs"] - c0["host_syncs"]) / steps, 2),
                "timing_events": 2 if not args.all_timing_events else None}

    dt, (relayed_all, out_all) = reduce_run(dt, [relayed, out_bytes], device=dev if backend == "nccl" else None,
                                          force=force_pg)
    # N > 1: the replicas' GOPs against their owners' (after the timing; bounded: a hung check is
    # reported and the process ends without waiting for it), and the steady-state exchange's cost
    xdev, hung = None, False
    if dist and world > 1 and rep is not None:
        if link is not None:
            def check():
                torch.cuda.set_device(local)          # (a thread of its own: HIP's device is per thread)
                return replica_check(ctx, link, gids, world)
            xdev, hung = run_bounded(check, 120.0)
            if not hung:
                per = [None] * world
                dist.all_gather_object(per, ((x1[0] - x0[0]) / steps, (x1[1] - x0[1]) / steps, (x1[2] - x0[2]) / steps))
                rep.update({
                    "sessions_per_rank": args.replicas, "subs_each": args.replica_subs,
                    "exchange_ms_per_step": round(1e3 * max(p[0] for p in per), 4),
                    "peer_wait_ms_per_step": round(1e3 * max(p[2] for p in per), 4),
                    "image_bytes_per_step": int(sum(p[1] for p in per)),
                    "transport": "peer mailboxes: images in the owners' HBM (IPC handles at the join), header "
                                 "words in shared memory; the replica's GPU imports over xGMI; no collective "
                                 "inside the timed steps",
                    "check": xdev})
                dist.barrier()                        # every rank is done with every mailbox
                link.close()
        else:
            xdev = {"ok": False, "error": rep["preflight"]["error"], "replicas": "skipped: IPC preflight failed"}

    # a failed or hung check may leave other ranks inside a collective: end without tearing the
    # process group down (which could wait on them)
    bail = hung or (xdev is not None and not xdev.get("ok"))
    if rank != 0:
        if bail:
            os._exit(0)
        if dist:
            dist.destroy_process_group()
        return

    fan_ms = float(np.mean(k_fan)) if k_fan else float("nan")
    achieved = (alg_bytes / max(launches, 1)) / (fan_ms / 1e3) / 1e9
    # HBM traffic per launch from the committed rocprofv3 PMC passes of exactly this kernel
    # variant and workload (tools/profile.sh + tools/summarize_profile.py); null otherwise
    traffic, traffic_source = None, None
    rewrite_desc = ("SSRC override with the stream's own SSRC (diagnostic: patch path, identity bytes)"
                    if args.rewrite_same_ssrc else
                    "per-subscriber seq/ts/SSRC" if args.rewrite else "identity (reference parity mode)")
    ing_traffic = None
    # the deframe walk's shape (edgpu_engine.cpp: EDGPU_TCP_WALK / EDGPU_TCP_SEG, segments of 4 by
    # default): part of the workload a traffic profile was taken on
    deframe_walk = None
    if args.ingest == "tcp":
        w = {"0": "parallel", "1": "serial", "2": "seg"}.get(os.environ.get("EDGPU_TCP_WALK", "seg"),
                                                             os.environ.get("EDGPU_TCP_WALK", "seg"))
        deframe_walk = f"seg{max(int(os.environ.get('EDGPU_TCP_SEG', '4')), 1)}" if w == "seg" else \
            ("serial" if w == "serial" else "parallel")
    for pmc in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_fanout_c2*.json"))):
        if world != 1:
            break
        try:
            pj = json.load(open(pmc))
            wl = pj.get("workload", {})
            if (pj.get("bench_fanout_kernel") == ctx.fanout_kernel() and wl.get("sessions_per_gpu") == args.sessions
                    and wl.get("subs_per_session") == args.subs and wl.get("ingest") == args.ingest
                    and wl.get("tick_ms", 1000) == args.tick_ms and wl.get("deframe_walk") == deframe_walk
                    and wl.get("rewrite", "identity (reference parity mode)") == rewrite_desc):
                traffic = pj.get("hbm_bytes_per_launch")
                ing_traffic = pj.get("ingest_hbm_bytes_per_launch")
                traffic_source = f"profiles/{pj.get('tag')}_pmc.json (rocprofv3 FETCH_SIZE/WRITE_SIZE passes)"
                break
        except Exception:
            traffic = None
    # the ingest side of a step (k_ingest, + the deframe kernels for RTSP-interleaved reads):
    # algorithmic bytes = packet bytes read (slots of the batch blob + 16-B descriptors, or the
    # '$'-framed TCP bytes) + slots written + 32-B packet metadata written
    timed = batches[warm:warm + steps]
    npk = float(np.mean([bt["n"] for bt in timed]))
    slot_b = float(np.mean([bt["bytes"] for bt in timed]))
    read_b = float(np.mean([bt["raw_bytes"] for bt in timed])) if args.ingest == "tcp" else slot_b + 16 * npk
    ing_alg = read_b + slot_b + 32 * npk
    ing_ms = float(np.mean(k_ing)) if k_ing else float("nan")
    ing_ach = ing_alg / (ing_ms / 1e3) / 1e9
    ingest = {"kernels": "k_ingest + k_tcp_* deframe" if args.ingest == "tcp" else "k_ingest",
              # HIP events on the context stream: with RTSP-interleaved reads the deframe kernels
              # run on a second stream beside the previous tick's fan-out (the host reads their
              # report, then enqueues k_ingest), so this is the time the ingest adds to the step
              "timing": ("exposed: the deframe runs beside the previous tick's fan-out; the context stream "
                         "sees k_ingest" if args.ingest == "tcp" else "k_ingest launch duration"),
              "alg_bytes_per_launch": int(ing_alg), "avg_ms": round(ing_ms, 4), "achieved": round(ing_ach, 1),
              "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ing_ach / HBM_PEAK_GBS, 4),
              "traffic": ing_traffic, "traffic_source": traffic_source if ing_traffic else None}
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline_reference(args)
        if cpu is None:             # no reference build travelled with the tree: the restatement
            cpu = cpu_baseline(args)
    res = {
        "metric": "relayed RTP packets/sec (whole node) + achieved HBM GB/s, 1080p H.264 fan-out",
        "value": round(relayed_all / dt, 1),
        "unit": "relayed RTP packets/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warm,
        "ms_per_step": round(dt / steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (PCG64 RTP/H.264 FU-A headers, GPU-random payload)",
        "config": {"workload": f"C2: {args.sessions} H.264 1080p30 4 Mb/s streams/GPU x {args.subs} UDP subs, "
                               f"{args.tick_ms}-ms ticks (ingest+keyframe+fan-out per step)"
                               + (", RTSP-interleaved TCP push reads deframed on the GPU" if args.ingest == "tcp" else "")
                               + (", batches in pinned host memory (PCIe H2D overlapped)" if args.ingest == "host" else ""),
                   "ingest": args.ingest,
                   **({"deframe_walk": deframe_walk} if deframe_walk else {}),
                   "sessions_per_gpu": args.sessions, "subs_per_session": args.subs,
                   "tick_ms": args.tick_ms,
                   "rewrite": rewrite_desc,
                   "engine_env": knobs,
                   **({"diagnostic_rings": {"video_ring_mb": args.ring_mb, "growth": not args.no_ring_growth}}
                      if args.ring_mb != 16 or args.no_ring_growth else {}),
                   "parallelism": f"stream-hash shards x{world}, no data-path collective"
                                  + (f"; C4 replicas: {args.replicas} sessions/rank fed through peer mailboxes"
                                     if link is not None else "")
                                  + ("" if backend == "nccl" or world == 1 else f" ({backend} rehearsal, ranks sharing GPUs)"),
                   "process_group": (backend if dist else None)},
        "relayed_GBps": round(out_all / dt / 1e9, 2),
        **({"pcie_H2D_GBps": round(sum(batches[i]["bytes"] + 16 * batches[i]["n"] for i in range(warm, warm + steps))
                                   / dt / 1e9, 2)} if args.ingest == "host" else {}),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_source,
                     "kernel": ctx.fanout_kernel(), "alg_bytes_per_launch": int(alg_bytes / max(launches, 1)),
                     "avg_kernel_ms": round(fan_ms, 4)},
        "kernel_ms": {"fanout": round(fan_ms, 4),
                      "tick_plan_plus_fanout": round(float(np.mean(k_tick)), 4) if k_tick else None,
                      "ingest": round(float(np.mean(k_ing)), 4) if k_ing else None,
                      "keyframe_index": round(float(np.mean(k_key)), 4) if k_key else None},
        # the fan-out alone (plan + copy: the reflect loop), like-for-like with cpu_baseline.value,
        # which times the reference's ReflectPackets apart from its PushPacket
        "reflect_loop": ({"relayed_per_s": round(relayed / max(launches, 1) / (float(np.mean(k_tick)) / 1e3), 1),
                          "timing": "tick_plan_plus_fanout kernel time per step"} if k_tick else None),
        "per_step": per_step,
        "timing_events": ("every kernel's, inside the timed steps" if args.all_timing_events else
                          f"the fan-out copy kernel's pair inside the timed steps; ingest, keyframe and plan "
                          f"from {extra} steps after them"),
        "ingest": ingest,
        "cpu_baseline": cpu,
        # the metric counts packets made send-ready in HBM; what reaches sockets is host-bound
        # (sendmmsg / writev over PCIe-copied bytes): tools/bench_egress.py, DESIGN.md §5.6
        "wire_note": ("value counts relayed packets made send-ready in HBM (the north_star metric); on sockets "
                      "the engine's egress is host-bound: tools/bench_egress.py, 46 M datagrams/s with UDP GSO "
                      "and 7.1-7.9 M in reference-exact one-datagram-per-send mode, 0.85-1.00x the reference's "
                      "sendto() path on the same box (profiles/r05z_wire/, DESIGN.md 5.6)"),
    }
    if rep is not None:
        res["replicas"] = rep
    elif xdev is not None:
        res["cross_device"] = xdev
    print(json.dumps(res), flush=True)
    if bail:
        os._exit(0)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
