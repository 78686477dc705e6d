"""Replays an event trace (easydarwin_amd/trace.py) through the GPU engine and returns the
capture in the same format the reference harness and the CPU restatement write, so parity
is a byte comparison.

Batch semantics: all PKT events since the previous TICK form one ``edgpu_ingest`` batch
(grouped by session, arrival order kept), followed by ``edgpu_keyframe_index``; JOINs since
the previous TICK become ``edgpu_subscriber_add``; the TICK itself is ``edgpu_fanout(now)``.
"""
from __future__ import annotations

import struct

import numpy as np

from . import edgpu
from .trace import JOIN, PKT, TICK, Trace


def _wire_images(subs, desc, arena, images):
    for s in subs:
        n = int(s["desc_count"])
        if n == 0:
            continue
        key = (int(s["subscriber"]), int(s["track"]), int(s["kind"]))
        d = desc[int(s["desc_base"]):int(s["desc_base"]) + n]
        tcp = int(s["transport"]) == edgpu.TRANSPORT_TCP
        parts = images[key]
        for off, ln in zip(d["offset"].tolist(), d["len"].tolist()):
            if tcp:
                parts.append(arena[off:off + ln].tobytes())
            else:
                parts.append(struct.pack(">H", ln) + arena[off:off + ln].tobytes())


def replay(trace: Trace, ctx: edgpu.Context | None = None, replica: str | None = None, **cfg):
    """Returns (capture_bytes, per-tick stats list).

    With overlap_ticks=1 in cfg, each tick's result is read only after the next tick's batch
    has been ingested and indexed, so that ingest runs while the previous fan-out copy may
    still be in flight (the pipelined mode's contract: results stay valid one extra tick).

    replica=None: subscribers join the context that ingests (the owner).
    replica="all" / "late": every subscriber joins a replica session on a second context,
    kept in step with the owner by session images (easydarwin_amd/replica.py); "all" creates
    every replica before the first packet; "late" creates a fresh replica for every joining
    subscriber at its join tick, from a full image taken mid-stream (the C4 fast-start
    path)."""
    own = ctx is None
    if own:
        ctx = edgpu.Context(**cfg)
    rep = link = None
    if replica is not None:
        from .replica import ReplicaLink
        assert replica in ("all", "late")
        dev = int(cfg.get("device", 0))
        rep = edgpu.Context(**cfg)
        link = ReplicaLink(ctx, dev, rep, dev)
    try:
        sess_tracks = []
        rsess = {}
        for sdp in trace.sdps:
            sid = ctx.session_add(sdp)
            assert sid == len(sess_tracks)
            sess_tracks.append(ctx.session_tracks(sid))
            if replica == "all":
                rsess[sid] = link.add(sid, sdp)
        subs_meta = {}          # handle -> (sub_id, session, tcp)
        images = {}
        pending, joins, stats = [], [], []
        lag = bool(cfg.get("overlap_ticks")) and replica is None
        unread = None                       # (ctx, result) of a tick not read back yet

        def drain():
            nonlocal unread
            if unread is not None:
                c, r, tt = unread
                st, subs, desc, arena = c.read_tick(r)
                stats.append((tt, st.relayed_packets, st.relayed_bytes))
                _wire_images(subs, desc, arena, images)
                unread = None

        clock = 0                           # the harness's virtual clock: max event time so far

        def flush():
            nonlocal pending
            if pending:
                desc, seg_off, seg_sess, blob = edgpu.build_batch(pending)
                ctx.ingest_host(desc, seg_off, seg_sess, blob)
                ctx.keyframe_index()
                pending = []

        for ev in trace.events:
            clock = max(clock, ev[1])
            if ev[0] == PKT:
                _, t, s, ch, data = ev
                pending.append((s, ch, t, data))
            elif ev[0] == JOIN:
                # an RTP-Info PLAY reads the queues as they are at the JOIN (HaveStreamBuffers):
                # ingest what precedes it first; other joins wait for the tick
                if ev[5] & 1 and rep is None:
                    flush()
                joins.append(ev + (clock,))
            elif ev[0] == TICK:
                t = ev[1]
                flush()
                if link is not None:
                    for (_, jt, s, sub_id, transport, _ua, _now) in joins:
                        if replica == "late" or s not in rsess:
                            rsess[s] = link.add(s, trace.sdps[s])     # "late": a fresh replica per join
                    link.sync(t)
                out = ctx if rep is None else rep
                for (_, jt, s, sub_id, transport, ua, now_j) in joins:
                    try:
                        h, _info = out.subscriber_play(s if rep is None else rsess[s],
                                                       edgpu.TRANSPORT_TCP if transport else edgpu.TRANSPORT_UDP,
                                                       rtp_info=bool(ua & 1), now_ms=now_j)
                    except edgpu.EdgpuError as e:      # deferred RTP-Info PLAY: not a subscriber
                        if e.code != edgpu.WOULD_BLOCK:
                            raise
                        continue
                    subs_meta[h] = (sub_id, s, transport)
                    for tr in range(sess_tracks[s]):
                        for k in (0, 1):
                            images[(h, tr, k)] = []
                joins = []
                if rep is not None:
                    ctx.fanout(t)                      # the owner ticks too (no subscribers here)
                drain()                              # the previous tick, after this batch's ingest
                unread = (out, out.fanout(t), t)
                if not lag:
                    drain()
        drain()
        # capture: one record per (subscriber, track, kind), sorted by subscriber id
        recs = []
        for (h, tr, k), parts in images.items():
            sub_id, s, transport = subs_meta[h]
            recs.append((sub_id, s, tr, k, transport, parts))
        recs.sort(key=lambda r: (r[0], r[2], r[3]))
        out = [b"EDCP", struct.pack("<I", len(recs))]
        for sub_id, s, tr, k, transport, parts in recs:
            data = b"".join(parts)
            out.append(struct.pack("<IIHBBQQ", sub_id, s, tr, k, transport, len(parts), len(data)))
            out.append(data)
        return b"".join(out), stats
    finally:
        if link is not None:
            link.close()
        if rep is not None:
            rep.close()
        if own:
            ctx.close()
