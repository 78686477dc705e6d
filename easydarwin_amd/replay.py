"""Replays an event trace (easydarwin_amd/trace.py) through the GPU engine and returns the
capture in the same format the reference harness and the CPU restatement write, so parity
is a byte comparison.

Batch semantics: all PKT events since the previous TICK form one ``edgpu_ingest`` batch
(grouped by session, arrival order kept), followed by ``edgpu_keyframe_index``; JOINs since
the previous TICK become ``edgpu_subscriber_add``; the TICK itself is ``edgpu_fanout(now)``.

Session lifecycle (trace v3, PUBLISH / UNPUBLISH): the replay keeps the module's reference
counts -- the pusher's and one per output -- and calls ``edgpu_session_remove`` when one
reaches 0 (with EDGPU_SESSION_KILL_OUTPUTS for an UNPUBLISH with kill); a PUBLISH of a removed
session adds a fresh engine session.  PUBLISH / UNPUBLISH end an ingest batch, and PKT / UPKT
events of a session without a pusher are dropped, as the reference harness drops them.
Without replicas, joins are made at their JOIN event (the engine applies them at the next
fan-out either way), so a join that finds no session fails then, as in the reference.

Preferences (trace v4): the stream prefs configure the context (edgpu_config), the module prefs
are kept as the module keeps them and change at PREFS events (RereadPrefs): a new session's SSRC
filter settings (edgpu_session_ssrc_prefs), a pusher's kill-clients attribute at its RECORD and
the kill at its leave, and which players take the RTP-Info PLAY (trace.rtp_info_player).

UPKT events (UDP pushers) are ingested like PKTs and their source addresses go to
``edgpu_udp_sources`` with the batch; the receiver reports each ``edgpu_fanout`` queues
(``edgpu_source_reports``) form the capture's EDRR trailer.  Each track's report identity is
set to what the reference harness's deterministic ``rand()`` gives it (trace.rr_ssrc).

``interleaved=seed`` feeds the same packets as a pusher's RTSP connection would carry them
('$' ch BE16(len) frames) through ``edgpu_ingest_interleaved`` instead: each session's
frames are cut into random TCP reads (cuts only between or inside frames of one arrival time,
so every frame completes in a read with its own arrival time), a random prefix of a
session's next-batch frame is sent early (carried on the device across calls), and RTSP
keep-alive requests sit between frames; the replay answers EDGPU_TCP_MESSAGE like the host
RTSP stack (consume the request through its blank line, resubmit the rest).
"""
from __future__ import annotations

import random
import re
import struct

import numpy as np

from . import edgpu
from .trace import (BLOCK, JOIN, LEAVE, PKT, PREFS, PUBLISH, TICK, UNPUBLISH, UPKT, Trace, pack_source_reports,
                    pref_bool, pref_values, rr_ssrc, rtp_info_player)


def _wire_images(subs, desc, arena, images, budgets=None, tag=0):
    """Appends each sub-stream's packets of the tick to its wire image.  `budgets` maps
    (tag, handle, track, kind) -> the writes its socket accepted this tick (BLOCK events); the
    rest would have blocked.  `tag` names the context (0 owner, 1 replica).  Returns the
    edgpu_fanout_blocked reports."""
    reports = []
    for q, s in enumerate(subs):
        n = int(s["desc_count"])
        if n == 0:
            continue
        key = (tag, int(s["subscriber"]), int(s["track"]), int(s["kind"]))
        if budgets and key in budgets and budgets[key] < n:
            n = budgets[key]
            reports.append((q, n))
            if n == 0:
                continue
        d = desc[int(s["desc_base"]):int(s["desc_base"]) + n]
        tcp = int(s["transport"]) == edgpu.TRANSPORT_TCP
        parts = images[key]
        for off, ln in zip(d["offset"].tolist(), d["len"].tolist()):
            if tcp:
                parts.append(arena[off:off + ln].tobytes())
            else:
                parts.append(struct.pack(">H", ln) + arena[off:off + ln].tobytes())
    return reports


RTSP_KEEPALIVE = (b"SET_PARAMETER rtsp://127.0.0.1/live/replay RTSP/1.0\r\nCSeq: 7\r\n"
                  b"Session: 51234\r\nContent-Length: 0\r\n\r\n")


def tcp_plan(batches, seed: int, messages: float = 0.1, carry: float = 0.5, barriers=()):
    """Per ingest batch (list of (session, channel, t, packet)): {session: [(read bytes, arrival)]}.
    No frame is carried from batch k into batch k + 1 for k in `barriers` (a pusher connection
    ends there)."""
    rng = random.Random(seed)
    per = []
    for b in batches:
        d = {}
        for s, ch, t, data in b:
            d.setdefault(s, []).append((t, struct.pack(">BBH", 0x24, ch, len(data)) + data))
        per.append(d)
    plan, carry_in = [], {}
    for k, d in enumerate(per):
        out = {}
        for s, frames in d.items():
            groups = []
            for t, fb in frames:
                if groups and groups[-1][0] == t:
                    groups[-1][1].append(fb)
                else:
                    groups.append((t, [fb]))
            pre = carry_in.pop(s, 0)
            reads = []
            for gi, (t, fbs) in enumerate(groups):
                data = b"".join(fbs)[pre if gi == 0 else 0:]
                if gi > 0 and rng.random() < messages:
                    data = RTSP_KEEPALIVE + data
                p = 0
                while p < len(data):
                    n = rng.choice([1, 3, rng.randint(1, 200), rng.randint(1, 4000), len(data)])
                    reads.append((data[p:p + n], t))
                    p += n
            if k + 1 < len(per) and s in per[k + 1] and k not in barriers and rng.random() < carry:
                first = per[k + 1][s][0][1]
                m = rng.randint(1, len(first) - 1)
                reads.append((first[:m], reads[-1][1] if reads else 0))
                carry_in[s] = m
            out[s] = reads
        plan.append(out)
    return plan


def ingest_tcp(ctx: edgpu.Context, reads_by_session: dict):
    """One batch of pusher reads through edgpu_ingest_interleaved (+ keyframe index), handing
    RTSP requests to a minimal "RTSP stack" that skips them and resubmits what follows."""
    todo = {s: list(rs) for s, rs in reads_by_session.items() if rs}
    calls = 0
    while todo:
        rows, blob = [], bytearray()
        for s, rs in todo.items():
            for b, t in rs:
                rows.append((s, len(b), len(blob), t))
                blob += b
        res = ctx.ingest_interleaved(np.array(rows, dtype=edgpu.TCP_READ_DTYPE), bytes(blob))
        ctx.keyframe_index()
        calls += 1
        nxt, i = {}, 0
        for s, rs in todo.items():
            r = res[i:i + len(rs)]
            i += len(rs)
            bad = np.nonzero(r["status"])[0]
            if not len(bad):
                continue
            j = int(bad[0])
            if int(r["status"][j]) != edgpu.TCP_MESSAGE:
                raise RuntimeError(f"session {s}: pusher connection dropped (status {int(r['status'][j])})")
            rest = [(rs[j][0][int(r["consumed"][j]):], rs[j][1])] + rs[j + 1:]
            buf = b"".join(b for b, _ in rest)
            end = buf.index(b"\r\n\r\n") + 4
            new, p = [], 0
            for b, t in rest:
                lo, p = p, p + len(b)
                if p > end:
                    new.append((b[max(0, end - lo):], t))
            if new:
                nxt[s] = new
        todo = nxt
    return calls


def _batches(trace: Trace, flush_on_rtpinfo: bool):
    """The pushers' interleaved packets of every ingest batch (a batch holding only UDP
    pushers' datagrams is an empty entry, so the list stays aligned with the flushes), and
    the indices of the batches a PUBLISH / UNPUBLISH ends (no frame is carried past them)."""
    out, cur, any_pkt, barriers = [], [], False, set()
    published = [True] * len(trace.sdps)
    prefs = trace.prefs
    for ev in trace.events:
        if ev[0] == PREFS:
            prefs = ev[2]
        if ev[0] == PKT:
            _, t, s, ch, data = ev
            if not published[s]:
                continue
            cur.append((s, ch, t, data))
            any_pkt = True
        elif ev[0] == UPKT:
            if published[ev[2]]:
                any_pkt = True
        elif (ev[0] == JOIN and rtp_info_player(prefs, ev[5]) and flush_on_rtpinfo) or ev[0] in (TICK, PUBLISH, UNPUBLISH):
            if any_pkt:
                out.append(cur)
                cur, any_pkt = [], False
            if ev[0] in (PUBLISH, UNPUBLISH):
                if out:
                    barriers.add(len(out) - 1)
                published[ev[2]] = ev[0] == PUBLISH
    return out, barriers


def replay(trace: Trace, ctx: edgpu.Context | None = None, replica: str | None = None,
           interleaved: int | None = None, sockets: dict | None = None, rewrite: dict | None = None,
           pinned: bool = False, tick_info: list | None = None, slots: dict | None = None, link_cls=None, **cfg):
    """Returns (capture_bytes, per-tick stats list).

    replica=None: subscribers join the context that ingests (the owner).
    replica="all" / "late" / "split": subscribers join a replica session on a second context,
    kept in step with the owner by session images (easydarwin_amd/replica.py; `link_cls`: the
    link class, ReplicaLink by default, replica.MailboxReplicaLink through a peer mailbox); "all" creates
    every replica before the first packet; "late" creates a fresh replica for every joining
    subscriber at its join tick, from a full image taken mid-stream (the C4 fast-start
    path); "split" sends the odd subscriber ids to one replica per session and keeps the even
    ones on the owner, so a session's outputs are served by two contexts at once.  A replica
    subscriber takes its bucket place from the owner (edgpu_session_remote_join, at its JOIN);
    `slots` (a dict) receives every subscriber's place by sub id.  The session lifecycle
    (PUBLISH / UNPUBLISH) reaches the replicas: a session that ends on the owner ends on them
    (its replica subscribers torn down with it by a kill), a fresh re-push gets fresh replicas.

    sockets={...}: every tick leaves through the engine's socket egress to loopback receivers
    (easydarwin_amd/egress.py SocketSink, constructed with these keyword arguments) and the
    capture is rebuilt from the bytes the receivers read.

    rewrite={sub_id: (seq_delta, ts_delta, ssrc or None)}: the per-output rewrite stage
    (edgpu_subscriber_rewrite) on every track of those subscribers, set at their join.

    pinned=True: every ingest batch is written into pinned host buffers (edgpu_host_alloc,
    two sets used alternately) and handed over as EDGPU_PTR_PINNED (asynchronous copy).

    tick_info=[]: receives, per tick read back, (copy passes, largest sub-stream's arena bytes,
    largest sub-stream's descriptors, the tick's arena bytes, its relayed packets) -- more than
    one pass when a tick exceeds out_arena_bytes or max_out_packets (edgpu_fanout_next)."""
    pv = pref_values(trace.prefs)           # the stream prefs: read once (ReflectorStream::Initialize)
    cfg = dict(cfg)
    cfg.setdefault("reflector_buffer_size_sec", int(pv["reflector_buffer_size_sec"]))
    cfg.setdefault("rtp_reflector_threshold_msec", max(1000, int(pv["rtp_reflector_threshold_msec"])))   # :101-102
    cfg.setdefault("reflector_rtp_info_offset_msec", int(pv["reflector_rtp_info_offset_msec"]) or edgpu.FALSE)
    cfg.setdefault("reflector_use_in_packet_receive_time", int(pref_bool(pv["reflector_use_in_packet_receive_time"])))
    cfg.setdefault("reflector_in_packet_max_receive_sec", int(pv["reflector_in_packet_max_receive_sec"]) or edgpu.FALSE)
    mod = {"prefs": dict(trace.prefs)}      # the module prefs (RereadPrefs at PREFS events)
    own = ctx is None
    if own:
        ctx = edgpu.Context(**cfg)
    rep = link = None
    if replica is not None:
        from .replica import ReplicaLink
        assert replica in ("all", "late", "split")
        if sockets is not None and replica == "split":
            raise ValueError("socket egress replays serve one context")
        dev = int(cfg.get("device", 0))
        rep = edgpu.Context(**cfg)
        link = (link_cls or ReplicaLink)(ctx, dev, rep, dev)
    try:
        sess_tracks = []
        rsess = {}
        rand_calls = 0
        # lifecycle: engine session of each trace session (None once removed), its pusher, and
        # the trace session of each engine session (receiver reports name the trace's)
        gen = [None] * len(trace.sdps)
        published = [True] * len(trace.sdps)
        kill_attr = [pref_bool(pref_values(mod["prefs"])["kill_clients_when_broadcast_stops"])] * len(trace.sdps)
        trace_of = {}

        def publish_fresh(i, now_s):
            nonlocal rand_calls
            sid = ctx.session_add(trace.sdps[i], udp_push=trace.udp_push(i))
            p = pref_values(mod["prefs"])       # SetupReflectorSession's SSRC filter: the prefs now
            ctx.session_ssrc_prefs(sid, pref_bool(p["use_one_SSRC_per_stream"]), int(p["timeout_stream_SSRC_secs"]))
            kill_attr[i] = pref_bool(p["kill_clients_when_broadcast_stops"])     # the RECORD
            gen[i] = sid
            trace_of[sid] = i
            for tr in range(ctx.session_tracks(sid)):
                ctx.source_identity(sid, tr, rr_ssrc(rand_calls), now_s)
                rand_calls += 1
            return sid

        for i, sdp in enumerate(trace.sdps):
            sid = publish_fresh(i, 0)
            assert sid == len(sess_tracks)
            sess_tracks.append(ctx.session_tracks(sid))
            if replica == "all":
                rsess[i] = link.add(sid, sdp, trace.udp_push(i))
        reports = []                        # (t, session, track, addr, port, bytes)
        sources = []                        # this batch's UDP datagram sources
        subs_meta = {}          # (tag, handle) -> (sub_id, session, tcp, place); tag 0 owner, 1 replica
        images = {}
        pending, joins, stats = [], [], []
        tick_info = tick_info if tick_info is not None else []
        unread = []                         # (ctx, tag, result, t, budgets) of ticks not read back yet

        def drain():
            nonlocal unread
            todo, unread = unread, []
            for c, tag, r, tt, budgets in todo:
                if sink is not None:
                    sink.tick(r, tt)
                    if link is not None and c is rep:
                        link.feedback()
                    st = c.stats()
                    stats.append((tt, st.relayed_packets, st.relayed_bytes))
                    continue
                reports, big = [], [0, 0, 0]

                def consume(st, subs, desc, arena):
                    reports.extend(_wire_images(subs, desc, arena, images, budgets, tag))
                    big[2] = max(big[2], int(st.relayed_packets))     # the tick's planned packets
                    if len(subs):
                        big[0] = max(big[0], int(subs["out_bytes"].max()))
                        big[1] = max(big[1], int(subs["desc_count"].max()))
                # every copy pass of the tick (more than one when it exceeds the arena)
                npass = c.read_passes(r, consume)
                if reports:
                    c.fanout_blocked(reports)
                if link is not None and c is rep:
                    link.feedback()                 # the replica's relocations reach the owner
                st = c.stats()
                stats.append((tt, st.relayed_packets, st.relayed_bytes))
                # (relayed_packets before the backpressure reports take the unsent ones off)
                tick_info.append((npass, big[0], big[1], int(st.arena_bytes), big[2]))

        pin_sets = [{}, {}]                 # pinned host batch buffers, used alternately
        pin_next = [0]

        def pin_ingest(desc, seg_off, seg_sess, blob):
            bufs = pin_sets[pin_next[0]]
            pin_next[0] ^= 1
            ptrs = []
            for k, a in (("desc", desc), ("seg", seg_off), ("sess", seg_sess), ("blob", blob)):
                raw = np.ascontiguousarray(a).view(np.uint8).ravel()
                if k not in bufs or bufs[k].nbytes < raw.nbytes:
                    if k in bufs:
                        bufs[k].free()
                    bufs[k] = ctx.host_alloc(max(raw.nbytes, 4096) * 2)
                bufs[k].array[:raw.nbytes] = raw
                ptrs.append(bufs[k].ptr)
            ctx.ingest_pinned(ptrs[0], len(desc), ptrs[1], ptrs[2], len(seg_sess), ptrs[3], blob.nbytes)

        clock = 0                           # the harness's virtual clock: max event time so far
        plan = None
        if interleaved is not None:
            bl, barriers = _batches(trace, True)
            plan = tcp_plan(bl, interleaved, barriers=barriers)
        nflush = 0

        def flush():
            nonlocal pending, nflush, sources
            if pending:
                udp = [p for p in pending if p[4]]
                if plan is not None:
                    if len(udp) < len(pending):
                        ingest_tcp(ctx, {gen[s]: rd for s, rd in plan[nflush].items()})
                    batch = udp                  # UDP pushers' datagrams: a plain batch
                else:
                    batch = pending
                if batch:
                    desc, seg_off, seg_sess, blob = edgpu.build_batch([(gen[p[0]],) + p[1:4] + (p[5],) for p in batch])
                    if pinned:
                        pin_ingest(desc, seg_off, seg_sess, blob)
                    else:
                        ctx.ingest_host(desc, seg_off, seg_sess, blob)
                    ctx.keyframe_index()
                nflush += 1
                pending = []
            if sources:
                ctx.udp_sources(sources)
                sources = []

        sink = None
        if sockets is not None:
            from .egress import SocketSink
            if any(ev[0] == BLOCK for ev in trace.events):
                raise ValueError("socket egress replays take no BLOCK events")
            kw = {k: v for k, v in sockets.items() if k not in ("report", "stats")}
            if kw.get("pacing") is not None:        # the gate's reflector prefs are the trace's
                kw["pacing"] = dict({"bucket_delay_ms": int(pv["reflector_bucket_offset_delay_msec"]),
                                     "over_buffer_ms": 1000 * int(cfg["reflector_buffer_size_sec"])}, **kw["pacing"])
            sink = SocketSink(ctx if rep is None else rep, **kw)
        blocks = {}                         # (sub_id, track, kind) -> budget for the next TICK
        gone = set()                        # (tag, handle)s removed by LEAVE or a kill

        def remote(sub_id):
            """Does this subscriber join a replica session?"""
            return rep is not None and (replica != "split" or sub_id % 2 == 1)

        def do_join(j):
            (_, jt, s, sub_id, transport, ua, now_j, place) = j
            tport = edgpu.TRANSPORT_TCP if transport else edgpu.TRANSPORT_UDP
            rtpi = rtp_info_player(mod["prefs"], ua)
            try:
                if remote(sub_id):
                    out, tag = rep, 1
                    h, _info, place = link.join(gen[s], rsess[s], tport, rtp_info=rtpi, now_ms=now_j, place=place)
                else:
                    out, tag = ctx, 0
                    h, _info = ctx.subscriber_play(gen[s], tport, rtp_info=rtpi, now_ms=now_j)
                    place = ctx.subscriber_slot(h)
            except edgpu.EdgpuError as e:      # deferred RTP-Info PLAY: not a subscriber
                if e.code != edgpu.WOULD_BLOCK:
                    raise
                return
            subs_meta[(tag, h)] = (sub_id, s, transport, place)
            if slots is not None:
                slots[sub_id] = place
            if rewrite and sub_id in rewrite:
                for tr in range(sess_tracks[s]):
                    out.subscriber_rewrite(h, tr, *rewrite[sub_id])
            if sink is not None:
                vid = sum(1 << t for t, m in enumerate(re.findall(r"(?m)^m=(\w+)", trace.sdps[s])) if m == "video")
                sink.join(h, sub_id, sess_tracks[s], bool(transport), play_time=now_j, video_tracks=vid)
            for tr in range(sess_tracks[s]):
                for k in (0, 1):
                    images[(tag, h, tr, k)] = []

        def outputs_of(s):
            return [th for th, meta in subs_meta.items() if meta[1] == s and th not in gone]

        def end_session(s, kill=False):
            """The owner session ends; its replicas with it (their subscribers too with a kill)."""
            drain()                         # (a session goes only after its last tick is read)
            if link is not None:
                link.remove(gen[s], kill_outputs=kill)
                rsess.pop(s, None)
            ctx.session_remove(gen[s], kill_outputs=kill)
            gen[s] = None

        def release_check(s):
            """A session without pusher or outputs dies (RemoveOutput's refcount-0 branch)."""
            if gen[s] is not None and not published[s] and not outputs_of(s) and not any(j[2] == s for j in joins):
                end_session(s)          # (a replica join waiting for its tick is an output already)

        for ev in trace.events:
            if ev[0] == BLOCK:
                blocks[(ev[2], ev[3], ev[4])] = ev[5]
                continue
            clock = max(clock, ev[1])
            if ev[0] == PKT:
                _, t, s, ch, data = ev
                if published[s]:
                    pending.append((s, ch, t, data, False, 0))
            elif ev[0] == UPKT:
                _, t, s, ch, addr, port, data = ev
                if published[s]:
                    pending.append((s, ch, t, data, True, edgpu.PKT_REMOTE_ODD if port & 1 else 0))
                    sources.append((gen[s], ch, addr, port, data))
            elif ev[0] == JOIN:
                # an RTP-Info PLAY reads the queues as they are at the JOIN (HaveStreamBuffers):
                # ingest what precedes it first
                # (on a replica too: its session is brought up to the owner's queues first)
                rtpi = rtp_info_player(mod["prefs"], ev[5])
                if rtpi:
                    flush()
                s = ev[2]
                if gen[s] is None:                      # no session: the SETUP fails
                    continue
                if not remote(ev[3]) or rtpi:
                    if remote(ev[3]):
                        if replica == "late" or s not in rsess:
                            rsess[s] = link.add(gen[s], trace.sdps[s], trace.udp_push(s))
                        link.sync(clock)
                    do_join(ev + (clock, None))
                else:
                    # replicas: made at the tick, the place taken on the owner now (AddOutput order)
                    joins.append(ev + (clock, ctx.session_remote_join(gen[s])))
            elif ev[0] == UNPUBLISH:
                _, t, s, kill = ev
                flush()
                if published[s]:
                    published[s] = False
                    # RemoveOutput's kill: the pusher's attribute or the pref now (:2156)
                    kill = kill or kill_attr[s] or pref_bool(pref_values(mod["prefs"])["kill_clients_when_broadcast_stops"])
                    if kill:                            # TearDownAllOutputs
                        for th in outputs_of(s):
                            gone.add(th)
                        joins = [j for j in joins if j[2] != s]   # (their places go with the session)
                        if gen[s] is not None:
                            end_session(s, kill=True)
                    release_check(s)
            elif ev[0] == PUBLISH:
                _, t, s = ev
                flush()
                if not published[s]:
                    published[s] = True
                    if gen[s] is None:
                        publish_fresh(s, clock // 1000)
                        if replica == "all":
                            rsess[s] = link.add(gen[s], trace.sdps[s], trace.udp_push(s))
                    else:                               # the surviving session's new RECORD
                        kill_attr[s] = pref_bool(pref_values(mod["prefs"])["kill_clients_when_broadcast_stops"])
            elif ev[0] == PREFS:
                mod["prefs"] = dict(ev[2])              # RereadPrefs
            elif ev[0] == LEAVE:
                # RemoveOutput applies at once: a join still waiting for its tick is made now
                # (the output existed, with nothing sent yet), and the output stops at the next
                # tick (edgpu_subscriber_remove)
                sub_id = ev[2]
                for j in [j for j in joins if j[3] == sub_id]:
                    if replica == "late" or j[2] not in rsess:
                        rsess[j[2]] = link.add(gen[j[2]], trace.sdps[j[2]], trace.udp_push(j[2]))
                    do_join(j)
                joins = [j for j in joins if j[3] != sub_id]
                for (tag, h), meta in subs_meta.items():
                    if meta[0] == sub_id and (tag, h) not in gone:
                        if tag:
                            link.leave(gen[meta[1]], h, meta[3])
                        else:
                            ctx.subscriber_remove(h)
                        gone.add((tag, h))
                        release_check(meta[1])
                        break
            elif ev[0] == TICK:
                t = ev[1]
                flush()
                if link is not None:
                    for (_, jt, s, sub_id, transport, _ua, _now, _place) in joins:
                        if replica == "late" or s not in rsess:
                            rsess[s] = link.add(gen[s], trace.sdps[s], trace.udp_push(s))   # "late": a fresh replica per join
                    link.sync(t)
                for j in joins:
                    do_join(j)
                joins = []
                drain()                              # the previous tick, after this batch's ingest
                by_handle = {}
                for (sub_id, trk, kind), b in blocks.items():
                    for (tag, h), meta in subs_meta.items():
                        if meta[0] == sub_id and (tag, h) not in gone:
                            by_handle[(tag, h, trk, kind)] = b
                blocks = {}
                # the owner ticks (with subscribers of its own in "split"), then the replica
                unread.append((ctx, 0, ctx.fanout(t), t, by_handle))
                reports.extend((t, trace_of[r[0]]) + tuple(r[1:]) for r in ctx.source_reports())
                if rep is not None:
                    if replica != "split":
                        unread.pop()                 # (no subscribers on the owner)
                    unread.append((rep, 1, rep.fanout(t), t, by_handle))
                drain()
        drain()
        wire = None
        if sink is not None:
            wire = sink.finish()
            sink.close()
            if isinstance(sockets, dict) and "report" in sockets:
                sockets["report"].extend(sink.blocked)
            if isinstance(sockets, dict) and "stats" in sockets:
                sockets["stats"].extend(sink.stats)
        # capture: one record per (subscriber, track, kind), sorted by subscriber id
        recs = []
        for (tag, h, tr, k), parts in images.items():
            sub_id, s, transport, _place = subs_meta[(tag, h)]
            if wire is not None:
                n, data = wire.get((h, tr, k), (0, b""))
            else:
                n, data = len(parts), b"".join(parts)
            recs.append((sub_id, s, tr, k, transport, n, data))
        recs.sort(key=lambda r: (r[0], r[2], r[3]))
        out = [b"EDCP", struct.pack("<I", len(recs))]
        for sub_id, s, tr, k, transport, n, data in recs:
            out.append(struct.pack("<IIHBBQQ", sub_id, s, tr, k, transport, n, len(data)))
            out.append(data)
        out.append(pack_source_reports(reports))
        return b"".join(out), stats
    finally:
        if link is not None:
            link.close()
        if rep is not None:
            rep.close()
        if own:
            ctx.close()
