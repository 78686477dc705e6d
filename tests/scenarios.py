"""Deterministic trace scenarios used for parity (golden fixtures, oracle pinning, GPU tests).

Each scenario function returns a :class:`easydarwin_amd.trace.Trace`.  Seeds derive from
``0xEA5D``.  The scenarios cover every row of SURVEY.md §8.a that has a
parity consequence:

* ``c1``            configs[0]: 1 H.264 720p30 push (2 s GOP) -> 4 UDP subscribers, two of
                    them joining mid-GOP at 3.3 s (Q3/Q4/Q5/Q7 key-pointer start, SPS/PPS not
                    replayed).
* ``mixed``         C5-style: H.264 / MP4V-ES / JPEG video with AAC / PCMA / PCMU audio,
                    jittered packet sizes, UDP and TCP-interleaved subscribers (Q2), pusher
                    RTCP SRs carried on the odd channel of a TCP push (Q12), staggered joins.
* ``clamp``         packets above the 2060-byte ReflectorPacket limit (Q11).
* ``ssrc``          SSRC switch mid-stream, zero-length survivors and the 30 s reset (Q13).
* ``nal``           crafted H.264 payloads: STAP-A/B, MTAP16/24, FU-A/FU-B with and without
                    the start bit, the 19/20-byte length boundary, CSRC counts (Q4).
* ``nokey``         a stream with no key frames: new subscribers start at the 1 s buffer
                    window, and a join while the pusher is stalled gets a NULL start (Q7).
* ``stall``         a 12 s pusher stall with subscribers attached (Q16 retention, bookmarks).
* ``anchor``        video + two audio tracks: the session-wide audio anchor flag (Q6).
* ``tiny``          a 1-session, 2-subscriber smoke case (used by ``smoke()``).
* ``rtpinfo``       RTP-Info players (UA "vlc"/"Android", ua_flags bit 0): the first-seq
                    filter (Q10) that starts them ~500 ms back instead of at the key pointer,
                    its u16 compare across a sequence wrap, the RTCP write that lifts it, and
                    PLAYs deferred for want of buffered packets (before the first packet, and
                    during a pusher stall).
* ``backpressure``  sockets that stop accepting writes mid-tick (QTSS_WouldBlock): bookmarks
                    at the blocked packet, Q9 relocation to the newest key frame after 2 s,
                    RTCP sub-streams, an RTP-Info player blocked before its first write.
* ``udppush``       UDP pushers (datagrams with source addresses on bound even/odd ports):
                    the RTCP SR-only gate (Q14), the pusher's RTCP address learnt from the
                    first datagram and moved by later SRs (NAT_WORKAROUND), and the receiver
                    reports with the eye count sent to it every 5 s.
* ``leave``         subscribers leaving (RemoveOutput): between ticks, while blocked, leave +
                    new output in one tick, join + leave before a tick, an RTP-Info player,
                    and the eye counts of the receiver reports after leaves.
* ``repush``        the session lifecycle: a pusher leaving with players attached and coming
                    back with a new SSRC inside the 30 s latch (the surviving session is
                    reused: zero-length packets, the old GOP for new joiners, until the
                    latch resets), the last player leaving a pusher-less session (it dies; a
                    join then fails; a re-push builds a fresh session: ids from 1, no stale
                    GOP), ``kill_clients`` tearing a UDP push's players down (fresh receiver-
                    report identities after the re-push), packets of a departed pusher
                    dropped, duplicate PUBLISH / UNPUBLISH ignored.
* ``threaded``      tick-invariant streams for the module's default (threaded) mode: players
                    joined before the first packet, no H.264 key frames, TCP and UDP pushers.
* ``prefs_buffer``  non-default ReflectorStream prefs (read once): a 3-s buffer window, the
                    RTP-Info offset, the 1000-ms relocation floor, the bucket delay.
* ``prefs_reread``  non-default module prefs and RereadPrefs (PREFS events): SSRC filtering off,
                    then a 5-s SSRC timeout for a session set up later; kill_clients by pref; the
                    RTP-Info player list, forcing and disabling RTP-Info; a 5000-ms relocation
                    threshold.
"""
from __future__ import annotations

import struct

import numpy as np

from easydarwin_amd.synth import (SEED_BASE, TrackSpec, make_sdp, rtp_header, rtcp_sr,
                                  session_packets)
from easydarwin_amd.trace import IDENT_PLAYER, IDENT_PUSHER, TCP, UDP, Trace


def _assemble(tr: Trace, per_session: list[list], tick_ms: int, end_ms: int,
              joins: list[tuple], tick_times=None, blocks=None, leaves=None, pubs=None, prefs=None, idents=None):
    # joins: (t, session, sub, transport) or (t, session, sub, transport, ua_flags)
    # blocks: {tick time: [(sub, track, kind, budget)]}
    # leaves: [(t, sub)]
    # pubs: [(t, "publish", session)] / [(t, "unpublish", session, kill)]
    # prefs: [(t, {pref overrides})] -- the server rewrites its prefs (RereadPrefs), before
    #        any PUBLISH or packet of the same time
    """Merge per-session packet lists (t, ch, bytes) with joins (t, sess, sub, transport)
    and ticks.  Within one tick interval the order is: packets and pusher PUBLISH / UNPUBLISH
    events (time order: a PUBLISH before and an UNPUBLISH after the packets of its time), then
    joins and leaves (time order; a join before a leave of the same time), then the tick's
    socket budgets (BLOCK), then the TICK at the interval end."""
    # a packet (t, ch, data, addr, port) is a UDP datagram from a pusher (UPKT)
    pkts = []
    for s, lst in enumerate(per_session):
        for k, p in enumerate(lst):
            pkts.append((p[0], s, k) + tuple(p[1:]))
    for p in (pubs or []):
        if p[1] == "publish":
            pkts.append((p[0], -1, 0, "P", p[2]))
        else:
            pkts.append((p[0], 1 << 30, 0, "U", p[2], p[3]))
    for k, (t, pr) in enumerate(prefs or []):
        pkts.append((t, -2, k, "R", pr))
    # idents: (t, session, role, addr, path, user, groups, realm) -- before a PUBLISH / JOIN of its time
    for k, idt in enumerate(idents or []):
        pkts.append((idt[0], -3, k, "I", idt[1:]))
    pkts.sort(key=lambda x: (x[0], x[1], x[2]))
    joins = sorted([(j[0], 0) + tuple(j[1:]) for j in joins] + [(t, 1, sub) for t, sub in (leaves or [])])
    ticks = tick_times if tick_times is not None else list(range(0, end_ms + 1, tick_ms))
    i = j = 0
    for tt in ticks:
        while i < len(pkts) and pkts[i][0] <= tt:
            t, s, _, ch, data = pkts[i][:5]
            if ch == "R":
                tr.reprefs(t, data)
            elif ch == "I":
                tr.ident(t, *data)
            elif ch == "P":
                tr.publish(t, data)
            elif ch == "U":
                tr.unpublish(t, data, pkts[i][5])
            elif len(pkts[i]) > 5:
                tr.upkt(t, s, ch, pkts[i][5], pkts[i][6], data)
            else:
                tr.pkt(t, s, ch, data)
            i += 1
        while j < len(joins) and joins[j][0] <= tt:
            if joins[j][1] == 1:
                tr.leave(joins[j][0], joins[j][2])
            else:
                t, _, s, sub, transport = joins[j][:5]
                tr.join(t, s, sub, transport, joins[j][5] if len(joins[j]) > 5 else 0)
            j += 1
        for sub, trk, kind, budget in (blocks or {}).get(tt, []):
            tr.block(tt, sub, trk, kind, budget)
        tr.tick(tt)
    return tr


def c1(duration_ms: int = 10_000) -> Trace:
    tracks = [TrackSpec("video", "H264/90000", 96, bitrate=2_000_000, gop=60, idr_bytes=40_000)]
    tr = Trace()
    tr.add_session(make_sdp(tracks))
    pk = session_packets(tracks, duration_ms, SEED_BASE + 0)
    joins = [(0, 0, 1, UDP), (0, 0, 2, UDP), (3300, 0, 3, UDP), (3300, 0, 4, UDP)]
    return _assemble(tr, [pk], 100, duration_ms, joins)


def mixed(duration_ms: int = 4_000) -> Trace:
    vids = [("H264/90000", True), ("MP4V-ES/90000", False), ("JPEG/90000", False)]
    auds = ["MPEG4-GENERIC/48000/2", "PCMA/8000", "PCMU/8000"]
    tr = Trace()
    per, joins = [], []
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + 4))
    sub = 100
    for s in range(6):
        vname, _ = vids[s % 3]
        tracks = [TrackSpec("video", vname, 96, bitrate=600_000, gop=30, idr_bytes=9_000,
                            jitter_sizes=(s % 2 == 1), rtcp_every_ms=(700 if s in (0, 3) else 0)),
                  TrackSpec("audio", auds[(s // 2) % 3], 97 if s % 3 == 0 else (8 if s % 3 == 1 else 0),
                            jitter_sizes=(s == 5))]
        tr.add_session(make_sdp(tracks))
        per.append(session_packets(tracks, duration_ms, SEED_BASE + 40 + s))
        for k in range(4):
            t = int(rng.integers(0, duration_ms - 500)) if k else 0
            joins.append((t, s, sub, TCP if (sub % 2) else UDP))
            sub += 1
    return _assemble(tr, per, 100, duration_ms, joins)


def clamp() -> Trace:
    tracks = [TrackSpec("video", "MP4V-ES/90000", 96)]
    tr = Trace()
    tr.add_session(make_sdp(tracks))
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + 7))
    ssrc = 0x1234ABCD
    pk = []
    for i, n in enumerate([100, 2059, 2060, 2061, 3000, 8000, 65535, 12, 20, 1400]):
        pay = rng.integers(0, 256, size=max(n - 12, 0), dtype=np.uint8).tobytes()
        pk.append((50 * i, 0, (rtp_header(1000 + i, 3000 * i, ssrc, 96, True) + pay)[:n]))
    joins = [(0, 0, 1, UDP), (0, 0, 2, TCP), (220, 0, 3, TCP)]
    return _assemble(tr, [pk], 100, 600, joins)


def ssrc() -> Trace:
    tracks = [TrackSpec("video", "H264/90000", 96)]
    tr = Trace()
    tr.add_session(make_sdp(tracks))
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + 8))
    pk, seq = [], 0

    def pkt(t, ssrc_v, nal=0x41, n=200):
        nonlocal seq
        seq += 1
        pay = bytes([nal]) + rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        pk.append((t, 0, rtp_header(seq, t * 90, ssrc_v, 96, True) + pay))

    pkt(0, 0xAAAA0001, 0x65)
    for t in range(200, 2000, 200):
        pkt(t, 0xAAAA0001)
    pkt(2100, 0)                       # SSRC 0 survives the filter
    pkt(2150, 0xAAAA0001)
    for t in range(2200, 40_000, 1000):  # new pusher SSRC: zero-length until the 30 s reset
        pkt(t, 0xBBBB0002, 0x65 if t % 5000 == 200 else 0x41)
    pkt(40_100, 0xAAAA0001)
    joins = [(0, 0, 1, UDP), (1000, 0, 2, TCP), (20_000, 0, 3, UDP), (35_000, 0, 4, TCP)]
    return _assemble(tr, [pk], 500, 41_000, joins)


def _h264_pkt(seq, t, payload: bytes, cc: int = 0, ssrc=0x51515151):
    csrc = b"".join(struct.pack(">I", 0x1000 + k) for k in range(cc))
    return rtp_header(seq, t * 90, ssrc, 96, False, cc=cc) + csrc + payload


def nal() -> Trace:
    """Crafted payloads through IsKeyFrameFirstPacket; a join after every candidate shows
    which packet became the key pointer (the new subscriber's first packet)."""
    tracks = [TrackSpec("video", "H264/90000", 96)]
    tr = Trace()
    tr.add_session(make_sdp(tracks))
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + 9))

    def rnd(n):
        return rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()

    cases = [
        bytes([0x41]) + rnd(30),                       # non-IDR slice
        bytes([0x65]) + rnd(30),                       # IDR            -> key
        bytes([0x67]) + rnd(7),                        # SPS, 20-B pkt  -> key (boundary)
        bytes([0x68]) + rnd(6),                        # PPS, 19-B pkt  -> not key (len < 20)
        bytes([0x78, 0, 4, 0x67]) + rnd(30),           # STAP-A(SPS)    -> key
        bytes([0x78, 0, 4, 0x41]) + rnd(30),           # STAP-A(slice)
        bytes([0x79, 0, 0, 0, 4, 0x65]) + rnd(30),     # STAP-B(IDR)    -> key
        bytes([0x7A, 0, 0, 0, 0, 0, 0, 0, 0x68]) + rnd(30),       # MTAP16(PPS) -> key
        bytes([0x7B, 0, 0, 0, 0, 0, 0, 0, 0, 0x65]) + rnd(30),    # MTAP24(IDR) -> key
        bytes([0x7B, 0, 0, 0, 0, 0, 0, 0, 0, 0x41]) + rnd(30),    # MTAP24(slice)
        bytes([0x7C, 0x85]) + rnd(30),                 # FU-A start IDR -> key
        bytes([0x7C, 0x05]) + rnd(30),                 # FU-A cont. IDR -> not key
        bytes([0x7C, 0x45]) + rnd(30),                 # FU-A end IDR   -> not key
        bytes([0x7D, 0x87]) + rnd(30),                 # FU-B start SPS -> key
        bytes([0x7C, 0x81]) + rnd(30),                 # FU-A start slice
        bytes([0x66]) + rnd(30),                       # SEI (type 6)
        bytes([0x78, 0, 4]),                           # STAP-A, too short to peek (len 15 < 20)
        bytes([0x78]) + rnd(6),                        # STAP-A, len 19
        bytes([0x78, 0, 4]) + rnd(5),                  # STAP-A, len 20, peek byte random
    ]
    pk = []
    t = 0
    seq = 7
    for i, pay in enumerate(cases):
        pk.append((t, 0, _h264_pkt(seq, t, pay)))
        seq += 1
        t += 100
    for cc in (1, 2):                                  # CSRC-shifted headers (h = 12 + 4cc < len)
        pk.append((t, 0, _h264_pkt(seq, t, bytes([0x65]) + rnd(40), cc=cc))); seq += 1; t += 100
        pk.append((t, 0, _h264_pkt(seq, t, bytes([0x41]) + rnd(40), cc=cc))); seq += 1; t += 100
    end = t + 200
    joins = [(tt, 0, 10 + k, UDP if k % 2 else TCP) for k, tt in enumerate(range(50, end, 100))]
    return _assemble(tr, [pk], 50, end, joins)


def nokey() -> Trace:
    tracks = [TrackSpec("video", "MP4V-ES/90000", 96, bitrate=300_000),
              TrackSpec("audio", "PCMU/8000", 0)]
    tr = Trace()
    tr.add_session(make_sdp(tracks))
    pk = session_packets(tracks, 3000, SEED_BASE + 10)
    pk += [(t + 6000, ch, d) for (t, ch, d) in session_packets(tracks, 1500, SEED_BASE + 11)]
    joins = [(0, 0, 1, UDP), (1500, 0, 2, TCP), (4500, 0, 3, UDP), (6500, 0, 4, TCP)]
    return _assemble(tr, [pk], 100, 7600, joins)


def stall() -> Trace:
    tracks = [TrackSpec("video", "H264/90000", 96, bitrate=300_000, gop=15, idr_bytes=4000),
              TrackSpec("audio", "PCMA/8000", 8)]
    tr = Trace()
    tr.add_session(make_sdp(tracks))
    pk = session_packets(tracks, 2000, SEED_BASE + 12)
    pk += [(t + 14_000, ch, d) for (t, ch, d) in session_packets(tracks, 1500, SEED_BASE + 13)]
    joins = [(0, 0, 1, TCP), (5000, 0, 2, UDP), (13_000, 0, 3, TCP), (14_500, 0, 4, UDP)]
    return _assemble(tr, [pk], 250, 16_000, joins)


def anchor() -> Trace:
    tracks = [TrackSpec("audio", "PCMA/8000", 8),
              TrackSpec("video", "H264/90000", 96, bitrate=400_000, gop=20, idr_bytes=5000),
              TrackSpec("audio", "MPEG4-GENERIC/48000/2", 97)]
    tr = Trace()
    tr.add_session(make_sdp(tracks))
    tracks2 = [TrackSpec("audio", "PCMU/8000", 0)]           # audio-only session: no anchor
    tr.add_session(make_sdp(tracks2))
    pk0 = session_packets(tracks, 3000, SEED_BASE + 14)
    pk1 = session_packets(tracks2, 3000, SEED_BASE + 15)
    joins = [(0, 0, 1, UDP), (750, 0, 2, TCP), (1400, 0, 3, UDP), (2100, 0, 4, TCP),
             (0, 1, 5, UDP), (1500, 1, 6, TCP)]
    ticks = sorted(set(list(range(0, 3001, 150)) + [333, 1001, 1777]))
    return _assemble(tr, [pk0, pk1], 150, 3000, joins, tick_times=ticks)


def tiny() -> Trace:
    tracks = [TrackSpec("video", "H264/90000", 96, bitrate=400_000, gop=15, idr_bytes=6000),
              TrackSpec("audio", "PCMA/8000", 8)]
    tr = Trace()
    tr.add_session(make_sdp(tracks))
    pk = session_packets(tracks, 1200, SEED_BASE + 16)
    joins = [(0, 0, 1, UDP), (600, 0, 2, TCP)]
    return _assemble(tr, [pk], 100, 1200, joins)


VLC = 1                                    # ua_flags bit 0: RTP-Info player profile


def rtpinfo() -> Trace:
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + 60))
    tr = Trace()
    # session 0: steady H.264 + PCMA push with pusher SRs on the video RTCP channel
    s0 = [TrackSpec("video", "H264/90000", 96, bitrate=600_000, gop=60, idr_bytes=9_000, rtcp_every_ms=900),
          TrackSpec("audio", "PCMA/8000", 8)]
    tr.add_session(make_sdp(s0))
    pk0 = session_packets(s0, 6000, SEED_BASE + 61)
    # session 1: starts at 1 s with its video sequence about to wrap, stalls 2.6-3.9 s
    s1 = [TrackSpec("video", "H264/90000", 96, bitrate=500_000, gop=45, idr_bytes=8_000,
                    extra={"seq0": 65536 - 30}),
          TrackSpec("audio", "PCMU/8000", 0)]
    tr.add_session(make_sdp(s1))
    pk1 = session_packets(s1, 1600, SEED_BASE + 62, t0=1000)
    pk1 += session_packets(s1, 2000, SEED_BASE + 63, t0=3900)
    # session 2: video only; at 2 s the pusher restarts its sequence numbers far below the
    # RTP-Info first seq of a player joining then, so the filter holds that player's RTP
    # sub-stream until its first RTCP write (an SR of the same NTP second passes the TCP
    # push's SSRC latch, Q12/Q13) lifts it
    s2 = [TrackSpec("video", "H264/90000", 96, bitrate=400_000, gop=30, idr_bytes=5_000,
                    ssrc=0x2222AAAA, extra={"seq0": 40_000})]
    tr.add_session(make_sdp(s2))
    s2b = [TrackSpec("video", "H264/90000", 96, bitrate=400_000, gop=30, idr_bytes=5_000,
                     rtcp_every_ms=250, ssrc=0x2222AAAA, extra={"seq0": 100})]
    pk2 = session_packets(s2, 2000, SEED_BASE + 64)
    pk2 += session_packets(s2b, 3000, SEED_BASE + 65, t0=2000)
    joins = [
        (0, 0, 1, UDP, VLC), (0, 0, 2, TCP),                    # at the first packets
        (1300, 0, 3, TCP, VLC), (1300, 0, 4, UDP),              # mid-GOP: ~500 ms back vs key
        (2700, 0, 5, UDP, VLC), (4450, 0, 6, TCP, VLC),
        (0, 1, 10, UDP, VLC),                                   # no packet yet: deferred
        (1800, 1, 11, TCP, VLC), (1800, 1, 12, UDP),            # after the seq wrap
        (3300, 1, 13, UDP, VLC), (3700, 1, 14, TCP, VLC),       # stalled pusher: deferred
        (4200, 1, 15, UDP, VLC),
        (1900, 2, 20, TCP, VLC), (1900, 2, 21, UDP),            # before the restart
        (1950, 2, 23, TCP, VLC),                                # at the restart: held by the filter
        (2300, 2, 22, UDP, VLC),
    ]
    del rng
    return _assemble(tr, [pk0, pk1, pk2], 100, 6000, joins)


def backpressure() -> Trace:
    """Egress backpressure: sockets that accept only part of a
    tick's writes (EAGAIN -> QTSS_WouldBlock).  SendPacketsToOutput stops at the blocked
    packet and bookmarks it; the next tick resumes there.  A socket blocked for longer than
    the 2 s relocation age has its bookmark moved to the newest key frame (Q9), which also
    arms the session's audio anchor (Q6).  Covers UDP and TCP subscribers, RTP and RTCP
    sub-streams (pusher SRs on the video RTCP channel), an RTP-Info player blocked before its
    first write (the first-seq filter stays armed), a subscriber blocked on its very first
    packet, and an audio-only session (no key frame: no relocation)."""
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + 70))
    tracks = [TrackSpec("video", "H264/90000", 96, bitrate=1_000_000, gop=30, idr_bytes=12_000,
                        rtcp_every_ms=500),
              TrackSpec("audio", "PCMA/8000", 8)]
    tracks2 = [TrackSpec("audio", "PCMU/8000", 0)]
    tr = Trace()
    tr.add_session(make_sdp(tracks))
    tr.add_session(make_sdp(tracks2))
    pk0 = session_packets(tracks, 8000, SEED_BASE + 71)
    pk1 = session_packets(tracks2, 8000, SEED_BASE + 72)
    joins = [(0, 0, 1, UDP), (0, 0, 2, TCP), (300, 0, 3, UDP), (1200, 0, 4, TCP),
             (1500, 0, 5, UDP, VLC), (2000, 0, 6, TCP), (0, 1, 7, UDP), (500, 1, 8, TCP)]
    ticks = list(range(0, 8001, 100))
    blocks = {}

    def add(t, *b):
        blocks.setdefault(t, []).append(b)
    for t in ticks:
        if t % 300 == 0 and t > 0:
            add(t, 2, 0, 0, int(rng.integers(0, 6)))          # TCP video: short budgets
            add(t, 2, 1, 0, int(rng.integers(0, 2)))          # TCP audio
        if 1000 <= t < 4200:
            add(t, 3, 0, 0, 0)                                # UDP video blocked > 2 s: Q9
        if 4200 <= t < 4600:
            add(t, 3, 0, 0, 1)                                # ... then a trickle
        if 1800 <= t < 2600 and t % 200 == 0:
            add(t, 4, 0, 1, 0)                                # RTCP sub-stream (pusher SRs)
        if t in (1500, 1600):
            add(t, 5, 0, 0, 0)                                # RTP-Info: blocked before a write
            add(t, 5, 0, 1, 0)
            add(t, 5, 1, 0, 0)
        if t == 1700:
            add(t, 5, 0, 0, 2)
        if t == 2000:
            add(t, 6, 0, 0, 0)                                # blocked on its first packet
        if 2000 <= t < 5000 and t % 100 == 0:
            add(t, 7, 0, 0, 0 if t < 4500 else 3)             # audio-only: no key to jump to
        if t % 700 == 0 and t >= 700:
            add(t, 8, 0, 0, int(rng.integers(0, 4)))
    return _assemble(tr, [pk0, pk1], 100, 8000, joins, tick_times=ticks, blocks=blocks)


def _ip(a, b, c, d):
    return a << 24 | b << 16 | c << 8 | d


def udppush() -> Trace:
    """UDP pushers: datagrams read from bound sockets with the
    pusher's address (ReflectorSocket::ProcessPacket, ReflectorStream.cpp:1769-1875).

    * session 0 (H.264 + PCMA, SRs every 700 ms): RTP from an even port (RTCP address =
      port + 1), SRs from the odd port, a NAT rebinding that moves the SRs to a new port,
      a receiver report (PT 201) and a truncated SR from elsewhere (rejected by the SR-only
      gate, Q14, so they neither relay nor move the address), an SR with a foreign SSRC
      (zero-length after the SSRC filter, but it still moves the address) and an oversized
      datagram (clamped to 2060);
    * session 1 (audio only): RTP from an odd port (no +1), first datagram only after the
      first 5 s report time, so that report is skipped and the timer still restarts;
    * session 2: an RTSP-interleaved (TCP) push, which never learns an address: no reports;
    * session 3: 130 subscribers, so the eye count has bit 7 set, which the reference's
      ``htonl(n) & 0x7fffffff`` clears on a little-endian host (ReflectorStream.cpp:519-521).
    Subscribers join over time, so the reports' eye counts change (ReflectorSession.cpp:
    215-268)."""
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + 80))
    dur = 16_500
    v = [TrackSpec("video", "H264/90000", 96, bitrate=500_000, gop=30, idr_bytes=6_000,
                   rtcp_every_ms=700),
         TrackSpec("audio", "PCMA/8000", 8)]
    a = [TrackSpec("audio", "PCMU/8000", 0)]
    tr = Trace()
    tr.add_session(make_sdp(v), udp_push=True)
    tr.add_session(make_sdp(a), udp_push=True)
    tr.add_session(make_sdp(a))
    tr.add_session(make_sdp(a), udp_push=True)
    src0, src1 = _ip(10, 0, 0, 5), _ip(192, 168, 7, 21)
    pk0 = []
    for t, ch, data in session_packets(v, dur, SEED_BASE + 81):
        port = 6000 + (ch & 1)
        if ch & 1 and t >= 7000:
            port = 7001                                   # NAT rebinding of the SR flow
        pk0.append((t, ch, data, src0, port))
    ssrc_v = struct.unpack(">I", pk0[0][2][8:12])[0]
    pk0 += [
        (2050, 1, struct.pack(">BBHI", 0x81, 201, 7, 0x1234) + bytes(24), _ip(10, 9, 9, 9), 9999),
        (2150, 1, rtcp_sr(ssrc_v, 2150, 0, 1, 1)[:20], _ip(10, 9, 9, 9), 9999),   # truncated
        (3050, 0, rtp_header(1, 0, ssrc_v, 96, False) + b"\x41" * 50, _ip(10, 1, 1, 1), 4000),
        (14750, 1, rtcp_sr(0x0BADF00D, 14750, 0, 1, 1), src0, 8001),   # foreign SSRC
        (12550, 0, rtp_header(2, 0, ssrc_v, 96, False) + b"\x41" +
         rng.integers(0, 256, size=2999, dtype=np.uint8).tobytes(), src0, 6000),
    ]
    pk0.sort(key=lambda p: p[0])
    pk1 = [(t, ch, data, src1, 5001) for t, ch, data in session_packets(a, dur, SEED_BASE + 82, t0=6000)
           if t >= 6000]
    pk2 = session_packets(a, dur, SEED_BASE + 83)
    pk3 = [(t, 0, rtp_header(t // 100, t * 8, 0x3333, 0, False) + bytes(40), _ip(172, 16, 0, 3), 30000)
           for t in range(0, 5301, 100)]
    joins = [(0, 0, 1, UDP), (3000, 0, 2, TCP), (9000, 0, 3, UDP), (500, 1, 4, UDP),
             (12000, 1, 5, TCP), (0, 2, 6, UDP)] + [(0, 3, 1000 + k, UDP) for k in range(130)]
    return _assemble(tr, [pk0, pk1, pk2, pk3], 100, dur, joins)


def leave() -> Trace:
    """Subscribers leaving (TEARDOWN / disconnect): QTSSReflectorModule's
    RemoveOutput -> ReflectorSession::RemoveOutput(output, isClient) + delete
    (QTSSReflectorModule.cpp:2133-2196, ReflectorSession.cpp:255-279, ReflectorStream.cpp:
    338-362).

    * session 0 (RTSP-interleaved push, H.264 + PCMA, pusher SRs on the video RTCP channel):
      a leave between two ticks (1), a TCP subscriber leaving while its socket is blocked (2),
      a leave and a new output of the same player in one tick interval (3 -> 4), a join and a
      leave before any tick (5: never receives), an RTP-Info player leaving (6), a control
      subscriber that stays (7);
    * session 1 (UDP push): subscribers come and go around the 5-s receiver-report times, so
      the eye counts the reports carry (DecEyeCount) change: 5, then 3, 4 and 2; a deferred
      RTP-Info PLAY (15: before the first packet, never an output) and a sub id that was
      never used leave without effect."""
    v = [TrackSpec("video", "H264/90000", 96, bitrate=600_000, gop=30, idr_bytes=8_000, rtcp_every_ms=600),
         TrackSpec("audio", "PCMA/8000", 8)]
    u = [TrackSpec("video", "H264/90000", 96, bitrate=400_000, gop=30, idr_bytes=5_000, rtcp_every_ms=700)]
    tr = Trace()
    tr.add_session(make_sdp(v))
    tr.add_session(make_sdp(u), udp_push=True)
    dur = 16_000
    pk0 = session_packets(v, 6000, SEED_BASE + 90)
    src = _ip(10, 0, 0, 9)
    pk1 = [(t, ch, data, src, 7000 + (ch & 1)) for t, ch, data in session_packets(u, dur, SEED_BASE + 91, t0=100)]
    joins = [(0, 0, 1, UDP), (0, 0, 2, TCP), (300, 0, 3, UDP), (1000, 0, 5, TCP), (1300, 0, 6, UDP, VLC),
             (0, 0, 7, TCP), (2550, 0, 4, UDP),
             (0, 1, 15, UDP, VLC), (100, 1, 10, UDP), (100, 1, 11, TCP), (200, 1, 12, UDP), (400, 1, 13, UDP),
             (600, 1, 14, TCP), (8000, 1, 16, UDP)]
    leaves = [(1550, 1), (2450, 2), (2550, 3), (1000, 5), (3000, 6), (500, 15), (6000, 10), (6000, 11),
              (11000, 12), (11000, 16), (11050, 99)]
    blocks = {}
    for t in range(2000, 2500, 100):
        blocks.setdefault(t, []).extend([(2, 0, 0, 0), (2, 1, 0, 1)])
    return _assemble(tr, [pk0, pk1], 100, dur, joins, blocks=blocks, leaves=leaves)


def repush() -> Trace:
    """Session lifecycle (QTSSReflectorModule.cpp:1379-1545, 2070-2196; the SSRC latch,
    ReflectorStream.cpp:1732-1767).

    * session 0 (RTSP-interleaved push, H.264 + PCMA, SRs on the video RTCP channel): players 1
      (UDP) and 2 (TCP) stay through a pusher leave at 2 s (no kill: the players keep the
      session alive); a new pusher with new SSRCs publishes at 3 s onto the surviving session,
      so its packets are zero-length no-ops until the latch resets 30 s after the old SSRC's
      last packet; player 3 joining at 4 s gets the OLD stream's GOP from the key pointer,
      player 4 joining after the reset the new stream;
    * session 1 (interleaved, video): its players leave at 1.5 s, its pusher at 2.5 s (the
      session dies), a player joining at 2.6 s finds no session, the re-push at 3 s builds a
      fresh session (packet ids from 1, unlatched filter, no stale GOP), player 13 joins it;
    * session 2 (UDP push, receiver reports): the pusher leaves at 6 s with kill_clients, so
      players 20 and 21 are torn down and the session dies; the re-push at 7 s draws new
      report identities (rand(), CNAME at 7 s); player 22 joins at 8 s;
    * session 3 (interleaved, video): the pusher leaves at 1 s with player 30 attached, its
      packets until 1.5 s are dropped (no pusher), a re-push at 1.5 s continues the same
      SSRC; a duplicate PUBLISH and an UNPUBLISH of a pusher-less session change nothing;
      player 31 joins at 2 s."""
    v0 = [TrackSpec("video", "H264/90000", 96, bitrate=200_000, gop=30, idr_bytes=3_000, rtcp_every_ms=900,
                    ssrc=0x0A0A0001),
          TrackSpec("audio", "PCMA/8000", 8, ssrc=0x0A0A0002)]
    v0b = [TrackSpec("video", "H264/90000", 96, bitrate=200_000, gop=30, idr_bytes=3_000, rtcp_every_ms=900,
                     ssrc=0x0B0B0001),
           TrackSpec("audio", "PCMA/8000", 8, ssrc=0x0B0B0002)]
    v1 = [TrackSpec("video", "H264/90000", 96, bitrate=300_000, gop=20, idr_bytes=4_000, ssrc=0x11110001)]
    v1b = [TrackSpec("video", "H264/90000", 96, bitrate=300_000, gop=20, idr_bytes=4_000, ssrc=0x1111BBBB)]
    u2 = [TrackSpec("video", "H264/90000", 96, bitrate=250_000, gop=30, idr_bytes=3_000, rtcp_every_ms=700,
                    ssrc=0x22220001)]
    u2b = [TrackSpec("video", "H264/90000", 96, bitrate=250_000, gop=30, idr_bytes=3_000, rtcp_every_ms=700,
                     ssrc=0x2222BBBB)]
    v3 = [TrackSpec("video", "MP4V-ES/90000", 96, bitrate=150_000, ssrc=0x33330001)]
    tr = Trace()
    tr.add_session(make_sdp(v0))
    tr.add_session(make_sdp(v1))
    tr.add_session(make_sdp(u2), udp_push=True)
    tr.add_session(make_sdp(v3))
    dur = 36_000
    pk0 = session_packets(v0, 2000, SEED_BASE + 100)
    pk0 += session_packets(v0b, dur - 3000, SEED_BASE + 101, t0=3000)
    pk1 = session_packets(v1, 2500, SEED_BASE + 102)
    pk1 += session_packets(v1b, 3000, SEED_BASE + 103, t0=3000)
    src = _ip(10, 2, 0, 7)
    pk2 = [(t, ch, d, src, 9000 + (ch & 1)) for t, ch, d in session_packets(u2, 6000, SEED_BASE + 104)]
    pk2 += [(t, ch, d, _ip(10, 2, 0, 8), 9100 + (ch & 1))
            for t, ch, d in session_packets(u2b, 5000, SEED_BASE + 105, t0=7000)]
    pk3 = session_packets(v3, 4000, SEED_BASE + 106)           # keeps sending while unpublished
    joins = [(0, 0, 1, UDP), (0, 0, 2, TCP), (4000, 0, 3, UDP), (33_500, 0, 4, TCP),
             (0, 1, 10, UDP), (0, 1, 11, TCP), (2600, 1, 12, UDP), (3500, 1, 13, TCP),
             (0, 2, 20, UDP), (0, 2, 21, TCP), (8000, 2, 22, UDP),
             (0, 3, 30, TCP), (2000, 3, 31, UDP)]
    leaves = [(1500, 10), (1500, 11)]
    pubs = [(2000, "unpublish", 0, 0), (3000, "publish", 0),
            (2500, "unpublish", 1, 0), (3000, "publish", 1),
            (6000, "unpublish", 2, 1), (7000, "publish", 2),
            (1000, "unpublish", 3, 0), (1200, "unpublish", 3, 1), (1500, "publish", 3), (1800, "publish", 3)]
    ticks = list(range(0, 3000, 100)) + list(range(3000, 12_000, 250)) + list(range(12_000, dur + 1, 500))
    return _assemble(tr, [pk0, pk1, pk2, pk3], 100, dur, joins, tick_times=ticks, leaves=leaves, pubs=pubs)


def threaded() -> Trace:
    """The module in its default mode (its own tick thread and UDP reader thread, two pusher
    threads; tests/test_gpu_qtss_module.py): every player joins before any packet, and no
    stream carries an H.264 key frame, so each output starts at the first packet its first
    tick sees inside the 1-s buffer window (the replay holds the pushers until every player has
    received once) and follows its bookmarks from there -- the per-sub-stream bytes do not
    depend on when the ticks run.  Two RTSP-interleaved pushers (MPEG-4 + PCMA, JPEG) and a UDP
    pusher (MPEG-4 + PCMU)."""
    a = [TrackSpec("video", "MP4V-ES/90000", 96, bitrate=400_000), TrackSpec("audio", "PCMA/8000", 8)]
    b = [TrackSpec("video", "JPEG/90000", 26, bitrate=300_000)]
    c = [TrackSpec("video", "MP4V-ES/90000", 96, bitrate=300_000), TrackSpec("audio", "PCMU/8000", 0)]
    tr = Trace()
    tr.add_session(make_sdp(a))
    tr.add_session(make_sdp(b))
    tr.add_session(make_sdp(c), udp_push=True)
    dur = 3000
    pk = [session_packets(a, dur, SEED_BASE + 120, t0=100), session_packets(b, dur, SEED_BASE + 121, t0=100)]
    src = _ip(10, 3, 0, 1)
    pk.append([(t, ch, d, src, 8000 + (ch & 1)) for t, ch, d in session_packets(c, dur, SEED_BASE + 122, t0=100)])
    joins = [(0, s, 10 * s + k, (UDP, TCP, UDP)[k]) for s in range(3) for k in range(3)]
    return _assemble(tr, pk, 100, dur + 200, joins)


def prefs_buffer() -> Trace:
    """ReflectorStream's prefs at non-default values (read once, ReflectorStream::Initialize,
    ReflectorStream.cpp:87-117):

    * reflector_buffer_size_sec 3: a new output of a stream without a key frame (session 1,
      MPEG-4) starts 3 s back instead of 1 (GetClientBufferStartPacketOffset, :1201-1231), the
      packet age limit becomes 30 s (:115) and a new RTP-Info window 3 s;
    * reflector_rtp_info_offset_msec 1000: an RTP-Info player starts at the oldest packet no older
      than 3000 - 1000 ms (GetFirstPacketInfo, :728-753);
    * rtp_reflector_threshold_msec 700 -> the 1000-ms floor (:101-102): a TCP player blocked for
      1.7 s has its bookmark moved to the newest key frame after 1 s (NeedRelocateBookMark,
      :1293-1322); another blocked for 0.8 s is not relocated;
    * reflector_bucket_offset_delay_msec 40: 19 outputs on session 0, three of them in the second
      bucket of 16, whose writes' transmit times are 40 ms earlier (RTPSessionOutput.cpp:603-608)."""
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + 80))
    s0 = [TrackSpec("video", "H264/90000", 96, bitrate=500_000, gop=45, idr_bytes=6_000, rtcp_every_ms=700),
          TrackSpec("audio", "PCMA/8000", 8)]
    s1 = [TrackSpec("video", "MP4V-ES/90000", 96, bitrate=300_000), TrackSpec("audio", "PCMU/8000", 0)]
    tr = Trace()
    tr.prefs = {"reflector_buffer_size_sec": "3", "reflector_rtp_info_offset_msec": "1000",
                "rtp_reflector_threshold_msec": "700", "reflector_bucket_offset_delay_msec": "40"}
    tr.add_session(make_sdp(s0))
    tr.add_session(make_sdp(s1))
    pk0 = session_packets(s0, 6000, SEED_BASE + 81)
    pk1 = session_packets(s1, 6000, SEED_BASE + 82)
    joins = [(0, 0, k, UDP) for k in range(1, 19)] + [(0, 0, 20, TCP)]
    joins += [(2500, 0, 21, UDP, VLC), (4100, 0, 22, TCP, VLC), (1500, 1, 30, UDP), (3700, 1, 31, TCP),
              (4600, 1, 32, UDP, VLC), (5000, 1, 33, TCP, VLC)]
    ticks = list(range(0, 6001, 100))
    blocks = {}
    for t in ticks:
        if 1000 <= t < 2700:
            blocks.setdefault(t, []).append((20, 0, 0, 0))          # TCP video: 1.7 s > 1 s floor
        if 3000 <= t < 3800:
            blocks.setdefault(t, []).append((5, 0, 0, 0))           # UDP video: 0.8 s, kept
        if t % 500 == 0 and t > 0:
            blocks.setdefault(t, []).append((31, 0, 0, int(rng.integers(0, 4))))
    return _assemble(tr, [pk0, pk1], 100, 6000, joins, tick_times=ticks, blocks=blocks)


def prefs_reread() -> Trace:
    """The module's prefs at non-default values and RereadPrefs (QTSSReflectorModule.cpp:
    454-537; a PREFS event is the server rewriting its prefs and sending QTSS_RereadPrefs_Role):

    * at start: use_one_SSRC_per_stream false (session 0's pusher switching SSRCs passes whole,
      FilterInvalidSSRCs off, ReflectorStream.cpp:1819-1820), kill_clients_when_broadcast_stops
      true (the pusher's leave at 3 s tears its players down although its own flag is off, :1884,
      2156; the session dies), rtp_reflector_threshold_msec 5000 (read once: a TCP player of
      session 1 blocked for 3.5 s keeps its bookmark);
    * 3.2 s: timeout_stream_SSRC_secs 5 and player_requires_rtp_header_info "EasyPlayer"; the
      SSRC filter is back on by default; kill_clients back off.  Session 0 re-pushed at 3.5 s is a
      fresh session set up with these: its pusher's new SSRC at 4.5 s is zero-length until 5 s
      after the old SSRC's last packet; an "EasyPlayer" joiner now takes the RTP-Info PLAY, a
      "vlc" one does not;
    * 7 s: force_rtp_info_sequence_and_time (every player RTP-Info); 8.5 s:
      disable_rtp_play_info (none); session 1's pusher leaves at 9.5 s without kill (players keep
      it) and returns at 9.8 s."""
    tr = Trace()
    tr.prefs = {"use_one_SSRC_per_stream": "false", "kill_clients_when_broadcast_stops": "true",
                "rtp_reflector_threshold_msec": "5000"}
    v0 = [TrackSpec("video", "H264/90000", 96, bitrate=200_000, gop=20, idr_bytes=3_000, ssrc=0x0C0C0001)]
    v0b = [TrackSpec("video", "H264/90000", 96, bitrate=200_000, gop=20, idr_bytes=3_000, ssrc=0x0C0C00BB)]
    s1 = [TrackSpec("video", "H264/90000", 96, bitrate=300_000, gop=30, idr_bytes=4_000, rtcp_every_ms=800),
          TrackSpec("audio", "PCMA/8000", 8)]
    tr.add_session(make_sdp(v0))
    tr.add_session(make_sdp(s1))
    dur = 11_000
    pk0 = [p for p in session_packets(v0, 1000, SEED_BASE + 90)]
    pk0 += session_packets(v0b, 1000, SEED_BASE + 91, t0=1000)            # SSRC switch: passes (filter off)
    pk0 += session_packets(v0, 800, SEED_BASE + 92, t0=2000)
    pk0 += session_packets(v0, 1000, SEED_BASE + 93, t0=3500)             # the fresh session latches ...
    pk0 += session_packets(v0b, dur - 4600, SEED_BASE + 94, t0=4500)      # ... then a new SSRC: held 5 s
    pk1 = session_packets(s1, dur, SEED_BASE + 95)
    joins = [(0, 0, 1, UDP), (500, 0, 2, TCP, VLC), (1500, 0, 3, UDP),
             (3600, 0, 4, UDP), (3700, 0, 5, TCP, VLC), (6000, 0, 6, UDP), (10_500, 0, 7, TCP),
             (0, 1, 10, UDP), (0, 1, 11, TCP), (1200, 1, 12, UDP, VLC), (4000, 1, 13, UDP),
             (7200, 1, 14, UDP), (7300, 1, 15, TCP, VLC), (8700, 1, 16, UDP, VLC), (8800, 1, 17, TCP),
             (9600, 1, 18, UDP)]
    ticks = list(range(0, dur + 1, 100))
    blocks = {t: [(11, 0, 0, 0)] for t in ticks if 3000 <= t < 6500}
    pubs = [(3000, "unpublish", 0, 0), (3500, "publish", 0), (9500, "unpublish", 1, 0), (9800, "publish", 1)]
    prefs = [(3200, {"timeout_stream_SSRC_secs": "5", "player_requires_rtp_header_info": "EasyPlayer"}),
             (7000, {"force_rtp_info_sequence_and_time": "true", "timeout_stream_SSRC_secs": "5"}),
             (8500, {"disable_rtp_play_info": "true", "force_rtp_info_sequence_and_time": "true"})]
    return _assemble(tr, [pk0, pk1], 100, dur, joins, tick_times=ticks, blocks=blocks, pubs=pubs, prefs=prefs)


def keepalive() -> Trace:
    """The pushers' client-session timeouts over 70 s (SURVEY §5 broadcaster keep-alive; the
    server closes a client session whose timeout passes without a refresh, TimeoutTask.cpp,
    RTPSession.cpp:496-501).  The module sets each pusher's timeout to max(30 s,
    timeout_broadcaster_session_secs) at its SETUPs (QTSSReflectorModule.cpp:1644, 483-487), and
    every socket refreshes it on a packet when it last did more than 10 s before
    (ReflectorSocket::ProcessPacket, ReflectorStream.cpp:1779-1786) -- each socket on its own
    clock, so the video RTP socket refreshes at the first packet after 10 s and its RTCP socket,
    with SRs every 5 s, only at 15 s.

    * session 0: a UDP push (video + SRs every 5 s).  Nothing but those refreshes keeps its pusher:
      its datagrams land on the module's sockets, the server never sees them.  kill_clients is on,
      so were the pusher to time out (the replay tools' EDGPU_REPLAY_NO_REFRESH) its players 1 and
      2 would be torn down at 30 s, the session would end and player 3 joining at 35 s would find
      none;
    * session 1: an RTSP-interleaved push, which the server refreshes on every '$' frame
      (RTSPSession.cpp:2157) besides the module's refreshes; player 10."""
    u = [TrackSpec("video", "H264/90000", 96, bitrate=100_000, gop=60, idr_bytes=2_000, rtcp_every_ms=5000)]
    v = [TrackSpec("video", "H264/90000", 96, bitrate=40_000, fps=10, gop=20, idr_bytes=1_500)]
    tr = Trace()
    tr.prefs = {"kill_clients_when_broadcast_stops": "true"}
    tr.add_session(make_sdp(u), udp_push=True)
    tr.add_session(make_sdp(v))
    dur = 70_000
    src = _ip(10, 3, 0, 9)
    pk0 = [(t, ch, d, src, 6100 + (ch & 1)) for t, ch, d in session_packets(u, dur, SEED_BASE + 120)]
    pk1 = session_packets(v, dur, SEED_BASE + 121)
    joins = [(0, 0, 1, UDP), (0, 0, 2, TCP), (35_000, 0, 3, UDP), (0, 1, 10, UDP)]
    return _assemble(tr, [pk0, pk1], 250, dur, joins)


def highrate() -> Trace:
    """A stream the engine's default rings cannot hold: 1080p at 12 Mb/s
    with a 10-s GOP.  The reference keeps every packet younger than 10 x the buffer and the key
    packet with everything after it in an unbounded queue (RemoveOldPackets, ReflectorStream.cpp:
    1233-1289), so players joining at 9 s are replayed the GOP from its key packet at 0 s: ~9,600
    packets / 13.5 MB, past the default 8,192-packet / 8-MiB video ring.  The engine grows that
    sender's rings before they lose what the reference retains (edgpu_config.ring_growth)."""
    v = [TrackSpec("video", "H264/90000", 96, bitrate=12_000_000, gop=300, idr_bytes=150_000, rtcp_every_ms=1000)]
    tr = Trace()
    tr.add_session(make_sdp(v))
    dur = 11_000
    pk = session_packets(v, dur, SEED_BASE + 140)
    joins = [(0, 0, 1, UDP), (9000, 0, 2, UDP), (9000, 0, 3, TCP), (10_500, 0, 4, UDP)]
    return _assemble(tr, [pk], 100, dur, joins)


def longbuffer() -> Trace:
    """reflector_buffer_size_sec = 3 (ReflectorStream.cpp:87-117: a 3-s new-output window and a 30-s
    packet age, sMaxPacketAgeMSec) on a 4 Mb/s stream with a 2-s GOP, and a TCP player held by
    backpressure for 8 s (BLOCK from 3 s to 11 s: its bookmark holds its packet, fNeededByOutput, until
    the relocation threshold moves it, Q9) -- at the engine's default ring capacities."""
    v = [TrackSpec("video", "H264/90000", 96, bitrate=4_000_000, gop=60, idr_bytes=60_000, rtcp_every_ms=1000),
         TrackSpec("audio", "PCMA/8000", 8)]
    tr = Trace()
    tr.prefs = {"reflector_buffer_size_sec": "3"}
    tr.add_session(make_sdp(v))
    dur = 14_000
    pk = session_packets(v, dur, SEED_BASE + 141)
    joins = [(0, 0, 1, UDP), (0, 0, 2, TCP), (5000, 0, 3, UDP), (12_000, 0, 4, TCP)]
    ticks = list(range(0, dur + 1, 100))
    blocks = {t: [(2, 0, 0, 0), (2, 1, 0, 0)] for t in ticks if 3000 <= t < 11_000}
    return _assemble(tr, [pk], 100, dur, joins, tick_times=ticks, blocks=blocks)


def prefs_push() -> Trace:
    """The module prefs that gate the push path, toggled by PREFS events (RereadPrefs,
    QTSSReflectorModule.cpp:454-541).  A scenario for the QTSS module only (tools/qtss_replay):
    its fixture comes from the REFERENCE module itself (oracle/_ref/libQTSSReflectorModule_ref.so)
    in the same fake server, since the harness and the engine-level replays have no ANNOUNCE or
    second pusher to model.

    * timeout_broadcaster_session_secs 45 at start (every push SETUP sets 45 s, :1644), 20 from
      5 s (clamped to 30, :486-487);
    * enable_broadcast_push off from 1 s to 2 s: session 0's RTSP-interleaved packets are dropped
      at RTSPIncomingData (:606) -- no refresh either; session 1's UDP datagrams are not;
    * enable_broadcast_announce off from 3 s to 4 s: session 0's pusher leaves at 3.1 s (its
      players keep the session), a new one is refused at ANNOUNCE at 3.2 s (:900), so nothing is
      pushed until the next one at 4.1 s;
    * allow_duplicate_broadcasts on from 5 s: a second pusher sets up session 0's live tracks at
      5.1 s and carries its packets (:1682), a second UDP pusher joins session 1 at 5.2 s; the
      second of session 0 leaves at 6 s, which clears every track's fSetupToReceive (:2089-2096),
      so with duplicates off again (6.1 s) a third pusher still sets up at 6.2 s; session 1's
      newest pusher leaves at 7 s, its first one keeps pushing."""
    v = [TrackSpec("video", "H264/90000", 96, bitrate=300_000, gop=30, idr_bytes=4_000, rtcp_every_ms=700),
         TrackSpec("audio", "PCMA/8000", 8)]
    u = [TrackSpec("video", "H264/90000", 96, bitrate=200_000, gop=30, idr_bytes=3_000, rtcp_every_ms=900)]
    tr = Trace()
    t45 = {"timeout_broadcaster_session_secs": "45"}
    tr.prefs = dict(t45)
    tr.add_session(make_sdp(v))
    tr.add_session(make_sdp(u), udp_push=True)
    dur = 9_000
    pk0 = session_packets(v, dur, SEED_BASE + 130)
    src = _ip(10, 4, 0, 2)
    pk1 = [(t, ch, d, src, 6200 + (ch & 1)) for t, ch, d in session_packets(u, dur, SEED_BASE + 131)]
    joins = [(0, 0, 1, UDP), (0, 0, 2, TCP), (1500, 0, 3, UDP), (3500, 0, 4, TCP), (5500, 0, 5, UDP),
             (0, 1, 10, UDP), (2500, 1, 11, TCP), (7500, 1, 12, UDP)]
    pubs = [(3100, "unpublish", 0, 0), (3200, "publish", 0), (4100, "publish", 0), (5100, "publish", 0),
            (5200, "publish", 1), (6000, "unpublish", 0, 0), (6200, "publish", 0), (7000, "unpublish", 1, 0)]
    prefs = [(1000, dict(t45, enable_broadcast_push="false")), (2000, dict(t45)),
             (3000, dict(t45, enable_broadcast_announce="false")), (4000, dict(t45)),
             (5000, {"allow_duplicate_broadcasts": "true", "timeout_broadcaster_session_secs": "20"}),
             (6100, {"timeout_broadcaster_session_secs": "20"})]
    return _assemble(tr, [pk0, pk1], 100, dur, joins, pubs=pubs, prefs=prefs)


def _aktt_tag(data: bytes, receive_ms: int) -> bytes:
    """A pusher's receive-time trailer: "aktt" + BE64 receive time (ms), appended to the packet
    (ReflectorStream.cpp:1960-1994 reads the packet's last 12 bytes)."""
    return data + b"aktt" + struct.pack(">Q", receive_ms & 0xFFFFFFFFFFFFFFFF)


def aktt() -> Trace:
    """reflector_use_in_packet_receive_time on (ReflectorStream.cpp:103-107), with
    reflector_in_packet_max_receive_sec 3 and a 2-s SSRC timeout: pushers append a 12-byte "aktt"
    BE64 receive-time trailer to most packets (ReflectorSocket::ProcessPacket, :1960-1994).  A
    tagged packet loses the trailer (every subscriber gets it 12 bytes shorter) and its arrival
    becomes the socket's anchor arrival plus its receive time's offset from the anchor's -- the
    anchor being the socket's first tagged packet since its SSRC changed -- clamped to now + 3 s.
    The rewritten arrivals drive the new-output window, retention, relocation and transmit times.

    * session 0, RTSP-interleaved H.264 + PCMA: receive clock 5e9 ms + t + jitter of +-40 ms (so
      arrivals are not monotone along a queue), 1 packet in 6 untagged; crafted packets: a
      13-byte SPS + trailer (the key-frame test sees 25 bytes, the queue keeps 13), a 24-byte one
      (an RTP header left), a packet shorter than 12 bytes ending in "aktt", a tagged packet whose
      receive time jumps 100 s ahead (clamped) and one 20 s back; the pusher's SSRC changes at
      3.5 s (zero-length for 2 s, then latched: the anchor restarts) and it leaves at 6 s and
      returns at 6.4 s with the same SSRC and a clock 40 s ahead (same session: the old anchor
      holds, arrivals clamp);
    * session 1, a UDP push of MPEG-4 video (no key frames: new outputs start in the 1-s window
      of the rewritten arrivals) with SRs from the odd port, which anchor on the RTCP SSRC word
      (GetSSRC by the remote port's parity);
    * UDP, TCP and RTP-Info players joining throughout; a TCP player blocked for 2.5 s (Q9
      relocation compares arrivals)."""
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + 150))
    v = [TrackSpec("video", "H264/90000", 96, bitrate=400_000, gop=30, idr_bytes=5_000, rtcp_every_ms=900,
                   ssrc=0x0AC7AA01),
         TrackSpec("audio", "PCMA/8000", 8, ssrc=0x0AC7AA02)]
    vb = [TrackSpec("video", "H264/90000", 96, bitrate=400_000, gop=30, idr_bytes=5_000, ssrc=0x0AC7AB0B),
          TrackSpec("audio", "PCMA/8000", 8, ssrc=0x0AC7AB0C)]
    u = [TrackSpec("video", "MP4V-ES/90000", 96, bitrate=300_000, rtcp_every_ms=700)]
    tr = Trace()
    tr.prefs = {"reflector_use_in_packet_receive_time": "true", "reflector_in_packet_max_receive_sec": "3",
                "timeout_stream_SSRC_secs": "2"}
    tr.add_session(make_sdp(v))
    tr.add_session(make_sdp(u), udp_push=True)
    dur = 9_000

    def tag(lst, base, skip_every=6):
        out = []
        for k, p in enumerate(lst):
            t, ch, d = p[:3]
            if k % skip_every != skip_every - 1:
                d = _aktt_tag(d, base + t + int(rng.integers(-40, 41)))
            out.append((t, ch, d) + tuple(p[3:]))
        return out

    pk0 = tag(session_packets(v, 3500, SEED_BASE + 151), 5_000_000_000)
    pk0 += tag(session_packets(vb, 2500, SEED_BASE + 152, t0=3500), 5_000_000_000)
    pk0 += tag(session_packets(vb, dur - 6400, SEED_BASE + 153, t0=6400), 5_000_040_000)
    ssrc0 = 0x0AC7AA01
    crafted = [
        (1210, 0, _aktt_tag(rtp_header(7, 90, ssrc0, 96, False) + bytes([0x67]), 5_000_001_210)),
        (1220, 0, _aktt_tag(rtp_header(8, 90, ssrc0, 96, False), 5_000_001_220)),
        (1230, 0, rtp_header(9, 90, ssrc0, 96, False)[:7] + b"aktt"),
        (2210, 0, _aktt_tag(rtp_header(10, 180, ssrc0, 96, False) + bytes(40), 5_000_102_210)),
        (2720, 0, _aktt_tag(rtp_header(11, 270, ssrc0, 96, False) + bytes(30), 4_999_982_720)),
    ]
    pk0 = sorted(pk0 + crafted, key=lambda p: p[0])
    src = _ip(10, 5, 0, 7)
    pk1 = [(t, ch, d, src, 7200 + (ch & 1)) for t, ch, d in
           tag(session_packets(u, dur, SEED_BASE + 154), 900_000, skip_every=5)]
    joins = [(0, 0, 1, UDP), (0, 0, 2, TCP), (1500, 0, 3, UDP), (2300, 0, 4, TCP, VLC), (3000, 0, 5, UDP, VLC),
             (4200, 0, 6, UDP), (6600, 0, 7, TCP), (8000, 0, 8, UDP, VLC),
             (0, 1, 10, UDP), (1200, 1, 11, TCP), (2500, 1, 12, UDP, VLC), (5000, 1, 13, UDP), (7700, 1, 14, TCP)]
    ticks = list(range(0, dur + 1, 100))
    blocks = {t: [(2, 0, 0, 0)] for t in ticks if 4000 <= t < 6500}
    pubs = [(6000, "unpublish", 0, 0), (6400, "publish", 0)]
    return _assemble(tr, [pk0, pk1], 100, dur, joins, tick_times=ticks, blocks=blocks, pubs=pubs)


def access() -> Trace:
    """The module's access roles (QTSSReflectorModule.cpp:2199-2304), for the QTSS module only: its
    fixture comes from the REFERENCE module in tools/qtss_replay, which now runs the RTSPRoute and
    RTSPAuthorize roles before the preprocessor (a request left not allowed is answered 403 by the
    server) and logs every request's route, authorization and response (EDGPU_REQ_LOG).  Prefs:
    ip_allow_list "10.7.*.*,192.168.1.20", redirect_broadcast_keyword "/live/" (trimmed to "live"),
    the redirect directory under the movie folder.  Session 0 (RTSP-interleaved) changes pushers:

    * 1.1 s a pusher from 10.9.0.1, no user: not accepted (not local, not listed), and QTAccessFile
      stops at the request's missing root directory -> 403;
    * 1.3 s one from 10.7.3.4 (the allow list's wildcard) -> pushes;
    * 2.6 s 203.0.113.5, user "alice" in groups editors,broadcaster (BroadcasterGroup) -> pushes;
    * 3.6 s 203.0.113.6, user "bob" (editors, realm "EasyRealm") -> 403;
    * 3.7 s bob again at /live/stream0.sdp: routed (root ./Movies/, path /stream0.sdp), so QTAccessFile
      reaches the movie folder's qtaccess, takes bob's realm, and still refuses the write -> 403;
    * 3.8 s a local pusher at /LIVE/stream0.sdp: routed (any case) to the same stream -> pushes;
    * 4.0 s a player at /live/stream0.sdp: routed, its lookup path (root + file name) names no
      session -> refused; players at /stream0.sdp keep playing;
    * 4.2 s authenticate_local_broadcast on: session 2's local pusher leaves and returns -> 403;
    * 5.0 s allow_broadcasts off: a player's SETUP and session 1's returning UDP pusher are answered
      403 "Broadcast is not allowed." (AllowBroadcast); 6.0 s on again: a player joins."""
    v = [TrackSpec("video", "H264/90000", 96, bitrate=300_000, gop=30, idr_bytes=4_000, rtcp_every_ms=700),
         TrackSpec("audio", "PCMA/8000", 8)]
    u = [TrackSpec("video", "H264/90000", 96, bitrate=200_000, gop=30, idr_bytes=3_000, rtcp_every_ms=900)]
    w = [TrackSpec("video", "H264/90000", 96, bitrate=150_000, gop=20, idr_bytes=2_000)]
    tr = Trace()
    base = {"ip_allow_list": "10.7.*.*,192.168.1.20", "redirect_broadcast_keyword": "/live/"}
    tr.prefs = dict(base)
    tr.add_session(make_sdp(v))
    tr.add_session(make_sdp(u), udp_push=True)
    tr.add_session(make_sdp(w))
    dur = 7_000
    pk0 = session_packets(v, dur, SEED_BASE + 160)
    src = _ip(10, 6, 0, 3)
    pk1 = [(t, ch, d, src, 6300 + (ch & 1)) for t, ch, d in session_packets(u, dur, SEED_BASE + 161)]
    pk2 = session_packets(w, dur, SEED_BASE + 162)
    P, L = IDENT_PUSHER, IDENT_PLAYER
    idents = [(1100, 0, P, _ip(10, 9, 0, 1), "", "", "", ""),
              (1300, 0, P, _ip(10, 7, 3, 4), "", "", "", ""),
              (2600, 0, P, _ip(203, 0, 113, 5), "", "alice", "editors,broadcaster", ""),
              (3600, 0, P, _ip(203, 0, 113, 6), "", "bob", "editors", "EasyRealm"),
              (3700, 0, P, _ip(203, 0, 113, 6), "/live/stream0.sdp", "bob", "editors", "EasyRealm"),
              (3800, 0, P, _ip(127, 0, 0, 1), "/LIVE/stream0.sdp", "", "", ""),
              (4000, 0, L, _ip(127, 0, 0, 1), "/live/stream0.sdp", "", "", "")]
    pubs = [(1000, "unpublish", 0, 0), (1100, "publish", 0), (1300, "publish", 0),
            (2500, "unpublish", 0, 0), (2600, "publish", 0), (3500, "unpublish", 0, 0), (3600, "publish", 0),
            (3700, "publish", 0), (3800, "publish", 0),
            (4300, "unpublish", 2, 0), (4400, "publish", 2), (5200, "unpublish", 1, 0), (5300, "publish", 1)]
    prefs = [(4200, dict(base, authenticate_local_broadcast="true")),
             (5000, dict(base, allow_broadcasts="false")), (6000, dict(base))]
    joins = [(0, 0, 1, UDP), (0, 0, 2, TCP), (0, 1, 10, UDP), (0, 2, 20, UDP), (1500, 0, 3, UDP),
             (4000, 0, 4, UDP), (4100, 0, 5, TCP), (5100, 0, 6, UDP), (6100, 0, 7, UDP), (6200, 1, 11, TCP)]
    return _assemble(tr, [pk0, pk1, pk2], 100, dur, joins, pubs=pubs, prefs=prefs, idents=idents)


# Scenarios for the QTSS module alone: fixtures from the reference module in tools/qtss_replay
MODULE_SCENARIOS = {"prefs_push": prefs_push, "access": access}


SCENARIOS = {
    "tiny": tiny, "c1": c1, "mixed": mixed, "clamp": clamp, "ssrc": ssrc, "nal": nal,
    "nokey": nokey, "stall": stall, "anchor": anchor, "rtpinfo": rtpinfo,
    "backpressure": backpressure, "udppush": udppush, "leave": leave, "repush": repush,
    "threaded": threaded, "prefs_buffer": prefs_buffer, "prefs_reread": prefs_reread,
    "keepalive": keepalive, "highrate": highrate, "longbuffer": longbuffer, "aktt": aktt,
}


def random_scenario(seed: int, lifecycle: bool = True) -> Trace:
    """A random mix of everything above, for differential tests on fresh inputs (the oracle
    pins itself on the fixtures; these traces are not committed): 1-3 sessions, each an
    RTSP-interleaved or a UDP push of H.264 / MPEG-4 / MJPEG video and/or AAC / G.711 audio,
    pusher SRs, jittered sizes; UDP, TCP and RTP-Info players joining at random times; random
    leaves; random socket budgets (BLOCK) on TCP and UDP sub-streams; ticks every 50-200 ms;
    pushers leaving and returning (PUBLISH / UNPUBLISH, with and without kill_clients); the
    server's prefs at random values and rewritten mid-trace (PREFS: RereadPrefs).
    Kept inside the parity scope of DESIGN.md §4.4 (no lag past the 10-s retention)."""
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + 1000 + seed))
    vids = ["H264/90000", "H264/90000", "MP4V-ES/90000", "JPEG/90000"]
    auds = [("MPEG4-GENERIC/48000/2", 97), ("PCMA/8000", 8), ("PCMU/8000", 0)]
    dur = int(rng.integers(2000, 6001))
    tick = int(rng.choice([50, 100, 100, 200]))
    tr = Trace()
    per, joins, leaves, blocks = [], [], [], {}
    sub = 1
    nsess = int(rng.integers(1, 4))
    for s in range(nsess):
        tracks = []
        kinds = int(rng.integers(0, 3))                 # 0 video, 1 audio, 2 both
        if kinds != 1:
            tracks.append(TrackSpec("video", str(rng.choice(vids)), 96, bitrate=int(rng.integers(200_000, 1_500_000)),
                                    gop=int(rng.choice([15, 30, 60])), idr_bytes=int(rng.integers(3_000, 20_000)),
                                    jitter_sizes=bool(rng.random() < 0.3),
                                    rtcp_every_ms=int(rng.choice([0, 0, 400, 900]))))
        if kinds != 0:
            name, pt = auds[int(rng.integers(0, 3))]
            tracks.append(TrackSpec("audio", name, pt, jitter_sizes=bool(rng.random() < 0.2),
                                    rtcp_every_ms=int(rng.choice([0, 0, 1000]))))
        udp = bool(rng.random() < 0.3)
        tr.add_session(make_sdp(tracks), udp_push=udp)
        t0 = int(rng.integers(0, 400))
        pk = session_packets(tracks, dur, SEED_BASE + 2000 + seed * 8 + s, t0=t0)
        if udp:
            src = _ip(10, 1, int(rng.integers(0, 256)), int(rng.integers(1, 255)))
            port = 6000 + 2 * int(rng.integers(0, 100))
            pk = [(t, ch, data, src, port + (ch & 1)) for t, ch, data in pk]
        per.append(pk)
        for _ in range(int(rng.integers(1, 6))):
            t = int(rng.integers(0, dur - 200)) if rng.random() < 0.7 else 0
            transport = TCP if rng.random() < 0.5 else UDP
            ua = VLC if rng.random() < 0.25 else 0
            joins.append((t, s, sub, transport, ua))
            if rng.random() < 0.3:
                leaves.append((int(rng.integers(t, dur)), sub))
            ntr = len(tracks)
            for _b in range(int(rng.integers(0, 4))):
                bt = (int(rng.integers(t, dur)) // tick) * tick
                for k in range(int(rng.integers(1, 6))):
                    tt = bt + k * tick
                    if tt <= dur:
                        blocks.setdefault(tt, []).append((sub, int(rng.integers(0, ntr)), int(rng.integers(0, 2)),
                                                          int(rng.integers(0, 5))))
            sub += 1
    # session lifecycle, from its own generator (the traces above stay as they were): a pusher
    # leaving (with or without kill_clients) and often coming back; its packets in between are
    # dropped; sometimes a duplicate PUBLISH or UNPUBLISH
    pubs = []
    if lifecycle:
        lrng = np.random.Generator(np.random.PCG64(SEED_BASE + 3000 + seed))
        for s in range(nsess):
            if lrng.random() >= 0.35:
                continue
            t1 = int(lrng.integers(200, max(dur - 400, 201)))
            pubs.append((t1, "unpublish", s, 1 if lrng.random() < 0.4 else 0))
            if lrng.random() < 0.2:
                pubs.append((t1 + 10, "unpublish", s, 0))                  # no pusher: no effect
            if lrng.random() < 0.7:
                t2 = t1 + int(lrng.integers(50, 1500))
                if t2 < dur:
                    pubs.append((t2, "publish", s))
                    if lrng.random() < 0.2:
                        pubs.append((t2 + 10, "publish", s))            # duplicate: refused
    # preferences, from a third generator: random overrides at start, sometimes a rewrite
    prefs = []
    if lifecycle:
        prng = np.random.Generator(np.random.PCG64(SEED_BASE + 4000 + seed))
        if prng.random() < 0.4:
            tr.prefs = _random_prefs(prng, stream=True)
        if prng.random() < 0.3:
            prefs.append((int(prng.integers(100, dur)), _random_prefs(prng, stream=False)))
    return _assemble(tr, per, tick, dur, joins, blocks=blocks, leaves=leaves, pubs=pubs, prefs=prefs)


def _random_prefs(rng, stream: bool) -> dict:
    """A random subset of the prefs a trace may set (easydarwin_amd/trace.py PREF_DEFAULTS)."""
    choices = {
        "kill_clients_when_broadcast_stops": lambda: str(bool(rng.random() < 0.5)).lower(),
        "use_one_SSRC_per_stream": lambda: str(bool(rng.random() < 0.5)).lower(),
        "timeout_stream_SSRC_secs": lambda: str(int(rng.integers(1, 40))),
        "disable_rtp_play_info": lambda: str(bool(rng.random() < 0.3)).lower(),
        "enable_player_compatibility": lambda: str(bool(rng.random() < 0.7)).lower(),
        "force_rtp_info_sequence_and_time": lambda: str(bool(rng.random() < 0.3)).lower(),
        "player_requires_rtp_header_info": lambda: str(rng.choice(["Android,vlc", "EasyPlayer", "*", "LibVLC",
                                                                   "nobody"])),
    }
    if stream:
        choices.update({
            "reflector_buffer_size_sec": lambda: str(int(rng.integers(1, 5))),
            "reflector_rtp_info_offset_msec": lambda: str(int(rng.integers(0, 2000))),
            "rtp_reflector_threshold_msec": lambda: str(int(rng.integers(0, 6000))),
            "reflector_bucket_offset_delay_msec": lambda: str(int(rng.integers(0, 150))),
        })
    keys = sorted(choices)
    pick = [k for k in keys if rng.random() < 0.4]
    return {k: choices[k]() for k in pick}


def spec_stress(tick_ms: int = 1000) -> Trace:
    """Refusals inside large ingest rounds, for k_ingest's speculative copy: the copy
    runs at each packet's guessed ring place before the header decides, so every refusal leaves
    a hole.  Not a golden: the oracle is pinned to the compiled reference on it (CPU test).

    * session 0, an 8 Mb/s H.264 push (~700 packets per 1-s tick, several 256-packet rounds):
      from 1.5 s a second pusher SSRC interleaves runs of 1 to 300 packets (zero-length after
      the SSRC filter, runs crossing round and tick boundaries), players joining inside runs;
    * session 1, a UDP push whose odd port also carries bursts of receiver reports and truncated
      SRs (refused by the SR gate, Q14: holes with no queue entry) between its SRs;
    * session 2, an audio-only push with the receive-time trailer on its odd packets.
    UDP and TCP players join throughout."""
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + 170))
    dur = 6_000
    v = [TrackSpec("video", "H264/90000", 96, bitrate=8_000_000, gop=30, idr_bytes=60_000, ssrc=0x5BEC0001),
         TrackSpec("audio", "MPEG4-GENERIC/48000/2", 97, ssrc=0x5BEC0002)]
    u = [TrackSpec("video", "H264/90000", 96, bitrate=2_000_000, gop=30, idr_bytes=20_000, rtcp_every_ms=300)]
    a = [TrackSpec("audio", "PCMA/8000", 8, ssrc=0x5BEC0A0A)]
    tr = Trace()
    tr.prefs = {"reflector_use_in_packet_receive_time": "true"}
    tr.add_session(make_sdp(v))
    tr.add_session(make_sdp(u), udp_push=True)
    tr.add_session(make_sdp(a))
    pk0 = []
    seq_b = 0
    for t, ch, data in session_packets(v, dur, SEED_BASE + 171):
        pk0.append((t, ch, data))
        if ch == 0 and t >= 1500 and rng.random() < 0.01:       # a run of the foreign SSRC
            for _ in range(int(rng.integers(1, 301))):
                seq_b += 1
                nal = 0x65 if rng.random() < 0.05 else 0x41
                pay = bytes([nal]) + rng.integers(0, 256, size=int(rng.integers(20, 1400)), dtype=np.uint8).tobytes()
                pk0.append((t, 0, rtp_header(seq_b, t * 90, 0x0BADBEEF, 96, False) + pay))
    src = _ip(10, 0, 7, 7)
    pk1 = []
    for t, ch, data in session_packets(u, dur, SEED_BASE + 172):
        pk1.append((t, ch, data, src, 6000 + (ch & 1)))
        if ch == 0 and rng.random() < 0.03:                       # refused on the odd port
            for _ in range(int(rng.integers(1, 40))):
                if rng.random() < 0.5:
                    rr = struct.pack(">BBHI", 0x81, 201, 7, 0x1234) + bytes(24)
                else:
                    rr = rtcp_sr(0x5BEC00FF, t, 0, 1, 1)[:int(rng.integers(8, 24))]
                pk1.append((t, 1, rr, src, 6001))
    pk2 = []
    for k, (t, ch, data) in enumerate(session_packets(a, dur, SEED_BASE + 173)):
        if k % 2:
            data = data + b"aktt" + struct.pack(">Q", 7_000_000_000 + t + int(rng.integers(0, 30)))
        pk2.append((t, ch, data))
    joins, sub = [], 1
    for t in sorted(int(x) for x in rng.integers(0, dur - 300, size=14)):
        joins.append((t, int(rng.integers(0, 3)), sub, TCP if rng.random() < 0.4 else UDP))
        sub += 1
    for s in range(3):
        joins.append((0, s, sub, UDP))
        sub += 1
    return _assemble(tr, [pk0, pk1, pk2], tick_ms, dur, joins)
