"""GPU + sockets: the engine's socket egress (edgpu_egress_*).

* Every golden scenario's ticks leave through edgpu_egress_send to loopback UDP receivers and
  RTSP-interleaved socketpairs; the capture rebuilt from the bytes the receivers read equals
  the reference reflector's capture.
* TCP backpressure over real sockets: small send buffers and readers held back for a while
  make the socket refuse writes (EAGAIN); the egress reports each blocked sub-stream to the
  engine (edgpu_fanout_blocked), and the bytes that finally arrive equal what the reference
  harness and the restatement produce when their sinks block at exactly the same writes
  (the reports replayed as BLOCK events).
"""
import hashlib
import json
import os
import subprocess

import pytest

from easydarwin_amd.replay import replay
from easydarwin_amd.trace import BLOCK, TICK, TCP, Trace, capture_summary, read_capture
import scenarios
from scenarios import SCENARIOS

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _fixture(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        return json.load(f)


@pytest.mark.gpu
# `highrate` replays a 13.5-MB GOP to two UDP players in one tick -- past what a loopback receive
# buffer holds (net.core.rmem_max): the receivers drain on their own threads while the egress sends
# (SocketSink, tools/udp_drain.c), so every datagram arrives
@pytest.mark.parametrize("name", [n for n in SCENARIOS                     # not the scripted BLOCKs
                                  if not any(ev[0] == BLOCK for ev in SCENARIOS[n]().events)])
def test_socket_egress_matches_reference(name):
    cap, _ = replay(SCENARIOS[name](), sockets={"threads": 3})
    fix = _fixture(name)
    got = capture_summary(read_capture(cap))
    bad = [k for k in fix["substreams"] if got.get(k) != fix["substreams"][k]]
    assert not bad, f"{len(bad)} sub-streams differ over sockets, e.g. {bad[:3]}"
    assert hashlib.sha256(cap).hexdigest() == fix["capture_sha256"]


def _with_blocks(tr: Trace, blocked) -> Trace:
    by_t = {}
    for t, sub, trk, kind, sent in blocked:
        by_t.setdefault(t, []).append((sub, trk, kind, sent))
    out = Trace(sdps=list(tr.sdps), flags=list(tr.flags), prefs=dict(tr.prefs))
    for ev in tr.events:
        if ev[0] == TICK:
            for sub, trk, kind, sent in by_t.get(ev[1], []):
                out.events.append((BLOCK, ev[1], sub, trk, kind, sent))
        out.events.append(ev)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["stall", "anchor", "mixed"])
def test_tcp_backpressure_over_sockets(name, oracle_bins, tmp_path):
    tr = SCENARIOS[name]()
    tcp_subs = {ev[3] for ev in tr.events if ev[0] == 2 and ev[4] == TCP}
    ticks = [ev[1] for ev in tr.events if ev[0] == TICK]
    # hold every TCP reader for a stretch of ticks in the middle of the run
    lo, hi = ticks[len(ticks) // 4], ticks[len(ticks) // 2]
    hold = {t: tcp_subs for t in ticks if lo <= t < hi}
    report = []
    cap, _ = replay(tr, sockets={"threads": 2, "tcp_sndbuf": 4096, "hold": hold, "report": report})
    assert report, "no write blocked: the test did not exercise backpressure"
    tb = _with_blocks(tr, report)
    p = tmp_path / "bp.edtr"
    tb.write(str(p))
    for which in ("port", "ref"):
        exe = oracle_bins[which]
        if exe is None:
            continue
        c = tmp_path / f"{which}.edcp"
        subprocess.run([exe, str(p), str(c)], check=True, stderr=subprocess.DEVNULL)
        want = capture_summary(read_capture(c.read_bytes()))
        got = capture_summary(read_capture(cap))
        bad = [k for k in want if got.get(k) != want[k]]
        assert not bad, f"{which}: {len(bad)} sub-streams differ, e.g. {bad[:3]}"


@pytest.mark.gpu
@pytest.mark.parametrize("dedup,gso", [("0", "1"), ("1", "1"), ("1", "0"), ("0", "0")])
@pytest.mark.parametrize("name", ["udppush", "c1", "mixed"])
def test_egress_copy_modes_match_reference(name, dedup, gso, monkeypatch):
    """EDGPU_EGRESS_DEDUP=1 (default) brings one region per identity sender over PCIe
    (edgpu_arena_gather) instead of the whole write-many arena; EDGPU_EGRESS_GSO=1 (default)
    sends runs of equal-length datagrams as UDP GSO messages: the same datagrams on the wire
    in every combination."""
    monkeypatch.setenv("EDGPU_EGRESS_DEDUP", dedup)
    monkeypatch.setenv("EDGPU_EGRESS_GSO", gso)
    cap, _ = replay(SCENARIOS[name](), sockets={"threads": 2})
    assert hashlib.sha256(cap).hexdigest() == _fixture(name)["capture_sha256"]


@pytest.mark.gpu
def test_egress_dedup_copies_less_and_reports_dead_peers():
    import numpy as np
    from easydarwin_amd import edgpu
    from easydarwin_amd.egress import SocketSink
    from easydarwin_amd.synth import TrackSpec, make_sdp, session_packets
    tracks = [TrackSpec("video", "H264/90000", 96, bitrate=800_000, gop=30, idr_bytes=9_000)]
    pk = session_packets(tracks, 3000, 0xEA5D + 99)
    with edgpu.Context() as ctx:
        s = ctx.session_add(make_sdp(tracks))
        sink = SocketSink(ctx, threads=2)
        hs = [ctx.subscriber_add(s, edgpu.TRANSPORT_UDP) for _ in range(4)]
        ht = [ctx.subscriber_add(s, edgpu.TRANSPORT_TCP) for _ in range(2)]
        for i, h in enumerate(hs + ht):
            sink.join(h, 100 + i, 1, h in ht)
        sent_copy, arena = [], []
        for tick in range(1, 31):
            t = tick * 100
            batch = [(s, ch, tt, d) for tt, ch, d in pk if t - 100 < tt <= t]
            if batch:
                desc, so, ss, blob = edgpu.build_batch(batch)
                ctx.ingest_host(desc, so, ss, blob)
                ctx.keyframe_index()
            r = ctx.fanout(t)
            st = sink.tick(r, t)
            sent_copy.append(st.copied_bytes)
            arena.append(ctx.stats().arena_bytes)
            if tick == 10:                          # the player's end goes away: EPIPE, not EAGAIN
                gone = sink.tcp.pop(ht[0])
                gone[1].close()
        # 6 copies in the arena (4 identical UDP + 2 TCP); the egress copies 3 of them (one UDP)
        assert sum(sent_copy) * 2 <= sum(arena) * 1.01
        assert sink.eg.disconnected() == [ht[0]]
        assert sink.eg.disconnected() == []         # reported once
        # the other TCP player and the UDP players kept receiving after the disconnect
        sink.drain()
        assert len(sink.tcp[ht[1]][2]) > 0 and all(len(sink.parts[(h, 0, 0)]) > 0 for h in hs)
        sink.close()
        gone[0].close()


@pytest.mark.gpu
@pytest.mark.parametrize("gso", ["1", "0"])
def test_udp_overload_loses_datagrams_without_reordering(gso, monkeypatch):
    """A UDP subscriber that cannot keep up loses datagrams, as RTPStream::Write's ignored
    SendTo result loses them (RTPStream.cpp:1145).  With GSO (EDGPU_EGRESS_GSO=1, the default)
    a refused send drops a whole message of up to 64 equal-length datagrams instead of one
    (include/edgpu.h, egress section); either way what arrives is, per sub-stream, an in-order
    subset of what the tick sent: no reordering, no duplicates."""
    import socket
    from easydarwin_amd import edgpu
    from easydarwin_amd.egress import SocketSink
    from easydarwin_amd.synth import TrackSpec, make_sdp, session_packets
    monkeypatch.setenv("EDGPU_EGRESS_GSO", gso)
    tracks = [TrackSpec("video", "H264/90000", 96, bitrate=8_000_000, gop=30, idr_bytes=60_000)]
    pk = session_packets(tracks, 4000, 0xEA5D + 98)
    with edgpu.Context() as ctx:
        s = ctx.session_add(make_sdp(tracks))
        sink = SocketSink(ctx, threads=2)
        hs = [ctx.subscriber_add(s, edgpu.TRANSPORT_UDP) for _ in range(3)]
        for i, h in enumerate(hs):
            sink.join(h, 200 + i, 1, False)
            sink.udp[(h, 0, 0)].setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)   # overloads
        lost = 0
        for tick in range(1, 5):
            t = tick * 1000
            batch = [(s, ch, tt, d) for tt, ch, d in pk if t - 1000 < tt <= t]
            desc, so, ss, blob = edgpu.build_batch(batch)
            ctx.ingest_host(desc, so, ss, blob)
            ctx.keyframe_index()
            r = ctx.fanout(t)
            st, subs, dsc, arena = ctx.read_tick(r)
            sent = {}
            for q in subs:
                if int(q["desc_count"]) and int(q["kind"]) == 0:
                    d = dsc[int(q["desc_base"]):int(q["desc_base"]) + int(q["desc_count"])]
                    sent[int(q["subscriber"])] = [arena[o:o + n].tobytes() for o, n in zip(d["offset"], d["len"])]
            before = {h: len(sink.parts[(h, 0, 0)]) for h in hs}
            sink.tick(r, t)
            for h in hs:
                got = [p[2:] for p in sink.parts[(h, 0, 0)][before[h]:]]
                want = sent.get(h, [])
                it = iter(want)
                assert all(any(g == w for w in it) for g in got), f"tick {t} handle {h}: reordered or duplicated"
                lost += len(want) - len(got)
        assert lost > 0, "the receivers kept up: the test did not overload them"
        sink.close()


def _gate_reference(tr: Trace, report, exe, tmp_path):
    """The reference harness with the server's write gate (EDTR_SERVER_GATE=1) and the socket
    budgets the egress met."""
    p = tmp_path / "gate.edtr"
    _with_blocks(tr, report).write(str(p))
    c = tmp_path / "gate.edcp"
    r = subprocess.run([exe, str(p), str(c)], check=True, stderr=subprocess.PIPE, text=True,
                       env=dict(os.environ, EDTR_SERVER_GATE="1"))
    stale = [int(ln.split()[-1]) for ln in r.stderr.splitlines() if "gate stale_dropped" in ln]
    return capture_summary(read_capture(c.read_bytes())), (stale[-1] if stale else None)


@pytest.mark.gpu
@pytest.mark.parametrize("name", [n for n in SCENARIOS
                                  if not any(ev[0] == BLOCK for ev in SCENARIOS[n]().events)])
def test_paced_egress_matches_the_reference_server_gate(name, oracle_bins, tmp_path):
    """Q20: with pacing on (edgpu_egress_pacing) the egress applies the server's RTPStream::Write
    gate -- the over-buffer window holds a new output's first packets until their transmit time
    (its buffer delay then becomes their age, RTPSessionOutput.cpp:612-622), and relocation,
    bookmarks and the next ticks follow from that -- and its sockets carry exactly what the
    reference harness writes through the same gate (compiled RTPOverbufferWindow)."""
    if oracle_bins["ref"] is None:
        pytest.skip("oracle/_ref/ref_harness not built")
    tr = SCENARIOS[name]()
    report = []
    cap, _ = replay(tr, sockets={"threads": 2, "pacing": {}, "report": report})
    want, _ = _gate_reference(tr, report, oracle_bins["ref"], tmp_path)
    got = capture_summary(read_capture(cap))
    bad = [k for k in want if got.get(k) != want[k]]
    assert not bad, (f"{len(bad)} sub-streams differ, e.g. {[(k, got.get(k), want[k]) for k in bad[:3]]}; "
                     f"{len(report)} socket blocks, e.g. {report[:12]}")


@pytest.mark.gpu
@pytest.mark.parametrize("seconds", [12, 16])
def test_paced_egress_thins_congested_tcp_audio_like_the_reference(seconds, oracle_bins, tmp_path):
    """Q20: TCP readers held for most of the run -- the interleaved connections stall, packets
    queue in the rings, and once an audio packet is more than drop_all_packets_delay (2.5 s) late
    RTPStream::UpdateQualityLevel drops it (RTPStream.cpp:936-1045).  The egress drops exactly the
    packets the reference harness's gate drops, and writes exactly what it writes.  A late packet
    must still be in the queue, so the 'mixed' scenario runs longer with a 10-s reflector buffer
    (reflector_buffer_size_sec); the send buffers hold about a second of a stream, so a reader
    that is drained again catches up (a smaller one starves the audio behind the video)."""
    if oracle_bins["ref"] is None:
        pytest.skip("oracle/_ref/ref_harness not built")
    tr = scenarios.mixed(seconds * 1000)
    tr.prefs = dict(tr.prefs, reflector_buffer_size_sec="10")
    tcp_subs = {ev[3] for ev in tr.events if ev[0] == 2 and ev[4] == TCP}
    ticks = [ev[1] for ev in tr.events if ev[0] == TICK]
    lo, hi = ticks[len(ticks) // 6], ticks[5 * len(ticks) // 6]
    hold = {t: tcp_subs for t in ticks if lo <= t < hi}
    report, stats = [], []
    cap, _ = replay(tr, sockets={"threads": 2, "tcp_sndbuf": 65536, "hold": hold, "pacing": {}, "report": report,
                                 "stats": stats})
    assert report, "no write blocked: the test did not congest the connections"
    want, ref_stale = _gate_reference(tr, report, oracle_bins["ref"], tmp_path)
    got = capture_summary(read_capture(cap))
    stale = sum(s.stale_dropped for s in stats)
    assert ref_stale, f"the reference dropped no stale packet: thinning was not exercised ({len(report)} blocks)"
    bad = [k for k in want if got.get(k) != want[k]]
    assert not bad, (f"{len(bad)} sub-streams differ, e.g. {[(k, got.get(k), want[k]) for k in bad[:3]]}; "
                     f"stale {stale} vs the reference's {ref_stale}")
    assert stale == ref_stale

@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_paced_egress_matches_the_reference_server_gate_on_random_traces(seed, oracle_bins, tmp_path):
    """Q20 on fresh random traces (random sessions, codecs, UDP / interleaved pushers, UDP / TCP /
    RTP-Info players, leaves, pusher lifecycle, random prefs; their socket budgets dropped -- the
    sockets' own take their place): the paced egress against the reference harness's gate."""
    from scenarios import random_scenario
    if oracle_bins["ref"] is None:
        pytest.skip("oracle/_ref/ref_harness not built")
    r0 = random_scenario(seed)
    tr = Trace(sdps=list(r0.sdps), events=[ev for ev in r0.events if ev[0] != BLOCK], flags=list(r0.flags),
               prefs=dict(r0.prefs))
    report = []
    cap, _ = replay(tr, sockets={"threads": 2, "pacing": {}, "report": report})
    want, _ = _gate_reference(tr, report, oracle_bins["ref"], tmp_path)
    got = capture_summary(read_capture(cap))
    bad = [k for k in want if got.get(k) != want[k]]
    assert not bad, (f"{len(bad)} sub-streams differ, e.g. {[(k, got.get(k), want[k]) for k in bad[:3]]}; "
                     f"{len(report)} socket blocks")
