"""GPU parity of the RTSP-interleaved push ingest (edgpu_ingest_interleaved, '$'-deframe on the
device) through the C ABI.

* Per-read reports (frames completed, bytes consumed, RTSP-message / dropped-connection
  status, carried bytes) equal the restatement's (oracle/interleave.py ingest_reads, itself
  pinned to the reference RTSPRequestStream in tests/test_interleave.py) on every seeded
  connection -- in one call and split over many calls (device-side carry).
* Frame contents, channels and arrival times: the golden scenarios replayed as TCP pushes
  (random read splits, carried prefixes, RTSP keep-alives between frames) reproduce the
  reference reflector's captures byte for byte.
* Many sessions at once, multi-chunk streams, '$'-dense payloads (sequential fallback walk),
  device-resident reads, capacity overflow, argument checks.
"""
import hashlib
import json
import os
import random
import struct

import numpy as np
import pytest

from easydarwin_amd import edgpu
from easydarwin_amd.replay import replay
from easydarwin_amd.synth import TrackSpec, make_sdp
from easydarwin_amd.trace import PKT, Trace
from interleave_cases import CASES, case, _frame, _split
from oracle.interleave import ingest_reads
from scenarios import SCENARIOS

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SDP = make_sdp([TrackSpec("video", "H264/90000"), TrackSpec("audio", "MPEG4-GENERIC/44100/2", pt=97)])
CFG = dict(max_batch_bytes=64 << 20, max_batch_packets=1 << 17, out_arena_bytes=16 << 20,
           max_out_packets=1 << 16)


def _rows(reads_by_session, t0=0):
    rows, blob = [], bytearray()
    for s, reads in reads_by_session:
        for k, r in enumerate(reads):
            rows.append((s, len(r), len(blob), t0 + k))
            blob += r
    return rows, bytes(blob)


def _call(ctx, rows, blob, device=False):
    arr = np.array(rows, dtype=edgpu.TCP_READ_DTYPE)
    if not device:
        return ctx.ingest_interleaved(arr, blob)
    # device-resident reads: a buffer from the context, filled through the HIP runtime libedgpu
    # itself uses (libamdhip64.so.7 is already loaded in this process)
    import ctypes as C
    buf = ctx.device_alloc(max(len(blob), 16))
    hip = C.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.c_int]
    assert hip.hipMemcpy(C.c_void_p(buf.ptr), blob, len(blob), 1) == 0      # hipMemcpyHostToDevice
    try:
        return ctx.ingest_interleaved(arr, len(blob), device_ptr=buf.ptr)
    finally:
        buf.free()


def _as_list(res):
    return [[int(r["frames"]), int(r["consumed"]), int(r["status"]), int(r["carry"])] for r in res]


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_report_matches_restatement_one_call(name):
    reads = case(name)
    rows, blob = _rows([(0, reads)])
    want, frames = ingest_reads({}, rows, blob)
    with edgpu.Context(**CFG) as ctx:
        ctx.session_add(SDP)
        got = _call(ctx, rows, blob)
        ctx.keyframe_index()
        assert _as_list(got) == want
        assert ctx.stats().ingested_packets == len(frames)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_report_matches_restatement_split_calls(name):
    reads = case(name)
    rng = random.Random(name)
    carry = {}
    with edgpu.Context(**CFG) as ctx:
        ctx.session_add(SDP)
        k = 0
        while k < len(reads):
            m = rng.choice([1, 2, 5, 40])
            rows, blob = _rows([(0, reads[k:k + m])], t0=k)
            want, _ = ingest_reads(carry, rows, blob)
            got = _as_list(_call(ctx, rows, blob))
            ctx.keyframe_index()
            assert got == want, f"call at read {k}"
            if any(r[2] for r in want):
                break
            k += m


@pytest.mark.gpu
def test_many_sessions_device_reads():
    """64 sessions in one call, each a different seeded connection shape, reads resident in
    HBM (EDGPU_PTR_DEVICE); then a second call continuing every session's carry."""
    _many_sessions()


# The deframe walk's three shapes (EDGPU_TCP_WALK, read at context creation; TcpParams.walk):
# every chunk from candidate windows at once, one serial chain per session, and segments of
# EDGPU_TCP_SEG chunks (the default, 4) -- seg 1 is the per-chunk walk, seg 3 ends segments
# mid-stream at odd chunk counts.  Each must give the restatement's reports and the reference's
# frames.
WALKS = [("parallel", 4), ("serial", 4), ("seg", 1), ("seg", 2), ("seg", 3), ("seg", 8)]


@pytest.mark.gpu
@pytest.mark.parametrize("walk,seg", WALKS, ids=[f"{w}{s if w == 'seg' else ''}" for w, s in WALKS])
def test_walk_shapes_match_restatement(walk, seg, monkeypatch):
    monkeypatch.setenv("EDGPU_TCP_WALK", walk)
    monkeypatch.setenv("EDGPU_TCP_SEG", str(seg))
    for name in CASES:
        reads = case(name)
        rows, blob = _rows([(0, reads)])
        want, frames = ingest_reads({}, rows, blob)
        with edgpu.Context(**CFG) as ctx:
            ctx.session_add(SDP)
            got = _call(ctx, rows, blob)
            ctx.keyframe_index()
            assert _as_list(got) == want, name
            assert ctx.stats().ingested_packets == len(frames), name
    _many_sessions()
    for name in ("anchor", "prefs_buffer"):
        cap, _ = replay(_trace(name), interleaved=1)
        with open(os.path.join(GOLD, name + ".json")) as f:
            assert hashlib.sha256(cap).hexdigest() == json.load(f)["capture_sha256"], name


def _many_sessions():
    rng = random.Random(5)
    conns = []
    for s in range(64):
        parts = [_frame(rng.randrange(4), rng.randbytes(rng.randint(0, 2043)) if rng.random() < 0.8
                        else b"$" * rng.randint(0, 2043)) for _ in range(rng.randint(0, 120))]
        data = b"".join(parts) + _frame(0, rng.randbytes(1000))[: rng.randint(0, 1003)]
        conns.append(_split(rng, data, 1, rng.choice([7, 300, 5000, 70000]), zero=0.02))
    carry = {}
    with edgpu.Context(**CFG) as ctx:
        for _ in range(64):
            ctx.session_add(SDP)
        for rnd in range(2):
            batch = []
            for s, reads in enumerate(conns):
                h = len(reads) // 2
                batch.append((s, reads[:h] if rnd == 0 else reads[h:]))
            rows, blob = _rows(batch, t0=1000 * rnd)
            want, frames = ingest_reads(carry, rows, blob)
            got = _as_list(_call(ctx, rows, blob, device=True))
            ctx.keyframe_index()
            assert got == want
            assert ctx.stats().ingested_packets == len(frames)


def _tcp_ok(trace):
    return all(len(ev[4]) <= 2043 for ev in trace.events if ev[0] == PKT)


def _trace(name):
    p = os.path.join(GOLD, name + ".edtr")
    if os.path.exists(p):
        with open(p, "rb") as f:
            return Trace.from_bytes(f.read())
    return SCENARIOS[name]()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
@pytest.mark.parametrize("name", list(SCENARIOS))
def test_interleaved_push_matches_reference(name, seed):
    tr = _trace(name)
    if not _tcp_ok(tr):
        pytest.skip("packets above 2043 bytes cannot travel RTSP-interleaved")
    cap, _ = replay(tr, interleaved=seed)
    with open(os.path.join(GOLD, name + ".json")) as f:
        fix = json.load(f)
    assert hashlib.sha256(cap).hexdigest() == fix["capture_sha256"]


@pytest.mark.gpu
def test_capacity_overflow_leaves_state_unchanged():
    reads = case("rtp_mix")
    rows, blob = _rows([(0, reads)])
    with edgpu.Context(max_batch_packets=64, max_batch_bytes=8 << 20, out_arena_bytes=1 << 20,
                       max_out_packets=1 << 12) as ctx:
        ctx.session_add(SDP)
        with pytest.raises(edgpu.EdgpuError) as e:
            _call(ctx, rows, blob)
        assert e.value.code == edgpu.OUT_OVERFLOW
        # the same bytes in small calls go through, with the same report as the restatement
        carry, k = {}, 0
        while k < len(reads):
            rows, blob = _rows([(0, reads[k:k + 10])], t0=k)
            want, _ = ingest_reads(carry, rows, blob)
            assert _as_list(_call(ctx, rows, blob)) == want
            ctx.keyframe_index()
            k += 10


@pytest.mark.gpu
def test_argument_checks():
    with edgpu.Context(**CFG) as ctx:
        tcp = ctx.session_add(SDP)
        udp = ctx.session_add(SDP, udp_push=True)
        f = _frame(0, b"x" * 20)
        bad = [
            [(udp, len(f), 0, 0)],                                  # UDP-push session
            [(tcp, 10, 0, 0), (tcp, 10, 12, 0)],                    # not contiguous
            [(tcp, 10, 0, 0), (5, 10, 10, 0)],                      # unknown session
            [(tcp, 30, 0, 0)],                                      # outside the bytes
        ]
        for rows in bad:
            with pytest.raises(edgpu.EdgpuError) as e:
                _call(ctx, rows, f)
            assert e.value.code == edgpu.BAD_ARGUMENT
        two = f + f
        rows = [(tcp, len(f), 0, 0), (tcp, len(f), len(f), 0)]
        assert _as_list(_call(ctx, rows, two)) == [[1, len(f), 0, 0], [1, len(f), 0, 0]]


@pytest.mark.gpu
def test_long_session_frames_match_restatement():
    """One session with ~9.5 MiB of frames in one call: more chunks than k_ingest keeps in LDS
    (256) and more reads than k_ingest / k_tcp_finish keep in LDS (64), so the frame lookups take
    their global-memory paths; audio bursts put > 32 frames into some chunks, which the walk does
    not record (k_tcp_finish re-walks them).  Every relayed datagram and its arrival time equal
    the restatement's frames, per channel, in order."""
    from oracle.interleave import FRAME, deframe
    rng = random.Random(11)
    frames, seq = [], [0, 0]
    for i in range(8800):
        if i % 200 < 170:
            ch, pt, body = 0, 96, bytes([0x41]) + rng.randbytes(rng.randint(980, 1380))
        else:
            ch, pt, body = 2, 97, rng.randbytes(rng.randint(40, 80))
        k = ch // 2
        hdr = struct.pack(">BBHII", 0x80, pt, seq[k] & 0xFFFF, 3000 * seq[k], 0x5EED0000 + k)
        seq[k] += 1
        frames.append(_frame(ch, hdr + body))
    data = b"".join(frames)
    reads, at = [], 0
    while at < len(data):
        n = rng.randint(80_000, 120_000)
        reads.append(data[at:at + n])
        at += n
    assert len(reads) > 64 and len(data) > 256 * 32768
    t0 = 50_000
    rows, blob = _rows([(0, reads)], t0=t0)
    want, _ = ingest_reads({}, rows, blob)
    cfg = dict(max_batch_bytes=16 << 20, max_batch_packets=1 << 15, out_arena_bytes=32 << 20,
               max_out_packets=1 << 15, video_ring_bytes=32 << 20, video_ring_packets=1 << 14,
               other_ring_packets=1 << 12)
    with edgpu.Context(**cfg) as ctx:
        s = ctx.session_add(SDP)
        ctx.subscriber_add(s)
        got = _call(ctx, rows, blob)
        ctx.keyframe_index()
        assert _as_list(got) == want
        r = ctx.fanout(t0 + len(reads))
        st, subs, desc, arena = ctx.read_tick(r)
        arr = ctx.fanout_arrivals(st.relayed_packets)
    exp = {0: [], 1: []}
    for kind, rd, ch, _, payload in deframe(reads):
        assert kind == FRAME
        exp[ch // 2].append((payload, t0 + rd))
    seen = set()
    for q in subs:
        if int(q["kind"]) != 0 or int(q["desc_count"]) == 0:
            continue
        tr = int(q["track"])
        b = int(q["desc_base"])
        d = desc[b:b + int(q["desc_count"])]
        pk = [arena[o:o + n].tobytes() for o, n in zip(d["offset"].tolist(), d["len"].tolist())]
        assert pk == [p for p, _ in exp[tr]], f"track {tr} bytes"
        assert arr[b:b + len(d)].tolist() == [t for _, t in exp[tr]], f"track {tr} arrivals"
        seen.add(tr)
    assert seen == {0, 1}
