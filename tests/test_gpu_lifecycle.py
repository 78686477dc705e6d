"""GPU: the session lifecycle of the engine (edgpu_session_remove) -- the end of a
ReflectorSession at reference count 0 and a fresh session for the next pusher
(QTSSReflectorModule.cpp:1379-1545, 2133-2196).

* 1000 create / join / ingest / fan-out / remove cycles leave the device's free memory flat
  (the rings, 16+ MiB per session, are freed; ids and table rows are reused);
* removal needs EDGPU_SESSION_KILL_OUTPUTS while subscribers are attached, and then takes them
  with it; a removed session and its subscribers are refused by every call that names them;
* a session added after a removal (same id) starts fresh: packet ids from 1, no key pointer,
  an unlatched SSRC filter -- while the subscribers of other sessions are undisturbed.
The byte-exact end-to-end check is the ``repush`` golden (tests/test_gpu_parity.py and the
adapter / module replays).
"""
import ctypes as C

import numpy as np
import pytest

from easydarwin_amd import edgpu
from easydarwin_amd.synth import TrackSpec, make_sdp

AV = [TrackSpec("video", "H264/90000", 96), TrackSpec("audio", "PCMA/8000", 8)]


def _rtp(seq, ts, ssrc=0x1234, payload=b"\x65" + b"\x00" * 40, pt=96):
    return bytes([0x80, pt, seq >> 8, seq & 0xFF]) + ts.to_bytes(4, "big") + ssrc.to_bytes(4, "big") + payload


def _ingest(ctx, pkts):
    desc, seg_off, seg_sess, blob = edgpu.build_batch(pkts)
    ctx.ingest_host(desc, seg_off, seg_sess, blob)
    ctx.keyframe_index()


def _free_bytes():
    hip = C.CDLL("libamdhip64.so")
    free, total = C.c_size_t(), C.c_size_t()
    assert hip.hipMemGetInfo(C.byref(free), C.byref(total)) == 0
    return free.value


def _relayed(ctx, t):
    r = ctx.fanout(t)
    st, subs, desc, arena = ctx.read_tick(r)
    return st, subs, desc, arena


@pytest.mark.gpu
def test_thousand_create_remove_cycles_keep_memory_flat():
    with edgpu.Context() as ctx:
        other = ctx.session_add(make_sdp(AV))            # a long-lived neighbour session
        h_other = ctx.subscriber_add(other)

        def cycle(k):
            s = ctx.session_add(make_sdp(AV))
            h = [ctx.subscriber_add(s, edgpu.TRANSPORT_UDP), ctx.subscriber_add(s, edgpu.TRANSPORT_TCP)]
            _ingest(ctx, [(s, 0, 10 * k, _rtp(1, 0)), (s, 2, 10 * k, _rtp(1, 0, pt=8, payload=b"\x11" * 160)),
                          (other, 0, 10 * k, _rtp(k & 0xFFFF, k))])
            st, *_ = _relayed(ctx, 10 * k)
            assert st.status == 0
            ctx.session_remove(s, kill_outputs=True)
            return s, h

        ids = set()
        for k in range(20):                              # warm-up: tables reach their size
            ids.add(cycle(k)[0])
        ctx.sync()
        base = _free_bytes()
        for k in range(20, 1020):
            ids.add(cycle(k)[0])
        ctx.sync()
        grown = base - _free_bytes()
        assert len(ids) == 1, f"session ids not reused: {sorted(ids)[:8]}"
        # without the removal this loop would hold 1000 x (2 x 8.25 MiB + 2 x 1.06 MiB) = 18 GiB
        assert grown < (64 << 20), f"device memory grew by {grown >> 20} MiB over 1000 cycles"
        st, subs, desc, _ = _relayed(ctx, 20_000)
        assert st.status == 0
        mine = [s for s in subs if int(s["subscriber"]) == h_other and int(s["kind"]) == 0 and int(s["track"]) == 0]
        assert mine, "the neighbour's subscriber lost its sub-streams"


@pytest.mark.gpu
def test_remove_with_outputs_needs_kill_and_invalidates_everything():
    with edgpu.Context() as ctx:
        s = ctx.session_add(make_sdp(AV))
        h = ctx.subscriber_add(s)
        with pytest.raises(edgpu.EdgpuError) as e:
            ctx.session_remove(s)
        assert e.value.code == edgpu.ERR
        ctx.subscriber_remove(h)
        ctx.session_remove(s)                            # no outputs left: plain removal
        for call in (lambda: ctx.session_tracks(s), lambda: ctx.subscriber_add(s),
                     lambda: ctx.session_remove(s), lambda: ctx.gop_span(s, 0),
                     lambda: ctx.source_identity(s, 0, 1, 0), lambda: ctx.session_eyes_add(s, 1)):
            with pytest.raises(edgpu.EdgpuError) as e:
                call()
            assert e.value.code == edgpu.BAD_ARGUMENT
        desc, seg_off, seg_sess, blob = edgpu.build_batch([(s, 0, 0, _rtp(1, 0))])
        with pytest.raises(edgpu.EdgpuError):
            ctx.ingest_host(desc, seg_off, seg_sess, blob)
        s2 = ctx.session_add(make_sdp(AV))
        h2 = ctx.subscriber_add(s2)
        ctx.session_remove(s2, kill_outputs=True)
        with pytest.raises(edgpu.EdgpuError):
            ctx.subscriber_remove(h2)                    # torn down with its session
        # a session with more tracks does not fit the removed one's rows; one with fewer takes them
        # (best fit: the tables do not grow under churn with mixed track counts)
        s3 = ctx.session_add(make_sdp(AV + AV[:1]))
        assert s3 != s2
        s4 = ctx.session_add(make_sdp(AV))
        assert s4 == s2
        ctx.session_remove(s4)
        s5 = ctx.session_add(make_sdp(AV[:1]))
        assert s5 == s2


@pytest.mark.gpu
def test_fresh_session_in_a_reused_slot_starts_from_scratch():
    """Old session: SSRC 0xAAAA latched, a key frame indexed, ids 1..3.  After removal the same
    id is a new session: a packet with a new SSRC is relayed (no latch), a joining subscriber
    gets nothing old (no stale key pointer), and packet ids restart at 1."""
    with edgpu.Context() as ctx:
        s = ctx.session_add(make_sdp(AV))
        _ingest(ctx, [(s, 0, 0, _rtp(1, 0, ssrc=0xAAAA)), (s, 0, 0, _rtp(2, 0, ssrc=0xAAAA, payload=b"\x41" * 40)),
                      (s, 0, 0, _rtp(3, 0, ssrc=0xAAAA, payload=b"\x41" * 40))])
        assert ctx.gop_span(s, 0)[0] == 3
        ctx.session_remove(s)
        s2 = ctx.session_add(make_sdp(AV))
        assert s2 == s
        assert ctx.gop_span(s2, 0) == (0, 0)             # no key pointer
        h = ctx.subscriber_add(s2)
        _ingest(ctx, [(s2, 0, 100, _rtp(7, 0, ssrc=0xBBBB, payload=b"\x41" * 40))])
        st, subs, desc, arena = _relayed(ctx, 100)
        rows = [i for i, q in enumerate(subs) if int(q["subscriber"]) == h and int(q["kind"]) == 0 and int(q["track"]) == 0]
        assert len(rows) == 1
        q = subs[rows[0]]
        assert int(q["desc_count"]) == 1                 # relayed: not a zero-length survivor
        d = desc[int(q["desc_base"])]
        assert int(d["packet_id"]) == 1                  # fStreamCountID restarts
        pkt = arena[int(d["offset"]):int(d["offset"]) + int(d["len"])].tobytes()
        assert pkt[8:12] == (0xBBBB).to_bytes(4, "big")
