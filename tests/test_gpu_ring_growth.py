"""GPU: sender rings that cover the reference's retention at the DEFAULT capacities (VERDICT r4
missing #2).

The reference keeps every packet younger than sMaxPacketAgeMSec = 10 x reflector_buffer_size_sec,
the key packet and everything after it, and what a blocked output still needs, in an unbounded
queue (RemoveOldPackets, ReflectorStream.cpp:1233-1289, 112-114).  The engine's rings start at
8,192 packets / 8 MiB per video sender and grow (edgpu_config.ring_growth): each fan-out's plan
measures that span per sender and a sender past half of a ring gets it doubled before the next
ingest, its packets moved to their new places.  ``highrate`` (12 Mb/s, a 10-s GOP, players joining
at 9 s) needs ~9,600 packets / 13.5 MB of its key packet's GOP; ``longbuffer`` runs a 3-s buffer
(30-s retention) with a TCP player held for 8 s.  Both must match the reference byte for byte with
no stream error -- and ``highrate`` must fail without growth, so the test exercises it."""
import hashlib

import pytest

from easydarwin_amd import edgpu
from easydarwin_amd.replay import replay
from easydarwin_amd.trace import pref_values
from test_gpu_parity import _fixture, _trace


def _ctx(tr, **cfg):
    pv = pref_values(tr.prefs)
    return edgpu.Context(reflector_buffer_size_sec=int(pv["reflector_buffer_size_sec"]),
                         rtp_reflector_threshold_msec=max(1000, int(pv["rtp_reflector_threshold_msec"])), **cfg)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["highrate", "longbuffer"])
@pytest.mark.parametrize("mode", ["host", "pinned", "interleaved"])
def test_default_rings_hold_what_the_reference_retains(name, mode):
    tr = _trace(name)
    kw = {"pinned": True} if mode == "pinned" else {"interleaved": 1} if mode == "interleaved" else {}
    with _ctx(tr) as ctx:
        cap, _ = replay(tr, ctx=ctx, **kw)
        errors = ctx.stream_errors()
        c = ctx.counters()
    assert errors == []
    assert hashlib.sha256(cap).hexdigest() == _fixture(name)["capture_sha256"]
    if name == "highrate":
        assert c["ring_grows"] >= 2                 # the video sender's packet and byte rings
        assert c["ring_bytes"] > (8 << 20) + (1 << 20)


@pytest.mark.gpu
def test_highrate_needs_the_growth():
    """The same stream with ring_growth off: the 9-s GOP replay no longer fits the 8-MiB ring, the
    joining players' session is marked (edgpu_stream_errors) and their bytes differ."""
    tr = _trace("highrate")
    with _ctx(tr, ring_growth=edgpu.FALSE) as ctx:
        cap, _ = replay(tr, ctx=ctx)
        errors = ctx.stream_errors()
        assert ctx.counters()["ring_grows"] == 0
    assert errors, "expected a ring overflow at the default capacities without growth"
    assert hashlib.sha256(cap).hexdigest() != _fixture("highrate")["capture_sha256"]


@pytest.mark.gpu
def test_growth_is_best_effort_when_device_memory_runs_out(monkeypatch):
    """A growth the device memory cannot hold (a ring pool limited to 16 MiB: the starting rings fit,
    the 16-MiB byte ring does not) is skipped and counted, and every ingest goes on: the replay
    completes, relays what the ungrown rings hold -- exactly what it relays with growth off -- and
    marks the session whose players lost packets (edgpu_stream_errors)."""
    tr = _trace("highrate")
    with _ctx(tr, ring_growth=edgpu.FALSE) as ctx:
        want, _ = replay(tr, ctx=ctx)
    monkeypatch.setenv("EDGPU_RING_POOL_LIMIT", str(16 << 20))
    with _ctx(tr) as ctx:
        cap, _ = replay(tr, ctx=ctx)
        errors = ctx.stream_errors()
        c = ctx.counters()
    assert c["ring_grow_failures"] >= 1 and c["ring_grows"] == 0
    assert c["ring_pool_bytes"] <= 16 << 20
    assert errors
    assert cap == want


@pytest.mark.gpu
def test_growth_stops_at_its_bound():
    """max_ring_bytes / max_ring_packets bound the growth (powers of two): with both at the
    starting capacities nothing grows."""
    tr = _trace("highrate")
    with _ctx(tr, max_ring_bytes=8 << 20, max_ring_packets=8192) as ctx:
        replay(tr, ctx=ctx)
        assert ctx.counters()["ring_grows"] == 0


@pytest.mark.gpu
def test_pooled_rings_are_reused_clean():
    """Rings come from a pool (edgpu_engine.cpp RingPool): a session that grew its rings and ended
    returns them, and the next session of the context takes them -- with whatever bytes the last
    owner left in them.  ``highrate`` replayed three times into one context, its session removed
    in between, must match the reference byte for byte each time, and the counters must come back
    to the empty context's rings."""
    tr = _trace("highrate")
    with _ctx(tr) as ctx:
        c0 = ctx.counters()
        for k in range(3):
            cap, _ = replay(tr, ctx=ctx)
            assert ctx.stream_errors() == []
            assert hashlib.sha256(cap).hexdigest() == _fixture("highrate")["capture_sha256"], k
            for s in range(len(tr.sdps)):            # (a removed session's id is reused by the next)
                ctx.session_remove(s, kill_outputs=True)
            c = ctx.counters()
            assert c["ring_bytes"] == c0["ring_bytes"], k
            assert c["ring_grows"] >= 2 * (k + 1)
