"""GPU: a fan-out tick larger than the output arena (or the descriptor array) is delivered whole,
in copy passes over consecutive sub-stream rows (include/edgpu.h edgpu_fanout_next), never
dropped.  The reference walks every output of every sender in each ReflectPackets
(ReflectorStream.cpp:1088-1120), so every capture must stay the reference's byte for byte when
the arena is forced down to the largest single sub-stream of the trace -- which splits nearly
every tick with more than one output into several passes -- through every host path: the C ABI
replay (serial and tick-pipelined), the C++ adapter, the QTSS module (transmit times included),
the socket egress, and the random traces.  A C4-style burst (hundreds of players joining mid-GOP
in one tick) through the module at its default 256-MiB arena gives every joiner its GOP replay
from the key pointer (ReflectorStream.cpp:1058-1069, 1138-1198)."""
import hashlib
import os
import re
import subprocess

import pytest

from easydarwin_amd import edgpu
from easydarwin_amd.replay import replay
from easydarwin_amd.trace import PKT, capture_summary, read_capture
from scenarios import SCENARIOS, random_scenario
from test_gpu_parity import _fixture, _trace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ADAPTER = os.path.join(ROOT, "tools", "adapter_replay")
MODULE = os.path.join(ROOT, "easydarwin_amd", "libQTSSReflectorModule.so")
QREPLAY = os.path.join(ROOT, "tools", "qtss_replay")


def _small(info):
    """The smallest capacities every tick of the replay fits: the largest sub-stream's bytes and
    descriptors (tick_info of a one-pass replay)."""
    assert info and all(t[0] == 1 for t in info), "the default arena holds every golden tick"
    arena = max(t[1] for t in info)
    desc = max(t[2] for t in info)
    return max(16, (arena + 15) // 16 * 16), max(1, desc)


def _split_ticks(info):
    return sum(1 for t in info if t[0] > 1)


def _check_split(info, arena, desc):
    """A tick that fits is one pass; some tick over the capacities is split."""
    assert all(t[0] == 1 for t in info if t[3] <= arena and t[4] <= desc)
    if any(t[3] > arena or t[4] > desc for t in info):
        assert _split_ticks(info) > 0, "no tick was split"


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(SCENARIOS))
def test_split_ticks_match_reference(name):
    tr = _trace(name)
    info = []
    cap, _ = replay(tr, tick_info=info)
    want = _fixture(name)["capture_sha256"]
    assert hashlib.sha256(cap).hexdigest() == want
    arena, desc = _small(info)
    for a, d in ((arena, desc), (2 * arena, 2 * desc), (arena, 1 << 20), (1 << 28, desc)):
        got_info = []
        got, _ = replay(tr, tick_info=got_info, out_arena_bytes=a, max_out_packets=d)
        if got != cap:
            g, w = capture_summary(read_capture(got)), capture_summary(read_capture(cap))
            bad = [k for k in w if g.get(k) != w[k]]
            pytest.fail(f"arena {a} / {d} descriptors: {len(bad)} sub-streams differ, e.g. {bad[:3]}")
        _check_split(got_info, a, d)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["tiny", "mixed", "nal", "ssrc", "anchor", "c1", "rtpinfo", "backpressure", "leave",
                                  "udppush", "repush", "prefs_buffer", "prefs_reread"])
def test_adapter_split_ticks_match_reference(name, tmp_path):
    info = []
    replay(_trace(name), tick_info=info)
    arena, desc = _small(info)
    t, c = tmp_path / "t.edtr", tmp_path / "c.edcp"
    t.write_bytes(_trace(name).to_bytes())
    r = subprocess.run([ADAPTER, str(t), str(c)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, EDGPU_ARENA_BYTES=str(arena), EDGPU_MAX_OUT_PACKETS=str(desc)))
    assert r.returncode == 0, r.stderr[-2000:]
    assert hashlib.sha256(c.read_bytes()).hexdigest() == _fixture(name)["capture_sha256"]
    ticks, passes = map(int, re.search(r"(\d+) ticks, (\d+) copy passes", r.stderr).groups())
    assert passes >= ticks
    if any(t[3] > arena or t[4] > desc for t in info):
        assert passes > ticks


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["tiny", "c1", "mixed", "clamp", "ssrc", "nal", "nokey", "stall", "anchor", "rtpinfo",
                                  "backpressure", "udppush", "leave", "repush", "prefs_buffer", "prefs_reread"])
def test_module_split_ticks_match_reference(name, tmp_path):
    """The module with a forced-small arena (EDGPU_QTSS_ARENA_BYTES): captures and every write's
    transmit time as the reference's (the bucket / buffer delays and the first-packet pass run
    across the passes as across one tick)."""
    info = []
    replay(_trace(name), tick_info=info)
    arena, desc = _small(info)
    t, c, tt = tmp_path / "t.edtr", tmp_path / "c.edcp", tmp_path / "t.edtt"
    t.write_bytes(_trace(name).to_bytes())
    env = dict(os.environ, EDGPU_TT_OUT=str(tt), EDGPU_QTSS_ARENA_BYTES=str(arena),
               EDGPU_QTSS_MAX_OUT_PACKETS=str(desc), EDGPU_GATHER_SPLIT_BYTES="0")
    r = subprocess.run([QREPLAY, MODULE, str(t), str(c)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    fx = _fixture(name)
    assert capture_summary(read_capture(c.read_bytes())) == fx["substreams"]
    assert hashlib.sha256(c.read_bytes()).hexdigest() == fx["capture_sha256"]
    assert hashlib.sha256(tt.read_bytes()).hexdigest() == fx["transmit_sha256"]
    passes, ticks = map(int, re.search(r"(\d+) copy passes in (\d+) ticks", r.stderr).groups())
    assert passes >= ticks
    if any(t[3] > arena or t[4] > desc for t in info):
        assert passes > ticks


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["tiny", "c1", "mixed", "udppush"])
def test_egress_split_ticks_match_reference(name):
    """The socket egress sends every pass of a split tick (edgpu_egress_send runs
    edgpu_fanout_next itself)."""
    info = []
    replay(_trace(name), tick_info=info)
    arena, desc = _small(info)
    cap, _ = replay(_trace(name), sockets={"threads": 2}, out_arena_bytes=arena, max_out_packets=desc)
    assert capture_summary(read_capture(cap)) == _fixture(name)["substreams"]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(0, 24, 3))
def test_random_traces_split_ticks_match_oracle(seed, oracle_bins, tmp_path):
    tr = random_scenario(seed)
    tb = tr.to_bytes()
    t, c = tmp_path / "p.edtr", tmp_path / "p.edcp"
    t.write_bytes(tb)
    subprocess.run([oracle_bins["port"], str(t), str(c)], check=True, stderr=subprocess.DEVNULL)
    want = c.read_bytes()
    info = []
    cap, _ = replay(tr, tick_info=info)
    assert cap == want
    arena, desc = _small(info)
    cap, _ = replay(tr, out_arena_bytes=arena, max_out_packets=desc)
    assert cap == want, "C ABI replay, split ticks"
    if all(len(ev[4]) <= 2043 for ev in tr.events if ev[0] == PKT):
        cap, _ = replay(tr, interleaved=1 + seed % 2, out_arena_bytes=arena, max_out_packets=desc)
        assert cap == want, "interleaved push, split ticks"
    m = tmp_path / "m.edcp"
    r = subprocess.run([QREPLAY, MODULE, str(t), str(m)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, EDGPU_QTSS_ARENA_BYTES=str(arena), EDGPU_QTSS_MAX_OUT_PACKETS=str(desc)))
    assert r.returncode == 0, r.stderr[-2000:]
    assert m.read_bytes() == want, "QTSS module, split ticks"


def _tiny_ctx_trace():
    """Two sessions, four players: enough rows that a one-sub-stream arena splits every tick."""
    return SCENARIOS["mixed"]()


@pytest.mark.gpu
def test_owed_pass_blocks_the_next_tick_and_skipped_passes_are_counted():
    """While the context knows a pass is owed, ingest / fan-out / session removal are refused
    (EDGPU_ERR); a host that fans out again without reading back loses the owed passes, and
    edgpu_counters.lost_passes says so."""
    tr = _tiny_ctx_trace()
    info = []
    replay(tr, tick_info=info)
    arena, desc = _small(info)
    pk = [ev for ev in tr.events if ev[0] == PKT]
    with edgpu.Context(out_arena_bytes=arena, max_out_packets=desc) as ctx:
        sessions = [ctx.session_add(sdp) for sdp in tr.sdps]
        for s in sessions:
            for _ in range(3):
                ctx.subscriber_add(s, edgpu.TRANSPORT_UDP)
        batch = [(e[2], e[3], e[1], e[4]) for e in pk[:400]]
        desc_a, seg, sess, blob = edgpu.build_batch(batch)
        ctx.ingest_host(desc_a, seg, sess, blob)
        ctx.keyframe_index()
        r = ctx.fanout(pk[399][1])
        st = ctx.stats()
        assert st.more_passes == 1 and st.pass_ == 0
        with pytest.raises(edgpu.EdgpuError) as e:
            ctx.ingest_host(desc_a, seg, sess, blob)
        assert e.value.code == edgpu.ERR
        with pytest.raises(edgpu.EdgpuError):
            ctx.fanout(pk[399][1])
        # (a pass's descriptors may start after a gap of at most one sub-stream: count the rows')
        n, total = 1, int(ctx.read_tick(r)[1]["desc_count"].sum())
        while (r := ctx.fanout_next()) is not None:
            st = ctx.stats()
            n += 1
            total += int(ctx.read_tick(r)[1]["desc_count"].sum())
            assert st.pass_ == n - 1
        assert n > 1 and total == st.relayed_packets
        assert ctx.counters()["lost_passes"] == 0
        # the next tick may go now; skip its passes without reading back: they are lost
        batch = [(e[2], e[3], e[1], e[4]) for e in pk[400:800]]
        desc_a, seg, sess, blob = edgpu.build_batch(batch)
        ctx.ingest_host(desc_a, seg, sess, blob)
        ctx.keyframe_index()
        ctx.fanout(pk[799][1])
        ctx.fanout(pk[799][1] + 1)          # the host never learnt of the owed passes
        c = ctx.counters()
        assert c["lost_passes"] > 0 and c["fanout_passes"] >= n + 2


@pytest.mark.gpu
def test_sub_stream_larger_than_the_arena_fails_the_tick():
    tr = SCENARIOS["c1"]()
    pk = [ev for ev in tr.events if ev[0] == PKT]
    with edgpu.Context(out_arena_bytes=4096) as ctx:
        s = ctx.session_add(tr.sdps[0])
        ctx.subscriber_add(s, edgpu.TRANSPORT_UDP)
        desc_a, seg, sess, blob = edgpu.build_batch([(e[2], e[3], e[1], e[4]) for e in pk[:200]])
        ctx.ingest_host(desc_a, seg, sess, blob)
        ctx.keyframe_index()
        ctx.fanout(pk[199][1])
        assert ctx.stats().status == edgpu.OUT_OVERFLOW


def _burst_trace(sessions=8, per_session=32):
    """C4-style: 8 pushers of 8 Mb/s H.264 (2-s GOP, ~2 MB) + AAC; at 3.3 s, `per_session`
    players join each of them in one tick (a third RTSP-interleaved): ~1.3 MB of GOP replay per
    joiner, more than the module's default 256-MiB arena in that tick."""
    from easydarwin_amd.synth import TrackSpec, make_sdp, session_packets
    from easydarwin_amd.trace import TCP, UDP, Trace
    from scenarios import _assemble
    tracks = [TrackSpec("video", "H264/90000", 96, bitrate=8_000_000, gop=60, idr_bytes=120_000),
              TrackSpec("audio", "MPEG4-GENERIC/48000/2", 97)]
    tr = Trace()
    per = []
    for s in range(sessions):
        tr.add_session(make_sdp(tracks))
        per.append(session_packets(tracks, 3600, 0xB0057 + s, t0=7 * s))
    joins = [(0, s, 1000 * s, UDP) for s in range(sessions)]
    joins += [(3300, s, 1000 * s + 1 + k, TCP if k % 3 == 2 else UDP) for s in range(sessions) for k in range(per_session)]
    return _assemble(tr, per, 100, 3600, joins)


@pytest.mark.gpu
def test_c4_burst_through_the_module_at_the_default_arena(oracle_bins, tmp_path):
    tr = _burst_trace()
    tb = tr.to_bytes()
    t, c, m = tmp_path / "b.edtr", tmp_path / "b.edcp", tmp_path / "m.edcp"
    t.write_bytes(tb)
    subprocess.run([oracle_bins["port"], str(t), str(c)], check=True, stderr=subprocess.DEVNULL)
    want = c.read_bytes()
    env = {k: v for k, v in os.environ.items() if not k.startswith("EDGPU_QTSS_")}
    r = subprocess.run([QREPLAY, MODULE, str(t), str(m)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    passes, ticks = map(int, re.search(r"(\d+) copy passes in (\d+) ticks", r.stderr).groups())
    assert passes > ticks, "the burst tick should exceed the default arena"
    got = m.read_bytes()
    if got != want:
        g, w = capture_summary(read_capture(got)), capture_summary(read_capture(want))
        bad = [k for k in w if g.get(k) != w[k]]
        pytest.fail(f"{len(bad)} sub-streams differ, e.g. {bad[:3]}")
    # every joiner got a GOP replay: its first video packet is an IDR's first FU-A fragment
    caps = read_capture(got)
    joiners = [ss for ss in caps.values() if ss.sub % 1000 != 0 and ss.track == 0 and ss.kind == 0]
    assert len(joiners) == 8 * 32
    for ss in joiners:
        first = ss.data[4:] if ss.tcp else ss.data[2:]
        assert first[12] & 0x1F == 7 or (first[12] & 0x1F == 28 and first[13] & 0x1F == 5), "not a key-frame start"


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["leave", "repush"])
def test_failed_pass_leaves_the_context_usable(name, tmp_path):
    """A sink error in the second copy pass of an over-capacity tick fails that tick only: the
    adapter drains the passes it still owed (edgpu_fanout_next, counted as lost) and reports the
    blocked sub-streams it had, so every later tick, output removal and session removal of the
    trace succeeds (a failed pass used to leave the context refusing all of them)."""
    info = []
    replay(_trace(name), tick_info=info)
    arena, desc = _small(info)
    t, c = tmp_path / "t.edtr", tmp_path / "c.edcp"
    t.write_bytes(_trace(name).to_bytes())
    r = subprocess.run([ADAPTER, str(t), str(c)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, EDGPU_ARENA_BYTES=str(arena), EDGPU_MAX_OUT_PACKETS=str(desc),
                                EDGPU_REPLAY_FAIL_PASS="1"))
    assert r.returncode == 0, r.stderr[-2000:]
    failed, after = map(int, re.search(r"(\d+) failed ticks, (\d+) good ticks after", r.stderr).groups())
    assert failed == 1 and after > 0, r.stderr[-2000:]


def _tick_bytes(ctx, r, out):
    """Appends each sub-stream's packets of one pass to out[(subscriber, track, kind)]."""
    _st, subs, desc, arena = ctx.read_tick(r)
    for q in subs:
        n = int(q["desc_count"])
        if not n:
            continue
        d = desc[int(q["desc_base"]):int(q["desc_base"]) + n]
        out.setdefault((int(q["subscriber"]), int(q["track"]), int(q["kind"])), []).extend(
            arena[o:o + ln].tobytes() for o, ln in zip(d["offset"], d["len"]))


@pytest.mark.gpu
def test_subscribers_change_between_passes():
    """include/edgpu.h edgpu_fanout_next: subscribers may come and go between the copy passes of a
    tick.  The passes keep the tick's table -- a subscriber added between passes gets nothing from
    this tick (its new-output start comes with the next one), a removed subscriber's rows still
    deliver the rest of the tick -- so a tick split into passes with a join and a leave landing
    between them delivers what the same tick in one pass delivers with the join and the leave
    after it, in this tick and the next (the module's concurrent delivery can land AddOutput /
    RemoveOutput there, reflector_adapter.cpp SetConcurrentDelivery)."""
    tr = _tiny_ctx_trace()
    info = []
    replay(tr, tick_info=info)
    arena, desc = _small(info)
    pk = [ev for ev in tr.events if ev[0] == PKT]
    batches = [[(e[2], e[3], e[1], e[4]) for e in pk[a:b]] for a, b in ((0, 400), (400, 800))]
    times = [pk[399][1], pk[799][1]]
    got = {}
    for mode, cfg in (("split", dict(out_arena_bytes=arena, max_out_packets=desc)), ("one", {})):
        ticks = []
        with edgpu.Context(**cfg) as ctx:
            sessions = [ctx.session_add(sdp) for sdp in tr.sdps]
            handles = {s: [ctx.subscriber_add(s, edgpu.TRANSPORT_UDP) for _ in range(3)] for s in sessions}
            leaving = handles[sessions[-1]][0]
            passes = 0
            for k, (batch, t) in enumerate(zip(batches, times)):
                out = {}
                d, seg, sess, blob = edgpu.build_batch(batch)
                ctx.ingest_host(d, seg, sess, blob)
                ctx.keyframe_index()
                r = ctx.fanout(t)
                _tick_bytes(ctx, r, out)
                passes += 1
                if k == 0 and mode == "split":
                    assert ctx.stats().more_passes == 1, "the tick should be split"
                    joined = ctx.subscriber_add(sessions[0], edgpu.TRANSPORT_UDP)   # between passes
                    ctx.subscriber_remove(leaving)
                while (r := ctx.fanout_next()) is not None:
                    _tick_bytes(ctx, r, out)
                    passes += 1
                if k == 0 and mode == "one":
                    joined = ctx.subscriber_add(sessions[0], edgpu.TRANSPORT_UDP)   # after the tick
                    ctx.subscriber_remove(leaving)
                assert ctx.stats().status == 0
                ticks.append(out)
            got[mode] = (ticks, joined, leaving, passes)
    (split, j1, l1, np1), (one, j2, l2, np2) = got["split"], got["one"]
    assert (j1, l1) == (j2, l2) and np1 > np2
    assert split == one
    assert any(key[0] == l1 for key in split[0]) and not any(key[0] == l1 for key in split[1])
    assert not any(key[0] == j1 for key in split[0]) and any(key[0] == j1 for key in split[1])


@pytest.mark.gpu
def test_fanout_active_compacts_each_pass():
    """edgpu_fanout_active: each pass's sub-streams with descriptors (or new), compacted in table order --
    the rows and indices a full read of the table (read_tick) filtered on the host gives; a
    capacity below the count truncates the rows and still reports the count."""
    tr = _tiny_ctx_trace()
    info = []
    replay(tr, tick_info=info)
    arena, desc = _small(info)
    pk = [ev for ev in tr.events if ev[0] == PKT]
    with edgpu.Context(out_arena_bytes=arena, max_out_packets=desc) as ctx:
        sessions = [ctx.session_add(sdp) for sdp in tr.sdps]
        for s in sessions:
            for k in range(5):
                ctx.subscriber_add(s, edgpu.TRANSPORT_TCP if k % 2 else edgpu.TRANSPORT_UDP)
        seen = 0
        for a, b in ((0, 300), (300, 700)):
            d, seg, sess, blob = edgpu.build_batch([(e[2], e[3], e[1], e[4]) for e in pk[a:b]])
            ctx.ingest_host(d, seg, sess, blob)
            ctx.keyframe_index()
            r = ctx.fanout(pk[b - 1][1])
            while r is not None:
                subs = ctx.read_tick(r)[1]
                idx = [i for i in range(len(subs)) if subs[i]["desc_count"] or subs[i]["flags"] & edgpu.SUB_NEW]
                rows, q, n = ctx.fanout_active(len(subs) + 3)
                assert n == len(idx) and q.tolist() == idx
                assert rows.tobytes() == subs[idx].tobytes()
                if n > 1:
                    rows2, q2, n2 = ctx.fanout_active(1)
                    assert n2 == n and q2.tolist() == idx[:1] and rows2.tobytes() == subs[idx[:1]].tobytes()
                seen += n
                r = ctx.fanout_next()
        assert seen > 0
