"""GPU: C-ABI call-order contracts and the timing history of the engine.

* edgpu_ingest refuses to run while the previous batch still needs edgpu_keyframe_index
  (two ingests in a row would otherwise drop the first batch's key pointers and audio anchor);
* every per-launch duration edgpu_kernel_times returns is >= 0 and a whole-tick duration is
  never shorter than its copy kernel's, over more ticks than the history holds and across a
  failed RTSP-interleaved ingest (which clears the pending batch without an index);
* an RTP-Info PLAY on a session with nothing buffered right after a PLAY that found packets
  reports EDGPU_WOULD_BLOCK (the stale-result regression of DESIGN §4.9);
* the copy kernel follows the active sub-streams' need for a per-output patch:
  k_fanout6<1024,16> while all are identity UDP, k_fanout4<1024,32> while one is TCP or
  rewrites, and every packet is relayed across the switches.
"""
import os

import ctypes as C

import numpy as np
import pytest

from easydarwin_amd import edgpu
from easydarwin_amd.synth import TrackSpec, make_sdp

H264 = [TrackSpec("video", "H264/90000", 96)]


def _rtp(seq, ts, ssrc=0x1234, payload=b"\x65" + b"\x00" * 40):
    return bytes([0x80, 96, seq >> 8, seq & 0xFF]) + ts.to_bytes(4, "big") + ssrc.to_bytes(4, "big") + payload


def _ingest(ctx, pkts):
    desc, seg_off, seg_sess, blob = edgpu.build_batch(pkts)
    ctx.ingest_host(desc, seg_off, seg_sess, blob)


@pytest.mark.gpu
def test_ingest_refused_while_index_pending():
    with edgpu.Context() as ctx:
        s = ctx.session_add(make_sdp(H264))
        _ingest(ctx, [(s, 0, 0, _rtp(1, 0))])
        with pytest.raises(edgpu.EdgpuError) as e:
            _ingest(ctx, [(s, 0, 1, _rtp(2, 0))])
        assert e.value.code == edgpu.ERR
        ctx.keyframe_index()
        _ingest(ctx, [(s, 0, 2, _rtp(3, 0))])
        ctx.keyframe_index()
        ctx.fanout(10)
        assert ctx.stats().status == 0


@pytest.mark.gpu
def test_kernel_times_nonnegative_and_paired():
    with edgpu.Context(max_batch_packets=64) as ctx:
        sess = [ctx.session_add(make_sdp(H264)) for _ in range(3)]
        for s in sess:
            ctx.subscriber_add(s, edgpu.TRANSPORT_UDP)
            ctx.subscriber_add(s, edgpu.TRANSPORT_TCP)
        seq = 0
        for tick in range(300):
            t = 10 * tick
            if tick == 150:
                # 100 frames > max_batch_packets: the interleaved ingest runs on the device and
                # fails (EDGPU_OUT_OVERFLOW) without a keyframe index
                raw = b"".join(b"$\x00" + len(p).to_bytes(2, "big") + p for p in (_rtp(k, 0) for k in range(100)))
                reads = np.zeros(1, dtype=edgpu.TCP_READ_DTYPE)
                reads[0] = (sess[0], len(raw), 0, t)
                with pytest.raises(edgpu.EdgpuError) as e:
                    ctx.ingest_interleaved(reads, raw)
                assert e.value.code == edgpu.OUT_OVERFLOW
            pkts = []
            for s in sess:
                for _ in range(2):
                    pkts.append((s, 0, t, _rtp(seq & 0xFFFF, 90 * t)))
                    seq += 1
            _ingest(ctx, pkts)
            ctx.keyframe_index()
            ctx.fanout(t)
            if tick % 100 == 99:
                ring = [ctx.kernel_times(w) for w in range(4)]
                assert len(ring[0]) == len(ring[1]) > 0
                for w in range(3):
                    assert ring[w] and min(ring[w]) >= 0.0, (w, ring[w][:8])
                assert ring[3] == []              # the keyframe index runs inside k_ingest
                assert all(b >= a for a, b in zip(ring[0], ring[1]))
        tm = ctx.timings()
        assert tm["tick_ms"] >= tm["fanout_ms"] >= 0.0 and tm["keyframe_ms"] >= 0.0


@pytest.mark.gpu
def test_timing_levels_select_the_recorded_pairs():
    with edgpu.Context() as ctx:
        with pytest.raises(edgpu.EdgpuError):
            ctx.set_timing(3)
        s = ctx.session_add(make_sdp(H264))
        ctx.subscriber_add(s, edgpu.TRANSPORT_UDP)

        def ticks(n, t0):
            for k in range(n):
                _ingest(ctx, [(s, 0, t0 + k, _rtp(t0 + k, 90 * k))])
                ctx.keyframe_index()
                ctx.fanout(t0 + k)

        ctx.set_timing(ctx.TIMING_NONE)          # nothing recorded yet: last timings are 0
        ticks(3, 0)
        assert [ctx.kernel_times(w) for w in range(4)] == [[], [], [], []]
        assert ctx.timings()["fanout_ms"] == 0.0
        ctx.set_timing(ctx.TIMING_FANOUT)
        ticks(4, 10)
        ring = [ctx.kernel_times(w) for w in range(4)]
        assert len(ring[0]) == 4 and min(ring[0]) >= 0.0 and ring[1:] == [[], [], []]
        ctx.set_timing(ctx.TIMING_ALL)
        ticks(5, 20)
        ring = [ctx.kernel_times(w) for w in range(4)]
        assert [len(r) for r in ring] == [5, 5, 5, 0]     # (no keyframe kernel: it is in k_ingest)
        assert all(b >= a for a, b in zip(ring[0], ring[1]))
        assert ctx.stats().status == 0


@pytest.mark.gpu
def test_prestaged_pinned_batches_relay_the_same_bytes():
    """edgpu_ingest_prestage: a pinned batch's blob prefix copied ahead in pieces, then the
    ingest copies the rest -- every tick's arena equals the one of a plain pinned ingest; a piece
    that does not extend the staged prefix, or runs past max_batch_bytes, is refused; a batch
    refused by validation drops what was copied ahead of it, and so does an explicit discard."""
    rng = np.random.default_rng(7)
    ticks = []
    seq = 0
    for t in range(30):
        pkts = []
        for s in range(3):
            for _ in range(int(rng.integers(1, 40))):
                n = int(rng.integers(20, 1400))
                pkts.append((s, 0, 10 * t, _rtp(seq & 0xFFFF, 90 * t, payload=bytes([0x41]) + rng.bytes(n))))
                seq += 1
        ticks.append(edgpu.build_batch(pkts))

    def run(prestage):
        out = []
        with edgpu.Context(max_batch_bytes=1 << 20) as ctx:
            for _ in range(3):
                ctx.subscriber_add(ctx.session_add(make_sdp(H264)), edgpu.TRANSPORT_UDP)
            bufs = []
            for k in range(2):
                bufs.append({n: ctx.host_alloc(1 << 20) for n in ("desc", "seg", "sess", "blob")})
            for t, (desc, seg, sess, blob) in enumerate(ticks):
                B = bufs[t % 2]
                for name, a in (("desc", desc), ("seg", seg), ("sess", sess), ("blob", blob)):
                    v = np.ascontiguousarray(a).view(np.uint8).ravel()
                    B[name].array[:v.nbytes] = v
                if prestage and t == 9:
                    # a prefix copied ahead and then discarded (edgpu_ingest_prestage(NULL, 0, 0): the
                    # host dropped the batch it belonged to) must not reach the next ingest: stage other
                    # bytes, discard, then write the batch and ingest it with nothing staged
                    v = np.ascontiguousarray(blob).view(np.uint8).ravel()
                    B["blob"].array[:v.nbytes] = v[::-1]
                    _check_ok(ctx.lib.edgpu_ingest_prestage(ctx.h, C.c_void_p(B["blob"].ptr), 0, blob.nbytes // 2 // 16 * 16))
                    _check_ok(ctx.lib.edgpu_ingest_prestage(ctx.h, None, 0, 0))
                    _check_ok(ctx.lib.edgpu_sync(ctx.h))       # (the discarded copy has read the buffer)
                    B["blob"].array[:v.nbytes] = v
                elif prestage:
                    cut = [0, blob.nbytes // 3, (2 * blob.nbytes) // 3]
                    for a, b in zip(cut, cut[1:]):
                        _check_ok(ctx.lib.edgpu_ingest_prestage(ctx.h, C.c_void_p(B["blob"].ptr), a, b - a))
                    if t == 5:              # a gap in the prefix: refused
                        assert ctx.lib.edgpu_ingest_prestage(ctx.h, C.c_void_p(B["blob"].ptr), cut[2] + 16, 16) != 0
                    if t == 6:              # past max_batch_bytes: refused
                        assert ctx.lib.edgpu_ingest_prestage(ctx.h, C.c_void_p(B["blob"].ptr), cut[2], 2 << 20) != 0
                ctx.ingest_pinned(B["desc"].ptr, len(desc), B["seg"].ptr, B["sess"].ptr, len(sess), B["blob"].ptr,
                                  blob.nbytes)
                ctx.keyframe_index()
                r = ctx.fanout(10 * t)
                st = ctx.stats()
                assert st.status == 0
                out.append(bytes(ctx.copy_to_host(r.arena, st.arena_bytes)))
            if prestage:                    # a refused batch drops what was copied ahead of it
                desc, seg, sess, blob = ticks[0]
                _check_ok(ctx.lib.edgpu_ingest_prestage(ctx.h, C.c_void_p(bufs[0]["blob"].ptr), 0, 64))
                with pytest.raises(edgpu.EdgpuError):
                    ctx.ingest_pinned(bufs[0]["desc"].ptr, len(desc), bufs[0]["seg"].ptr, bufs[0]["sess"].ptr,
                                      len(sess), bufs[0]["blob"].ptr, 2 << 20)
                _check_ok(ctx.lib.edgpu_ingest_prestage(ctx.h, C.c_void_p(bufs[0]["blob"].ptr), 0, 64))
        return out

    assert run(True) == run(False)


def _check_ok(rc):
    assert rc == 0, edgpu.last_error() if hasattr(edgpu, "last_error") else rc


@pytest.mark.gpu
def test_rtp_info_play_on_empty_session_after_a_found_play():
    with edgpu.Context() as ctx:
        full = ctx.session_add(make_sdp(H264))
        empty = ctx.session_add(make_sdp(H264))
        _ingest(ctx, [(full, 0, 100 + k, _rtp(500 + k, 9000 * k)) for k in range(5)])
        ctx.keyframe_index()
        _h, info = ctx.subscriber_play(full, rtp_info=True, now_ms=200)
        assert info == [(500, 0)]
        with pytest.raises(edgpu.EdgpuError) as e:
            ctx.subscriber_play(empty, rtp_info=True, now_ms=200)
        assert e.value.code == edgpu.WOULD_BLOCK


@pytest.mark.gpu
def test_contexts_run_concurrently_from_threads():
    """One context per thread (calls on a context are serialized by the caller,
    many contexts run at once): four host threads each replay a different golden scenario on
    their own context at the same time, and each capture is the reference's."""
    import hashlib
    import json
    import os
    import threading

    from easydarwin_amd.replay import replay
    from scenarios import SCENARIOS
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    names = ["mixed", "rtpinfo", "backpressure", "udppush"]
    traces = {n: SCENARIOS[n]() for n in names}
    out, errs = {}, []

    def run(n):
        try:
            out[n] = replay(traces[n])[0]
        except Exception as e:          # surfaced below
            errs.append((n, repr(e)))
    th = [threading.Thread(target=run, args=(n,)) for n in names]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for n in names:
        want = json.load(open(os.path.join(gold, n + ".json")))["capture_sha256"]
        assert hashlib.sha256(out[n]).hexdigest() == want, n


@pytest.mark.gpu
@pytest.mark.skipif("EDGPU_FANOUT" in os.environ, reason="EDGPU_FANOUT pins one variant")
def test_fanout_kernel_follows_patching_substreams():
    plain, patching = "k_fanout6<1024,16,", "k_fanout4<1024,32,"
    with edgpu.Context() as ctx:
        s = ctx.session_add(make_sdp(H264))
        u = ctx.subscriber_add(s, edgpu.TRANSPORT_UDP)
        seq, relayed = 0, 0

        def tick(expect_kernel, expect_relayed):
            nonlocal seq, relayed
            # one IDR packet (the key pointer) first, then non-key slices
            pk = [(s, 0, 10 * seq + k, _rtp(seq + k, 3000 * seq, payload=(b"\x65" if seq + k == 0 else b"\x41") + b"\x00" * 40))
                  for k in range(5)]
            seq += 5
            _ingest(ctx, pk)
            ctx.keyframe_index()
            ctx.fanout(10 * seq)
            st = ctx.stats()
            assert st.status == 0
            assert st.relayed_packets == expect_relayed
            assert ctx.fanout_kernel().startswith(expect_kernel)     # the kernel that tick used

        tick(plain, 5)                       # the first tick: the UDP output starts at the key packet
        t = ctx.subscriber_add(s, edgpu.TRANSPORT_TCP)
        tick(patching, 15)                   # UDP: 5 new; the joining TCP output: key packet -> newest
        ctx.subscriber_remove(t)
        tick(plain, 5)
        ctx.subscriber_rewrite(u, 0, seq_delta=7)
        tick(patching, 5)
        ctx.subscriber_rewrite(u, 0)         # identity again
        tick(plain, 5)
        # a join burst (new outputs: at least 4096 sub-stream rows and a quarter of the tick's)
        # replays the GOP to each through the 32-packet kernel; the tick after is steady again
        for _ in range(2100):
            ctx.subscriber_add(s, edgpu.TRANSPORT_UDP)
        tick(patching, 5 + 2100 * 30)
        tick(plain, 5 * 2101)


@pytest.mark.gpu
def test_churn_keeps_the_tables_bounded():
    """Sessions of mixed track counts and their subscribers come and go: a removed session's
    sender rows and a removed subscriber's sub-stream rows are reused, best fit, by any later one
    that fits, so the tables stay at the size of the most that were live at once."""
    def sdp(n):
        return "v=0\r\n" + "".join(f"m=video 0 RTP/AVP 96\r\na=rtpmap:96 H264/90000\r\na=control:trackID={i + 1}\r\n"
                                   for i in range(n))
    sizes = []
    with edgpu.Context() as ctx:
        for cycle in range(6):
            live = []
            for n in ((3, 1, 2) if cycle % 2 == 0 else (2, 2, 1)):
                s = ctx.session_add(sdp(n))
                live.append((s, [ctx.subscriber_add(s, edgpu.TRANSPORT_UDP) for _ in range(2)]))
            ctx.fanout(1000 * cycle)
            ctx.stats()
            for s, subs in live:
                for h in subs:
                    ctx.subscriber_remove(h)
                ctx.session_remove(s)
            ctx.fanout(1000 * cycle + 500)         # freed sub-stream rows are reusable from this tick
            ctx.stats()
            c = ctx.counters()
            sizes.append((c["senders"], c["substream_rows"]))
    # 6 tracks live at most: 12 senders; 2 subscribers x 2 sub-streams per track: 24 rows
    assert sizes == [(12, 24)] * 6


@pytest.mark.gpu
def test_fanout_rows_equal_descriptors_arrivals_and_sources():
    """edgpu_fanout_rows: for each selected sub-stream, its descriptors with their arrivals and batch
    slots (edgpu_fanout_packet_info) at the rows asked for; identity sub-streams of one sender are
    suffixes of the longest one's rows (what the module adapter reads back instead of every
    descriptor)."""
    with edgpu.Context() as ctx:
        s = ctx.session_add(make_sdp(H264))
        ctx.subscriber_add(s, edgpu.TRANSPORT_UDP)
        ctx.subscriber_add(s, edgpu.TRANSPORT_TCP)
        rng = np.random.default_rng(5)

        def batch(t, seq0, n, key):
            return edgpu.build_batch([(s, 0, t + k, _rtp(seq0 + k, 90 * t, payload=bytes([0x65 if k == 0 and key else 0x41])
                                                         + rng.bytes(int(rng.integers(20, 1300))))) for k in range(n)])

        for t, seq0, n, key, join in ((10, 100, 12, True, False), (40, 200, 7, False, True)):
            ctx.ingest_host(*batch(t, seq0, n, key))
            ctx.keyframe_index()
            if join:
                ctx.subscriber_add(s, edgpu.TRANSPORT_UDP)     # a GOP replay: longer than the others
            r = ctx.fanout(0)
            st, subs, d, arena = ctx.read_tick(r)
            arr = ctx.fanout_arrivals(st.pass_packets)
            src = ctx.fanout_sources(st.pass_packets)
            live = [q for q in range(len(subs)) if subs[q]["desc_count"]]
            sel, base = [], 0
            for q in live:
                sel.append((q, base))
                base += int(subs[q]["desc_count"])
            rows = ctx.fanout_rows_n(sel, base)
            for q, b in sel:
                n_q, db = int(subs[q]["desc_count"]), int(subs[q]["desc_base"])
                got = rows[b:b + n_q]
                assert (got["offset"] == d["offset"][db:db + n_q]).all()
                assert (got["len"] == d["len"][db:db + n_q]).all()
                assert (got["packet_id"] == d["packet_id"][db:db + n_q]).all()
                assert (got["arrival"] == arr[db:db + n_q]).all()
                assert (got["source"] == src[db:db + n_q]).all()
            ident = [q for q in live if subs[q]["flags"] & edgpu.SUB_IDENTITY and subs[q]["kind"] == 0]
            if join:
                assert len({int(subs[q]["desc_count"]) for q in ident}) == 2
            longest = max(ident, key=lambda q: int(subs[q]["desc_count"]))
            lb = dict(sel)[longest]
            for q in ident:                      # a suffix of the longest one's rows
                n_q, b = int(subs[q]["desc_count"]), dict(sel)[q]
                tail = rows[lb + int(subs[longest]["desc_count"]) - n_q:lb + int(subs[longest]["desc_count"])]
                for f in ("len", "packet_id", "arrival", "source"):
                    assert (tail[f] == rows[b:b + n_q][f]).all()
            # rows past nrows are not written
            short = ctx.fanout_rows_n(sel[:1], 1)
            assert len(short) == 1 and short[0]["packet_id"] == rows[0]["packet_id"]


@pytest.mark.gpu
def test_fanout_sources_point_into_the_last_host_batch():
    """edgpu_fanout_packet_info's sources: a descriptor whose packet came with the last host batch
    names its blob slot, and the packet bytes there are the identity UDP wire bytes in the arena;
    packets of an earlier batch (a new output's GOP replay) and of a device batch have none."""
    with edgpu.Context() as ctx:
        s = ctx.session_add(make_sdp(H264))
        ctx.subscriber_add(s, edgpu.TRANSPORT_UDP)
        rng = np.random.default_rng(3)

        def batch(t, seq0, n, key):
            return edgpu.build_batch([(s, 0, t, _rtp(seq0 + k, 90 * t, payload=bytes([0x65 if k == 0 and key else 0x41])
                                                     + rng.bytes(int(rng.integers(20, 1300))))) for k in range(n)])

        def check(b, want_sources):
            desc, seg_off, seg_sess, blob = b
            r = ctx.fanout(0)
            st, subs, d, arena = ctx.read_tick(r)
            src = ctx.fanout_sources(st.pass_packets)
            got = 0
            for q in subs:
                for i in range(int(q["desc_count"])):
                    k = int(q["desc_base"]) + i
                    off, ln = int(d["offset"][k]), int(d["len"][k])
                    if src[k] == edgpu.NO_SOURCE:
                        continue
                    got += 1
                    assert bytes(blob[int(src[k]) * 16 + 4:int(src[k]) * 16 + 4 + ln]) == bytes(arena[off:off + ln])
            assert got == want_sources, (got, want_sources)
            return int(st.pass_packets)

        b1 = batch(10, 100, 12, True)
        ctx.ingest_host(*b1)
        ctx.keyframe_index()
        assert check(b1, 12) == 12                 # every packet came with this batch
        b2 = batch(20, 200, 5, False)              # no key frame: the key stays in batch 1
        ctx.ingest_host(*b2)
        ctx.keyframe_index()
        ctx.subscriber_add(s, edgpu.TRANSPORT_UDP)  # a new output: the GOP from batch 1 + batch 2
        n = check(b2, 10)                           # 5 new packets x 2 outputs have sources
        assert n == 5 + 12 + 5


@pytest.mark.gpu
def test_device_local_cpus_are_the_gpus_node_within_the_allowed_set():
    """edgpu_device_local_cpus: the GPU's NUMA node (its PCI function's sysfs local_cpulist), only
    CPUs this process may run on, and non-empty on an MI355X host."""
    import os
    cpus = edgpu.device_local_cpus(0)
    assert cpus and len(set(cpus)) == len(cpus)
    assert set(cpus) <= os.sched_getaffinity(0)
