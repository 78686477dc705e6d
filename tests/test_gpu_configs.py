"""GPU: BASELINE configs C3 (per-GPU shape) and C4 (10k mid-GOP joins) at full size.

* C3 = 8192 streams x 64 UDP subscribers sharded by FNV-1a(stream ID) over 8 GPUs.  One GPU's
  share is rank 0's shard (~1024 sessions) x 64 subscribers; the test runs that shard through
  the engine and checks size-independent properties: exact relayed packet / byte counts
  (first tick = key pointer -> newest per session, ReflectorStream.cpp:1058-1069; later ticks
  = the tick's packets), every sub-stream's descriptor count, and full bytes of a sample of
  sub-streams against the ingested packets.
* C4 = 10,000 subscribers join the C2 stream set mid-GOP; a subscriber's egress GPU is
  hash(subID) % 8 (tools/bench_c4.py), so 7/8 join a replica session fed by a full session
  image.  Checked: each joiner's first tick is exactly the owner ring's key pointer -> newest
  (count and bytes), the remote-join / replica-session accounting, and the image size
  (header + per-sender records + metadata + slot bytes of key pointer (or the RTP-Info window
  start, whichever is older) -> newest).
"""
import numpy as np
import pytest

from easydarwin_amd import edgpu
from easydarwin_amd.workload import H264Fleet, fnv1a64, shard_sessions
from test_gpu_scale import _host_batch


def _is_key(b):
    """IsKeyFrameFirstPacket (ReflectorStream.cpp:1403-1513) over the workload's packets:
    SPS (36 B) / PPS (20 B, exactly the Len >= 20 boundary) single NALs, FU-A start of an IDR."""
    t0 = b["fu"][:, 0] & 0x1F
    t1 = b["fu"][:, 1]
    return (b["len"] >= 20) & ((t0 == 7) | (t0 == 8) | ((t0 == 28) & ((t1 & 0x80) != 0) & ((t1 & 0x1F) == 5)))


def _expected_first_tick(batches, upto, now):
    """Per session: packets a new output receives at the fan-out after batch `upto`, and the
    global indices (batch, packet) of its first packet -- key pointer -> newest, else the
    new-output window (arrival >= now - 1000 ms)."""
    n = len(batches[0]["seg_off"]) - 1
    out = []
    for s in range(n):
        pk = []          # (batch, index) of the session's packets in arrival order
        keys = []
        arr = []
        for t in range(upto + 1):
            b = batches[t]
            lo, hi = int(b["seg_off"][s]), int(b["seg_off"][s + 1])
            k = _is_key(b)[lo:hi]
            for i in range(lo, hi):
                pk.append((t, i))
            keys.extend(k.tolist())
            arr.extend(b["arrival"][lo:hi].tolist())
        key_idx = [i for i, v in enumerate(keys) if v]
        if key_idx:
            first = key_idx[-1]
        else:
            first = next(i for i, a in enumerate(arr) if a >= now - 1000)
        out.append((len(pk) - first, pk[first:]))
    return out


@pytest.mark.gpu
def test_c3_per_gpu_shape_properties():
    gids = shard_sessions(8192, 0, 8)               # rank 0's share of C3 at 8 GPUs
    n_sess, subs, ticks = len(gids), 64, 2
    assert 900 < n_sess < 1150
    fleet = H264Fleet(gids, tick_ms=1000)
    rng = np.random.Generator(np.random.PCG64(13))
    batches = [fleet.next_batch() for _ in range(ticks)]
    mats = [_host_batch(b, rng) for b in batches]
    max_pk = max(b["n"] for b in batches)
    max_bytes = max(int(b["slot_bytes"].sum()) for b in batches)
    first = _expected_first_tick(batches, 0, batches[0]["t_end"])
    with edgpu.Context(video_ring_packets=8192, video_ring_bytes=16 << 20, other_ring_packets=256,
                       other_ring_bytes=64 << 10, out_arena_bytes=int(max_bytes * subs * 1.05) // 16 * 16,
                       max_out_packets=int(max_pk * subs * 1.05), max_batch_packets=max_pk + 1,
                       max_batch_bytes=max_bytes + 16) as ctx:
        for _ in range(n_sess):
            s = ctx.session_add(fleet.sdp())
            for _k in range(subs):
                ctx.subscriber_add(s, edgpu.TRANSPORT_UDP)
        samp_rng = np.random.Generator(np.random.PCG64(17))
        for t, (b, (desc, blob, slot_off)) in enumerate(zip(batches, mats)):
            ctx.ingest_host(desc, b["seg_off"], np.arange(n_sess, dtype=np.uint32), blob)
            ctx.keyframe_index()
            r = ctx.fanout(b["t_end"])
            st = ctx.stats()
            assert st.status == 0
            seg = b["seg_off"].astype(np.int64)
            per_sess = np.diff(seg)
            want = np.array([c for c, _ in first]) if t == 0 else per_sess
            assert st.relayed_packets == int(want.sum()) * subs
            subs_tab = ctx.copy_to_host(r.substreams, r.n_substreams * edgpu.SUB_DTYPE.itemsize).view(edgpu.SUB_DTYPE)
            rtp = subs_tab[subs_tab["kind"] == 0]
            assert len(rtp) == n_sess * subs
            assert np.all(subs_tab[subs_tab["kind"] == 1]["desc_count"] == 0)
            sess_of = rtp["subscriber"].astype(np.int64) // subs
            assert np.array_equal(rtp["desc_count"].astype(np.int64), want[sess_of])
            # bytes of a sample of sub-streams: exactly the tick's packets (t >= 1) or the
            # first tick's key pointer -> newest (t == 0, all inside batch 0)
            d = ctx.copy_to_host(r.desc, st.relayed_packets * 16).view(edgpu.OUT_DTYPE)
            for qi in samp_rng.choice(len(rtp), size=32, replace=False):
                q = rtp[qi]
                s = int(sess_of[qi])
                n = int(q["desc_count"])
                dd = d[int(q["desc_base"]):int(q["desc_base"]) + n]
                idx = range(int(seg[s + 1]) - n, int(seg[s + 1]))
                assert np.array_equal(dd["len"], b["len"][seg[s + 1] - n:seg[s + 1]].astype(np.uint32))
                region = ctx.copy_to_host(r.arena + int(q["out_base"]), int(q["out_bytes"]))
                for (o, ln), i in zip(zip(dd["offset"].tolist(), dd["len"].tolist()), idx):
                    src = blob[int(slot_off[i]) + 4:int(slot_off[i]) + 4 + ln]
                    assert np.array_equal(region[o - int(q["out_base"]):o - int(q["out_base"]) + ln], src)


@pytest.mark.gpu
def test_c4_burst_joins_match_owner_gop():
    n_sess, joins, gpus, warm = 1024, 10_000, 8, 3
    fleet = H264Fleet(np.arange(n_sess), tick_ms=1000)
    rng = np.random.Generator(np.random.PCG64(23))
    batches = [fleet.next_batch() for _ in range(warm)]
    mats = [_host_batch(b, rng) for b in batches]
    now = batches[-1]["t_end"]
    expect = _expected_first_tick(batches, warm - 1, now)
    max_pk = max(b["n"] for b in batches)
    max_bytes = max(int(b["slot_bytes"].sum()) for b in batches)
    cfg = dict(video_ring_packets=8192, video_ring_bytes=16 << 20, other_ring_packets=256,
               other_ring_bytes=64 << 10, out_arena_bytes=12 << 30, max_out_packets=joins * 1200,
               max_batch_packets=max_pk + 1, max_batch_bytes=max_bytes + 16)
    # the replica on a second GPU when there is one: the image crosses devices over xGMI
    import torch
    rdev = 1 if torch.cuda.device_count() > 1 else 0
    with edgpu.Context(**cfg) as owner, edgpu.Context(device=rdev, **cfg) as replica:
        sdp = fleet.sdp()
        osess = [owner.session_add(sdp) for _ in range(n_sess)]
        rsess = [replica.session_add(sdp) for _ in range(n_sess)]
        for b, (desc, blob, _so) in zip(batches, mats):
            owner.ingest_host(desc, b["seg_off"], np.arange(n_sess, dtype=np.uint32), blob)
            owner.keyframe_index()
            owner.fanout(b["t_end"])
        assert owner.stats().status == 0

        subs = np.arange(joins)
        sess_of = subs % n_sess
        remote = np.array([fnv1a64(f"sub{int(k)}") % gpus != 0 for k in subs])
        need = np.unique(sess_of[remote])
        assert 8000 < int(remote.sum()) < 9500 and len(need) == n_sess     # bench_c4.py accounting
        offs, _ = owner.session_export([osess[g] for g in need], now)
        total = int(offs[-1])
        # image size: 64-B header, one 16-B stream record, two 96-B sender records, then the
        # video RTP sender's packets from min(key pointer, RTP-Info window start) to newest
        for j, g in enumerate(need[:64]):
            pk = []
            for t in range(warm):
                b = batches[t]
                lo, hi = int(b["seg_off"][g]), int(b["seg_off"][g + 1])
                pk.extend(zip(b["arrival"][lo:hi].tolist(), b["slot_bytes"][lo:hi].tolist()))
            key_first = len(pk) - expect[g][0]
            win_first = next(i for i, (a, _) in enumerate(pk) if a >= now - 1000)
            f = min(key_first, win_first)
            size = 64 + 16 + 2 * 96 + 32 * (len(pk) - f) + sum(sb for _, sb in pk[f:])
            assert int(offs[j + 1] - offs[j]) == (size + 15) // 16 * 16
        img_src = owner.device_alloc(total)
        img_dst = replica.device_alloc(total)
        offs2, _ = owner.session_export([osess[g] for g in need], now, img_src.ptr, img_src.nbytes)
        assert np.array_equal(offs, offs2)
        replica.memcpy_peer(img_dst.ptr, 0, img_src.ptr, total)          # owner GPU 0 -> replica GPU
        replica.session_import(img_dst.ptr, offs, [rsess[g] for g in need])
        h_own = owner.subscribers_add([osess[g] for g in sess_of[~remote]], edgpu.TRANSPORT_UDP)
        h_rep = replica.subscribers_add([rsess[g] for g in sess_of[remote]], edgpu.TRANSPORT_UDP)
        c0o, c0r = owner.counters(), replica.counters()
        ro = owner.fanout(now)
        rr = replica.fanout(now)
        c1o, c1r = owner.counters(), replica.counters()
        relayed = (c1o["relayed_packets"] - c0o["relayed_packets"]) + (c1r["relayed_packets"] - c0r["relayed_packets"])
        assert relayed == sum(expect[int(g)][0] for g in sess_of)
        # each joiner's first tick = the owner ring's key pointer -> newest, count and bytes
        check = np.random.Generator(np.random.PCG64(29))
        for ctx, r, handles, sess in ((owner, ro, h_own, sess_of[~remote]), (replica, rr, h_rep, sess_of[remote])):
            st = ctx.stats()
            assert st.status == 0
            tab = ctx.copy_to_host(r.substreams, r.n_substreams * edgpu.SUB_DTYPE.itemsize).view(edgpu.SUB_DTYPE)
            rtp = tab[tab["kind"] == 0]
            by_handle = {int(q["subscriber"]): q for q in rtp}
            counts = np.array([int(by_handle[int(h)]["desc_count"]) for h in handles])
            assert np.array_equal(counts, np.array([expect[int(g)][0] for g in sess]))
            d = ctx.copy_to_host(r.desc, st.relayed_packets * 16).view(edgpu.OUT_DTYPE)
            for k in check.choice(len(handles), size=12, replace=False):
                q = by_handle[int(handles[k])]
                g = int(sess[k])
                n = int(q["desc_count"])
                dd = d[int(q["desc_base"]):int(q["desc_base"]) + n]
                region = ctx.copy_to_host(r.arena + int(q["out_base"]), int(q["out_bytes"]))
                for (o, ln), (t, i) in zip(zip(dd["offset"].tolist(), dd["len"].tolist()), expect[g][1]):
                    desc, blob, slot_off = mats[t]
                    assert ln == int(desc["len"][i])
                    src = blob[int(slot_off[i]) + 4:int(slot_off[i]) + 4 + ln]
                    assert np.array_equal(region[o - int(q["out_base"]):o - int(q["out_base"]) + ln], src)
        img_src.free()
        img_dst.free()
