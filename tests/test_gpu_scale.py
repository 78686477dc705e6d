"""GPU: the benchmark workload (BASELINE.json configs[1], C2) through the engine.

* small slice of the same generator (8 sessions) -> bit-exact against the CPU oracle
  (oracle/relay_model, itself pinned to the reference by tests/test_oracle.py);
* full size (1024 sessions x 16 UDP subscribers, 1-s ticks) -> size-independent properties:
  exact relayed packet/byte counts, per-sub-stream descriptor structure (offsets, lengths,
  packet ids), and full byte comparison of a random sample of sub-streams against the
  ingested packets.
"""
import os
import struct
import subprocess
import tempfile

import numpy as np
import pytest

from easydarwin_amd import edgpu
from easydarwin_amd.trace import Trace, read_capture
from easydarwin_amd.workload import H264Fleet

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _host_batch(b, rng):
    """Materialise a workload batch on the host: random payload + synthetic headers."""
    slot_bytes = b["slot_bytes"]
    slot_off = np.concatenate([[0], np.cumsum(slot_bytes)[:-1]]).astype(np.int64)
    blob = rng.integers(0, 256, size=int(slot_bytes.sum()), dtype=np.uint8)
    for k in range(16):
        blob[slot_off + k] = b["hdr"][:, k]
    blob[slot_off + 16] = b["fu"][:, 0]
    blob[slot_off + 17] = b["fu"][:, 1]
    desc = np.zeros(b["n"], dtype=edgpu.PKT_DTYPE)
    desc["slot"] = slot_off // 16
    desc["len"] = b["len"]
    desc["channel"] = b["channel"]
    desc["arrival_ms"] = b["arrival"]
    return desc, blob, slot_off


def _run_slice(n_sess, subs, ticks, seed=7):
    fleet = H264Fleet(np.arange(n_sess), tick_ms=1000)
    rng = np.random.Generator(np.random.PCG64(seed))
    batches = [fleet.next_batch() for _ in range(ticks)]
    mats = [_host_batch(b, rng) for b in batches]
    return fleet, batches, mats


@pytest.mark.gpu
def test_workload_slice_matches_oracle(oracle_bins):
    n_sess, subs, ticks = 8, 3, 4
    fleet, batches, mats = _run_slice(n_sess, subs, ticks)
    # trace for the oracle
    tr = Trace()
    for _ in range(n_sess):
        tr.add_session(fleet.sdp())
    sub_id = 0
    for t, (b, (desc, blob, slot_off)) in enumerate(zip(batches, mats)):
        sess_of = np.searchsorted(b["seg_off"], np.arange(b["n"]), side="right") - 1
        # trace events must be time-ordered (the virtual clock never goes back)
        for i in sorted(range(b["n"]), key=lambda i: (int(desc["arrival_ms"][i]), int(sess_of[i]), i)):
            off = int(slot_off[i]) + 4
            tr.pkt(int(desc["arrival_ms"][i]), int(sess_of[i]), 0, blob[off:off + int(desc["len"][i])].tobytes())
        if t == 0:
            for s in range(n_sess):
                for k in range(subs):
                    tr.join(b["t_end"], s, sub_id, k % 2)      # UDP and TCP subscribers
                    sub_id += 1
        tr.tick(b["t_end"])
    with tempfile.TemporaryDirectory() as td:
        p, c = os.path.join(td, "w.edtr"), os.path.join(td, "w.edcp")
        tr.write(p)
        subprocess.run([oracle_bins["port"], p, c], check=True)
        want = open(c, "rb").read()
    from easydarwin_amd.replay import replay
    got, _ = replay(tr)
    assert got == want


@pytest.mark.gpu
def test_c2_full_size_properties():
    n_sess, subs, ticks = 1024, 16, 3
    fleet, batches, mats = _run_slice(n_sess, subs, ticks, seed=11)
    max_pk = max(b["n"] for b in batches)
    max_bytes = max(int(b["slot_bytes"].sum()) for b in batches)
    with edgpu.Context(video_ring_packets=8192, video_ring_bytes=16 << 20, other_ring_packets=256,
                       other_ring_bytes=64 << 10, out_arena_bytes=int(max_bytes * subs * 1.05) // 16 * 16,
                       max_out_packets=int(max_pk * subs * 1.05), max_batch_packets=max_pk + 1,
                       max_batch_bytes=max_bytes + 16) as ctx:
        for _ in range(n_sess):
            s = ctx.session_add(fleet.sdp())
            for _k in range(subs):
                ctx.subscriber_add(s, edgpu.TRANSPORT_UDP)
        rng = np.random.Generator(np.random.PCG64(5))
        prev_first_tick = None
        for t, (b, (desc, blob, slot_off)) in enumerate(zip(batches, mats)):
            ctx.ingest_host(desc, b["seg_off"], np.arange(n_sess, dtype=np.uint32), blob)
            ctx.keyframe_index()
            r = ctx.fanout(b["t_end"])
            st = ctx.stats()
            assert st.status == 0
            seg = b["seg_off"].astype(np.int64)
            per_sess = np.diff(seg)
            if t >= 1:
                # steady state: every subscriber receives exactly this tick's packets
                assert st.relayed_packets == int(per_sess.sum()) * subs
                assert st.relayed_bytes == int(b["len"].astype(np.int64).sum()) * subs
            subs_tab = ctx.copy_to_host(r.substreams, r.n_substreams * edgpu.SUB_DTYPE.itemsize).view(edgpu.SUB_DTYPE)
            d = ctx.copy_to_host(r.desc, st.relayed_packets * 16).view(edgpu.OUT_DTYPE)
            rtp = subs_tab[subs_tab["kind"] == 0]
            assert len(rtp) == n_sess * subs
            assert np.all(subs_tab[subs_tab["kind"] == 1]["desc_count"] == 0)
            # structure: offsets increasing, lengths = ingested lengths in order
            samp = rng.choice(len(rtp), size=48, replace=False)
            for qi in samp:
                q = rtp[qi]
                s = int(q["subscriber"]) // subs
                n = int(q["desc_count"])
                dd = d[int(q["desc_base"]):int(q["desc_base"]) + n]
                lens = b["len"][seg[s + 1] - n:seg[s + 1]]
                assert np.array_equal(dd["len"], lens.astype(np.uint32))
                assert np.all(np.diff(dd["offset"].astype(np.int64)) > 0)
                assert np.all(np.diff(dd["packet_id"].astype(np.int64)) == 1)
                # bytes: the sub-stream's arena region vs the ingested packets
                base, nb = int(q["out_base"]), int(q["out_bytes"])
                region = ctx.copy_to_host(r.arena + base, nb)
                for (o, ln), i in zip(zip(dd["offset"].tolist(), dd["len"].tolist()),
                                      range(seg[s + 1] - n, seg[s + 1])):
                    src = blob[int(slot_off[i]) + 4:int(slot_off[i]) + 4 + ln]
                    assert np.array_equal(region[o - base:o - base + ln], src)
            if t == 0:
                prev_first_tick = st.relayed_packets
        assert prev_first_tick > 0
