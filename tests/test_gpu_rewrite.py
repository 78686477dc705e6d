"""GPU: the per-output rewrite stage (edgpu_subscriber_rewrite, north_star item 3).

The reference never rewrites a relayed packet (Q1): RTPSessionOutput::PacketShouldBeThinned
returns false on its first line (RTPSessionOutput.cpp:685-687) and the RTCP rewrite
(RewriteRTCP / TrackRTCPPackets, :403-561) is not called (:600-601).  So:

* identity parameters reproduce the reference capture byte for byte (every parity test runs
  that way; here a subscriber explicitly set to the identity is checked too);
* non-identity parameters must equal the reference capture transformed on the host by the
  documented rule (include/edgpu.h, edgpu_subscriber_rewrite) -- seq += d (mod 2^16),
  ts += d (mod 2^32), SSRC replaced, for RTP packets of >= 12 bytes; RTCP sender SSRC and an
  SR's RTP timestamp.  The host restatement below is this test's oracle for the transform
  (there is no live reference for dead code); the untransformed capture is the reference's.
"""
import hashlib
import os
import struct
import subprocess
import tempfile

import pytest

from easydarwin_amd.replay import replay
from easydarwin_amd.trace import JOIN, read_capture, split_wire_image
from scenarios import SCENARIOS
from test_gpu_parity import _fixture, _trace


def rewrite_params(sub_id: int):
    """Deterministic per-subscriber parameters; every fourth subscriber keeps the identity."""
    if sub_id % 4 == 3:
        return None
    seq = (sub_id * 7919 + 1) & 0xFFFF
    ts = (sub_id * 0x9E3779B1 + 0x1000) & 0xFFFFFFFF
    ssrc = (0xABC00000 + sub_id) if sub_id % 2 == 0 else None
    return seq, ts, ssrc


def rewrite_packet(pkt: bytes, kind: int, seq_d: int, ts_d: int, ssrc) -> bytes:
    b = bytearray(pkt)
    if kind == 0:
        if len(b) >= 12:
            b[2:4] = ((int.from_bytes(b[2:4], "big") + seq_d) & 0xFFFF).to_bytes(2, "big")
            b[4:8] = ((int.from_bytes(b[4:8], "big") + ts_d) & 0xFFFFFFFF).to_bytes(4, "big")
            if ssrc is not None:
                b[8:12] = ssrc.to_bytes(4, "big")
    else:
        if ssrc is not None and len(b) >= 8:
            b[4:8] = ssrc.to_bytes(4, "big")
        if len(b) >= 20 and b[1] == 200:
            b[16:20] = ((int.from_bytes(b[16:20], "big") + ts_d) & 0xFFFFFFFF).to_bytes(4, "big")
    return bytes(b)


def transform_capture(cap: bytes, params: dict) -> bytes:
    """The reference capture with each subscriber's packets rewritten (same record order)."""
    recs = read_capture(cap)
    out = [b"EDCP", struct.pack("<I", len(recs))]
    for key in sorted(recs):
        ss = recs[key]
        data = ss.data
        p = params.get(ss.sub)
        if p is not None:
            parts = []
            for pkt in split_wire_image(data, ss.tcp):
                q = rewrite_packet(pkt, ss.kind, *p)
                if ss.tcp:
                    ch = data[1] if data else 0
                    parts.append(struct.pack(">BBH", 0x24, ch, len(q)) + q)
                else:
                    parts.append(struct.pack(">H", len(q)) + q)
            data = b"".join(parts)
        out.append(struct.pack("<IIHBBQQ", ss.sub, ss.session, ss.track, ss.kind, ss.tcp, ss.n_packets, len(data)))
        out.append(data)
    # receiver reports to pushers are not subscriber output: keep the trailer as is
    n = 8 + sum(28 + len(r.data) for r in recs.values())
    return b"".join(out) + cap[n:]


def _reference_capture(name, oracle_bins):
    """The full reference capture: the committed bytes, or the restatement's replay checked
    against the fixture's digest of the reference capture."""
    tr = _trace(name)
    with tempfile.TemporaryDirectory() as td:
        t, c = os.path.join(td, "t.edtr"), os.path.join(td, "c.edcp")
        tr.write(t)
        subprocess.run([oracle_bins["port"], t, c], check=True)
        cap = open(c, "rb").read()
    assert hashlib.sha256(cap).hexdigest() == _fixture(name)["capture_sha256"]
    return tr, cap


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["mixed", "c1", "udppush", "nal", "clamp", "rtpinfo", "backpressure"])
def test_rewrite_matches_transformed_reference(name, oracle_bins):
    tr, ref = _reference_capture(name, oracle_bins)
    subs = sorted({ev[3] for ev in tr.events if ev[0] == JOIN})
    params = {s: rewrite_params(s) for s in subs}
    rw = {s: p for s, p in params.items() if p is not None}
    got, _ = replay(tr, rewrite=rw)
    want = transform_capture(ref, rw)
    if got != want:
        g, w = read_capture(got), read_capture(want)
        bad = [k for k in w if g[k].data != w[k].data]
        raise AssertionError(f"{len(bad)} sub-streams differ, e.g. {bad[:4]}")
    assert got != ref or not rw


@pytest.mark.gpu
def test_identity_rewrite_is_reference():
    tr, ref = _reference_capture("mixed", oracle_bins={"port": os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "oracle", "relay_model")})
    subs = sorted({ev[3] for ev in tr.events if ev[0] == JOIN})
    got, _ = replay(tr, rewrite={s: (0, 0, None) for s in subs})
    assert got == ref
