"""CPU: the cold-path parsers pinned to the reference.

* SDP (a22): every case of tests/golden/sdp_vectors.json -- lowercase and trailing-blank
  payload names, two rtpmap lines per track, rtpmap before any m=, m=application, RTP/AVP/TCP,
  LF / CR / blank-line endings, a=control forms, non-"m=" m lines -- through the engine's parse
  (edgpu_sdp_parse, the one edgpu_session_add applies) must give the payload type, payload
  name and trackID the REAL SDPSourceInfo::Parse gave (oracle/_ref/ref_vectors sdp).  The
  H.264 keyframe gate (Q3) follows from the name: exactly b"H264/90000".
* CKeyFrameCache (a21): the op scripts of tests/golden/keyframecache_vectors.json through the
  engine's class (tools/kfc_run) must give the reference's results op for op: return values,
  the caller's buffer after PutOnePacket (the buf[13] rewrite), curdatalen, GetOnePacket bytes.
* The restatement's own choices where the reference is undefined (no pin): a PutOnePacket of
  more than 5116 bytes is refused, and a start packet shorter than 14 bytes is not written past.
"""
import json
import os
import struct
import subprocess

import pytest

from easydarwin_amd import edgpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
KFC = os.path.join(ROOT, "tools", "kfc_run")
SDP = json.load(open(os.path.join(GOLD, "sdp_vectors.json")))["cases"]
KFCV = json.load(open(os.path.join(GOLD, "keyframecache_vectors.json")))["scripts"]


@pytest.mark.parametrize("k", range(len(SDP)))
def test_sdp_parse_matches_reference(k):
    case = SDP[k]
    sdp = bytes.fromhex(case["sdp_hex"])
    got = edgpu.sdp_parse(sdp)
    want = [(s["type"], bytes.fromhex(s["name"]), s["track_id"]) for s in case["streams"]]
    assert got == want


def test_h264_gate_cases_present():
    names = [bytes.fromhex(s["name"]) for c in SDP for s in c["streams"]]
    assert b"h264/90000" in names and b"H264/90000  " in names and b"  H264/90000" in names


def _pack(ops):
    out = [struct.pack("<I", len(ops))]
    for code, a, b, data in ops:
        d = bytes.fromhex(data) if isinstance(data, str) else data
        out.append(struct.pack("<BiiI", code, a, b, len(d)) + d)
    return b"".join(out)


def _run_kfc(ops, tmp_path):
    p = tmp_path / "s.bin"
    p.write_bytes(_pack(ops))
    r = subprocess.run([KFC, str(p)], capture_output=True, text=True, check=True)
    return json.loads(r.stdout)


@pytest.mark.parametrize("k", range(len(KFCV)))
def test_keyframecache_matches_reference(k, tmp_path):
    sc = KFCV[k]
    assert _run_kfc(sc["ops"], tmp_path) == sc["results"]


def test_keyframecache_unpinned_choices(tmp_path):
    big = bytes(5117)
    short = bytes(range(13))
    res = _run_kfc([(0, 1 << 20, 0, b""), (1, 5, 1, big), (1, 5, 1, short), (1, 7, 1, bytes(14))], tmp_path)
    assert res[1]["ok"] == 0 and res[1]["curdatalen"] == 0         # refused (the reference overruns)
    assert res[2]["ok"] == 1 and res[2]["buf"] == short.hex()      # nothing written past the packet
    assert bytes.fromhex(res[3]["buf"])[13] == 0x67 and res[3]["curdatalen"] == 18
