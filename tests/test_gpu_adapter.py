"""GPU: the C++ module-side adapter (easydarwin_amd/csrc/reflector_adapter.h), driven the way
the reflector module drives its seams (tools/adapter_replay.cpp), reproduces the reference
harness's captures; CKeyFrameCache served from the GPU GOP index."""
import hashlib
import json
import os
import subprocess

import pytest

from easydarwin_amd import edgpu
from easydarwin_amd.replay import replay
from easydarwin_amd.trace import PKT, TICK, Trace, capture_summary, read_capture
from scenarios import SCENARIOS

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
TOOL = os.path.join(ROOT, "tools", "adapter_replay")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["tiny", "mixed", "nal", "ssrc", "anchor", "c1", "rtpinfo", "backpressure", "leave",
                                  "udppush", "repush", "prefs_buffer", "prefs_reread", "keepalive", "highrate",
                                  "longbuffer", "aktt"])
def test_adapter_replay_matches_reference(name, tmp_path):
    fix = json.load(open(os.path.join(GOLD, name + ".json")))
    t, c = tmp_path / "t.edtr", tmp_path / "c.edcp"
    t.write_bytes(SCENARIOS[name]().to_bytes())
    r = subprocess.run([TOOL, str(t), str(c)], check=True, capture_output=True, text=True)
    assert "0 stream errors" in r.stderr, r.stderr[-2000:]
    cap = c.read_bytes()
    if hashlib.sha256(cap).hexdigest() != fix["capture_sha256"]:
        got = capture_summary(read_capture(cap))
        bad = {k: (got.get(k, [None])[:2], fix["substreams"][k][:2]) for k in fix["substreams"]
               if got.get(k) != fix["substreams"][k]}
        pytest.fail(f"{len(bad)} sub-streams differ ([packets, bytes] got vs want): {dict(list(bad.items())[:6])}")


@pytest.mark.gpu
def test_gop_copy_is_key_pointer_to_newest():
    """After the c1 push, the GOP served to a joining player (CKeyFrameCache TLV) is every
    packet from the last IDR's first FU-A fragment to the newest packet."""
    tr = SCENARIOS["c1"]()
    with edgpu.Context() as ctx:
        replay(tr, ctx=ctx)
        img, n = ctx.gop_copy(0, 0)
    pk = [e[4] for e in tr.events if e[0] == PKT]
    last_key = max(i for i, p in enumerate(pk) if len(p) > 13 and p[12] & 0x1F == 28 and p[13] == 0x85)
    want = b"".join(b"\x28" + len(p).to_bytes(2, "big") + p + b"\x29" for p in pk[last_key:])
    assert n == len(pk) - last_key
    assert img == want
