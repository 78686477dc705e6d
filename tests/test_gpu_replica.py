"""GPU: cross-GPU keyframe fast start through session images.

Every subscriber of a golden scenario joins a *replica* session on a second engine context
while the owner context ingests; the replica follows the owner through full + delta session
images (edgpu_session_export / edgpu_memcpy_peer / edgpu_session_import).  The replica's
per-subscriber output must equal the reference reflector's capture byte for byte -- i.e. a
subscriber served by a non-owner GPU is indistinguishable from one served by the owner.
Both contexts live on device 0 here (the box has one GPU); the peer copy is then a plain
device copy, and the kernels are the same ones a two-GPU link runs.
"""
import hashlib

import numpy as np
import pytest

from easydarwin_amd import edgpu
from easydarwin_amd.replay import replay
from scenarios import SCENARIOS
from test_gpu_parity import _fixture, _trace


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["all", "late"])
@pytest.mark.parametrize("name", list(SCENARIOS))
def test_replica_matches_reference(name, mode):
    tr = _trace(name)
    if tr.has_lifecycle:
        pytest.skip("replica replays model no session lifecycle (a replica follows a live owner session)")
    cap, _ = replay(tr, replica=mode)
    if hashlib.sha256(cap).hexdigest() != _fixture(name)["capture_sha256"]:
        from easydarwin_amd.trace import capture_summary, read_capture
        g, w = capture_summary(read_capture(cap)), _fixture(name)["substreams"]
        bad = [k for k in w if g.get(k) != w[k]]
        pytest.fail(f"{len(bad)} sub-streams differ, e.g. {[(k, g.get(k), w[k]) for k in bad[:3]]}")


@pytest.mark.gpu
def test_image_rejects_mismatch_and_gaps():
    tr = _trace("anchor")
    with edgpu.Context() as a, edgpu.Context() as b:
        s = a.session_add(tr.sdps[0])
        # one-track replica for a multi-track image: rejected
        one = "v=0\r\nm=video 0 RTP/AVP 96\r\na=rtpmap:96 H264/90000\r\n"
        r_bad = b.session_add(one)
        r_ok = b.session_add(tr.sdps[0])
        offs, heads = a.session_export([s], 0)
        buf = a.device_alloc(int(offs[-1]))
        a.session_export([s], 0, buf.ptr, buf.nbytes)
        with pytest.raises(edgpu.EdgpuError):
            b.session_import(buf.ptr, offs, [r_bad])
        b.session_import(buf.ptr, offs, [r_ok])
        # a delta that does not start at the replica's head: rejected
        since = np.ones(len(heads), dtype=np.uint64)
        with pytest.raises(edgpu.EdgpuError):
            a.session_export([s], 0, buf.ptr, buf.nbytes, since=since)   # from > head
        buf.free()
