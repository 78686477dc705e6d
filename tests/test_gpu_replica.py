"""GPU: cross-GPU keyframe fast start through session images.

Every subscriber of a golden scenario joins a *replica* session on a second engine context
while the owner context ingests; the replica follows the owner through full + delta session
images (edgpu_session_export / edgpu_memcpy_peer / edgpu_session_import).  The replica's
per-subscriber output must equal the reference reflector's capture byte for byte -- i.e. a
subscriber served by a non-owner GPU is indistinguishable from one served by the owner.
Both contexts live on device 0 here (the box has one GPU); the peer copy is then a plain
device copy, and the kernels are the same ones a two-GPU link runs.

Every golden runs, the session lifecycle ones included (a pusher's leave, the session's end with
or without its outputs, a fresh re-push, RereadPrefs): the lifecycle reaches the replicas
(ReplicaLink.remove), a re-pushed session gets fresh ones.  "split" serves the odd subscriber
ids from a replica and the even ones from the owner, and the bucket places of all of them are
the ones a single context gives -- the reference's one array (ReflectorStream::AddOutput,
ReflectorStream.cpp:281-334) -- so the transmit times' bucket lateness is the reference's too.
Each mode runs a second time with the images and relocations going through a peer mailbox in
the owner's memory (replica.MailboxReplicaLink), so every golden pins the mailbox protocol the
one-process-per-GPU link uses, the import straight from the mailbox slot included.
"""
import hashlib

import numpy as np
import pytest

from easydarwin_amd import edgpu
from easydarwin_amd.replay import replay
from easydarwin_amd.replica import MailboxReplicaLink
from scenarios import SCENARIOS
from test_gpu_parity import _fixture, _trace


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["all", "late", "split",
                                  "all+mailbox", "late+mailbox", "split+mailbox"])
@pytest.mark.parametrize("name", list(SCENARIOS))
def test_replica_matches_reference(name, mode):
    """"+mailbox": the images and the relocation feedback travel through a peer mailbox
    (MailboxReplicaLink: the protocol DistReplicaLink runs between processes, both ends here)."""
    tr = _trace(name)
    mode, _, via = mode.partition("+")
    cap, _ = replay(tr, replica=mode, link_cls=MailboxReplicaLink if via else None)
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


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["udppush", "nal", "prefs_buffer", "leave", "repush", "prefs_reread"])
def test_split_session_places_match_one_context(name):
    """A session's outputs split over the owner and a replica are numbered in one bucket array: every
    subscriber's place equals the one it gets when a single context serves them all (udppush: 130
    players, nine buckets; leave: places freed and reused)."""
    tr = _trace(name)
    one, split = {}, {}
    replay(tr, slots=one)
    replay(tr, replica="split", slots=split)
    assert one and split == one
    if name == "udppush":
        assert max(one.values()) >= 16 * 8


@pytest.mark.gpu
def test_remote_places_first_empty():
    """edgpu_session_remote_join / _leave / edgpu_subscriber_set_slot against AddOutput's rule: the
    first empty place, a freed one reused, remote and local outputs in one array, the eye count."""
    sdp = _trace("anchor").sdps[0]
    with edgpu.Context() as own, edgpu.Context() as rep:
        s = own.session_add(sdp)
        r = rep.session_add(sdp)
        h0 = own.subscriber_add(s)
        p1 = own.session_remote_join(s)
        h2 = own.subscriber_add(s)
        p3 = own.session_remote_join(s)
        assert (own.subscriber_slot(h0), p1, own.subscriber_slot(h2), p3) == (0, 1, 2, 3)
        own.session_remote_leave(s, p1)
        assert own.session_remote_join(s) == 1            # the freed place, reused
        own.subscriber_remove(h0)
        assert own.session_remote_join(s) == 0
        with pytest.raises(edgpu.EdgpuError):
            own.session_remote_leave(s, 2)                 # a local output's place
        a = rep.subscriber_add(r)
        b = rep.subscriber_add(r)
        rep.subscriber_set_slot(a, 3)
        assert (rep.subscriber_slot(a), rep.subscriber_slot(b)) == (3, 1)
        with pytest.raises(edgpu.EdgpuError):
            rep.subscriber_set_slot(b, 3)                  # taken
        rep.subscriber_set_slot(b, 40)
        c = rep.subscriber_add(r)
        assert rep.subscriber_slot(c) == 0                 # the first empty one
        own.session_remove(s, kill_outputs=True)
        rep.session_remove(r, kill_outputs=True)
