"""Cross-GPU keyframe fast start (BASELINE config C4): replica sessions.

A stream is owned by one GPU (``dist.owner``).  A subscriber whose egress GPU differs joins
a *replica session* on its own GPU.  The owner exports a session image (the serveable part
of every sender ring: key pointer -> newest, or the new-output window when there is no key;
``edgpu_session_export``), the image crosses xGMI once per (session, destination GPU), and
the replica imports it (``edgpu_session_import``).  After that, each tick ships only a delta
image (the packets after the heads of the previous export), so the replica follows its
owner without re-sending the GOP.  A subscriber of the replica receives exactly the bytes it
would have received from the owner; ``tests/test_gpu_replica.py`` checks them against the
reference reflector's captures.

Transport:

* in one process (two contexts, possibly on two GPUs): ``ReplicaLink`` exports into a buffer
  on the owner's GPU and pulls it with ``edgpu_memcpy_peer`` (hipMemcpyPeerAsync);
* one process per GPU: ``dist.exchange_images`` moves images with RCCL point-to-point
  send/recv, batched the way ``ncclGroupStart``/``ncclSend``/``ncclRecv`` batch them.
"""
from __future__ import annotations

import numpy as np

from . import edgpu


class ReplicaLink:
    """Keeps replica sessions on `replica` in step with their owner sessions on `owner`."""

    def __init__(self, owner: edgpu.Context, owner_device: int, replica: edgpu.Context,
                 replica_device: int):
        self.owner, self.replica = owner, replica
        self.odev, self.rdev = owner_device, replica_device
        self.pairs: list[tuple[int, int]] = []      # (owner session, replica session)
        self.heads: dict[int, np.ndarray] = {}      # pair index -> heads after its last export
        self.bytes_shipped = 0
        self._src = None
        self._dst = None

    def add(self, owner_session: int, sdp: str, udp_push: bool = False) -> int:
        """Creates the replica session; its first sync ships a full image."""
        rs = self.replica.session_add(sdp, udp_push)
        self.pairs.append((owner_session, rs))
        return rs

    def _buffers(self, nbytes: int):
        if self._src is None or self._src.nbytes < nbytes:
            cap = max(nbytes, 1 << 20) * 5 // 4
            if self._src is not None:
                self._src.free()
                self._dst.free()
            self._src = self.owner.device_alloc(cap)
            self._dst = self.replica.device_alloc(cap)
        return self._src, self._dst

    def close(self):
        if self._src is not None:
            self._src.free()
            self._dst.free()
            self._src = self._dst = None

    def sync(self, now_ms: int) -> int:
        """Ships full images for new replicas and deltas for the rest; returns bytes moved."""
        if not self.pairs:
            return 0
        osess = [o for o, _ in self.pairs]
        nsnd = [self.owner.senders_of([o]) for o in osess]
        since = np.concatenate([self.heads[i] if i in self.heads
                                else np.full(n, edgpu.IMAGE_FULL, dtype=np.uint64)
                                for i, n in enumerate(nsnd)])
        offsets, heads = self.owner.session_export(osess, now_ms, since=since)     # size query
        total = int(offsets[-1])
        src, dst = self._buffers(total)
        offsets, heads = self.owner.session_export(osess, now_ms, src.ptr, src.nbytes, since=since)
        self.replica.memcpy_peer(dst.ptr, self.odev, src.ptr, total)
        self.replica.session_import(dst.ptr, offsets, [r for _, r in self.pairs])
        k = 0
        for i, n in enumerate(nsnd):
            self.heads[i] = heads[k:k + n].copy()
            k += n
        self.bytes_shipped += total
        return total
