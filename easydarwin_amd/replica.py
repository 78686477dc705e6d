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
        self.heads: dict[tuple[int, int], np.ndarray] = {}   # pair -> heads after its last export
        self.bytes_shipped = 0
        self._src = None
        self._dst = None

    def add(self, owner_session: int, sdp: str, udp_push: bool = False) -> int:
        """Creates the replica session; its first sync ships a full image."""
        rs = self.replica.session_add(sdp, udp_push)
        self.pairs.append((owner_session, rs))
        return rs

    def join(self, owner_session: int, replica_session: int, transport: int, rtp_info: bool = False,
             now_ms: int = 0, place: int | None = None):
        """A subscriber of the replica session: (handle, rtp-info, place).  Its place in the session's
        bucket arrays is taken on the owner (edgpu_session_remote_join, which counts its eye there)
        unless `place` was reserved already, so that the owner's and every replica's subscribers are
        numbered in one array as the reference's AddOutput numbers them (ReflectorStream.cpp:281-334)."""
        h, info = self.replica.subscriber_play(replica_session, transport, rtp_info=rtp_info, now_ms=now_ms)
        if place is None:
            place = self.owner.session_remote_join(owner_session)
        self.replica.subscriber_set_slot(h, place)
        return h, info, place

    def leave(self, owner_session: int, handle: int, place: int):
        """RemoveOutput of a replica subscriber: gone from the replica, its place and eye from the owner."""
        self.replica.subscriber_remove(handle)
        self.owner.session_remote_leave(owner_session, place)

    def remove(self, owner_session: int, kill_outputs: bool = False):
        """The owner session ends (edgpu_session_remove on the owner follows): its replica sessions go
        with it, their subscribers too with kill_outputs (TearDownAllOutputs)."""
        keep = []
        for pr in self.pairs:
            if pr[0] == owner_session:
                self.replica.session_remove(pr[1], kill_outputs=kill_outputs)
                self.heads.pop(pr, None)
            else:
                keep.append(pr)
        self.pairs = keep

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
        since = np.concatenate([self.heads[pr] if pr in self.heads
                                else np.full(n, edgpu.IMAGE_FULL, dtype=np.uint64)
                                for pr, n in zip(self.pairs, nsnd)])
        offsets, heads = self.owner.session_export(osess, now_ms, since=since)     # size query
        total = int(offsets[-1])
        src, dst = self._buffers(total)
        offsets, heads = self.owner.session_export(osess, now_ms, src.ptr, src.nbytes, since=since)
        self.replica.memcpy_peer(dst.ptr, self.odev, src.ptr, total)
        self.replica.session_import(dst.ptr, offsets, [r for _, r in self.pairs])
        k = 0
        for pr, n in zip(self.pairs, nsnd):
            self.heads[pr] = heads[k:k + n].copy()
            k += n
        self.bytes_shipped += total
        return total

    def feedback(self) -> list:
        """Relocations on the replica sessions since the last call (a backpressure report moved an
        output to the newest key frame) set the owners' video-key-update flag, so the owner's next
        audio packet becomes the session's audio key pointer as in the reference
        (edgpu_session_relocations -> edgpu_session_key_update).  Call it after the replica's
        backpressure reports and before the owner's next keyframe index.  Returns the owner
        sessions updated."""
        if not self.pairs:
            return []
        hit = set(self.replica.session_relocations([r for _, r in self.pairs]))
        upd = sorted({o for o, r in self.pairs if r in hit})
        if upd:
            self.owner.session_key_update(upd)
        return upd


class DistReplicaLink:
    """The one-process-per-GPU form of ReplicaLink: the owner of global session g is rank
    ``dist.owner(g, world)``; a rank that serves subscribers of a session it does not own keeps
    a replica of it, and every ``sync`` round moves full images (first time) or deltas from the
    owners with ``dist.exchange_images`` (RCCL point-to-point under the nccl backend, device
    buffers; gloo in CPU-side tests, host buffers).  Every rank calls ``sync`` at the same
    points (it is collective)."""

    def __init__(self, ctx: edgpu.Context, world: int, rank: int, comm: str = "cuda"):
        import torch
        self.torch = torch
        self.ctx, self.world, self.rank = ctx, world, rank
        self.comm = comm                              # "cuda": RCCL device buffers; "cpu": gloo
        self.local_of: dict[int, int] = {}            # owned global session -> engine session
        self.replica_of: dict[int, int] = {}          # replicated global session -> engine session
        self.heads: dict[tuple[int, int], np.ndarray] = {}   # (global session, dst rank) -> heads
        self.bytes_sent = self.bytes_received = 0

    def own(self, g: int, local: int):
        self.local_of[int(g)] = int(local)

    def want(self, g: int, sdp: str, udp_push: bool = False) -> int:
        """Creates the replica of global session g here; its first sync brings the full image."""
        rs = self.ctx.session_add(sdp, udp_push)
        self.replica_of[int(g)] = rs
        return rs

    def places(self, events):
        """dist.route_places over this context: the owners here take / free the places of every
        rank's replica joins / leaves (events as route_places takes them); returns {key: place}
        for this rank's joins, each to be given to its subscriber with subscriber_set_slot."""
        from .dist import route_places
        return route_places(events, lambda g: self.ctx.session_remote_join(self.local_of[g]),
                            lambda g, p: self.ctx.session_remote_leave(self.local_of[g], p),
                            self.world, self.rank)

    def _export(self, sessions, dst_rank, now_ms):
        local = [self.local_of[g] for g in sessions]
        nsnd = [self.ctx.senders_of([s]) for s in local]
        since = np.concatenate([self.heads.get((g, dst_rank), np.full(n, edgpu.IMAGE_FULL, dtype=np.uint64))
                                for g, n in zip(sessions, nsnd)])
        offsets, _ = self.ctx.session_export(local, now_ms, since=since)              # size query
        total = int(offsets[-1])
        dev = self.torch.empty(max(total, 16), dtype=self.torch.uint8, device="cuda")
        self.torch.cuda.synchronize()
        offsets, heads = self.ctx.session_export(local, now_ms, dev.data_ptr(), dev.numel(), since=since)
        k = 0
        for g, n in zip(sessions, nsnd):
            self.heads[(g, dst_rank)] = heads[k:k + n].copy()
            k += n
        return (dev if self.comm == "cuda" else dev.cpu()), offsets

    def _import(self, buf, offsets, sessions, src_rank):
        dev = buf if buf.is_cuda else buf.cuda()
        self.torch.cuda.synchronize()
        self.ctx.session_import(dev.data_ptr(), offsets, [self.replica_of[g] for g in sessions])

    def sync(self, now_ms: int):
        from .dist import exchange_images
        sent, recv = exchange_images(
            sorted(self.replica_of), lambda s, r: self._export(s, r, now_ms), self._import,
            lambda n: self.torch.empty(n, dtype=self.torch.uint8, device="cuda" if self.comm == "cuda" else "cpu"),
            self.world, self.rank)
        self.bytes_sent += sent
        self.bytes_received += recv
        return sent, recv

    def feedback(self) -> list:
        """ReplicaLink.feedback across ranks (dist.route_relocations): this rank's replicas'
        relocations go to the owners, and the owned sessions other ranks relocated get their
        flag set here.  Collective; call it after the replicas' backpressure reports and before
        the owners' next keyframe index.  Returns the owned global sessions updated."""
        from .dist import route_relocations
        g_of = {v: g for g, v in self.replica_of.items()}
        hit = self.ctx.session_relocations(sorted(g_of)) if g_of else []
        return route_relocations([g_of[s] for s in hit],
                                 lambda gs: self.ctx.session_key_update([self.local_of[g] for g in gs]),
                                 self.world, self.rank)
