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
* one process per GPU: ``DistReplicaLink`` -- at the join each owner hands every replica rank
  the IPC handle of a mailbox in its HBM (easydarwin_amd/mailbox.py); after that the owner
  exports into it and the replica's GPU imports straight out of it over xGMI, with no
  collective on the steady-state path.
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


class MailboxReplicaLink(ReplicaLink):
    """ReplicaLink whose images and relocations travel through a peer mailbox in the owner's HBM
    (easydarwin_amd/mailbox.py), as DistReplicaLink's do between processes -- both ends in one
    process: the replica end reads the owner's buffer directly instead of through an IPC mapping
    (a process cannot open an IPC handle of its own memory); the control words are the same
    shared-memory region.  So every golden pins the mailbox
    protocol, the import straight from the mailbox slot and the lockstep relocation feedback on
    the GPU (tests/test_gpu_replica.py, mode "mailbox")."""

    def __init__(self, owner: edgpu.Context, owner_device: int, replica: edgpu.Context,
                 replica_device: int, session_bytes: int = 4 << 20):
        super().__init__(owner, owner_device, replica, replica_device)
        self.session_bytes = session_bytes
        self.out_mb = self.in_mb = None
        self._retired = []

    def _boxes(self, n: int, nbytes: int):
        from .mailbox import DeviceRegion, Mailbox, SameProcessRegion
        mb = self.out_mb
        if mb is not None and n <= mb.max_sessions and nbytes <= mb.slot_room:
            return
        room = max(n, 2 * (mb.max_sessions if mb else 0), 8)
        slot = max(room * self.session_bytes, 2 * nbytes)
        if mb is not None:
            self._retired += [self.in_mb, mb]
        self.out_mb = Mailbox(DeviceRegion, self.owner, room, slot)
        self.in_mb = Mailbox(SameProcessRegion, self.replica, room, slot,
                             handle=(self.out_mb.data.base, self.out_mb.ctl.handle))

    def sync(self, now_ms: int) -> int:
        if not self.pairs:
            return 0
        osess = [o for o, _ in self.pairs]
        nsnd = [self.owner.senders_of([o]) for o in osess]
        since = np.concatenate([self.heads[pr] if pr in self.heads
                                else np.full(n, edgpu.IMAGE_FULL, dtype=np.uint64)
                                for pr, n in zip(self.pairs, nsnd)])
        offsets, _ = self.owner.session_export(osess, now_ms, since=since)     # size query
        self._boxes(len(self.pairs), int(offsets[-1]))
        pairs = list(self.pairs)

        def export_fn(dst, cap):
            offsets, heads = self.owner.session_export(osess, now_ms, dst, cap, since=since)
            k = 0
            for pr, n in zip(pairs, nsnd):
                self.heads[pr] = heads[k:k + n].copy()
                k += n
            return offsets
        self.out_mb.publish(export_fn, len(pairs))
        total = self.in_mb.consume(lambda ptr, offs: self.replica.session_import(ptr, offs, [r for _, r in pairs]),
                                   len(pairs))
        self.bytes_shipped += total
        return total

    def feedback(self) -> list:
        if self.in_mb is None:              # nothing published yet: nothing to relocate either
            return super().feedback()
        if not self.pairs:
            return []
        hit = set(self.replica.session_relocations([r for _, r in self.pairs]))
        self.in_mb.feedback([o for o, r in self.pairs if r in hit])
        upd = sorted(set(self.out_mb.collect(lockstep=True)))
        if upd:
            self.owner.session_key_update(upd)
        return upd

    def close(self):
        for mb in self._retired + [self.in_mb, self.out_mb]:
            if mb is not None:
                mb.close()
        self._retired, self.in_mb, self.out_mb = [], None, None
        super().close()


class DistReplicaLink:
    """The one-process-per-GPU form of ReplicaLink.  The owner of global session g is rank
    ``dist.owner(g, world)``; a rank that serves subscribers of a session it does not own keeps a
    replica of it.

    Joins are the control plane, and the only collective: ``connect`` gathers every rank's
    replicated sessions, each owner sizes one peer mailbox per replica rank (``mailbox.Mailbox``:
    double-buffered image slots in its own HBM, the header words in POSIX shared memory) and hands
    the IPC handle and the shared-memory name over, and the replica maps them (``edgpu_ipc_open``); ``places`` numbers the joiners in their
    owners' bucket arrays (``dist.route_places``).  The steady state has no collective: ``sync``
    exports each owned session's images (full the first time per replica rank, deltas after)
    straight into the mailboxes and imports this rank's replicas straight from the owners'
    mailboxes -- the replica's GPU reads the owner's HBM over xGMI -- and ``feedback`` carries the
    replicas' relocations back through the same mailboxes.  Every rank calls ``connect`` /
    ``places`` at the same (join) ticks and ``sync`` / ``feedback`` at every tick.

    lockstep: ``feedback`` waits for every replica's relocations of the tick (exact one-process
    semantics, the parity tests); without it a relocation may reach its owner a tick late.
    pull: "copy" (default) brings each publication into a local staging buffer with one peer DMA
    copy (hipMemcpyPeerAsync over xGMI) and imports from there; "direct" lets the import kernel read
    the owner's mapped HBM itself (one HBM write + read less per image byte).
    session_bytes: mailbox slot room per replicated session (full images are key -> newest:
    about 2 s of stream; default EDGPU_MAILBOX_SESSION_MB or 4 MiB)."""

    def __init__(self, ctx: edgpu.Context, world: int, rank: int, lockstep: bool = True,
                 session_bytes: int | None = None, timeout_s: float = 60.0, region_cls=None,
                 pull: str = "copy"):
        import os

        from .mailbox import DeviceRegion
        self.region_cls = region_cls or DeviceRegion     # mailbox.HostRegion: the CPU rehearsal
        if pull not in ("copy", "direct"):
            raise ValueError("pull: 'copy' or 'direct'")
        self.pull = pull if region_cls is None else "direct"   # (host regions: the stand-in reads them)
        self._stage = None                                # local staging buffer (pull="copy")
        self.ctx, self.world, self.rank = ctx, world, rank
        self.lockstep = lockstep
        self.session_bytes = session_bytes or int(float(os.environ.get("EDGPU_MAILBOX_SESSION_MB", "4")) * (1 << 20))
        self.timeout_s = timeout_s
        self.local_of: dict[int, int] = {}            # owned global session -> engine session
        self.replica_of: dict[int, int] = {}          # replicated global session -> engine session
        self.heads: dict[tuple[int, int], np.ndarray] = {}   # (global session, dst rank) -> heads
        self.out: dict[int, tuple] = {}               # dst rank -> (Mailbox, [global sessions])
        self.inbox: dict[int, tuple] = {}             # src rank -> (Mailbox, [global sessions])
        self._retired: list = []                      # replaced mailboxes, freed at the next connect
        self.bytes_sent = self.bytes_received = 0
        self.sync_s = 0.0                             # host time inside sync()

    def own(self, g: int, local: int):
        self.local_of[int(g)] = int(local)

    def want(self, g: int, sdp: str, udp_push: bool = False) -> int:
        """Creates the replica of global session g here; the next connect() brings it into its
        owner's mailbox and the sync after that its full image."""
        rs = self.ctx.session_add(sdp, udp_push)
        self.replica_of[int(g)] = rs
        return rs

    def places(self, events):
        """dist.route_places over this context (collective, at joins): the owners here take / free
        the places of every rank's replica joins / leaves; returns {key: place} for this rank's
        joins, each to be given to its subscriber with subscriber_set_slot."""
        from .dist import route_places
        return route_places(events, lambda g: self.ctx.session_remote_join(self.local_of[g]),
                            lambda g, p: self.ctx.session_remote_leave(self.local_of[g], p),
                            self.world, self.rank)

    def connect(self):
        """The join round (collective): every rank's replicated sessions reach their owners, which
        (re)create the mailboxes whose session lists grew past their room and hand the new
        handles over.  A mailbox keeps its sequence when only its list changes."""
        import torch.distributed as dist

        from .dist import owner
        from .mailbox import Mailbox
        for mb in self._retired:
            mb.close()
        self._retired = []
        wants = [None] * self.world
        dist.all_gather_object(wants, sorted(self.replica_of))
        made = {}
        for r in range(self.world):
            if r == self.rank:
                continue
            mine = [g for g in wants[r] if owner(g, self.world) == self.rank]
            cur = self.out.get(r)
            if not mine:
                if cur:
                    self._retired.append(cur[0])
                    self.out.pop(r)
                continue
            if cur is None or len(mine) > cur[0].max_sessions:
                room = max(len(mine), 2 * (cur[0].max_sessions if cur else 0), 8)
                mb = Mailbox(self.region_cls, self.ctx, room, room * self.session_bytes, timeout_s=self.timeout_s)
                if cur:
                    self._retired.append(cur[0])
                self.out[r] = (mb, mine)
                made[r] = (mb.handle, room, room * self.session_bytes, getattr(self.ctx, "device", 0))
            else:
                self.out[r] = (cur[0], mine)
        handles = [None] * self.world
        dist.all_gather_object(handles, made)
        for src in range(self.world):
            if src == self.rank:
                continue
            mine = [g for g in sorted(self.replica_of) if owner(g, self.world) == src]
            if self.rank in handles[src]:
                h, room, slot_bytes, dev = handles[src][self.rank]
                if src in self.inbox:
                    self._retired.append(self.inbox[src][0])
                mb = Mailbox(self.region_cls, self.ctx, room, slot_bytes, handle=h, timeout_s=self.timeout_s)
                mb.src_device = dev
                self.inbox[src] = (mb, mine)
            elif src in self.inbox:
                if mine:
                    self.inbox[src] = (self.inbox[src][0], mine)
                else:
                    self._retired.append(self.inbox.pop(src)[0])

    def _export_fn(self, sessions, dst_rank, now_ms):
        local = [self.local_of[g] for g in sessions]
        nsnd = [self.ctx.senders_of([s]) for s in local]
        since = np.concatenate([self.heads.get((g, dst_rank), np.full(n, edgpu.IMAGE_FULL, dtype=np.uint64))
                                for g, n in zip(sessions, nsnd)])

        def fn(dst, cap):
            offsets, heads = self.ctx.session_export(local, now_ms, dst, cap, since=since)
            k = 0
            for g, n in zip(sessions, nsnd):
                self.heads[(g, dst_rank)] = heads[k:k + n].copy()
                k += n
            return offsets
        return fn

    def sync(self, now_ms: int):
        """Publishes this rank's images to every replica rank, then imports this rank's replicas
        from every owner (no collective).  Returns (bytes sent, bytes received)."""
        import time as _time
        t0 = _time.perf_counter()
        sent = recv = 0
        for r, (mb, sessions) in sorted(self.out.items()):
            sent += mb.publish(self._export_fn(sessions, r, now_ms), len(sessions))
        for src, (mb, sessions) in sorted(self.inbox.items()):
            local = [self.replica_of[g] for g in sessions]
            recv += mb.consume(lambda ptr, offs, mb=mb: self._import(mb, ptr, offs, local), len(sessions))
        self.bytes_sent += sent
        self.bytes_received += recv
        self.sync_s += _time.perf_counter() - t0
        return sent, recv

    def _import(self, mb, ptr, offsets, local):
        if self.pull == "direct":
            self.ctx.session_import(ptr, offsets, local)
            return
        nbytes = int(offsets[-1])
        if self._stage is None or self._stage.nbytes < nbytes:
            if self._stage is not None:
                self._stage.free()
            self._stage = self.ctx.device_alloc(max(nbytes * 5 // 4, 1 << 20))
        # one peer DMA copy over xGMI, then the import from local HBM (stream-ordered after it)
        self.ctx.memcpy_peer(self._stage.ptr, mb.src_device, ptr, nbytes)
        self.ctx.session_import(self._stage.ptr, offsets, local)

    def feedback(self) -> list:
        """The replicas' relocations to their owners (ReplicaLink.feedback across ranks, through
        the mailboxes): call it after this rank's backpressure reports and before its next ingest.
        Returns the owned global sessions whose key-update flag was set here."""
        g_of = {v: g for g, v in self.replica_of.items()}
        hit = set(g_of[s] for s in self.ctx.session_relocations(sorted(g_of))) if g_of else set()
        for _src, (mb, sessions) in sorted(self.inbox.items()):
            mb.feedback([g for g in sessions if g in hit])
        mine = set()
        for _r, (mb, _sessions) in sorted(self.out.items()):
            mine.update(mb.collect(self.lockstep))
        upd = sorted(g for g in mine if g in self.local_of)
        if upd:
            self.ctx.session_key_update([self.local_of[g] for g in upd])
        return upd

    @property
    def wanted_by_others(self) -> set:
        """Owned global sessions some other rank replicates (as of the last connect)."""
        return {g for _mb, ss in self.out.values() for g in ss}

    def stats(self) -> dict:
        boxes = [mb for mb, _ in self.out.values()] + [mb for mb, _ in self.inbox.values()]
        return {"bytes_sent": self.bytes_sent, "bytes_received": self.bytes_received,
                "sync_s": round(self.sync_s, 6), "peer_wait_s": round(sum(mb.wait_s for mb in boxes), 6),
                "mailboxes_out": len(self.out), "mailboxes_in": len(self.inbox)}

    def close(self):
        for mb in self._retired:
            mb.close()
        for mb, _ in list(self.inbox.values()):
            mb.close()
        for mb, _ in list(self.out.values()):
            mb.close()
        self._retired, self.inbox, self.out = [], {}, {}
        if self._stage is not None:
            self._stage.free()
            self._stage = None
