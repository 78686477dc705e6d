"""Peer mailboxes: the steady-state replica feed between processes, without a collective
("xGMI peer copies (RCCL only for the cross-GPU subscriber join)").

One mailbox carries one owner rank's session images to one replica rank, in two regions the
owner creates and hands over at the join:
  * data: the image slots, in the owner's device memory (edgpu_device_alloc); the replica maps
    it once (edgpu_ipc_open) and its GPU reads the images straight out of the owner's HBM over
    xGMI (edgpu_session_import takes the mapped pointer, or a peer copy of it);
  * control: the header words, the feedback ids and each slot's header and offsets, in POSIX
    shared memory (the ranks of a node share its host memory) -- polled and written by the two
    processes directly, so a step's handshake costs no device transfers.  The CPU rehearsal
    (gloo tests, no GPU) keeps the images in shared memory as well.

Control layout (bytes):
  [0, 64)      owner writes:   collected u64 at 24 (the feedback round it took last)
  [64, 128)    replica writes: ack u64 (the last publication imported), nfb u32, fb_seq u64
               (the last publication imported when the feedback was written), fb_round u64
               (the feedback round: one per feedback call, so a replica that reports twice
               between two publications loses neither report)
  [128, FB)    replica writes: feedback -- global ids of sessions one of its outputs relocated
               (ReflectorSender::NeedRelocateBookMark -> SetHasVideoKeyFrameUpdate, ReflectorStream.cpp:
               1311-1317), at most `max_sessions`
  slot k meta  the header of the publication in data slot k (seq u64, slot/n u32, bytes u64),
               then its offsets u64[n + 1]; publication p goes to slot p & 1, so a replica one
               publication behind still finds its own

Protocol -- every rank calls the steps at the same points of its ticks:

  publish   owner    waits until ack >= seq - 1 (the slot it is about to reuse was imported),
                     exports the images (full the first time a session is sent to this replica,
                     deltas after) into data slot (seq + 1) & 1 (the export is complete when it
                     returns), writes their offsets, then the slot's header with the new seq
  consume   replica  waits until the slot of the publication it expects holds it, reads the
                     offsets, imports from the mapped slot (complete when it returns) and writes
                     ack = seq
  feedback  replica  (after its tick's backpressure reports) the relocations it saw, fb_seq = seq,
                     fb_round + 1
  collect   owner    takes the feedback -- in lockstep mode waiting for fb_seq == seq, so a
                     relocation reaches the owner before its next ingest as in the one-process
                     reference.  Without lockstep a round the owner has not taken yet is carried
                     into the replica's next one (a relocation arrives a tick or two late, as
                     between two servers)

Waits poll the header with a bound (`timeout_s`) and raise TimeoutError naming the peer: a dead
peer ends the run instead of hanging it.
"""
from __future__ import annotations

import time

import numpy as np

HDR_BYTES = 128
SLOT_ALIGN = 256


class DeviceRegion:
    """A mailbox in device memory: the owner's buffer (edgpu_device_alloc) or a replica's mapping
    of it (edgpu_ipc_open).  `base` is the pointer this process's GPU uses."""

    def __init__(self, ctx, nbytes: int = 0, handle: bytes | None = None):
        self.ctx = ctx
        if handle is None:
            self.buf = ctx.device_alloc(nbytes)
            self.base, self.nbytes = self.buf.ptr, nbytes
            self.handle = ctx.ipc_export(self.base)
        else:
            self.buf = None
            self.base, self.nbytes, self.handle = ctx.ipc_open(handle), nbytes, handle

    def read(self, off: int, n: int) -> np.ndarray:
        return self.ctx.copy_to_host(self.base + off, n)

    def write(self, off: int, data) -> None:
        self.ctx.copy_to_device(self.base + off, data)

    def addr(self, off: int) -> int:
        return self.base + off

    def close(self):
        if self.buf is not None:
            self.buf.free()
            self.buf = None
        elif self.base:
            self.ctx.ipc_close(self.base)
        self.base = 0


class SameProcessRegion(DeviceRegion):
    """The replica end of a mailbox whose owner lives in this process (replica.MailboxReplicaLink):
    the owner's device pointer itself stands for the handle."""

    def __init__(self, ctx, nbytes: int = 0, handle: int | None = None):
        self.ctx, self.buf = ctx, None
        self.base, self.nbytes, self.handle = int(handle), nbytes, handle

    def close(self):
        self.base = 0


_created_here: set = set()           # shared-memory names this process created


class HostRegion:
    """The CPU rehearsal's mailbox: POSIX shared memory (the handle is its name)."""

    def __init__(self, ctx=None, nbytes: int = 0, handle: bytes | None = None):
        from multiprocessing import shared_memory
        if handle is None:
            self.shm = shared_memory.SharedMemory(create=True, size=max(nbytes, HDR_BYTES))
            self.owner = True
            self.handle = self.shm.name.encode()
            _created_here.add(self.shm.name)
        else:
            self.shm = shared_memory.SharedMemory(name=handle.decode())
            self.owner = False
            self.handle = handle
            # the creating rank owns the segment's lifetime: this process's resource tracker must
            # not unlink it at exit (Python < 3.13 registers every attach)
            if self.shm.name not in _created_here:
                from multiprocessing import resource_tracker
                try:
                    resource_tracker.unregister(self.shm._name, "shared_memory")
                except Exception:
                    pass
        self.nbytes = self.shm.size
        self.view = np.ndarray((self.nbytes,), dtype=np.uint8, buffer=self.shm.buf)
        if self.owner:
            self.view[:HDR_BYTES] = 0

    def read(self, off: int, n: int) -> np.ndarray:
        return self.view[off:off + n].copy()

    def write(self, off: int, data) -> None:
        a = np.frombuffer(bytes(data), dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else \
            np.ascontiguousarray(data).view(np.uint8).ravel()
        self.view[off:off + a.size] = a

    def addr(self, off: int):
        return self.view[off:]

    def close(self):
        if self.shm is not None:
            del self.view
            self.shm.close()
            if self.owner:
                _created_here.discard(self.shm.name)
                self.shm.unlink()
            self.shm = None


def slot_meta(max_sessions: int) -> int:
    """A slot's header (64 B) + offsets in the control region, 64-B aligned."""
    return -(-(64 + 8 * (max_sessions + 1)) // 64) * 64


def ctl_layout(max_sessions: int):
    """(feedback region end, slot 0 meta, slot 1 meta, control bytes)."""
    fb_end = HDR_BYTES + 4 * max_sessions
    m0 = -(-fb_end // 64) * 64
    sm = slot_meta(max_sessions)
    return fb_end, m0, m0 + sm, m0 + 2 * sm


class Mailbox:
    """One direction owner -> replica.  The owner creates it (handle=None) and hands `handle`
    (the data region's handle, the control region's name) over at the join; the replica opens it
    with the same sizes.  `region_cls` holds the image slots (DeviceRegion, or HostRegion in the
    rehearsal); the control words are always a HostRegion."""

    def __init__(self, region_cls, ctx, max_sessions: int, slot_bytes: int, handle=None,
                 timeout_s: float = 60.0):
        self.max_sessions, self.slot_bytes = int(max_sessions), int(slot_bytes)
        self.fb_end, m0, m1, ctl_bytes = ctl_layout(self.max_sessions)
        self.slot_meta_at = (m0, m1)
        self.slot_room = -(-self.slot_bytes // SLOT_ALIGN) * SLOT_ALIGN
        h_data, h_ctl = handle if handle is not None else (None, None)
        self.ctl = HostRegion(None, ctl_bytes, h_ctl)
        try:
            self.data = region_cls(ctx, 2 * self.slot_room, h_data)
        except Exception:
            self.ctl.close()
            raise
        self.handle = (self.data.handle, self.ctl.handle)
        self.seq = 0                      # owner: last published; replica: last imported
        self.collected = 0                # owner: the feedback round it took last
        self.fb_round = 0                 # replica: its last feedback round
        self.fb_last: list = []           # replica: its last feedback round's ids
        self.timeout_s = timeout_s
        self.bytes_moved = 0
        self.wait_s = 0.0                 # time spent waiting for the peer

    def _hdr(self) -> dict:
        h = self.ctl.read(0, HDR_BYTES)
        u64 = h[0:32].view(np.uint64)
        r64 = h[64:96].view(np.uint64)
        return {"collected": int(u64[3]), "ack": int(r64[0]),
                "nfb": int(h[72:76].view(np.uint32)[0]), "fb_seq": int(r64[2]), "fb_round": int(r64[3])}

    def _wait(self, pred, what: str) -> dict:
        t0 = time.perf_counter()
        delay = 0.0
        while True:
            h = self._hdr()
            if pred(h):
                self.wait_s += time.perf_counter() - t0
                return h
            if time.perf_counter() - t0 > self.timeout_s:
                raise TimeoutError(f"peer mailbox: {what} not seen in {self.timeout_s:.0f} s (peer rank gone?)")
            if delay:
                time.sleep(delay)
            delay = min(max(delay * 2, 5e-6), 1e-3)

    # ---- owner side ----
    def publish(self, export_fn, n: int) -> int:
        """export_fn(dst, cap) -> offsets[n + 1] writes n sessions' images at dst (a device
        pointer; a host view in the rehearsal), complete when it returns.  Returns the bytes
        published."""
        if n > self.max_sessions:
            raise ValueError(f"mailbox holds {self.max_sessions} sessions, {n} published")
        if self.seq >= 2:
            want = self.seq - 1
            self._wait(lambda h: h["ack"] >= want, f"import of publication {want}")
        k = (self.seq + 1) & 1
        offsets = np.asarray(export_fn(self.data.addr(k * self.slot_room), self.slot_room), dtype=np.uint64)
        if len(offsets) != n + 1:
            raise ValueError("export_fn must return n + 1 offsets")
        total = int(offsets[-1])
        if total > self.slot_room:
            raise ValueError(f"publication of {total} bytes exceeds the mailbox slot ({self.slot_room})")
        meta = self.slot_meta_at[k]
        self.ctl.write(meta + 64, offsets)
        self.seq += 1
        hdr = np.zeros(24, np.uint8)
        hdr[0:8] = np.array([self.seq], np.uint64).view(np.uint8)
        hdr[8:16] = np.array([k, n], np.uint32).view(np.uint8)
        hdr[16:24] = np.array([total], np.uint64).view(np.uint8)
        self.ctl.write(meta, hdr)          # the slot's seq: its images and offsets are complete already
        self.bytes_moved += total
        return total

    def collect(self, lockstep: bool) -> list:
        """The replica's relocations since the last collect (lockstep: waits for the feedback
        round of the last publication).  Returns global session ids."""
        if lockstep and self.seq:
            h = self._wait(lambda h: h["fb_seq"] >= self.seq, f"feedback of publication {self.seq}")
        else:
            h = self._hdr()
        if h["fb_round"] <= self.collected:
            return []
        ids = self.ctl.read(HDR_BYTES, 4 * h["nfb"]).view(np.uint32).tolist() if h["nfb"] else []
        self.collected = h["fb_round"]
        self.ctl.write(24, np.array([self.collected], np.uint64))
        return ids

    # ---- replica side ----
    def consume(self, import_fn, n: int) -> int:
        """Waits for the next publication, applies it (import_fn(src, offsets), src the mapped
        slot's images, complete when it returns) and acks it.  Returns the bytes imported."""
        want = self.seq + 1
        k = want & 1
        meta = self.slot_meta_at[k]
        t0 = time.perf_counter()
        delay = 0.0
        while True:                                    # the slot's own header
            sh = self.ctl.read(meta, 64 + 8 * (n + 1))
            seq = int(sh[0:8].view(np.uint64)[0])
            if seq >= want:
                break
            if time.perf_counter() - t0 > self.timeout_s:
                raise TimeoutError(f"peer mailbox: publication {want} not seen in {self.timeout_s:.0f} s "
                                   f"(peer rank gone?)")
            if delay:
                time.sleep(delay)
            delay = min(max(delay * 2, 5e-6), 1e-3)
        self.wait_s += time.perf_counter() - t0
        if seq != want:
            raise RuntimeError(f"peer mailbox: slot holds publication {seq} while {want} was expected")
        kk, nn = sh[8:16].view(np.uint32)
        nbytes = int(sh[16:24].view(np.uint64)[0])
        if int(nn) != n:
            raise RuntimeError(f"peer mailbox: publication of {int(nn)} sessions, {n} replicated")
        offsets = sh[64:64 + 8 * (n + 1)].view(np.uint64)
        if nbytes:
            import_fn(self.data.addr(k * self.slot_room), offsets)
        self.seq = want
        self.ctl.write(64, np.array([self.seq], np.uint64))
        self.bytes_moved += nbytes
        return nbytes

    def feedback(self, relocated=()) -> None:
        """This tick's relocations (global ids), as a feedback round after the last publication."""
        fb = set(int(g) for g in relocated)
        if self.fb_last and self._hdr()["collected"] < self.fb_round:   # the last round not taken yet
            fb |= set(self.fb_last)
        ids = np.asarray(sorted(fb), dtype=np.uint32)
        if len(ids) > self.max_sessions:
            raise ValueError("more relocations than replicated sessions")
        self.fb_last = ids.tolist()
        if len(ids):
            self.ctl.write(HDR_BYTES, ids)
        self.fb_round += 1
        w = np.zeros(24, np.uint8)
        w[0:4] = np.array([len(ids)], np.uint32).view(np.uint8)
        w[8:24] = np.array([self.seq, self.fb_round], np.uint64).view(np.uint8)
        self.ctl.write(72, w)              # nfb, fb_seq, fb_round: the ids are written already

    def close(self):
        self.data.close()
        self.ctl.close()
