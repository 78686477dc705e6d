"""Subscribers on real sockets for the engine's socket egress (include/edgpu.h edgpu_egress_*).

``SocketSink`` gives every UDP subscriber track a pair of loopback receiver sockets (RTP,
RTCP) and every RTSP-interleaved subscriber a stream socketpair, lets ``edgpu_egress_send``
write each fan-out tick to them, and rebuilds each sub-stream's wire image from what the
receivers read -- the capture format of easydarwin_amd/trace.py, so the bytes that crossed
the kernel's socket layer compare directly with the reference's captures.

TCP backpressure: ``hold`` (tick time -> set of subscriber ids) leaves a subscriber's reader
undrained at that tick, so its small send buffer fills and the egress sees EAGAIN; the reports
the egress filed with the engine are kept per tick (``blocked``, as BLOCK events) so the same
budgets can be replayed through the reference harness.

Q20: ``pacing`` (a dict of edgpu_pacing_config fields, {} for the defaults) turns the server's
write gate on for every subscriber (edgpu_egress_pacing: over-buffer window, TCP-audio thinning),
with the PLAY time and the video tracks ``join`` is given and the tick's clock; then ``blocked``
keeps only the writes the socket refused (with the writes it took), since the reference harness
applies the gate itself (EDTR_SERVER_GATE=1).
"""
from __future__ import annotations

import ctypes as C
import os
import socket
import struct

from . import edgpu

_DRAIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "libudp_drain.so")
_drain_lib = None


def _drain():
    """tools/libudp_drain.so: a thread per UDP receiver that takes datagrams (recvmmsg) while the
    egress sends -- a tick replaying a whole GOP to a new player outruns any receive buffer
    net.core.rmem_max allows, and loopback UDP drops what does not fit."""
    global _drain_lib
    if _drain_lib is None:
        lib = C.CDLL(_DRAIN)
        lib.udpd_start.restype = C.c_void_p
        lib.udpd_start.argtypes = [C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_int]
        lib.udpd_stop.argtypes = [C.c_void_p]
        lib.udpd_size.restype = C.c_size_t
        lib.udpd_size.argtypes = [C.c_void_p, C.c_int]
        lib.udpd_count.restype = C.c_size_t
        lib.udpd_count.argtypes = [C.c_void_p, C.c_int]
        lib.udpd_take.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        lib.udpd_free.argtypes = [C.c_void_p]
        _drain_lib = lib
    return _drain_lib


class SocketSink:
    def __init__(self, ctx: edgpu.Context, threads: int = 2, tcp_sndbuf: int | None = None,
                 hold: dict | None = None, pacing: dict | None = None):
        self.eg = edgpu.Egress(ctx, threads)
        self.pacing = pacing
        if pacing is not None:
            self.eg.pacing_config(**pacing)
        self.tcp_sndbuf = tcp_sndbuf
        self.hold = hold or {}
        self.udp = {}           # (handle, track, kind) -> receiver socket
        self.tcp = {}           # handle -> [sender end, reader end, bytearray]
        self.parts = {}         # (handle, track, kind) -> wire image parts (UDP)
        self.npk = {}           # (handle, track, kind) -> datagrams received (UDP)
        self.q_of = []          # sub-stream index -> (handle, track, kind)
        self.sub_id = {}        # handle -> subscriber id
        self.blocked = []       # (tick time, sub_id, track, kind, sent)
        self.stats = []

    def join(self, handle: int, sub_id: int, ntracks: int, tcp: bool, play_time: int = 0, video_tracks: int = 0):
        self.sub_id[handle] = sub_id
        for t in range(ntracks):
            for k in (0, 1):
                self.q_of.append((handle, t, k))
                self.parts[(handle, t, k)] = []
                self.npk[(handle, t, k)] = 0
        if tcp:
            a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)
            if self.tcp_sndbuf:
                a.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, self.tcp_sndbuf)
                b.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, self.tcp_sndbuf)
            else:           # (clamped to net.core.wmem_max) a GOP replay should not block the egress
                a.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 32 << 20)
            a.setblocking(False)
            b.setblocking(False)
            self.eg.tcp(handle, a.fileno())
            self.tcp[handle] = [a, b, bytearray()]
        else:
            for t in range(ntracks):
                ports = []
                for k in (0, 1):
                    r = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
                    r.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 16 << 20)
                    r.bind(("127.0.0.1", 0))
                    r.setblocking(False)
                    self.udp[(handle, t, k)] = r
                    ports.append(r.getsockname()[1])
                self.eg.udp(handle, t, "127.0.0.1", ports[0], ports[1])
        if self.pacing is not None:
            self.eg.pacing(handle, play_time, video_tracks)

    def tick(self, result, t: int):
        if self.pacing is not None:
            self.eg.clock(t)
        # the receivers drain on their own threads while the egress sends (tools/udp_drain.c):
        # every UDP socket, and the TCP players this tick does not hold
        held = self.hold.get(t, set())
        keys = list(self.udp)
        tcp = [h for h in self.tcp if self.sub_id[h] not in held]
        lib = _drain()
        n_rx = len(keys) + len(tcp)
        fds = (C.c_int * max(1, n_rx))(*([self.udp[k].fileno() for k in keys] + [self.tcp[h][1].fileno() for h in tcp]))
        stream = (C.c_int * max(1, n_rx))(*([0] * len(keys) + [1] * len(tcp)))
        h = lib.udpd_start(fds, stream, n_rx) if n_rx else None
        try:
            st = self.eg.send(result)
        finally:
            if h:
                lib.udpd_stop(h)
                for i in range(n_rx):
                    n = lib.udpd_size(h, i)
                    if not n:
                        continue
                    b = C.create_string_buffer(n)
                    lib.udpd_take(h, i, b)
                    raw = b.raw
                    if i >= len(keys):
                        self.tcp[tcp[i - len(keys)]][2] += raw
                        continue
                    k, o = keys[i], 0
                    while o < n:                    # one part per datagram, as drain() keeps them
                        ln = (raw[o] << 8) | raw[o + 1]
                        self.parts[k].append(raw[o:o + 2 + ln])
                        o += 2 + ln
                    self.npk[k] += lib.udpd_count(h, i)
                lib.udpd_free(h)
        self.stats.append(st)
        for q, _sent, written, cause in self.eg.block_info():
            if cause != 0:                          # the write gate held it, not the socket
                continue
            h, trk, kind = self.q_of[q]
            self.blocked.append((t, self.sub_id[h], trk, kind, written))
        self.drain(skip={h for h, sid in self.sub_id.items() if sid in held})
        return st

    def drain(self, skip=()):
        for key, r in self.udp.items():
            while True:
                try:
                    d = r.recv(65536)
                except BlockingIOError:
                    break
                self.parts[key].append(struct.pack(">H", len(d)) + d)
                self.npk[key] += 1
        for h, (_a, b, buf) in self.tcp.items():
            if h in skip:
                continue
            while True:
                try:
                    d = b.recv(1 << 20)
                except BlockingIOError:
                    break
                if not d:
                    break
                buf += d

    def finish(self) -> dict:
        """Flushes buffered TCP tails, drains everything, and returns the wire images
        {(handle, track, kind): (packets, bytes)}."""
        for _ in range(10000):
            self.drain()
            if self.eg.flush() == 0:
                break
        self.drain()
        images = {k: (self.npk[k], b"".join(v)) for k, v in self.parts.items()}
        for h, (_a, _b, buf) in self.tcp.items():
            per = {}
            p = 0
            while p + 4 <= len(buf):
                assert buf[p] == 0x24, "TCP stream lost frame sync"
                ln = buf[p + 2] << 8 | buf[p + 3]
                per.setdefault(buf[p + 1], []).append(bytes(buf[p:p + 4 + ln]))
                p += 4 + ln
            assert p == len(buf), "partial frame at the end of a TCP stream"
            for ch, frames in per.items():
                images[(h, ch >> 1, ch & 1)] = (len(frames), b"".join(frames))
        return images

    def close(self):
        for r in self.udp.values():
            r.close()
        for a, b, _ in self.tcp.values():
            a.close()
            b.close()
        self.eg.close()
