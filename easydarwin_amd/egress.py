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

import socket
import struct

from . import edgpu


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
        if tcp:
            a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)
            if self.tcp_sndbuf:
                a.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, self.tcp_sndbuf)
                b.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, self.tcp_sndbuf)
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
        st = self.eg.send(result)
        self.stats.append(st)
        for q, _sent, written, cause in self.eg.block_info():
            if cause != 0:                          # the write gate held it, not the socket
                continue
            h, trk, kind = self.q_of[q]
            self.blocked.append((t, self.sub_id[h], trk, kind, written))
        held = self.hold.get(t, set())
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
        images = {k: (len(v), b"".join(v)) for k, v in self.parts.items()}
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
