"""Deterministic synthetic RTP push streams (BASELINE.md / SURVEY.md §8.d input specs).

Every stream is generated from a numpy PCG64 seeded with ``0xEA5D + config_index`` (then
per session).  Payload bytes are uniform random except the headers the reflector reads:
the RTP fixed header (RFC 3550) and the H.264 NAL / FU-A indicator and header bytes
(RFC 6184) that ``ReflectorSender::IsKeyFrameFirstPacket`` inspects
(ReflectorStream.cpp:1403-1513).

``session_packets`` returns one session's push as a time-ordered list of
``(t_ms, channel, bytes)`` tuples (channel = 2*track + is_rtcp, the RTSP-interleaved channel
``ProcessRTPData`` maps back to a track, QTSSReflectorModule.cpp:654-671).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

import numpy as np

SEED_BASE = 0xEA5D


@dataclass
class TrackSpec:
    media: str                     # "video" | "audio"
    payload: str                   # rtpmap payload name, e.g. "H264/90000"
    pt: int = 96
    bitrate: int = 2_000_000       # video bits/s
    fps: int = 30
    gop: int = 60                  # frames per GOP (2 s at 30 fps)
    idr_bytes: int = 40_000
    mtu: int = 1400                # max RTP packet size (12 RTP + 2 FU + 1386)
    jitter_sizes: bool = False     # C5: packet sizes uniform [20, 2059]
    rtcp_every_ms: int = 0         # emit an RTCP SR on the odd channel every N ms (0 = never)
    ssrc: int | None = None
    extra: dict = field(default_factory=dict)


def make_sdp(tracks: list[TrackSpec], name: str = "EasyPusher") -> str:
    lines = ["v=0", "o=- 0 0 IN IP4 127.0.0.1", f"s={name}", "c=IN IP4 127.0.0.1", "t=0 0"]
    for i, tr in enumerate(tracks):
        lines.append(f"m={tr.media} 0 RTP/AVP {tr.pt}")
        lines.append(f"a=rtpmap:{tr.pt} {tr.payload}")
        lines.append(f"a=control:trackID={i + 1}")
    return "\r\n".join(lines) + "\r\n"


def rtp_header(seq: int, ts: int, ssrc: int, pt: int, marker: bool, cc: int = 0) -> bytes:
    return struct.pack(">BBHII", 0x80 | (cc & 0x0F), (0x80 if marker else 0) | (pt & 0x7F),
                       seq & 0xFFFF, ts & 0xFFFFFFFF, ssrc & 0xFFFFFFFF)


def rtcp_sr(ssrc: int, ntp_ms: int, rtp_ts: int, pkts: int, octets: int) -> bytes:
    ntp_sec = 2208988800 + ntp_ms // 1000
    ntp_frac = ((ntp_ms % 1000) << 32) // 1000
    return struct.pack(">BBHIIIIII", 0x80, 200, 6, ssrc, ntp_sec & 0xFFFFFFFF, ntp_frac,
                       rtp_ts & 0xFFFFFFFF, pkts, octets)


class _RTP:
    def __init__(self, rng, tr: TrackSpec):
        self.rng = rng
        self.tr = tr
        self.seq = int(rng.integers(0, 1 << 16))
        if "seq0" in tr.extra:                  # pinned initial sequence number (wrap tests)
            self.seq = int(tr.extra["seq0"]) & 0xFFFF
        self.ts0 = int(rng.integers(0, 1 << 32))
        self.ssrc = tr.ssrc if tr.ssrc is not None else int(rng.integers(1, 1 << 32))
        self.sent = 0
        self.octets = 0

    def packet(self, ts: int, marker: bool, payload: bytes) -> bytes:
        p = rtp_header(self.seq, self.ts0 + ts, self.ssrc, self.tr.pt, marker) + payload
        self.seq = (self.seq + 1) & 0xFFFF
        self.sent += 1
        self.octets += len(payload)
        return p

    def rand(self, n: int) -> bytes:
        return self.rng.integers(0, 256, size=max(n, 0), dtype=np.uint8).tobytes()


def _h264_nal_packets(r: _RTP, nal_hdr: int, nal_len: int, ts: int, last_in_frame: bool):
    """Packetise one NAL unit of ``nal_len`` bytes (incl. its 1-byte header): single NAL unit
    packet if it fits, else FU-A fragments (RFC 6184 §5.8)."""
    mtu = r.tr.mtu
    if 12 + nal_len <= mtu:
        return [r.packet(ts, last_in_frame, bytes([nal_hdr]) + r.rand(nal_len - 1))]
    out = []
    body = nal_len - 1
    frag = mtu - 14
    ind = (nal_hdr & 0xE0) | 28
    typ = nal_hdr & 0x1F
    off = 0
    while off < body:
        n = min(frag, body - off)
        s = off == 0
        e = off + n >= body
        fu_hdr = (0x80 if s else 0) | (0x40 if e else 0) | typ
        out.append(r.packet(ts, last_in_frame and e, bytes([ind, fu_hdr]) + r.rand(n)))
        off += n
    return out


def _video_h264(rng, tr: TrackSpec, duration_ms: int, t0: int):
    r = _RTP(rng, tr)
    gop_bytes = tr.bitrate // 8 * tr.gop // tr.fps
    p_mean = max(200, (gop_bytes - tr.idr_bytes - 40) // max(tr.gop - 1, 1))
    out = []
    nframes = duration_ms * tr.fps // 1000
    for i in range(nframes):
        t = t0 + (i * 1000) // tr.fps
        ts = i * (90000 // tr.fps)
        pk = []
        if i % tr.gop == 0:
            pk += _h264_nal_packets(r, 0x67, 24, ts, False)        # SPS: 36-B packet
            pk += _h264_nal_packets(r, 0x68, 8, ts, False)         # PPS: 20-B packet (Q4 boundary)
            pk += _h264_nal_packets(r, 0x65, tr.idr_bytes, ts, True)
        else:
            sz = int(p_mean * rng.uniform(0.8, 1.2))
            pk += _h264_nal_packets(r, 0x41, sz, ts, True)
        out += [(t, p) for p in pk]
    return r, out


def _video_opaque(rng, tr: TrackSpec, duration_ms: int, t0: int):
    """MP4V-ES / JPEG video: the reflector never looks past the RTP header of these
    (keyframe indexing is gated on "H264/90000", ReflectorStream.cpp:1879)."""
    r = _RTP(rng, tr)
    frame_bytes = tr.bitrate // 8 // tr.fps
    out = []
    nframes = duration_ms * tr.fps // 1000
    for i in range(nframes):
        t = t0 + (i * 1000) // tr.fps
        ts = i * (90000 // tr.fps)
        left = int(frame_bytes * rng.uniform(0.7, 1.3))
        while left > 0:
            if tr.jitter_sizes:
                n = int(rng.integers(20, 2060)) - 12
            else:
                n = min(tr.mtu - 12, left)
            left -= n
            out.append((t, r.packet(ts, left <= 0, r.rand(n))))
    return r, out


def _audio(rng, tr: TrackSpec, duration_ms: int, t0: int):
    r = _RTP(rng, tr)
    name = tr.payload.upper()
    if name.startswith("MPEG4-GENERIC"):
        rate, spp, size = 48000, 1024, None
    else:                                   # PCMA / PCMU 8 kHz, 20 ms
        rate, spp, size = 8000, 160, 160
    out = []
    n = duration_ms * rate // (spp * 1000)
    for i in range(n):
        t = t0 + (i * spp * 1000) // rate
        if tr.jitter_sizes:
            sz = int(rng.integers(20, 2060)) - 12
        elif size is None:
            sz = int(rng.integers(200, 401))
        else:
            sz = size
        out.append((t, r.packet(i * spp, True, r.rand(sz))))
    return r, out


def session_packets(tracks: list[TrackSpec], duration_ms: int, seed: int, t0: int = 0):
    """All packets of one push session, merged in arrival order (stable by track)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    merged = []
    for ti, tr in enumerate(tracks):
        if tr.media == "video" and tr.payload == "H264/90000":
            r, pk = _video_h264(rng, tr, duration_ms, t0)
        elif tr.media == "video":
            r, pk = _video_opaque(rng, tr, duration_ms, t0)
        else:
            r, pk = _audio(rng, tr, duration_ms, t0)
        for k, (t, p) in enumerate(pk):
            merged.append((t, ti, 0, k, p))
        if tr.rtcp_every_ms:
            for k, t in enumerate(range(t0 + tr.rtcp_every_ms, t0 + duration_ms, tr.rtcp_every_ms)):
                merged.append((t, ti, 1, k, rtcp_sr(r.ssrc, t, t * 90, r.sent, r.octets)))
    merged.sort(key=lambda x: (x[0], x[1], x[2], x[3]))
    return [(t, 2 * ti + rt, p) for (t, ti, rt, _, p) in merged]
