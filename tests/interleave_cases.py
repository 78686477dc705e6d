"""Seeded RTSP-interleaved pusher connections (lists of TCP reads) for the '$'-deframe tests.

Each case is one pusher's connection as the server's socket reads see it: '$' ch BE16(len)
frames (RTSPSessionInterface.cpp:329-344 framing, as EasyPusher sends RTP/RTCP over RTSP),
split at arbitrary byte positions into reads.  The shapes cover what RTSPRequestStream::
ReadRequest distinguishes (RTSPRequestStream.cpp:65-171): frames split anywhere (header split,
1-byte reads, many frames per read), zero-length frames and reads, the largest frame the 2047-
byte request buffer holds, an RTSP request between frames, an oversized frame (connection
dropped), an oversized frame whose bytes have not all arrived, and payloads full of '$' bytes
(adversarial for a speculative parallel walk).
"""
from __future__ import annotations

import random
import struct

RTSP_REQ = (b"SET_PARAMETER rtsp://127.0.0.1/live/cam RTSP/1.0\r\nCSeq: 9\r\n"
            b"Session: 1234\r\nContent-Length: 0\r\n\r\n")


def _frame(ch, payload):
    return struct.pack(">BBH", 0x24, ch, len(payload)) + payload


def _split(rng, data, lo, hi, zero=0.0):
    reads, p = [], 0
    while p < len(data):
        if zero and rng.random() < zero:
            reads.append(b"")
        n = rng.randint(lo, hi)
        reads.append(data[p:p + n])
        p += n
    return reads


def _payload(rng, n, fill=None):
    if fill is not None:
        return bytes([fill]) * n
    return rng.randbytes(n)


def _frames(rng, count, lmin, lmax, channels=4, fill=None, dollar=0.0):
    out = []
    for _ in range(count):
        n = rng.randint(lmin, lmax)
        if dollar and rng.random() < dollar:
            pl = _payload(rng, n, 0x24)
        else:
            pl = _payload(rng, n, fill)
        out.append(_frame(rng.randrange(channels), pl))
    return out


def case(name: str) -> list[bytes]:
    rng = random.Random(f"deframe-{name}")
    if name == "rtp_mix":
        data = b"".join(_frames(rng, 400, 0, 1500))
        return _split(rng, data, 1, 4000, zero=0.02)
    if name == "tiny_reads":
        data = b"".join(_frames(rng, 60, 0, 300))
        return _split(rng, data, 1, 7)
    if name == "max_frame":
        data = b"".join(_frame(rng.randrange(4), _payload(rng, rng.choice([2043, 2042, 2040, 2043])))
                        for _ in range(40))
        return _split(rng, data, 1, 5000)
    if name == "rtsp_tail":
        data = b"".join(_frames(rng, 50, 12, 1400)) + RTSP_REQ + b"".join(_frames(rng, 10, 12, 1400))
        return _split(rng, data, 100, 3000)
    if name == "oversize":
        data = (b"".join(_frames(rng, 20, 12, 1400)) + _frame(1, _payload(rng, 2044))
                + b"".join(_frames(rng, 5, 12, 1400)))
        return _split(rng, data, 1, 2500)
    if name == "oversize_short":
        data = b"".join(_frames(rng, 20, 12, 1400)) + _frame(0, _payload(rng, 60000))[:1500]
        return _split(rng, data, 1, 2500)
    if name == "dollar_payload":
        data = b"".join(_frames(rng, 300, 0, 1500, dollar=0.5))
        return _split(rng, data, 1, 9000)
    if name == "big":
        data = b"".join(_frames(rng, 6000, 12, 1460, dollar=0.05))
        return _split(rng, data, 1, 65536)
    if name in ("fua_runs", "fua_oversize", "fua_partial"):
        # runs of equal-length FU-A frames (the walk's guessed headers all hold) broken by
        # shorter tails, audio frames, and -- where a guess would land -- an RTSP message, an
        # oversize frame or the end of the stream mid-frame
        out = []
        for run in range(10):
            out += [_frame(0, _payload(rng, 1400)) for _ in range(rng.randint(5, 40))]
            if name == "fua_runs" and run == 6:
                out.append(RTSP_REQ)
            if name == "fua_oversize" and run == 7:
                out.append(_frame(0, _payload(rng, 2044)))
            out.append(_frame(0, _payload(rng, rng.randint(12, 1399))))
            if rng.random() < 0.5:
                out.append(_frame(2, _payload(rng, rng.randint(200, 400))))
        data = b"".join(out)
        if name == "fua_partial":
            data += b"".join(_frame(0, _payload(rng, 1400)) for _ in range(9)) + _frame(0, _payload(rng, 1400))[:700]
        return _split(rng, data, 1, 20000)
    raise KeyError(name)


CASES = ["rtp_mix", "tiny_reads", "max_frame", "rtsp_tail", "oversize", "oversize_short",
         "dollar_payload", "big", "fua_runs", "fua_oversize", "fua_partial"]
