"""oracle/interleave.py -- TEST INFRASTRUCTURE ONLY (the checker, never the product).

Clean-room restatement of how EasyDarwin splits a pusher's RTSP connection into interleaved
packets (RTSP-interleaved TCP push, the EasyPusher default), pinned against the real
reference code by oracle/_ref/ref_deframe (Server.tproj/RTSPRequestStream.cpp compiled from
the reference) in tests/test_interleave.py:

* RTSPRequestStream::ReadRequest (RTSPRequestStream.cpp:65-171): the connection's bytes
  collect in a 2048-byte request buffer of which 2047 bytes are usable (QTSS_MAX_REQUEST_BUFFER_SIZE,
  QTSS.h:47; the read length at :122-123, the full-buffer check at :90-100).  When the buffer
  starts with '$' it waits for 4 header bytes, then for BE16(len) + 4 bytes, and returns that
  frame as a data packet (:156-171), keeping the rest for the next call ("retreat bytes").
  A frame longer than 2047 bytes can never complete: once the buffer is full ReadRequest asks
  the socket for 0 bytes (:123-124), recv returns 0 and Socket::Read reports ENOTCONN
  (Socket.cpp:383-388) -- the pusher's connection is dropped and the frame never delivered.
* Anything else at a frame boundary is an RTSP request (header parse, :172-260) -- handled
  by the RTSP session, outside this path.
* ProcessRTPData (QTSSReflectorModule.cpp:604-678): channel = byte 1, track = channel / 2,
  RTCP = channel & 1, packet = the frame after its 4-byte header.

``deframe(reads)`` returns the events ref_deframe writes: (kind, read, channel, a, bytes) with
kind FRAME (a = payload length, bytes = payload, read = the read that completed it),
MESSAGE (a = stream bytes consumed before it) or TOO_LONG (connection dropped; a = bytes
consumed before the frame, read = the read that filled the buffer).
"""
from __future__ import annotations

import struct

MAX_FRAME = 2047                 # usable request-buffer bytes (2048 - 1)
FRAME, MESSAGE, TOO_LONG = 1, 2, 3


def deframe(reads: list[bytes]) -> list[tuple]:
    buf = b""
    consumed = 0
    out = []
    for r, data in enumerate(reads):
        buf += data
        while buf:
            if buf[0] != 0x24:
                out.append((MESSAGE, r, 0, consumed, None))
                return out
            if len(buf) < 4:
                break
            flen = 4 + (buf[2] << 8 | buf[3])
            if flen > MAX_FRAME:
                if len(buf) >= MAX_FRAME:
                    out.append((TOO_LONG, r, 0, consumed, b""))
                    return out
                break
            if len(buf) < flen:
                break
            out.append((FRAME, r, buf[1], flen - 4, buf[4:flen]))
            consumed += flen
            buf = buf[flen:]
    return out


def frame(channel: int, packet: bytes) -> bytes:
    """'$' ch BE16(len) + packet (RTSPSessionInterface.cpp:329-344)."""
    return struct.pack(">BBH", 0x24, channel, len(packet)) + packet


def write_reads(path: str, reads: list[bytes]):
    with open(path, "wb") as f:
        f.write(b"EDRD" + struct.pack("<I", len(reads)))
        for r in reads:
            f.write(struct.pack("<I", len(r)) + r)


def read_events(path: str) -> list[tuple]:
    d = open(path, "rb").read()
    assert d[:4] == b"EDDF"
    (n,) = struct.unpack_from("<I", d, 4)
    p, out = 8, []
    for _ in range(n):
        kind, read, ch, a, blen = struct.unpack_from("<BIBII", d, p)
        p += 14
        data = d[p:p + blen]
        p += blen
        out.append((kind, read, ch, a, data if kind == FRAME else (b"" if kind == TOO_LONG else None)))
    return out


# ---- the engine boundary's per-read report (include/edgpu.h, edgpu_ingest_interleaved) ----
TCP_MESSAGE, TCP_DROPPED = 1, 2


def ingest_reads(carry: dict, rows, blob: bytes):
    """Restatement of edgpu_ingest_interleaved on the framing above.

    carry: session -> carried bytes (updated).  rows: (session, len, offset, arrival_ms) with a
    session's reads consecutive and contiguous.  Returns (results, frames): results[i] =
    [frames, consumed, status, carry] per read; frames = [(session, channel, arrival, packet)]
    in stream order (a frame's arrival is that of the read holding its last byte)."""
    import bisect
    results = [[0, 0, 0, 0] for _ in rows]
    frames = []
    i, n = 0, len(rows)
    while i < n:
        s = rows[i][0]
        j = i
        while j < n and rows[j][0] == s:
            j += 1
        stream = carry.get(s, b"")
        starts = []
        for k in range(i, j):
            starts.append(len(stream))
            stream += blob[rows[k][2]:rows[k][2] + rows[k][1]]
        L, pos, code = len(stream), 0, "end"
        while pos < L:
            if stream[pos] != 0x24:
                code = "message"
                break
            if pos + 4 > L:
                code = "partial"
                break
            flen = 4 + (stream[pos + 2] << 8 | stream[pos + 3])
            if flen > MAX_FRAME:
                code = "dropped" if L - pos >= MAX_FRAME else "partial"
                break
            if pos + flen > L:
                code = "partial"
                break
            r = bisect.bisect_right(starts, pos + flen - 1) - 1
            frames.append((s, stream[pos + 1], rows[i + r][3], stream[pos + 4:pos + flen]))
            results[i + r][0] += 1
            pos += flen
        carry[s] = stream[pos:] if code == "partial" else b""
        for k in range(i, j):
            st, ln = starts[k - i], rows[k][1]
            consumed, status = ln, 0
            if code in ("message", "dropped"):
                consumed = max(0, min(pos - st, ln))
                at = pos if code == "message" else pos + MAX_FRAME - 1
                if st + ln > at:
                    status = TCP_MESSAGE if code == "message" else TCP_DROPPED
            results[k][1:] = [consumed, status, len(carry[s])]
        i = j
    return results, frames
