"""Vectorised synthetic workload for the benchmark configs (BASELINE.json configs[1..2]).

C2: ``n_sessions`` pushed H.264/90000 1080p30 streams at 4 Mb/s, 2 s GOP (IDR ~120 KB,
SPS 36-B and PPS 20-B packets before it), FU-A at 1400-byte RTP packets, marker on each
frame's last packet, 90 kHz timestamps (+3000 per frame), random initial seq / ts / SSRC,
a random GOP phase and a random capture offset (0-33 ms: pushers are not frame-synchronous) per
session; ``subs_per_session`` UDP subscribers each.  Packets arrive at their frame time; one
batch = the packets that arrived in one tick interval (default 1 s; at 20-ms ticks about 60 % of
the sessions have a frame in each batch).

Only the RTP/FU headers are synthesised on the host; payload bytes are filled on the GPU
(they are never inspected by the relay, only moved).  Session ids are global so that a
multi-GPU run shards one workload: rank r owns the sessions whose FNV-1a-64 stream-ID hash
is r mod N; the benchmark's population (owned_sessions) gives every rank the
same number of them.
"""
from __future__ import annotations

import numpy as np

from .synth import SEED_BASE, TrackSpec, make_sdp

FPS = 30
GOP = 60
MTU = 1400
FRAG = MTU - 14           # FU-A payload bytes per fragment


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def stream_id(g: int) -> str:
    # ReflectorSession source id "<path>-<channel>" (QTSSReflectorModule.cpp:1384)
    return f"live/stream{g}.sdp-1"


def shard_sessions(n_global: int, rank: int, world: int) -> np.ndarray:
    return np.array([g for g in range(n_global) if fnv1a64(stream_id(g)) % world == rank], dtype=np.int64)


def owned_sessions(per_rank: int, rank: int, world: int) -> np.ndarray:
    """The first `per_rank` stream IDs (in ID order) whose FNV-1a hash owner is `rank`: a global
    population of world x per_rank streams in which every GPU owns exactly per_rank, so a weak-
    scaling run keeps the per-GPU work fixed while streams still shard by hash.  For world = 1
    this is range(per_rank)."""
    out, g = [], 0
    while len(out) < per_rank:
        if fnv1a64(stream_id(g)) % world == rank:
            out.append(g)
        g += 1
    return np.array(out, dtype=np.int64)


class H264Fleet:
    """State of a fleet of synthetic H.264 pushers (one video track each)."""

    def __init__(self, session_ids: np.ndarray, bitrate: int = 4_000_000, idr_bytes: int = 120_000,
                 tick_ms: int = 1000, config_index: int = 1):
        self.gids = np.asarray(session_ids, dtype=np.int64)
        n = len(self.gids)
        self.n = n
        rngs = [np.random.Generator(np.random.PCG64(SEED_BASE + config_index * 1_000_003 + int(g))) for g in self.gids]
        self.seq = np.array([r.integers(0, 1 << 16) for r in rngs], dtype=np.int64)
        self.ts0 = np.array([r.integers(0, 1 << 32) for r in rngs], dtype=np.int64)
        self.ssrc = np.array([r.integers(1, 1 << 32) for r in rngs], dtype=np.int64)
        self.phase = np.array([r.integers(0, GOP) for r in rngs], dtype=np.int64)
        self.offset = np.array([r.integers(0, 1000 // FPS + 1) for r in rngs], dtype=np.int64)   # ms
        self.fdone = np.zeros(n, dtype=np.int64)     # frames of each session batched so far
        self.rng = np.random.Generator(np.random.PCG64(SEED_BASE + config_index))
        self.idr_bytes = idr_bytes
        gop_bytes = bitrate // 8 * GOP // FPS
        self.p_mean = (gop_bytes - idr_bytes - 40) // (GOP - 1)
        self.tick_ms = tick_ms
        self.tracks = [TrackSpec("video", "H264/90000", 96, bitrate=bitrate, gop=GOP, idr_bytes=idr_bytes)]

    def sdp(self) -> str:
        return make_sdp(self.tracks)

    def next_batch(self):
        """Packets of the next tick for every session, grouped by session in arrival order.

        Returns dict with: ``desc`` (edgpu_pkt_desc records without slots), ``seg_off``,
        ``hdr`` (n x 16 bytes: the slot's first 16 bytes = 4-B reserved + 12-B RTP header),
        ``fu`` (n x 2: bytes 16-17 of the slot = FU indicator/header or NAL header + 1 byte),
        ``slot_bytes`` (n), ``t_end`` (tick time)."""
        # frame f of session s arrives at f * 1000 // FPS + offset[s]; this tick takes the frames
        # that arrived before its end (a tick shorter than a frame interval may carry none of a
        # session's)
        self.t_ms = getattr(self, "t_ms", 0) + self.tick_ms
        span = self.t_ms - self.offset
        due = np.where(span > 0, (span * FPS + 999) // 1000, 0)        # frames arrived before t_ms
        f0s = self.fdone
        nfs = due - f0s
        self.fdone = due
        n = self.n
        nf = int(nfs.max()) if n else 0                                # frame columns (ragged: masked)
        fidx = f0s[:, None] + np.arange(nf)[None, :]                   # (n, nf)
        valid = np.arange(nf)[None, :] < nfs[:, None]
        gop_pos = (fidx + self.phase[:, None]) % GOP
        is_idr = gop_pos == 0
        psize = (self.p_mean * self.rng.uniform(0.8, 1.2, size=(n, nf))).astype(np.int64)
        size = np.where(is_idr, self.idr_bytes, psize)                 # NAL bytes incl. header
        nfrag = (size - 1 + FRAG - 1) // FRAG                          # FU-A fragments
        npk = np.where(valid, nfrag + np.where(is_idr, 2, 0), 0)       # + SPS + PPS
        # per-packet expansion (session-major, frame order, packet order)
        tot = int(npk.sum())
        sess_of_frame = np.repeat(np.arange(n), nf)
        frame_of_pk = np.repeat(np.arange(n * nf), npk.ravel())
        sess = sess_of_frame[frame_of_pk]
        fl = frame_of_pk % nf
        first_pk_of_frame = np.concatenate([[0], np.cumsum(npk.ravel())[:-1]])
        k = np.arange(tot) - first_pk_of_frame[frame_of_pk]           # packet index within frame
        idr = is_idr.ravel()[frame_of_pk]
        nfr = nfrag.ravel()[frame_of_pk]
        sz = size.ravel()[frame_of_pk]
        fu_k = np.where(idr, k - 2, k)                                 # fragment index (-2,-1 = SPS,PPS)
        last = fu_k == nfr - 1
        body = np.where(last, (sz - 1) - (nfr - 1) * FRAG, FRAG)
        plen = np.where(fu_k == -2, 36, np.where(fu_k == -1, 20, 14 + body))
        # seq numbers continue per session
        pk_per_sess = npk.sum(axis=1)
        sess_first = np.concatenate([[0], np.cumsum(pk_per_sess)[:-1]])
        seq = (self.seq[sess] + (np.arange(tot) - sess_first[sess])) & 0xFFFF
        self.seq = (self.seq + pk_per_sess) & 0xFFFF
        fr = f0s[sess] + fl
        ts = (self.ts0[sess] + 3000 * fr) & 0xFFFFFFFF
        arrival = fr * 1000 // FPS + self.offset[sess]
        marker = last
        hdr = np.zeros((tot, 16), dtype=np.uint8)
        hdr[:, 4] = 0x80
        hdr[:, 5] = (0x80 * marker + 96).astype(np.uint8)
        hdr[:, 6] = seq >> 8
        hdr[:, 7] = seq & 0xFF
        for i in range(4):
            hdr[:, 8 + i] = (ts >> (24 - 8 * i)) & 0xFF
            hdr[:, 12 + i] = (self.ssrc[sess] >> (24 - 8 * i)) & 0xFF
        fu = np.zeros((tot, 2), dtype=np.uint8)
        nal_type = np.where(idr, 5, 1)
        nri = np.where(idr, 0x60, 0x40)
        fu[:, 0] = np.where(fu_k == -2, 0x67, np.where(fu_k == -1, 0x68, nri | 28))
        fu_hdr = (np.where(fu_k == 0, 0x80, 0) | np.where(last, 0x40, 0) | nal_type)
        fu[:, 1] = np.where(fu_k < 0, 0x42, fu_hdr)
        slot_bytes = ((plen + 4 + 15) // 16) * 16
        seg_off = np.concatenate([[0], np.cumsum(pk_per_sess)]).astype(np.uint32)
        return {
            "n": tot, "len": plen.astype(np.uint16), "channel": np.zeros(tot, np.uint8),
            "arrival": arrival.astype(np.int64), "hdr": hdr, "fu": fu,
            "slot_bytes": slot_bytes.astype(np.int64), "seg_off": seg_off,
            "t_end": int(self.t_ms),
        }
