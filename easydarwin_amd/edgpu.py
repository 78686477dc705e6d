"""ctypes binding of libedgpu.so (include/edgpu.h) -- the host-side mirror of the reflector's
module interface for this path.

There is no CPU fallback: if the HIP extension is missing or no gfx950 device is visible the
calls raise.  ``EdgpuError`` carries the QTSS_Error-compatible status code.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# EDGPU_LIB: a measurement build (make -C easydarwin_amd/csrc ab) instead of the shipped library
LIB_PATH = os.environ.get("EDGPU_LIB") or os.path.join(HERE, "libedgpu.so")

OK, ERR, BAD_ARGUMENT, WOULD_BLOCK = 0, -1, -10, -14
NO_DEVICE, OUT_OF_MEMORY, RING_OVERFLOW, OUT_OVERFLOW, TIMEOUT = -101, -102, -103, -104, -105
TRANSPORT_UDP, TRANSPORT_TCP = 0, 1
PTR_HOST, PTR_DEVICE, PTR_PINNED = 0, 1, 2
PLAY_RTP_INFO = 1
SESSION_KILL_OUTPUTS = 1          # edgpu_session_remove flags
FALSE = 0xFFFFFFFF

EXPORTED = [
    "edgpu_version", "edgpu_last_error", "edgpu_config_default", "edgpu_ctx_create",
    "edgpu_ctx_destroy", "edgpu_sync", "edgpu_session_add", "edgpu_session_tracks",
    "edgpu_subscriber_add", "edgpu_subscriber_remove", "edgpu_ingest", "edgpu_keyframe_index",
    "edgpu_fanout", "edgpu_tick_stats_get", "edgpu_copy_to_host", "edgpu_last_timings",
    "edgpu_gop_span", "edgpu_counters_get", "edgpu_kernel_times", "edgpu_gop_copy",
    "edgpu_session_export", "edgpu_session_import", "edgpu_session_relocations", "edgpu_session_key_update",
    "edgpu_stream_errors", "edgpu_fanout_packet_info", "edgpu_fanout_rows", "edgpu_fanout_active",
    "edgpu_memcpy_peer", "edgpu_device_alloc",
    "edgpu_device_free", "edgpu_fanout_kernel", "edgpu_subscriber_play",
    "edgpu_subscribers_add", "edgpu_ingest_interleaved", "edgpu_fanout_blocked",
    "edgpu_egress_create", "edgpu_egress_destroy", "edgpu_egress_last_error", "edgpu_egress_udp",
    "edgpu_egress_tcp", "edgpu_egress_send", "edgpu_egress_flush", "edgpu_egress_blocked",
    "edgpu_udp_sources", "edgpu_source_reports", "edgpu_source_identity", "edgpu_session_eyes_add",
    "edgpu_subscriber_rewrite", "edgpu_sdp_parse", "edgpu_host_alloc", "edgpu_host_free",
    "edgpu_arena_gather", "edgpu_egress_disconnected", "edgpu_fanout_arrivals", "edgpu_session_remove",
    "edgpu_set_timing", "edgpu_ingest_prestage", "edgpu_fanout_next", "edgpu_session_ssrc_prefs",
    "edgpu_subscriber_slot", "edgpu_egress_pacing_config", "edgpu_egress_pacing", "edgpu_egress_clock",
    "edgpu_egress_block_info", "edgpu_session_remote_join", "edgpu_session_remote_leave",
    "edgpu_subscriber_set_slot", "edgpu_device_local_cpus", "edgpu_debug_stall",
    "edgpu_ipc_export", "edgpu_ipc_open", "edgpu_ipc_close", "edgpu_copy_to_device",
]
IPC_HANDLE_BYTES = 64
TCP_MESSAGE, TCP_DROPPED = 1, 2
PKT_REMOTE_ODD = 1          # edgpu_pkt_desc.flags: a UDP datagram from an odd source port
IMAGE_FULL = 0xFFFFFFFFFFFFFFFF
NO_SOURCE = 0xFFFFFFFF


class Config(C.Structure):
    _fields_ = [
        ("device", C.c_int32),
        ("reflector_buffer_size_sec", C.c_uint32),
        ("rtp_reflector_threshold_msec", C.c_uint32),
        ("timeout_stream_SSRC_secs", C.c_uint32),
        ("use_one_SSRC_per_stream", C.c_uint32),
        ("video_ring_packets", C.c_uint32),
        ("video_ring_bytes", C.c_uint64),
        ("other_ring_packets", C.c_uint32),
        ("other_ring_bytes", C.c_uint64),
        ("out_arena_bytes", C.c_uint64),
        ("max_out_packets", C.c_uint32),
        ("max_batch_packets", C.c_uint32),
        ("max_batch_bytes", C.c_uint64),
        ("reflector_rtp_info_offset_msec", C.c_uint32),
        ("ring_growth", C.c_uint32),
        ("max_ring_packets", C.c_uint32),
        ("max_ring_bytes", C.c_uint64),
        ("reflector_use_in_packet_receive_time", C.c_uint32),
        ("reflector_in_packet_max_receive_sec", C.c_uint32),
        ("watchdog_ms", C.c_uint32),
        ("ingest_spec_min", C.c_uint32),
    ]


class RtpInfo(C.Structure):
    _fields_ = [("seq", C.c_uint16), ("_pad", C.c_uint16), ("rtptime", C.c_uint32)]


REWRITE_SSRC = 1


class Rewrite(C.Structure):
    _fields_ = [("seq_delta", C.c_uint16), ("flags", C.c_uint16), ("ts_delta", C.c_uint32), ("ssrc", C.c_uint32)]


class SdpTrack(C.Structure):
    _fields_ = [("payload_type", C.c_uint32), ("track_id", C.c_uint32), ("name_len", C.c_uint32),
                ("name", C.c_char * 244)]


class PktDesc(C.Structure):
    _fields_ = [("slot", C.c_uint32), ("len", C.c_uint16), ("channel", C.c_uint8),
                ("flags", C.c_uint8), ("arrival_ms", C.c_int64)]


class OutDesc(C.Structure):
    _fields_ = [("offset", C.c_uint64), ("len", C.c_uint32), ("packet_id", C.c_uint32)]


class SubstreamOut(C.Structure):
    _fields_ = [("subscriber", C.c_uint32), ("track", C.c_uint16), ("kind", C.c_uint8),
                ("transport", C.c_uint8), ("desc_base", C.c_uint32), ("desc_count", C.c_uint32),
                ("out_base", C.c_uint64), ("out_bytes", C.c_uint64), ("sender", C.c_uint32),
                ("flags", C.c_uint32)]


class FanoutResult(C.Structure):
    _fields_ = [("arena", C.c_void_p), ("desc", C.c_void_p), ("substreams", C.c_void_p),
                ("n_substreams", C.c_uint32)]


class TickStats(C.Structure):
    _fields_ = [("relayed_packets", C.c_uint64), ("relayed_bytes", C.c_uint64),
                ("arena_bytes", C.c_uint64), ("ingested_packets", C.c_uint64),
                ("ingested_bytes", C.c_uint64), ("status", C.c_int32), ("nwork", C.c_uint32),
                ("pass_arena_bytes", C.c_uint64), ("pass_packets", C.c_uint32), ("pass_", C.c_uint32),
                ("more_passes", C.c_uint32), ("stream_errors", C.c_uint32)]


class EgressStats(C.Structure):
    _fields_ = [("udp_datagrams", C.c_uint64), ("udp_bytes", C.c_uint64), ("udp_dropped", C.c_uint64),
                ("tcp_frames", C.c_uint64), ("tcp_bytes", C.c_uint64), ("blocked_substreams", C.c_uint32),
                ("_pad", C.c_uint32), ("copy_ms", C.c_double), ("send_ms", C.c_double),
                ("copied_bytes", C.c_uint64), ("stale_dropped", C.c_uint64)]


PACE_OVERBUFFER = 1


class Pacing(C.Structure):
    _fields_ = [("play_time_ms", C.c_int64), ("video_tracks", C.c_uint32), ("flags", C.c_uint32)]


class PacingConfig(C.Structure):
    _fields_ = [("bucket_delay_ms", C.c_int64), ("over_buffer_ms", C.c_int64), ("drop_all_packets_ms", C.c_int64),
                ("thin_all_the_way_ms", C.c_int64), ("start_thinning_ms", C.c_int64), ("bucket_size", C.c_uint32),
                ("send_interval_ms", C.c_uint32), ("max_send_ahead_s", C.c_uint32), ("overbuffer_rate", C.c_float)]


class Counters(C.Structure):
    _fields_ = [("relayed_packets", C.c_uint64), ("relayed_bytes", C.c_uint64),
                ("fanout_in_bytes", C.c_uint64), ("fanout_launches", C.c_uint64),
                ("ingested_packets", C.c_uint64), ("ingested_bytes", C.c_uint64),
                ("fanout_passes", C.c_uint64), ("lost_passes", C.c_uint64),
                ("senders", C.c_uint32), ("substream_rows", C.c_uint32),
                ("ring_grows", C.c_uint64), ("ring_bytes", C.c_uint64), ("ring_pool_bytes", C.c_uint64),
                ("ring_grow_failures", C.c_uint64), ("watchdog_timeouts", C.c_uint64),
                ("kernel_launches", C.c_uint64), ("host_syncs", C.c_uint64)]


# numpy mirrors (same layout as the C structs)
PKT_DTYPE = np.dtype([("slot", "<u4"), ("len", "<u2"), ("channel", "u1"), ("flags", "u1"),
                      ("arrival_ms", "<i8")])
OUT_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("packet_id", "<u4")])
SUB_DTYPE = np.dtype([("subscriber", "<u4"), ("track", "<u2"), ("kind", "u1"), ("transport", "u1"),
                      ("desc_base", "<u4"), ("desc_count", "<u4"), ("out_base", "<u8"),
                      ("out_bytes", "<u8"), ("sender", "<u4"), ("flags", "<u4")])
SUB_IDENTITY = 1
SUB_NEW = 2             # the output had no bookmark on this sender when the tick began
TCP_READ_DTYPE = np.dtype([("session", "<u4"), ("len", "<u4"), ("offset", "<u8"), ("arrival_ms", "<i8")])
TCP_RESULT_DTYPE = np.dtype([("frames", "<u4"), ("consumed", "<u4"), ("status", "<i4"), ("carry", "<u4")])
UDP_SOURCE_DTYPE = np.dtype([("session", "<u4"), ("channel", "u1"), ("_pad", "u1"), ("port", "<u2"),
                             ("addr", "<u4"), ("len", "<u4"), ("head", "u1", (4,))])
RR_MAX = 96
SOURCE_REPORT_DTYPE = np.dtype([("session", "<u4"), ("track", "<u2"), ("port", "<u2"), ("addr", "<u4"),
                                ("len", "<u4"), ("bytes", "u1", (RR_MAX,))])
assert UDP_SOURCE_DTYPE.itemsize == 20 and SOURCE_REPORT_DTYPE.itemsize == 112
assert TCP_READ_DTYPE.itemsize == 24 and TCP_RESULT_DTYPE.itemsize == 16
assert PKT_DTYPE.itemsize == C.sizeof(PktDesc) == 16
assert OUT_DTYPE.itemsize == C.sizeof(OutDesc) == 16
assert SUB_DTYPE.itemsize == C.sizeof(SubstreamOut) == 40


class EdgpuError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"edgpu error {code}: {msg}")
        self.code = code


_lib = None


def load(path: str = LIB_PATH):
    """Load libedgpu.so.  Raises (loudly) when the extension has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} missing: build it with `make -C easydarwin_amd/csrc` "
                                "(or __graft_entry__.build()); there is no CPU fallback")
    lib = C.CDLL(path)
    P, U32, U64, I32, I64 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int, C.c_int64
    sig = {
        "edgpu_version": (C.c_char_p, []),
        "edgpu_last_error": (C.c_char_p, []),
        "edgpu_config_default": (None, [C.POINTER(Config)]),
        "edgpu_ctx_create": (I32, [C.POINTER(Config), C.POINTER(P)]),
        "edgpu_ctx_destroy": (I32, [P]),
        "edgpu_sync": (I32, [P]),
        "edgpu_session_add": (I32, [P, C.c_char_p, U32, I32, C.POINTER(U32)]),
        "edgpu_session_tracks": (I32, [P, U32, C.POINTER(U32)]),
        "edgpu_session_ssrc_prefs": (I32, [P, U32, U32, U32]),
        "edgpu_session_remove": (I32, [P, U32, U32]),
        "edgpu_subscriber_add": (I32, [P, U32, I32, C.POINTER(U32)]),
        "edgpu_subscriber_remove": (I32, [P, U32]),
        "edgpu_ingest": (I32, [P, P, U32, P, P, U32, P, U64, I32]),
        "edgpu_keyframe_index": (I32, [P]),
        "edgpu_fanout": (I32, [P, I64, C.POINTER(FanoutResult)]),
        "edgpu_fanout_next": (I32, [P, C.POINTER(FanoutResult), C.POINTER(U32)]),
        "edgpu_tick_stats_get": (I32, [P, C.POINTER(TickStats)]),
        "edgpu_copy_to_host": (I32, [P, P, P, U64]),
        "edgpu_last_timings": (I32, [P, C.POINTER(C.c_float)]),
        "edgpu_gop_span": (I32, [P, U32, U32, C.POINTER(U64), C.POINTER(U64)]),
        "edgpu_counters_get": (I32, [P, C.POINTER(Counters)]),
        "edgpu_kernel_times": (I32, [P, I32, C.POINTER(C.c_float), U32, C.POINTER(U32)]),
        "edgpu_set_timing": (I32, [P, I32]),
        "edgpu_ingest_prestage": (I32, [P, P, C.c_uint64, C.c_uint64]),
        "edgpu_gop_copy": (I32, [P, U32, U32, P, U64, C.POINTER(U64), C.POINTER(U32)]),
        "edgpu_session_export": (I32, [P, P, U32, I64, P, P, U64, P, P]),
        "edgpu_session_import": (I32, [P, P, P, U32, P]),
        "edgpu_session_relocations": (I32, [P, P, U32, P]),
        "edgpu_session_key_update": (I32, [P, P, U32]),
        "edgpu_stream_errors": (I32, [P, P, P, U32, P]),
        "edgpu_fanout_packet_info": (I32, [P, P, P, U32, I32]),
        "edgpu_fanout_rows": (I32, [P, P, U32, P, U64, I32]),
        "edgpu_fanout_active": (I32, [P, P, P, U32, C.POINTER(U32), I32]),
        "edgpu_memcpy_peer": (I32, [P, P, I32, P, U64]),
        "edgpu_device_alloc": (I32, [P, U64, C.POINTER(P)]),
        "edgpu_device_free": (I32, [P, P]),
        "edgpu_ipc_export": (I32, [P, P, P]),
        "edgpu_ipc_open": (I32, [P, P, C.POINTER(P)]),
        "edgpu_ipc_close": (I32, [P, P]),
        "edgpu_copy_to_device": (I32, [P, P, P, U64]),
        "edgpu_fanout_kernel": (C.c_char_p, [P]),
        "edgpu_subscriber_play": (I32, [P, U32, I32, U32, I64, C.POINTER(U32), P]),
        "edgpu_subscribers_add": (I32, [P, U32, P, P, P]),
        "edgpu_ingest_interleaved": (I32, [P, P, U32, P, U64, I32, P]),
        "edgpu_fanout_blocked": (I32, [P, P, U32]),
        "edgpu_egress_create": (I32, [P, U32, C.POINTER(P)]),
        "edgpu_egress_destroy": (I32, [P]),
        "edgpu_egress_last_error": (C.c_char_p, [P]),
        "edgpu_egress_udp": (I32, [P, U32, U32, I32, I32, U32, C.c_uint16, C.c_uint16]),
        "edgpu_egress_tcp": (I32, [P, U32, I32]),
        "edgpu_egress_send": (I32, [P, C.POINTER(FanoutResult), C.POINTER(EgressStats)]),
        "edgpu_egress_flush": (I32, [P, C.POINTER(U64)]),
        "edgpu_egress_blocked": (I32, [P, P, U32, C.POINTER(U32)]),
        "edgpu_udp_sources": (I32, [P, P, U32]),
        "edgpu_source_reports": (I32, [P, P, U32, C.POINTER(U32)]),
        "edgpu_source_identity": (I32, [P, U32, U32, U32, I64]),
        "edgpu_session_eyes_add": (I32, [P, U32, C.c_int32]),
        "edgpu_subscriber_rewrite": (I32, [P, U32, U32, C.POINTER(Rewrite)]),
        "edgpu_sdp_parse": (I32, [C.c_char_p, U32, C.POINTER(SdpTrack), U32, C.POINTER(U32)]),
        "edgpu_host_alloc": (I32, [P, U64, C.POINTER(P)]),
        "edgpu_host_free": (I32, [P, P]),
        "edgpu_arena_gather": (I32, [P, C.POINTER(FanoutResult), P, U32, P, U64]),
        "edgpu_egress_disconnected": (I32, [P, P, U32, C.POINTER(U32)]),
        "edgpu_subscriber_slot": (I32, [P, U32, C.POINTER(C.c_int32)]),
        "edgpu_session_remote_join": (I32, [P, U32, C.POINTER(C.c_int32)]),
        "edgpu_session_remote_leave": (I32, [P, U32, C.c_int32]),
        "edgpu_subscriber_set_slot": (I32, [P, U32, C.c_int32]),
        "edgpu_device_local_cpus": (I32, [C.c_int, P, U32, P]),
        "edgpu_egress_pacing_config": (I32, [P, C.POINTER(PacingConfig)]),
        "edgpu_egress_pacing": (I32, [P, U32, C.POINTER(Pacing)]),
        "edgpu_egress_clock": (I32, [P, C.c_int64]),
        "edgpu_egress_block_info": (I32, [P, P, U32, C.POINTER(U32)]),
        "edgpu_fanout_arrivals": (I32, [P, P, U32, I32]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _check(rc: int):
    if rc != OK:
        raise EdgpuError(rc, _lib.edgpu_last_error().decode(errors="replace"))


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def sdp_parse(sdp: bytes) -> list:
    """The engine's SDP parse (edgpu_sdp_parse, host only): [(payload type, name bytes, trackID)]."""
    lib = load()
    n = C.c_uint32()
    cap = 64
    buf = (SdpTrack * cap)()
    _check(lib.edgpu_sdp_parse(sdp, len(sdp), buf, cap, C.byref(n)))
    return [(buf[i].payload_type, bytes(buf[i].name[:buf[i].name_len]), buf[i].track_id) for i in range(n.value)]


def device_local_cpus(device: int = 0) -> list:
    """The host CPUs of the GPU's NUMA node this process may run on (edgpu_device_local_cpus;
    initialises HIP)."""
    lib = load()
    cap = 4096
    buf = (C.c_uint32 * cap)()
    n = C.c_uint32()
    _check(lib.edgpu_device_local_cpus(device, buf, cap, C.byref(n)))
    return [int(buf[i]) for i in range(min(n.value, cap))]


class Context:
    """One engine context (one GPU).  Mirrors the module-side calls of the reflector."""

    def __init__(self, device: int = 0, **cfg):
        lib = load()
        c = Config()
        lib.edgpu_config_default(C.byref(c))
        c.device = device
        for k, v in cfg.items():
            setattr(c, k, v)
        h = C.c_void_p()
        _check(lib.edgpu_ctx_create(C.byref(c), C.byref(h)))
        self.h = h
        self.lib = lib
        self.device = int(device)
        self._ntracks = {}          # session -> tracks (senders_of without a C call per session)

    def close(self):
        if self.h:
            _check(self.lib.edgpu_ctx_destroy(self.h))
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def session_add(self, sdp: str, udp_push: bool = False) -> int:
        b = sdp.encode()
        out = C.c_uint32()
        _check(self.lib.edgpu_session_add(self.h, b, len(b), int(udp_push), C.byref(out)))
        self._ntracks[out.value] = self.session_tracks(out.value)
        return out.value

    def session_tracks(self, session: int) -> int:
        out = C.c_uint32()
        _check(self.lib.edgpu_session_tracks(self.h, session, C.byref(out)))
        return out.value

    def session_ssrc_prefs(self, session: int, use_one_ssrc: bool, timeout_s: int):
        """The session's SSRC filter prefs (edgpu_session_ssrc_prefs)."""
        _check(self.lib.edgpu_session_ssrc_prefs(self.h, session, 1 if use_one_ssrc else 0, int(timeout_s)))

    def session_remove(self, session: int, kill_outputs: bool = False):
        """The end of a ReflectorSession (reference count 0); kill_outputs tears its subscribers
        down with it (kill_clients_when_broadcast_stops)."""
        _check(self.lib.edgpu_session_remove(self.h, session, SESSION_KILL_OUTPUTS if kill_outputs else 0))
        self._ntracks.pop(session, None)

    def subscriber_add(self, session: int, transport: int = TRANSPORT_UDP) -> int:
        out = C.c_uint32()
        _check(self.lib.edgpu_subscriber_add(self.h, session, transport, C.byref(out)))
        return out.value

    def subscriber_play(self, session: int, transport: int = TRANSPORT_UDP, rtp_info: bool = False,
                        now_ms: int = 0):
        """PLAY of a player; rtp_info=True for an RTP-Info player (UA vlc / Android).  Returns
        (handle, [(first seq, first rtptime)] per track).  Raises EdgpuError with code
        WOULD_BLOCK when an RTP-Info PLAY finds a track with nothing buffered."""
        n = self.session_tracks(session)
        info = (RtpInfo * max(n, 1))()
        out = C.c_uint32()
        _check(self.lib.edgpu_subscriber_play(self.h, session, transport, PLAY_RTP_INFO if rtp_info else 0,
                                              int(now_ms), C.byref(out), info))
        return out.value, [(info[i].seq, info[i].rtptime) for i in range(n)]

    def subscribers_add(self, sessions, transports) -> np.ndarray:
        """Burst join: one subscriber per (session, transport); returns their handles."""
        ses = np.ascontiguousarray(sessions, dtype=np.uint32)
        trn = np.ascontiguousarray(np.broadcast_to(transports, ses.shape), dtype=np.int32)
        out = np.zeros(len(ses), dtype=np.uint32)
        _check(self.lib.edgpu_subscribers_add(self.h, len(ses), _ptr(ses), _ptr(trn), _ptr(out)))
        return out

    def subscriber_rewrite(self, handle: int, track: int, seq_delta: int = 0, ts_delta: int = 0,
                           ssrc: int | None = None):
        """Per-output rewrite of one subscriber track (identity: all defaults)."""
        rw = Rewrite(seq_delta & 0xFFFF, REWRITE_SSRC if ssrc is not None else 0, ts_delta & 0xFFFFFFFF,
                     (ssrc or 0) & 0xFFFFFFFF)
        _check(self.lib.edgpu_subscriber_rewrite(self.h, handle, track, C.byref(rw)))

    def subscriber_remove(self, handle: int):
        _check(self.lib.edgpu_subscriber_remove(self.h, handle))

    def subscriber_slot(self, handle: int) -> int:
        """Its place in the session's bucket arrays (ReflectorStream::AddOutput / FindBucket)."""
        v = C.c_int32()
        _check(self.lib.edgpu_subscriber_slot(self.h, handle, C.byref(v)))
        return v.value

    def subscriber_set_slot(self, handle: int, slot: int):
        """Moves the subscriber to bucket place `slot` (the place its owner gave a replica's output)."""
        _check(self.lib.edgpu_subscriber_set_slot(self.h, handle, int(slot)))

    def ingest_host(self, desc: np.ndarray, seg_off: np.ndarray, seg_sess: np.ndarray, blob: np.ndarray):
        desc = np.ascontiguousarray(desc, dtype=PKT_DTYPE)
        seg_off = np.ascontiguousarray(seg_off, dtype=np.uint32)
        seg_sess = np.ascontiguousarray(seg_sess, dtype=np.uint32)
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        _check(self.lib.edgpu_ingest(self.h, _ptr(desc), len(desc), _ptr(seg_off), _ptr(seg_sess),
                                     len(seg_sess), _ptr(blob), blob.nbytes, PTR_HOST))

    def ingest_device(self, desc_ptr: int, n: int, seg_ptr: int, seg_sess_ptr: int, nseg: int,
                      blob_ptr: int, blob_bytes: int):
        _check(self.lib.edgpu_ingest(self.h, C.c_void_p(desc_ptr), n, C.c_void_p(seg_ptr),
                                     C.c_void_p(seg_sess_ptr), nseg, C.c_void_p(blob_ptr),
                                     blob_bytes, PTR_DEVICE))

    def ingest_pinned(self, desc_ptr: int, n: int, seg_ptr: int, seg_sess_ptr: int, nseg: int,
                      blob_ptr: int, blob_bytes: int):
        """A batch in pinned host memory (edgpu_host_alloc): copied on the copy stream, asynchronous."""
        _check(self.lib.edgpu_ingest(self.h, C.c_void_p(desc_ptr), n, C.c_void_p(seg_ptr),
                                     C.c_void_p(seg_sess_ptr), nseg, C.c_void_p(blob_ptr),
                                     blob_bytes, PTR_PINNED))

    def host_alloc(self, nbytes: int) -> "HostBuffer":
        return HostBuffer(self, nbytes)

    def ingest_interleaved(self, reads: np.ndarray, data, device_ptr: int | None = None) -> np.ndarray:
        """RTSP-interleaved push ingest: `reads` (TCP_READ_DTYPE: session, len, offset,
        arrival_ms; a session's reads consecutive and contiguous in the bytes) over `data`
        (host bytes / uint8 array), or over device memory at `device_ptr` (then `data` is its
        byte count).  Returns the per-read results (TCP_RESULT_DTYPE)."""
        reads = np.ascontiguousarray(reads, dtype=TCP_READ_DTYPE)
        out = np.zeros(len(reads), dtype=TCP_RESULT_DTYPE)
        if device_ptr is None:
            buf = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else \
                np.ascontiguousarray(data, dtype=np.uint8)
            _check(self.lib.edgpu_ingest_interleaved(self.h, _ptr(reads), len(reads), _ptr(buf), buf.nbytes,
                                                     PTR_HOST, _ptr(out)))
        else:
            _check(self.lib.edgpu_ingest_interleaved(self.h, _ptr(reads), len(reads), C.c_void_p(device_ptr),
                                                     int(data), PTR_DEVICE, _ptr(out)))
        return out

    def fanout_blocked(self, reports):
        """Egress backpressure for the last tick: [(substream index, packets sent)]."""
        a = np.ascontiguousarray(np.array(list(reports), dtype=np.uint32).reshape(-1, 2))
        if len(a):
            _check(self.lib.edgpu_fanout_blocked(self.h, _ptr(a), len(a)))

    def keyframe_index(self):
        _check(self.lib.edgpu_keyframe_index(self.h))

    def udp_sources(self, rows):
        """Source addresses of UDP-pushed datagrams, in arrival order:
        [(session, channel, addr, port, datagram bytes)] (only len and the first 4 bytes
        travel)."""
        a = np.zeros(len(rows), dtype=UDP_SOURCE_DTYPE)
        for i, (s, ch, addr, port, data) in enumerate(rows):
            h = bytes(data[:4]).ljust(4, b"\0")
            a[i] = (s, ch, 0, port, addr, len(data), np.frombuffer(h, dtype=np.uint8))
        if len(a):
            _check(self.lib.edgpu_udp_sources(self.h, _ptr(a), len(a)))

    def source_reports(self) -> list:
        """Receiver reports queued by the last fanout: [(session, track, addr, port, bytes)]."""
        n = C.c_uint32(0)
        cap = 64
        while True:
            buf = np.zeros(cap, dtype=SOURCE_REPORT_DTYPE)
            rc = self.lib.edgpu_source_reports(self.h, _ptr(buf), cap, C.byref(n))
            if rc == 0:
                break
            if n.value <= cap:
                _check(rc)
            cap = n.value
        return [(int(r["session"]), int(r["track"]), int(r["addr"]), int(r["port"]),
                 bytes(r["bytes"][:int(r["len"])])) for r in buf[:n.value]]

    def source_identity(self, session: int, track: int, ssrc: int, cname_secs: int):
        _check(self.lib.edgpu_source_identity(self.h, session, track, ssrc, int(cname_secs)))

    def session_eyes_add(self, session: int, delta: int):
        """Subscribers of an owned session joined (+) or left (-) on another context."""
        _check(self.lib.edgpu_session_eyes_add(self.h, session, int(delta)))

    def session_remote_join(self, session: int) -> int:
        """A subscriber of this owned session joined on another context: its eye and its place in
        the session's bucket arrays (returned)."""
        v = C.c_int32()
        _check(self.lib.edgpu_session_remote_join(self.h, session, C.byref(v)))
        return v.value

    def session_remote_leave(self, session: int, place: int):
        _check(self.lib.edgpu_session_remote_leave(self.h, session, int(place)))

    def fanout(self, now_ms: int) -> FanoutResult:
        r = FanoutResult()
        _check(self.lib.edgpu_fanout(self.h, int(now_ms), C.byref(r)))
        return r

    def fanout_next(self):
        """The next copy pass of an over-capacity tick (edgpu_fanout_next): its result, or None
        when the tick is complete."""
        r = FanoutResult()
        launched = C.c_uint32()
        _check(self.lib.edgpu_fanout_next(self.h, C.byref(r), C.byref(launched)))
        return r if launched.value else None

    def stats(self) -> TickStats:
        s = TickStats()
        _check(self.lib.edgpu_tick_stats_get(self.h, C.byref(s)))
        return s

    def sync(self):
        _check(self.lib.edgpu_sync(self.h))

    def debug_stall(self, us: int):
        """edgpu_debug_stall: one wave on the context stream waits `us` microseconds of the device
        clock -- work the GPU watchdog (watchdog_ms) can time out on."""
        _check(self.lib.edgpu_debug_stall(self.h, C.c_uint32(us)))

    def timings(self):
        a = (C.c_float * 4)()
        _check(self.lib.edgpu_last_timings(self.h, a))
        return {"fanout_ms": a[0], "tick_ms": a[1], "ingest_ms": a[2], "keyframe_ms": a[3]}

    def fanout_kernel(self) -> str:
        """Name of the fan-out copy kernel this context launches."""
        return self.lib.edgpu_fanout_kernel(self.h).decode()

    def counters(self) -> dict:
        c = Counters()
        _check(self.lib.edgpu_counters_get(self.h, C.byref(c)))
        return {k: getattr(c, k) for k, _ in Counters._fields_}

    TIMING_NONE, TIMING_FANOUT, TIMING_ALL = 0, 1, 2

    def set_timing(self, level: int):
        """Which per-launch timing events are recorded (edgpu_set_timing): TIMING_ALL (default),
        TIMING_FANOUT (the fan-out copy kernel's pair only) or TIMING_NONE."""
        _check(self.lib.edgpu_set_timing(self.h, level))

    def kernel_times(self, which: int) -> list:
        """which: 0 fan-out kernel, 1 whole fan-out tick, 2 ingest, 3 keyframe index."""
        buf = (C.c_float * 256)()
        n = C.c_uint32()
        _check(self.lib.edgpu_kernel_times(self.h, which, buf, 256, C.byref(n)))
        return [buf[i] for i in range(n.value)]

    def gop_span(self, session: int, track: int):
        p, b = C.c_uint64(), C.c_uint64()
        _check(self.lib.edgpu_gop_span(self.h, session, track, C.byref(p), C.byref(b)))
        return p.value, b.value

    def gop_copy(self, session: int, track: int, cap: int = 8 << 20) -> tuple:
        """CKeyFrameCache TLV image of the track's GOP (key pointer -> newest)."""
        buf = np.empty(cap, dtype=np.uint8)
        n, k = C.c_uint64(), C.c_uint32()
        _check(self.lib.edgpu_gop_copy(self.h, session, track, _ptr(buf), cap, C.byref(n), C.byref(k)))
        return buf[:n.value].tobytes(), k.value

    # ---- cross-GPU keyframe fast start (session images) ----
    def senders_of(self, sessions) -> int:
        nt = self._ntracks
        return int(sum(2 * (nt[s] if s in nt else self.session_tracks(s)) for s in map(int, sessions)))

    def session_export(self, sessions, now_ms: int, dst_ptr: int = 0, cap: int = 0, since=None):
        """Export session images.  dst_ptr 0 = size query.  `since`: None (full images) or,
        per sender of each session in order, IMAGE_FULL or a previous call's head.
        Returns (offsets[n+1], heads[n_senders])."""
        sess = np.ascontiguousarray(sessions, dtype=np.uint32)
        offsets = np.zeros(len(sess) + 1, dtype=np.uint64)
        heads = np.zeros(self.senders_of(sess), dtype=np.uint64)
        frm = None if since is None else np.ascontiguousarray(since, dtype=np.uint64)
        if frm is not None and len(frm) != len(heads):
            raise ValueError("`since` needs one entry per sender")
        _check(self.lib.edgpu_session_export(self.h, _ptr(sess), len(sess), int(now_ms),
                                             None if frm is None else _ptr(frm),
                                             C.c_void_p(dst_ptr) if dst_ptr else None, int(cap),
                                             _ptr(offsets), _ptr(heads)))
        return offsets, heads

    def session_import(self, images_ptr: int, offsets, sessions):
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        sess = np.ascontiguousarray(sessions, dtype=np.uint32)
        if len(offsets) != len(sess) + 1:
            raise ValueError("offsets must have len(sessions) + 1 entries")
        _check(self.lib.edgpu_session_import(self.h, C.c_void_p(images_ptr), _ptr(offsets), len(sess), _ptr(sess)))

    def session_relocations(self, sessions) -> list:
        """Sessions (of `sessions`, on this context) whose outputs a backpressure report relocated
        since the last call (a replica's feedback for its owner); the indication is cleared."""
        sess = np.ascontiguousarray(sessions, dtype=np.uint32)
        out = np.zeros(max(len(sess), 1), dtype=np.uint8)
        _check(self.lib.edgpu_session_relocations(self.h, _ptr(sess), len(sess), _ptr(out)))
        return [int(x) for x, f in zip(sess, out) if f]

    def stream_errors(self) -> list:
        """[(session, code)] the ticks marked since the last call (edgpu_stream_errors); clears them."""
        n = C.c_uint32()
        _check(self.lib.edgpu_stream_errors(self.h, None, None, 0, C.byref(n)))      # how many
        cap = max(n.value, 1)
        ss = np.zeros(cap, dtype=np.uint32)
        cs = np.zeros(cap, dtype=np.int32)
        _check(self.lib.edgpu_stream_errors(self.h, _ptr(ss), _ptr(cs), cap, C.byref(n)))
        return [(int(a), int(b)) for a, b in zip(ss[:min(n.value, cap)], cs[:min(n.value, cap)])]

    def session_key_update(self, sessions):
        """The owner's side: ReflectorSession::SetHasVideoKeyFrameUpdate(true) on `sessions`."""
        sess = np.ascontiguousarray(sessions, dtype=np.uint32)
        _check(self.lib.edgpu_session_key_update(self.h, _ptr(sess), len(sess)))

    def memcpy_peer(self, dst_ptr: int, src_device: int, src_ptr: int, nbytes: int):
        _check(self.lib.edgpu_memcpy_peer(self.h, C.c_void_p(dst_ptr), int(src_device), C.c_void_p(src_ptr), int(nbytes)))

    def device_alloc(self, nbytes: int) -> "DeviceBuffer":
        return DeviceBuffer(self, nbytes)

    def ipc_export(self, dev_ptr: int) -> bytes:
        """The inter-process handle of a buffer from device_alloc (edgpu_ipc_export)."""
        h = (C.c_uint8 * IPC_HANDLE_BYTES)()
        _check(self.lib.edgpu_ipc_export(self.h, C.c_void_p(dev_ptr), h))
        return bytes(h)

    def ipc_open(self, handle: bytes) -> int:
        """Maps another process's buffer (edgpu_ipc_open); returns the pointer this GPU uses."""
        h = (C.c_uint8 * IPC_HANDLE_BYTES).from_buffer_copy(handle)
        out = C.c_void_p()
        _check(self.lib.edgpu_ipc_open(self.h, h, C.byref(out)))
        return int(out.value)

    def ipc_close(self, ptr: int):
        _check(self.lib.edgpu_ipc_close(self.h, C.c_void_p(ptr)))

    def copy_to_device(self, dev_ptr: int, data):
        a = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else data)
        if a.nbytes:
            _check(self.lib.edgpu_copy_to_device(self.h, C.c_void_p(dev_ptr), _ptr(a), int(a.nbytes)))

    def copy_to_host(self, dev_ptr, nbytes: int) -> np.ndarray:
        out = np.empty(int(nbytes), dtype=np.uint8)
        if nbytes:
            _check(self.lib.edgpu_copy_to_host(self.h, _ptr(out), C.c_void_p(dev_ptr), int(nbytes)))
        return out

    def fanout_arrivals(self, n: int) -> np.ndarray:
        """Arrival time (ms) of each of the last tick's `n` descriptors (edgpu_fanout_arrivals)."""
        out = np.zeros(max(int(n), 1), dtype=np.int64)
        _check(self.lib.edgpu_fanout_arrivals(self.h, _ptr(out), out.size, PTR_HOST))
        return out[:n]

    def fanout_sources(self, n: int) -> np.ndarray:
        """Per descriptor of the current pass: its packet's blob slot in the last host batch, or
        NO_SOURCE (edgpu_fanout_packet_info)."""
        out = np.zeros(max(int(n), 1), dtype=np.uint32)
        _check(self.lib.edgpu_fanout_packet_info(self.h, None, _ptr(out), out.size, PTR_HOST))
        return out[:n]

    ROW_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("packet_id", "<u4"), ("arrival", "<i8"),
                          ("source", "<u4"), ("_pad", "<u4")])

    def fanout_rows(self, sel) -> np.ndarray:
        """edgpu_fanout_rows: `sel` = [(substream row, first output row), ...]; returns the rows
        (offset, len, packet_id, arrival, source) of those sub-streams' descriptors."""
        sel = np.ascontiguousarray(np.asarray(sel, dtype=np.uint32).reshape(-1, 2))
        nrows = int(sel[:, 1].max()) + 1 if sel.size else 0
        return self._rows(sel, nrows)

    def fanout_rows_n(self, sel, nrows: int) -> np.ndarray:
        sel = np.ascontiguousarray(np.asarray(sel, dtype=np.uint32).reshape(-1, 2))
        return self._rows(sel, int(nrows))

    def _rows(self, sel, nrows):
        out = np.zeros(max(nrows, 1), dtype=self.ROW_DTYPE)
        _check(self.lib.edgpu_fanout_rows(self.h, _ptr(sel), len(sel), _ptr(out), nrows, PTR_HOST))
        return out[:nrows]

    def fanout_active(self, cap: int):
        """The current pass's sub-streams with descriptors, compacted in table order
        (edgpu_fanout_active): (rows as SUB_DTYPE, their table indices, total count)."""
        rows = np.zeros(max(int(cap), 1), dtype=SUB_DTYPE)
        q = np.zeros(max(int(cap), 1), dtype=np.uint32)
        n = C.c_uint32()
        _check(self.lib.edgpu_fanout_active(self.h, _ptr(rows), _ptr(q), int(cap), C.byref(n), PTR_HOST))
        k = min(n.value, int(cap))
        return rows[:k], q[:k], n.value

    def read_tick(self, r: FanoutResult):
        """(stats, substream table, descriptors, arena) of the current copy pass of the last
        fan-out (the whole tick unless it exceeded the arena: st.more_passes, fanout_next), on
        the host."""
        st = self.stats()
        if st.status != OK:
            raise EdgpuError(st.status, "device-side status after fan-out")
        subs = self.copy_to_host(r.substreams, r.n_substreams * SUB_DTYPE.itemsize).view(SUB_DTYPE)
        desc = self.copy_to_host(r.desc, st.pass_packets * OUT_DTYPE.itemsize).view(OUT_DTYPE)
        arena = self.copy_to_host(r.arena, st.pass_arena_bytes)
        return st, subs, desc, arena

    def read_passes(self, r: FanoutResult, consume):
        """Reads every copy pass of the tick whose first pass is `r`: consume(stats, subs, desc,
        arena) per pass, in sub-stream row order.  Returns the number of passes."""
        n = 0
        while r is not None:
            consume(*self.read_tick(r))
            n += 1
            r = self.fanout_next()
        return n


class Egress:
    """Socket egress of fan-out ticks (edgpu_egress_*): UDP via sendmmsg, RTSP-interleaved TCP
    via writev with the reference's all-or-nothing buffering; TCP backpressure is reported to
    the engine automatically."""

    def __init__(self, ctx: Context, threads: int = 1):
        self.ctx, self.lib = ctx, ctx.lib
        h = C.c_void_p()
        _check(self.lib.edgpu_egress_create(ctx.h, threads, C.byref(h)))
        self.h = h

    def _chk(self, rc):
        if rc != OK:
            raise EdgpuError(rc, self.lib.edgpu_egress_last_error(self.h).decode(errors="replace"))

    def udp(self, subscriber: int, track: int, ip: str, rtp_port: int, rtcp_port: int,
            rtp_fd: int = -1, rtcp_fd: int = -1):
        import socket
        ip_be = int.from_bytes(socket.inet_aton(ip), "little")
        self._chk(self.lib.edgpu_egress_udp(self.h, subscriber, track, rtp_fd, rtcp_fd, ip_be,
                                            socket.htons(rtp_port), socket.htons(rtcp_port)))

    def tcp(self, subscriber: int, fd: int):
        self._chk(self.lib.edgpu_egress_tcp(self.h, subscriber, fd))

    def send(self, r: FanoutResult) -> EgressStats:
        s = EgressStats()
        self._chk(self.lib.edgpu_egress_send(self.h, C.byref(r), C.byref(s)))
        return s

    def blocked(self):
        """The (sub-stream, sent) reports of the last send."""
        cap = 1 << 16
        buf = np.zeros((cap, 2), dtype=np.uint32)
        n = C.c_uint32()
        self._chk(self.lib.edgpu_egress_blocked(self.h, _ptr(buf), cap, C.byref(n)))
        return [tuple(map(int, x)) for x in buf[:min(n.value, cap)]]

    def pacing_config(self, bucket_delay_ms=73, over_buffer_ms=1000, drop_all_packets_ms=2500,
                      thin_all_the_way_ms=1500, start_thinning_ms=0, bucket_size=16, send_interval_ms=50,
                      max_send_ahead_s=25, overbuffer_rate=2.0):
        c = PacingConfig(bucket_delay_ms, over_buffer_ms, drop_all_packets_ms, thin_all_the_way_ms,
                         start_thinning_ms, bucket_size, send_interval_ms, max_send_ahead_s, overbuffer_rate)
        self._chk(self.lib.edgpu_egress_pacing_config(self.h, C.byref(c)))

    def pacing(self, subscriber: int, play_time_ms: int | None, video_tracks: int = 0, flags: int = 0):
        """The server's write gate for this subscriber (None: off): edgpu_egress_pacing."""
        if play_time_ms is None:
            self._chk(self.lib.edgpu_egress_pacing(self.h, subscriber, None))
        else:
            p = Pacing(play_time_ms, video_tracks, flags)
            self._chk(self.lib.edgpu_egress_pacing(self.h, subscriber, C.byref(p)))

    def clock(self, now_ms: int):
        self._chk(self.lib.edgpu_egress_clock(self.h, int(now_ms)))

    def block_info(self):
        """(sub-stream, sent, written, cause) of the last send's stopped sub-streams; cause 0 = the
        socket, 1 = the write gate."""
        cap = 1 << 16
        buf = np.zeros((cap, 4), dtype=np.uint32)
        n = C.c_uint32()
        self._chk(self.lib.edgpu_egress_block_info(self.h, _ptr(buf), cap, C.byref(n)))
        return [tuple(map(int, x)) for x in buf[:min(n.value, cap)]]

    def disconnected(self) -> list:
        """Subscribers whose RTSP connection failed (not EAGAIN) since the last call."""
        buf = np.zeros(4096, dtype=np.uint32)
        n = C.c_uint32()
        self._chk(self.lib.edgpu_egress_disconnected(self.h, _ptr(buf), len(buf), C.byref(n)))
        return [int(x) for x in buf[:min(n.value, len(buf))]]

    def flush(self) -> int:
        left = C.c_uint64()
        self._chk(self.lib.edgpu_egress_flush(self.h, C.byref(left)))
        return left.value

    def close(self):
        if self.h:
            self.lib.edgpu_egress_destroy(self.h)
            self.h = None


class HostBuffer:
    """Pinned host memory owned by a context (edgpu_host_alloc); `.array` is a uint8 view."""

    def __init__(self, ctx: Context, nbytes: int):
        out = C.c_void_p()
        _check(ctx.lib.edgpu_host_alloc(ctx.h, int(nbytes), C.byref(out)))
        self.ctx, self.ptr, self.nbytes = ctx, int(out.value), int(nbytes)
        self.array = np.ctypeslib.as_array((C.c_uint8 * max(self.nbytes, 1)).from_address(self.ptr))[:self.nbytes]

    def free(self):
        if self.ptr and self.ctx.h:
            self.array = None
            _check(self.ctx.lib.edgpu_host_free(self.ctx.h, C.c_void_p(self.ptr)))
        self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DeviceBuffer:
    """Device memory owned by a context (edgpu_device_alloc); freed with the object."""

    def __init__(self, ctx: Context, nbytes: int):
        out = C.c_void_p()
        _check(ctx.lib.edgpu_device_alloc(ctx.h, int(nbytes), C.byref(out)))
        self.ctx, self.ptr, self.nbytes = ctx, int(out.value), int(nbytes)

    def free(self):
        if self.ptr and self.ctx.h:
            _check(self.ctx.lib.edgpu_device_free(self.ctx.h, C.c_void_p(self.ptr)))
        self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def build_batch(pkts):
    """Host-side batch builder: ``pkts`` is a list of (session, channel, arrival_ms, bytes) or
    (session, channel, arrival_ms, bytes, flags) in arrival order (flags: PKT_REMOTE_ODD).  Groups them by session (stable) into the edgpu_ingest layout: 16-B
    slots with the packet 4 bytes in, a descriptor per packet, per-session segments."""
    order = sorted(range(len(pkts)), key=lambda i: (pkts[i][0], i))
    n = len(pkts)
    desc = np.zeros(n, dtype=PKT_DTYPE)
    sizes = [((min(len(pkts[i][3]), 65535) + 4 + 15) // 16) * 16 for i in order]
    total = int(sum(sizes))
    blob = np.zeros(max(total, 16), dtype=np.uint8)
    seg_off, seg_sess = [0], []
    off = 0
    last = None
    for k, i in enumerate(order):
        s, ch, t, data = pkts[i][:4]
        fl = pkts[i][4] if len(pkts[i]) > 4 else 0
        data = data[:65535]
        if s != last:
            if last is not None:
                seg_off.append(k)
            seg_sess.append(s)
            last = s
        desc[k] = (off // 16, len(data), ch, fl, t)
        blob[off + 4:off + 4 + len(data)] = np.frombuffer(data, dtype=np.uint8)
        off += sizes[k]
    seg_off.append(n)
    if n == 0:
        seg_off = [0]
    return desc, np.array(seg_off, dtype=np.uint32), np.array(seg_sess, dtype=np.uint32), blob
