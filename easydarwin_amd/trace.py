"""Event-trace and capture formats shared by the reference harness (oracle/ref_harness.cpp),
the CPU restatement (oracle/relay_model.cpp) and the GPU engine's replay driver.

A *trace* is what a reflector sees: push sessions (one SDP each), then a time-ordered event
list.  It mirrors the reference's entry points:

* ``PKT``  -> ``ReflectorStream::PushPacket`` for an RTSP-interleaved push
  (QTSSReflectorModule.cpp:604-678: track = channel/2, RTCP = channel & 1);
* ``JOIN`` -> SETUP+PLAY of one subscriber on every track of a session
  (QTSSReflectorModule.cpp:1610-1622, 1942-1946);
* ``TICK`` -> ``ReflectorSender::ReflectPackets`` on every sender
  (ReflectorStream.cpp:1709-1714);
* ``BLOCK`` -> during the next TICK, one subscriber sub-stream's socket accepts ``budget``
  more writes and then returns QTSS_WouldBlock (EAGAIN) for the rest of that tick
  (egress backpressure: SendPacketsToOutput's blocked branch, ReflectorStream.cpp:1158-1190);
* ``LEAVE`` -> a subscriber's TEARDOWN / disconnect: ``ReflectorSession::RemoveOutput(output,
  isClient=true)`` then ``delete`` of the RTPSessionOutput, as QTSSReflectorModule's
  RemoveOutput does (QTSSReflectorModule.cpp:2133-2196; ReflectorSession.cpp:255-279,
  ReflectorStream.cpp:338-362): the output leaves every track's bucket and the eye count
  drops (DecEyeCount, ReflectorStream.h:445).  It takes effect immediately (a LEAVE before the
  subscriber's first TICK means it never receives anything); a LEAVE of a subscriber that is
  not an output (a deferred RTP-Info PLAY) changes nothing.
* ``UPKT`` -> a UDP datagram from a pusher's address arriving on a UDP-push session's RTP
  (even) or RTCP (odd) port: ``ReflectorSocket::GetIncomingData`` -> ``ProcessPacket`` with
  the remote address (ReflectorStream.cpp:1716-1735, 1769-1875), which also records the
  source's RTCP address for the receiver reports (NAT_WORKAROUND, :1843-1855).

Every event carries the virtual clock value (ms) that ``OS::Milliseconds`` returns while it
is applied.  The GPU engine's batch boundary is the TICK: all PKTs since the previous TICK
form one ingest batch (a UDP read event is the same natural boundary in the reference,
ReflectorStream.cpp:1676-1714).

Binary layout (little endian)::

    trace   := "EDTR" u32 version u32 n_sessions { u32 sdp_len sdp_bytes [u8 flags] }*
               [ u32 prefs_len prefs_bytes ]                                 (version 4)
               event* u8 0
               (version 1: no flags byte; version 2: flags bit 0 = UDP push;
                version 3: as 2, with PUBLISH / UNPUBLISH events;
                version 4: as 3, with the server's preferences and PREFS events;
                version 5: as 4, with IDENT events -- read by tools/qtss_replay alone)
    event   := u8 1 i64 t u32 session u8 channel u32 len bytes[len]          (PKT)
             | u8 2 i64 t u32 session u32 sub_id u8 transport u8 ua_flags    (JOIN)
             | u8 3 i64 t                                                    (TICK)
             | u8 4 i64 t u32 sub_id u16 track u8 kind u32 budget           (BLOCK)
             | u8 5 i64 t u32 session u8 channel u32 addr u16 port u32 len bytes[len]
                                                                             (UPKT, v2)
             | u8 6 i64 t u32 sub_id                                         (LEAVE)
             | u8 7 i64 t u32 session u8 kill                                (UNPUBLISH, v3)
             | u8 8 i64 t u32 session                                        (PUBLISH, v3)
             | u8 9 i64 t u32 len bytes[len]                                 (PREFS, v4)
             | u8 10 i64 t u32 session u8 role u32 addr u8 scheme
               { u16 len bytes[len] } x 4 (path, user, groups, realm)        (IDENT, v5)
    capture := "EDCP" u32 n { u32 sub u32 session u16 track u8 kind u8 tcp
                             u64 n_packets u64 n_bytes bytes[n_bytes] }*
               [ "EDRR" u32 m { i64 t u32 session u16 track u32 addr u16 port u32 len
                               bytes[len] }* ]

``prefs_bytes`` (and a PREFS event's bytes) are ``name=value`` lines: the preferences the
server's prefs objects hold (WinNTSupport/easydarwin.xml), every unnamed one at the reference's
default (:data:`PREF_DEFAULTS`).  They are the QTSSReflectorModule prefs ReflectorStream::
Initialize reads once (ReflectorStream.cpp:87-117) and the ones RereadPrefs reads
(QTSSReflectorModule.cpp:454-537), plus the server pref ``player_requires_rtp_header_info``
(comma-separated; QTSServerPrefs, read at every PLAY by HavePlayerProfile, QTSSModuleUtils.cpp:
1012-1046).  A PREFS event is the server rewriting its prefs file and sending the
QTSS_RereadPrefs_Role: the module prefs take the new values (new sessions get the SSRC ones,
QTSSReflectorModule.cpp:1457); ReflectorStream's are not re-read.  A JOIN's ``ua_flags`` bit 0
picks the player's user agent: "vlc/3.0.8 LibVLC/3.0.8" (else "EasyPlayer/1.0"); whether it
is an RTP-Info player follows from the prefs (:func:`rtp_info_player`).

``kind`` is 0 for the RTP sub-stream, 1 for RTCP.  The capture bytes are the sub-stream's
*wire image*: UDP = ``BE16(len) + datagram`` per packet; TCP = the exact interleaved byte
stream ``'$' ch BE16(len) + packet`` (RTSPSessionInterface.cpp:329-344).  The optional
``EDRR`` trailer lists the receiver reports sent to UDP pushers
(ReflectorStream::SendReceiverReport, ReflectorStream.cpp:510-527), in send order; it is
present only when at least one was sent.  ``addr`` is IPv4 in host order.

The reference draws each ReflectorStream's receiver-report SSRC from ``rand()``
(ReflectorStream.cpp:167) and its CNAME from the clock (RTCPSRPacket.cpp:87-117).  The
harness makes ``rand()`` deterministic (:func:`rr_ssrc` of the call count: one call per
ReflectorStream, in session then track order) and runs on a virtual clock that is 0 when the
sessions are created, so a replay feeds the engine the same identities.
"""
from __future__ import annotations

import hashlib
import struct
from dataclasses import dataclass, field

PKT, JOIN, TICK, BLOCK, UPKT, LEAVE, UNPUBLISH, PUBLISH, PREFS, IDENT = 1, 2, 3, 4, 5, 6, 7, 8, 9, 10
IDENT_PUSHER, IDENT_PLAYER = 0, 1
UDP, TCP = 0, 1

# The reference's defaults of the prefs a trace may set (ReflectorStream.cpp:53-59,
# QTSSReflectorModule.cpp:100-166, and the shipped easydarwin.xml's player list, :98-101).
PREF_DEFAULTS = {
    "reflector_bucket_offset_delay_msec": "73",
    "reflector_buffer_size_sec": "1",
    "rtp_reflector_threshold_msec": "2000",
    "reflector_rtp_info_offset_msec": "500",
    "kill_clients_when_broadcast_stops": "false",
    "use_one_SSRC_per_stream": "true",
    "timeout_stream_SSRC_secs": "30",
    "disable_rtp_play_info": "false",
    "enable_player_compatibility": "true",
    "force_rtp_info_sequence_and_time": "false",
    "player_requires_rtp_header_info": "Android,vlc",
    "enable_broadcast_announce": "true",
    "enable_broadcast_push": "true",
    "allow_duplicate_broadcasts": "false",
    "timeout_broadcaster_session_secs": "30",
    "reflector_use_in_packet_receive_time": "false",
    "reflector_in_packet_max_receive_sec": "60",
    # the module's access prefs (QTSSReflectorModule.cpp:141-175, 489-538; RTSPAuthorize, RTSPRoute)
    "allow_broadcasts": "true",
    "authenticate_local_broadcast": "false",
    "BroadcasterGroup": "broadcaster",
    "ip_allow_list": "127.0.0.*",
    "redirect_broadcast_keyword": "",
    "redirect_broadcasts_dir": "",
    "allow_non_sdp_urls": "true",
}
USER_AGENTS = ("EasyPlayer/1.0", "vlc/3.0.8 LibVLC/3.0.8")    # by JOIN ua_flags bit 0


def pref_values(prefs: dict) -> dict:
    """Every pref of PREF_DEFAULTS with the trace's overrides applied."""
    unknown = set(prefs) - set(PREF_DEFAULTS)
    assert not unknown, f"unknown prefs {sorted(unknown)}"
    out = dict(PREF_DEFAULTS)
    out.update({k: str(v) for k, v in prefs.items()})
    return out


def pref_bool(v: str) -> bool:
    return v.strip().lower() == "true"


def rtp_info_player(prefs: dict, ua_flags: int) -> bool:
    """DoPlay's rtpInfoEnabled (QTSSReflectorModule.cpp:1962-1969): the player profile (a
    case-sensitive substring of the user agent in player_requires_rtp_header_info, "*" = any,
    QTSSModuleUtils.cpp:983-1010) when enable_player_compatibility, forced on by
    force_rtp_info_sequence_and_time, off with disable_rtp_play_info."""
    p = pref_values(prefs)
    ua = USER_AGENTS[ua_flags & 1]
    on = False
    if pref_bool(p["enable_player_compatibility"]):
        on = any(x == "*" or (x and x in ua) for x in p["player_requires_rtp_header_info"].split(","))
    if pref_bool(p["force_rtp_info_sequence_and_time"]):
        on = True
    if pref_bool(p["disable_rtp_play_info"]):
        on = False
    return on


def pack_prefs(prefs: dict) -> bytes:
    return "".join(f"{k}={v}\n" for k, v in sorted(prefs.items())).encode()


def unpack_prefs(b: bytes) -> dict:
    out = {}
    for line in b.decode().splitlines():
        if line:
            k, v = line.split("=", 1)
            out[k] = v
    return out


@dataclass
class Trace:
    sdps: list[str] = field(default_factory=list)
    events: list[tuple] = field(default_factory=list)   # (type, t, ...) in file order
    flags: list[int] = field(default_factory=list)      # per session: bit 0 = UDP push
    prefs: dict = field(default_factory=dict)           # the server's pref overrides (version 4)

    def add_session(self, sdp: str, udp_push: bool = False) -> int:
        self.sdps.append(sdp)
        self.flags.append(1 if udp_push else 0)
        return len(self.sdps) - 1

    def udp_push(self, session: int) -> bool:
        return bool(self.flags[session] & 1) if session < len(self.flags) else False

    @property
    def version(self) -> int:
        if any(ev[0] == IDENT for ev in self.events):
            return 5
        if self.prefs or any(ev[0] == PREFS for ev in self.events):
            return 4
        if any(ev[0] in (PUBLISH, UNPUBLISH) for ev in self.events):
            return 3
        return 2 if any(self.flags) or any(ev[0] == UPKT for ev in self.events) else 1

    @property
    def has_lifecycle(self) -> bool:
        return any(ev[0] in (PUBLISH, UNPUBLISH) for ev in self.events)

    def pkt(self, t: int, session: int, channel: int, data: bytes):
        self.events.append((PKT, int(t), session, channel, bytes(data)))

    def join(self, t: int, session: int, sub_id: int, transport: int = UDP, ua_flags: int = 0):
        self.events.append((JOIN, int(t), session, sub_id, transport, ua_flags))

    def tick(self, t: int):
        self.events.append((TICK, int(t)))

    def block(self, t: int, sub_id: int, track: int, kind: int, budget: int):
        self.events.append((BLOCK, int(t), sub_id, track, kind, budget))

    def leave(self, t: int, sub_id: int):
        self.events.append((LEAVE, int(t), sub_id))

    def upkt(self, t: int, session: int, channel: int, addr: int, port: int, data: bytes):
        self.events.append((UPKT, int(t), session, channel, int(addr), int(port), bytes(data)))

    def unpublish(self, t: int, session: int, kill: bool = False):
        self.events.append((UNPUBLISH, int(t), session, 1 if kill else 0))

    def publish(self, t: int, session: int):
        self.events.append((PUBLISH, int(t), session))

    def ident(self, t: int, session: int, role: int, addr: int, path: str = "", user: str = "",
              groups: str = "", realm: str = "", scheme: int = 0):
        """Who opens the session's next RTSP connection of `role` (IDENT_PUSHER: its next
        PUBLISH; IDENT_PLAYER: its next JOIN) -- for the module's RTSPRoute / RTSPAuthorize roles
        (tools/qtss_replay): the client's IPv4 address, the request path ("" = the session's
        own), the user the server authenticated with its groups (comma-separated) and realm, and
        the request's auth scheme."""
        self.events.append((IDENT, int(t), session, role, int(addr), path, user, groups, realm, scheme))

    def reprefs(self, t: int, prefs: dict):
        """The server rewrites its prefs (these overrides replace the previous ones) and sends
        QTSS_RereadPrefs_Role."""
        pref_values(prefs)
        self.events.append((PREFS, int(t), dict(prefs)))

    # -- serialisation ------------------------------------------------------------------
    def to_bytes(self) -> bytes:
        # PKT and TICK times drive the virtual clock and must not go back; a JOIN's time is
        # informational (the join takes effect at the next TICK, like a new output being
        # picked up by the next ReflectPackets), and so is a LEAVE's (it applies in order).
        times = [ev[1] for ev in self.events if ev[0] not in (JOIN, BLOCK, LEAVE)]
        assert all(a <= b for a, b in zip(times, times[1:])), "trace events must be time-ordered"
        ver = self.version
        out = [b"EDTR", struct.pack("<II", ver, len(self.sdps))]
        for i, s in enumerate(self.sdps):
            b = s.encode()
            out.append(struct.pack("<I", len(b)))
            out.append(b)
            if ver >= 2:
                out.append(struct.pack("<B", self.flags[i] if i < len(self.flags) else 0))
        if ver >= 4:
            pb = pack_prefs(self.prefs)
            out.append(struct.pack("<I", len(pb)) + pb)
        for ev in self.events:
            if ev[0] == PKT:
                _, t, s, ch, data = ev
                out.append(struct.pack("<BqIBI", PKT, t, s, ch, len(data)))
                out.append(data)
            elif ev[0] == JOIN:
                _, t, s, sub, tr, ua = ev
                out.append(struct.pack("<BqIIBB", JOIN, t, s, sub, tr, ua))
            elif ev[0] == BLOCK:
                _, t, sub, trk, kind, budget = ev
                out.append(struct.pack("<BqIHBI", BLOCK, t, sub, trk, kind, budget))
            elif ev[0] == UPKT:
                _, t, s, ch, addr, port, data = ev
                out.append(struct.pack("<BqIBIHI", UPKT, t, s, ch, addr, port, len(data)))
                out.append(data)
            elif ev[0] == LEAVE:
                out.append(struct.pack("<BqI", LEAVE, ev[1], ev[2]))
            elif ev[0] == UNPUBLISH:
                out.append(struct.pack("<BqIB", UNPUBLISH, ev[1], ev[2], ev[3]))
            elif ev[0] == PUBLISH:
                out.append(struct.pack("<BqI", PUBLISH, ev[1], ev[2]))
            elif ev[0] == PREFS:
                pb = pack_prefs(ev[2])
                out.append(struct.pack("<BqI", PREFS, ev[1], len(pb)) + pb)
            elif ev[0] == IDENT:
                _, t, s, role, addr, path, user, groups, realm, scheme = ev
                out.append(struct.pack("<BqIBIB", IDENT, t, s, role, addr, scheme))
                for txt in (path, user, groups, realm):
                    b = txt.encode()
                    out.append(struct.pack("<H", len(b)) + b)
            else:
                out.append(struct.pack("<Bq", TICK, ev[1]))
        out.append(b"\x00")
        return b"".join(out)

    def write(self, path: str):
        with open(path, "wb") as f:
            f.write(self.to_bytes())

    @staticmethod
    def from_bytes(buf: bytes) -> "Trace":
        assert buf[:4] == b"EDTR"
        ver, n = struct.unpack_from("<II", buf, 4)
        assert ver in (1, 2, 3, 4, 5)
        p = 12
        tr = Trace()
        for _ in range(n):
            (ln,) = struct.unpack_from("<I", buf, p)
            p += 4
            tr.sdps.append(buf[p:p + ln].decode())
            p += ln
            fl = 0
            if ver >= 2:
                fl = buf[p]
                p += 1
            tr.flags.append(fl)
        if ver >= 4:
            (ln,) = struct.unpack_from("<I", buf, p)
            tr.prefs = unpack_prefs(buf[p + 4:p + 4 + ln])
            p += 4 + ln
        while p < len(buf):
            typ = buf[p]
            if typ == 0:
                break
            if typ == PKT:
                _, t, s, ch, ln = struct.unpack_from("<BqIBI", buf, p)
                p += 18
                tr.events.append((PKT, t, s, ch, bytes(buf[p:p + ln])))
                p += ln
            elif typ == JOIN:
                _, t, s, sub, trn, ua = struct.unpack_from("<BqIIBB", buf, p)
                p += 19
                tr.events.append((JOIN, t, s, sub, trn, ua))
            elif typ == TICK:
                _, t = struct.unpack_from("<Bq", buf, p)
                p += 9
                tr.events.append((TICK, t))
            elif typ == BLOCK:
                _, t, sub, trk, kind, budget = struct.unpack_from("<BqIHBI", buf, p)
                p += 20
                tr.events.append((BLOCK, t, sub, trk, kind, budget))
            elif typ == LEAVE:
                _, t, sub = struct.unpack_from("<BqI", buf, p)
                p += 13
                tr.events.append((LEAVE, t, sub))
            elif typ == UNPUBLISH:
                _, t, s, kill = struct.unpack_from("<BqIB", buf, p)
                p += 14
                tr.events.append((UNPUBLISH, t, s, kill))
            elif typ == PUBLISH:
                _, t, s = struct.unpack_from("<BqI", buf, p)
                p += 13
                tr.events.append((PUBLISH, t, s))
            elif typ == PREFS:
                _, t, ln = struct.unpack_from("<BqI", buf, p)
                tr.events.append((PREFS, t, unpack_prefs(buf[p + 13:p + 13 + ln])))
                p += 13 + ln
            elif typ == IDENT:
                _, t, s, role, addr, scheme = struct.unpack_from("<BqIBIB", buf, p)
                p += 19
                txt = []
                for _ in range(4):
                    (ln,) = struct.unpack_from("<H", buf, p)
                    txt.append(bytes(buf[p + 2:p + 2 + ln]).decode())
                    p += 2 + ln
                tr.events.append((IDENT, t, s, role, addr) + tuple(txt) + (scheme,))
            elif typ == UPKT:
                _, t, s, ch, addr, port, ln = struct.unpack_from("<BqIBIHI", buf, p)
                p += 24
                tr.events.append((UPKT, t, s, ch, addr, port, bytes(buf[p:p + ln])))
                p += ln
            else:
                raise ValueError(f"bad event {typ} at {p}")
        return tr


@dataclass
class SubStream:
    sub: int
    session: int
    track: int
    kind: int          # 0 RTP, 1 RTCP
    tcp: int
    n_packets: int
    data: bytes

    @property
    def key(self):
        return (self.sub, self.track, self.kind)

    def digest(self) -> str:
        return hashlib.sha256(self.data).hexdigest()


def read_capture(path_or_bytes) -> dict:
    buf = path_or_bytes
    if isinstance(path_or_bytes, str):
        with open(path_or_bytes, "rb") as f:
            buf = f.read()
    assert buf[:4] == b"EDCP", "bad capture magic"
    (n,) = struct.unpack_from("<I", buf, 4)
    p = 8
    out = {}
    for _ in range(n):
        sub, sess, track, kind, tcp, npk, nb = struct.unpack_from("<IIHBBQQ", buf, p)
        p += 28
        data = bytes(buf[p:p + nb])
        p += nb
        ss = SubStream(sub, sess, track, kind, tcp, npk, data)
        out[ss.key] = ss
    return out


def rr_ssrc(k: int) -> int:
    """The harness's deterministic rand(): the value of its k-th call (0-based)."""
    return ((k + 1) * 0x9E3779B1 + 0x7F4A7C15) & 0x7FFFFFFF


def pack_source_reports(reports) -> bytes:
    """reports: [(t, session, track, addr, port, bytes)] -> the capture's EDRR trailer."""
    if not reports:
        return b""
    out = [b"EDRR", struct.pack("<I", len(reports))]
    for t, s, trk, addr, port, data in reports:
        out.append(struct.pack("<qIHIHI", t, s, trk, addr, port, len(data)))
        out.append(bytes(data))
    return b"".join(out)


def read_source_reports(buf: bytes) -> list:
    """The EDRR trailer of a capture: [(t, session, track, addr, port, bytes)]."""
    assert buf[:4] == b"EDCP", "bad capture magic"
    (n,) = struct.unpack_from("<I", buf, 4)
    p = 8
    for _ in range(n):
        nb = struct.unpack_from("<Q", buf, p + 20)[0]
        p += 28 + nb
    if p >= len(buf):
        return []
    assert buf[p:p + 4] == b"EDRR", "bad capture trailer"
    (m,) = struct.unpack_from("<I", buf, p + 4)
    p += 8
    out = []
    for _ in range(m):
        t, s, trk, addr, port, ln = struct.unpack_from("<qIHIHI", buf, p)
        p += 24
        out.append((t, s, trk, addr, port, bytes(buf[p:p + ln])))
        p += ln
    return out


def capture_summary(cap: dict) -> dict:
    """Digest form used by the committed golden fixtures."""
    return {f"{k[0]}/{k[1]}/{k[2]}": [v.n_packets, len(v.data), v.digest()]
            for k, v in sorted(cap.items())}


def split_wire_image(data: bytes, tcp: int) -> list[bytes]:
    """Wire image -> list of packets (inverse of the framing described above)."""
    out, p = [], 0
    hdr = 4 if tcp else 2
    while p < len(data):
        if tcp:
            assert data[p] == 0x24
        ln = (data[p + hdr - 2] << 8) | data[p + hdr - 1]
        out.append(data[p + hdr:p + hdr + ln])
        p += hdr + ln
    return out
