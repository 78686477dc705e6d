// oracle/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured as
// the product).  Drives the REAL EasyDarwin reflector hot path, compiled from the
// read-only reference sources by oracle/_ref/Makefile, with a fake QTSS server:
//
//   * a callback table (QTSS_Private.h:52-127) whose dictionary calls are served by a
//     tiny in-memory attribute store, whose QTSS_Write (index 10) captures the bytes
//     per subscriber sub-stream, and whose Milliseconds is a virtual clock;
//   * OS::Milliseconds is link-wrapped (-Wl,--wrap) onto the same virtual clock;
//   * push sessions are built exactly as FindOrCreateSession does for an RTSP-TCP
//     (interleaved, EasyPusher-default) push (QTSSReflectorModule.cpp:1379-1460):
//     SDPSourceInfo -> ReflectorSession -> SetupReflectorSession(kMarkSetup|kIsPushSession,
//     one SSRC per stream = true, 30 s);
//   * subscribers are built as DoSetup/DoPlay do (QTSSReflectorModule.cpp:1610-1622,
//     1766-1786, 1942-1946): RTPSessionOutput + ReflectorSession::AddOutput, one RTP
//     stream object per track carrying the ReflectorStream cookie, then InitializeStreams
//     and state = playing;
//   * PKT events call ReflectorStream::PushPacket (as ProcessRTPData does,
//     QTSSReflectorModule.cpp:604-678: track = channel/2, RTCP = channel&1);
//   * TICK events call ReflectPackets on every sender (RTP then RTCP, track order), as
//     ReflectorSocket::Run does (ReflectorStream.cpp:1709-1714);
//   * BLOCK events give one sub-stream's socket a write budget for the next TICK: after
//     `budget` accepted writes QTSS_Write returns QTSS_WouldBlock (EAGAIN, RTPStream.cpp:
//     1145-1147) until the TICK ends -- the blocked-client path of SendPacketsToOutput;
//   * UDP-push sessions (trace v2, session flag bit 0) get their socket pair bound on
//     loopback to an even/odd port pair, as UDPSocketPool::CreateUDPSocketPair binds it
//     (UDPSocketPool.cpp), so GetLocalPort()&1 tells RTCP from RTP; UPKT events are the
//     datagrams GetIncomingData reads (ReflectorStream.cpp:1716-1735): clamped to the
//     2060-byte receive buffer, then ReflectorSocket::ProcessPacket(now, packet, remote
//     addr, remote port), which applies the UDP RTCP SR gate (Q14) and records the pusher's
//     RTCP address (NAT_WORKAROUND, :1843-1855).  The session is still set up through the
//     TCP-transport branch of BindSockets (no UDPSocketPool search, no event registration);
//     the transport type is read nowhere on the packet path;
//   * UDPSocket::SendTo is link-wrapped: the only caller on this path is
//     ReflectorStream::SendReceiverReport (:510-527, every kRRInterval from the RTCP sender's
//     ReflectPackets, :1039-1047), whose datagrams go to the capture's EDRR trailer;
//   * LEAVE events remove a subscriber as QTSSReflectorModule's RemoveOutput does
//     (QTSSReflectorModule.cpp:2133-2196): ReflectorSession::RemoveOutput(output, true) -- out
//     of every track's bucket, DecEyeCount -- then delete the RTPSessionOutput; its capture so
//     far is kept;
//   * rand() is link-wrapped to a deterministic sequence (trace.py rr_ssrc): its only caller
//     on this path is the ReflectorStream constructor's receiver-report SSRC (:167);
//   * session lifecycle (trace v3): sessions live in a real OSRefTable, registered and resolved
//     as FindOrCreateSession does (QTSSReflectorModule.cpp:1388, 1469-1477) -- the pusher holds
//     one reference, every output one.  UNPUBLISH runs DestroySession's broadcaster branch
//     (:2082-2109: fSetupToReceive cleared, RemoveSessionFromOutput) and RemoveOutput(NULL,
//     session, kill) (:2133-2196): TearDownAllOutputs reaches every output's
//     RTPSessionOutput::TearDown -> QTSS_Teardown (callback 22), after which the fake server
//     closes those client sessions (DestroySession's player branch -> RemoveOutput(output)); at
//     reference count 0 the session is UnRegistered and killed.  PUBLISH reuses a session that
//     still exists (Resolve, not set up again, :1479-1536) or builds a fresh one (:1391-1478).
//     PKT / UPKT of a session without a pusher are dropped; a JOIN of a session that no longer
//     exists fails (FindOrCreateSession returns NULL for a player, :1391-1396).
//   * preferences (trace v4): the trace's overrides are values of a module prefs object and of
//     the server prefs object, read through the reference's own QTSSModuleUtils::GetAttribute /
//     HavePlayerProfile over this fake server's dictionary callbacks (GetAttrInfoByName,
//     GetNumValues, GetValueAsString); a pref the trace does not name is missing, so the
//     reference falls back to its default.  ReflectorStream::Initialize reads its prefs once
//     (ReflectorStream.cpp:87-117); the module prefs are read as RereadPrefs reads them
//     (QTSSReflectorModule.cpp:454-537) at start and at every PREFS event, and used where the
//     module uses them: SetupReflectorSession's SSRC filter (:1457), RECORD's kill-clients
//     attribute (:1884) and RemoveOutput's kill (:2156), DoPlay's rtpInfoEnabled (:1962-1969).
//
// Usage: ref_harness <trace.edtr> <capture.edcp>
//        ref_harness --bench <trace.edtr>    (memcpy sinks, no capture; prints the replay's
//                                             relayed packets / bytes and seconds as JSON)
//        ref_harness --bench-udp <trace.edtr> (the same, but every UDP subscriber write is a
//                                             real sendto() to a loopback socket, one syscall
//                                             per packet as RTPStream::Write's SendTo,
//                                             RTPStream.cpp:1139-1145)
// Trace / capture formats: see easydarwin_amd/trace.py (shared with the port oracle and
// the GPU engine's replay driver).

#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>
#include <memory>
#include <algorithm>
#include <climits>

#include "QTSS.h"
#include "QTSS_Private.h"
#include "OS.h"
#include "OSQueue.h"
#include "MyAssert.h"
#include "SDPSourceInfo.h"
#include "ReflectorSession.h"
#include "ReflectorStream.h"
#include "RTPSessionOutput.h"
#include "RTPOverbufferWindow.h"
#include "QTSServerInterface.h"
#include "QTSSModuleUtils.h"
#include "OSRef.h"

// ---------------------------------------------------------------------------------------
// The two server-side module tables ReflectorSession::SetSessionName reads
// (QTSServerInterface.h:356-357).  The harness *is* the server, with zero modules
// registered in any role.
QTSSModule** QTSServerInterface::sModuleArray[QTSSModule::kNumRoles];
UInt32       QTSServerInterface::sNumModulesInRole[QTSSModule::kNumRoles];

// ---------------------------------------------------------------------------------------
// A ReflectorSocket's own free-packet queue (private; reached by explicit instantiation, which
// the language exempts from access checks, as oracle/ref_module_host.cpp reaches the session
// map): ReflectorSocket::Run hands it to ReflectPackets (ReflectorStream.cpp:1713), so the
// packets RemoveOldPackets frees go back to the socket and GetPacket reuses them (:2039-2047).
namespace {
template <typename Tag, typename Tag::type M> struct Steal { friend typename Tag::type get(Tag) { return M; } };
struct FreeQueueMember { typedef OSQueue ReflectorSocket::*type; friend type get(FreeQueueMember); };
template struct Steal<FreeQueueMember, &ReflectorSocket::fFreeQueue>;
}
// ReflectorSocket::Run's reflect step for one stream: each sender under its socket's demuxer
// mutex, with that socket's free queue (ReflectorStream.cpp:1687, 1709-1714)
static void reflect_stream(ReflectorStream* st) {
    UDPSocketPair* pr = st->GetSocketPair();
    ReflectorSocket* a = (ReflectorSocket*)pr->GetSocketA();
    ReflectorSocket* b = (ReflectorSocket*)pr->GetSocketB();
    SInt64 wake = 0;
    {
        OSMutexLocker l(a->GetDemuxer()->GetMutex());
        st->GetRTPSender()->ReflectPackets(&wake, &(a->*get(FreeQueueMember())));
    }
    wake = 0;
    {
        OSMutexLocker l(b->GetDemuxer()->GetMutex());
        st->GetRTCPSender()->ReflectPackets(&wake, &(b->*get(FreeQueueMember())));
    }
}

// ---------------------------------------------------------------------------------------
// Virtual clock.
static SInt64 g_now = 0;
extern "C" SInt64 __wrap__ZN2OS12MillisecondsEv() { return g_now; }

// Deterministic rand() (easydarwin_amd/trace.py rr_ssrc).
static UInt32 g_rand_calls = 0;
extern "C" int __wrap_rand() {
    const UInt32 k = g_rand_calls++;
    return (int)(((k + 1) * 0x9E3779B1u + 0x7F4A7C15u) & 0x7FFFFFFFu);
}

// Receiver reports to UDP pushers: UDPSocket::SendTo(addr, port, buf, len).
struct SentReport { SInt64 t; UInt32 session; UInt16 track; UInt32 addr; UInt16 port; std::string bytes; };
static std::vector<SentReport> g_reports;
static std::map<const void*, std::pair<UInt32, UInt16>> g_rtcp_sockets;   // socket B -> (session, track)
extern "C" OS_Error __wrap__ZN9UDPSocket6SendToEjtPvj(void* self, UInt32 addr, UInt16 port, void* buf, UInt32 len) {
    auto it = g_rtcp_sockets.find(self);
    SentReport r;
    r.t = g_now;
    r.session = it == g_rtcp_sockets.end() ? 0xFFFFFFFFu : it->second.first;
    r.track = it == g_rtcp_sockets.end() ? 0xFFFF : it->second.second;
    r.addr = addr; r.port = port;
    r.bytes.assign((const char*)buf, len);
    g_reports.push_back(r);
    return OS_NoErr;
}

// ---------------------------------------------------------------------------------------
// Attribute store.  Values have stable storage because RTPSessionOutput writes through
// pointers returned by QTSS_GetValuePtr (RTPSessionOutput.cpp:647-651).
struct Value { std::vector<char> buf; UInt32 len = 0; };
struct FakeObj {
    std::map<UInt32, std::vector<std::unique_ptr<Value>>> attrs;
    std::map<std::string, std::pair<UInt32, UInt32>> named;   // attribute name -> (id, data type)
    // capture side (RTP stream objects only)
    bool is_stream = false;
    UInt32 sub_id = 0, session = 0, track = 0, transport = 0;
    UInt32 rtp_channel = 0, rtcp_channel = 1;
    std::string cap[2];          // [0] RTP writes, [1] RTCP writes (wire image)
    UInt64 npk[2] = {0, 0};
    SInt64 budget[2] = {-1, -1}; // writes the socket accepts this tick (-1: unlimited)
    std::vector<SInt64> tt[2];   // QTSS_PacketStruct.packetTransmitTime of each accepted write
    // EDTR_SERVER_GATE: the server's RTPStream::Write gate (below)
    FakeObj* client = nullptr;   // the stream's client session
    bool video = false;          // qtssRTPStrPayloadType is video (the SDP's m= media)
    SInt64 last_delay = 0;       // RTPStream::fLastCurrentPacketDelay
    UInt64 stale_dropped = 0;    // fStalePacketsDropped
    // the client session's RTPSession part (on the client object)
    RTPOverbufferWindow* window = nullptr;
    // a pusher's client session: its timeout (RTPSessionInterface's fTimeoutTask), who it is
    SInt64 to_ms = 0, deadline = 0;
    int push_s = -1, push_k = -1;
    SInt64 play_time = 0, last_check = 0, last_check_media = 0;
    bool started_thinning = false;
};
static std::vector<std::unique_ptr<FakeObj>> g_objs;
static FakeObj* new_obj() { g_objs.emplace_back(new FakeObj()); return g_objs.back().get(); }

static void set_value(FakeObj* o, UInt32 id, UInt32 idx, const void* p, UInt32 len) {
    auto& vec = o->attrs[id];
    if (vec.size() <= idx) vec.resize(idx + 1);
    if (!vec[idx]) vec[idx].reset(new Value());
    Value& v = *vec[idx];
    if (v.buf.size() < len) v.buf.resize(std::max<size_t>(len, 16));
    if (len) memcpy(v.buf.data(), p, len);
    v.len = len;
}
static Value* get_value(FakeObj* o, UInt32 id, UInt32 idx) {
    auto it = o->attrs.find(id);
    if (it == o->attrs.end() || idx >= it->second.size() || !it->second[idx]) return nullptr;
    return it->second[idx].get();
}

static std::map<std::string, UInt32> g_attr_ids;

// Preferences: the module prefs object and the server prefs object (trace v4).
static const char* const kPrefDefaults[][2] = {            // easydarwin_amd/trace.py PREF_DEFAULTS
    {"reflector_bucket_offset_delay_msec", "73"}, {"reflector_buffer_size_sec", "1"},
    {"rtp_reflector_threshold_msec", "2000"}, {"reflector_rtp_info_offset_msec", "500"},
    {"kill_clients_when_broadcast_stops", "false"}, {"use_one_SSRC_per_stream", "true"},
    {"timeout_stream_SSRC_secs", "30"}, {"disable_rtp_play_info", "false"},
    {"enable_player_compatibility", "true"}, {"force_rtp_info_sequence_and_time", "false"},
    {"player_requires_rtp_header_info", "Android,vlc"},
    {"enable_broadcast_announce", "true"}, {"enable_broadcast_push", "true"},
    {"allow_duplicate_broadcasts", "false"}, {"timeout_broadcaster_session_secs", "30"},
        {"reflector_use_in_packet_receive_time", "false"}, {"reflector_in_packet_max_receive_sec", "60"},
        {"allow_broadcasts", "true"}, {"authenticate_local_broadcast", "false"}, {"BroadcasterGroup", "broadcaster"},
        {"ip_allow_list", "127.0.0.*"}, {"redirect_broadcast_keyword", ""}, {"redirect_broadcasts_dir", ""},
        {"allow_non_sdp_urls", "true"},
};
static FakeObj* g_mod_prefs = nullptr;      // QTSSReflectorModule's prefs object
static FakeObj* g_srv_prefs = nullptr;      // the server's prefs object
// the trace's overrides (name -> value); a named pref becomes an attribute of the right type
static void load_prefs(const std::map<std::string, std::string>& over) {
    for (FakeObj* o : {g_mod_prefs, g_srv_prefs}) { o->attrs.clear(); o->named.clear(); }
    UInt32 next = 0x20000000u;
    for (const auto& kv : over) {
        const std::string& k = kv.first;
        const std::string& v = kv.second;
        if (k == "player_requires_rtp_header_info") {          // a LIST-PREF, one value per entry
            size_t p = 0, idx = 0;
            while (p <= v.size()) {
                size_t e = v.find(',', p);
                if (e == std::string::npos) e = v.size();
                std::string one = v.substr(p, e - p);
                set_value(g_srv_prefs, qtssPrefsPlayersReqRTPHeader, (UInt32)idx++, one.data(), (UInt32)one.size());
                p = e + 1;
            }
            continue;
        }
        const bool isBool = v == "true" || v == "false";
        const UInt32 id = next++;
        g_mod_prefs->named[k] = std::make_pair(id, (UInt32)(isBool ? qtssAttrDataTypeBool16 : qtssAttrDataTypeUInt32));
        if (isBool) { bool b = v == "true"; set_value(g_mod_prefs, id, 0, &b, sizeof(b)); }
        else { UInt32 u = (UInt32)strtoul(v.c_str(), nullptr, 10); set_value(g_mod_prefs, id, 0, &u, sizeof(u)); }
    }
}
// RereadPrefs' module prefs used on this path (QTSSReflectorModule.cpp:454-537: same names,
// types and defaults, :100-166), read through the reference's QTSSModuleUtils::GetAttribute
struct ModulePrefs {
    bool killClients = false, oneSSRC = true, rtpInfoDisabled = false, playerCompat = true, forceRTPInfo = false;
    UInt32 timeoutSSRC = 30;
    UInt32 broadcasterTimeoutSecs = 30;      // timeout_broadcaster_session_secs, at least 30 (:483-487)
};
static ModulePrefs g_mp;
static void reread_prefs() {
    static bool dFalse = false, dTrue = true;
    static UInt32 d30 = 30;
    QTSS_ModulePrefsObject o = (QTSS_ModulePrefsObject)g_mod_prefs;
    QTSSModuleUtils::GetAttribute(o, (char*)"disable_rtp_play_info", qtssAttrDataTypeBool16, &g_mp.rtpInfoDisabled, &dFalse, sizeof(dFalse));
    QTSSModuleUtils::GetAttribute(o, (char*)"kill_clients_when_broadcast_stops", qtssAttrDataTypeBool16, &g_mp.killClients, &dFalse, sizeof(dFalse));
    QTSSModuleUtils::GetAttribute(o, (char*)"use_one_SSRC_per_stream", qtssAttrDataTypeBool16, &g_mp.oneSSRC, &dTrue, sizeof(dTrue));
    QTSSModuleUtils::GetAttribute(o, (char*)"timeout_stream_SSRC_secs", qtssAttrDataTypeUInt32, &g_mp.timeoutSSRC, &d30, sizeof(d30));
    QTSSModuleUtils::GetAttribute(o, (char*)"enable_player_compatibility", qtssAttrDataTypeBool16, &g_mp.playerCompat, &dTrue, sizeof(dTrue));
    QTSSModuleUtils::GetAttribute(o, (char*)"force_rtp_info_sequence_and_time", qtssAttrDataTypeBool16, &g_mp.forceRTPInfo, &dFalse, sizeof(dFalse));
    QTSSModuleUtils::GetAttribute(o, (char*)"timeout_broadcaster_session_secs", qtssAttrDataTypeUInt32, &g_mp.broadcasterTimeoutSecs, &d30, sizeof(d30));
    if (g_mp.broadcasterTimeoutSecs < 30) g_mp.broadcasterTimeoutSecs = 30;
}

// ---------------------------------------------------------------------------------------
// The pushers' client-session timeouts, as tools/qtss_replay keeps them for a loaded module (the same
// model and the same EDGPU_KEEPALIVE_LOG lines): the module sets qtssCliSesTimeoutMsec to
// max(30, timeout_broadcaster_session_secs) s at every push SETUP (QTSSReflectorModule.cpp:1644) and
// names the pusher on its sockets (AddBroadcasterClientSession, :1715); the server moves the deadline
// on at the pusher's RTSP requests (RTSPSession.cpp:1669) and every '$' frame of an interleaved push
// (:2157); the reference's own ReflectorSocket::ProcessPacket calls QTSS_RefreshTimeOut on it every
// 10 s of packets (ReflectorStream.cpp:1779-1786); a session whose deadline passes is closed as a
// pusher that hung up (DestroySession, with its RECORD's kill flag).  EDGPU_REPLAY_NO_REFRESH=1: the
// module's refreshes are logged but ignored.
static FILE* g_ka_log = nullptr;
static bool g_no_refresh = false;
static void ka_log(char kind, SInt64 t, const FakeObj* c, const char* extra = "") {
    if (g_ka_log) fprintf(g_ka_log, "%c %lld push %d.%d%s\n", kind, (long long)t, c->push_s, c->push_k, extra);
}
static QTSS_Error cb_refresh_timeout(void* client, ...) {
    FakeObj* c = (FakeObj*)client;
    if (!c || c->push_s < 0) return QTSS_BadArgument;
    ka_log('R', g_now, c);
    if (!g_no_refresh && c->deadline) c->deadline = g_now + c->to_ms;
    return QTSS_NoErr;
}
static std::map<std::string, std::string> parse_prefs(const std::string& b) {
    std::map<std::string, std::string> m;
    size_t p = 0;
    while (p < b.size()) {
        size_t e = b.find('\n', p);
        if (e == std::string::npos) e = b.size();
        const std::string line = b.substr(p, e - p);
        const size_t q = line.find('=');
        if (q != std::string::npos) m[line.substr(0, q)] = line.substr(q + 1);
        p = e + 1;
    }
    return m;
}
// a user agent of the trace (easydarwin_amd/trace.py USER_AGENTS: JOIN ua_flags bit 0)
static const char* kUserAgents[2] = {"EasyPlayer/1.0", "vlc/3.0.8 LibVLC/3.0.8"};
static UInt32 g_cookie_attr = 0;

// ---------------------------------------------------------------------------------------
// Callbacks (all reached through QTSS_Private.cpp's varargs stubs).
static QTSS_Error cb_fail(...) { return QTSS_RequestFailed; }
static QTSS_Error cb_ok(...) { return QTSS_NoErr; }
static QTSS_Error cb_milliseconds(SInt64* out, ...) { *out = g_now; return QTSS_NoErr; }
// QTSS_Teardown(client session): the server closes it later (ClientSessionClosing); recorded here
static std::vector<void*> g_torn_down;
static QTSS_Error cb_teardown(void* client, ...) { g_torn_down.push_back(client); return QTSS_NoErr; }
static QTSS_Error cb_id_for_tag(UInt32 type, const char* tag, QTSS_AttributeID* out, ...) {
    std::string key = std::to_string(type) + ":" + tag;
    auto it = g_attr_ids.find(key);
    if (it == g_attr_ids.end()) {
        UInt32 id = 0x40000000u + (UInt32)g_attr_ids.size();
        it = g_attr_ids.emplace(key, id).first;
    }
    *out = it->second;
    return QTSS_NoErr;
}
// A real QTSSDictionary refuses qtssIllegalAttrID (QTSS.h:342) with QTSS_AttrDoesntExist;
// QTSSModuleUtils::CreateAttribute relies on that when a pref is missing.
static QTSS_Error cb_get_value_ptr(void* obj, UInt32 id, UInt32 idx, void** out, UInt32* len, ...) {
    if (!obj) return QTSS_BadArgument;
    if (id == (UInt32)qtssIllegalAttrID) return QTSS_AttrDoesntExist;
    Value* v = get_value((FakeObj*)obj, id, idx);
    if (!v) { if (len) *len = 0; return QTSS_ValueNotFound; }
    *out = v->buf.data();
    if (len) *len = v->len;
    return QTSS_NoErr;
}
static QTSS_Error cb_get_value(void* obj, UInt32 id, UInt32 idx, void* buf, UInt32* len, ...) {
    if (!obj) return QTSS_BadArgument;
    if (id == (UInt32)qtssIllegalAttrID) return QTSS_AttrDoesntExist;
    Value* v = get_value((FakeObj*)obj, id, idx);
    if (!v) return QTSS_ValueNotFound;
    if (*len < v->len) { *len = v->len; return QTSS_NotEnoughSpace; }
    memcpy(buf, v->buf.data(), v->len);
    *len = v->len;
    return QTSS_NoErr;
}
// QTSS_GetAttrInfoByName: an attribute-info object with qtssAttrID / qtssAttrDataType
static QTSS_Error cb_attr_info_by_name(void* obj, const char* name, void** out, ...) {
    FakeObj* o = (FakeObj*)obj;
    if (!o || !name) return QTSS_BadArgument;
    auto it = o->named.find(name);
    if (it == o->named.end()) return QTSS_AttrDoesntExist;
    FakeObj* info = new_obj();
    set_value(info, qtssAttrID, 0, &it->second.first, sizeof(UInt32));
    set_value(info, qtssAttrDataType, 0, &it->second.second, sizeof(UInt32));
    *out = info;
    return QTSS_NoErr;
}
static QTSS_Error cb_num_values(void* obj, UInt32 id, UInt32* n, ...) {
    if (!obj || !n) return QTSS_BadArgument;
    auto it = ((FakeObj*)obj)->attrs.find(id);
    *n = it == ((FakeObj*)obj)->attrs.end() ? 0 : (UInt32)it->second.size();
    return QTSS_NoErr;
}
// QTSS_GetValueAsString of a char-array value: a new[] copy the caller deletes
static QTSS_Error cb_value_as_string(void* obj, UInt32 id, UInt32 idx, char** out, ...) {
    if (!obj || !out) return QTSS_BadArgument;
    *out = nullptr;
    Value* v = get_value((FakeObj*)obj, id, idx);
    if (!v) return QTSS_ValueNotFound;
    char* c = new char[v->len + 1];
    memcpy(c, v->buf.data(), v->len);
    c[v->len] = 0;
    *out = c;
    return QTSS_NoErr;
}
static QTSS_Error cb_set_value(void* obj, UInt32 id, UInt32 idx, const void* buf, UInt32 len, ...) {
    if (!obj) return QTSS_BadArgument;
    if (id == (UInt32)qtssIllegalAttrID) return QTSS_AttrDoesntExist;
    set_value((FakeObj*)obj, id, idx, buf, len);
    return QTSS_NoErr;
}
// QTSS_Write(stream, QTSS_PacketStruct*, len, outLen, flags): RTPStream::Write's framing
// (RTPStream.cpp:1098-1145) -- UDP datagram, or '$' ch BE16(len) + packet on the RTP or
// RTCP channel (RTSPSessionInterface.cpp:329-344).  A sink blocks only when a BLOCK event
// set its budget for this tick.
// Bench mode (--bench): the sink is a memcpy into a scratch buffer (no capture), counted.
static bool g_bench = false;
static UInt64 g_bench_pkts = 0, g_bench_bytes = 0;
// --bench-steady: the reflect loop's own time (TICKs) apart from the ingest's (PKTs)
static double g_reflect_s = 0, g_push_s = 0;
static UInt64 g_ticks = 0, g_pushed = 0;
static char g_scratch[70000];
static int g_udp_fd = -1;                      // --bench-udp: the subscribers' UDP socket
static sockaddr_in g_udp_dst;                  // an unread loopback socket (drops when full)
//
// EDTR_SERVER_GATE=1: QTSS_Write also applies what the server's RTPStream::Write does before its
// socket write (Server.tproj/RTPStream.cpp:1048-1147) -- Q20, for the engine's own egress
// (edgpu_egress pacing): the session's over-buffer window, the REFERENCE's RTPOverbufferWindow
// (RTPOverbufferWindow.cpp, compiled in) built as RTPSessionInterface builds it (send_interval
// 50 ms, window kUInt32_Max, max_send_ahead_time 25 s, overbuffer_rate 2.0: RTPSessionInterface.cpp:
// 131, QTSServerPrefs.cpp:132-160) with overbuffering off -- DoSetup turns it off for every
// player without a dynamic-rate header (QTSSReflectorModule.cpp:1772-1777), which is every player
// here -- gates RTP and (overbuffering off) RTCP writes: a packet whose transmit time is past
// now + the send interval waits (QTSS_WouldBlock); then RTP packets of TCP non-video streams go
// through RTPStream::UpdateQualityLevel (:936-1045) with SetThinningParams' defaults (:897-918:
// late tolerance 1.5 s -> no adjustment; drop_all_packets_delay 2500, thin_all_the_way 1500,
// start_thinning 0, start_thicking 250 ms, QTSServerPrefs.cpp:110-148), restated below: with the
// reflector's two quality levels (ReflectorSession.h:152-154) only its stale-packet drop can
// change what is written.  A dropped packet is written nowhere but counts as written.  Only then
// does the socket budget apply, and an accepted RTP write enters the window (:1208-1213).
static bool g_gate = false;
static bool update_quality_level(FakeObj* st, FakeObj* cs, SInt64 tt, SInt64 delay, SInt64 now) {
    if (tt <= cs->play_time) return true;
    if (st->video) return true;                            // no thinning for video (:946-951)
    if (st->transport != qtssRTPTransportTypeTCP) return true;
    if (cs->last_check == 0) {
        cs->last_check = now; cs->last_check_media = tt; st->last_delay = delay;
        return true;
    }
    if (!cs->started_thinning) {
        if (delay > 0 && delay - st->last_delay < 250) {   // fStartThinningDelay 0
            if (delay < st->last_delay) st->last_delay = delay;
            return true;
        }
        cs->started_thinning = true;
    }
    if (cs->last_check == 0 || delay > 1500) {             // fThinAllTheWayDelay
        cs->last_check = now; cs->last_check_media = tt; st->last_delay = delay;
        if (delay > 1500 && delay > 2500) {                // SetMinQuality; fDropAllPacketsForThisStreamDelay
            st->stale_dropped++;
            return false;
        }
    }
    return true;                                           // two quality levels: nothing else drops
}

static QTSS_Error cb_write(void* stream, const void* buf, UInt32 len, UInt32* outLen, UInt32 flags, ...) {
    FakeObj* s = (FakeObj*)stream;
    const QTSS_PacketStruct* pkt = (const QTSS_PacketStruct*)buf;
    int k = (flags & qtssWriteFlagsIsRTCP) ? 1 : 0;
    if (len == 0) return QTSS_NoErr;
    if (g_gate && s->client) {
        FakeObj* cs = s->client;
        const SInt64 now = g_now;
        const SInt64 delay = now - pkt->packetTransmitTime;
        // overbuffering is off: RTCP is gated too (:1085-1096)
        if (cs->window->CheckTransmitTime(pkt->packetTransmitTime, now, (SInt32)len) > now) return QTSS_WouldBlock;
        if (!k && !update_quality_level(s, cs, pkt->packetTransmitTime, delay, now)) {
            if (outLen) *outLen = len;
            return QTSS_NoErr;                             // stale: not written, counted as written
        }
    }
    if (s->budget[k] == 0) return QTSS_WouldBlock;
    if (s->budget[k] > 0) s->budget[k]--;
    if (g_bench) {
        const UInt32 h = s->transport == qtssRTPTransportTypeTCP ? 4 : 0;
        if (g_udp_fd >= 0 && h == 0)
            (void)::sendto(g_udp_fd, pkt->packetData, len, 0, (const sockaddr*)&g_udp_dst, sizeof(g_udp_dst));
        else
            memcpy(g_scratch + h, pkt->packetData, len);
        g_bench_pkts++;
        g_bench_bytes += len + h;
        if (outLen) *outLen = len;
        return QTSS_NoErr;
    }
    if (g_gate && s->client && !k) s->client->window->AddPacketToWindow((SInt32)len);
    std::string& c = s->cap[k];
    if (s->transport == qtssRTPTransportTypeTCP) {
        c.push_back('$');
        c.push_back((char)(k ? s->rtcp_channel : s->rtp_channel));
    }
    c.push_back((char)(len >> 8));
    c.push_back((char)(len & 0xff));
    c.append((const char*)pkt->packetData, len);
    s->npk[k]++;
    s->tt[k].push_back(pkt->packetTransmitTime);
    if (outLen) *outLen = len;
    return QTSS_NoErr;
}

struct NoopAssert : public AssertLogger {
    unsigned long count = 0;
    void LogAssert(char* m) override { if (getenv("EDTR_SHOW_ASSERTS")) fprintf(stderr, "assert: %s\n", m); ++count; }
};

// ---------------------------------------------------------------------------------------
// Trace reader (format: easydarwin_amd/trace.py).
struct Reader {
    std::vector<unsigned char> d; size_t p = 0;
    template <class T> T get() { T v; memcpy(&v, &d[p], sizeof(T)); p += sizeof(T); return v; }
    bool done() const { return p >= d.size(); }
};

struct Sub {
    UInt32 id, session;
    FakeObj* client;
    std::vector<FakeObj*> streams;
    RTPSessionOutput* output;
    ReflectorSession* rsess;        // the ReflectorSession it is an output of
};

// One trace session (one stream name): the ReflectorSession registered under it, if any, and
// whether a pusher is attached.
struct Live {
    ReflectorSession* sess = nullptr;
    FakeObj* bcast = nullptr;       // the pusher's client session
    bool published = false;
    bool killAttr = false;          // its QTSSReflectorModuleTearDownClients, set at RECORD (:1884)
    int pubs = 0;                   // pusher connections so far (their ordinals in the keep-alive log)
};

int main(int argc, char** argv) {
    int reps = 1;
    // --bench-steady <trace> <loops> <warm_ms>: the trace's packets and ticks replayed `loops` times
    // back to back on the same sessions and players, the clock running on (loop k at k x the last
    // TICK's time), so the queues reach the reference's steady state -- packets older than
    // sMaxPacketAgeMSec freed to their socket's queue and reused (RemoveOldPackets,
    // ReflectorStream.cpp:1233-1289; GetPacket :2039-2047) -- and only what happens at or after
    // virtual time warm_ms is counted: relayed packets, the TICKs' reflect time and, apart from it,
    // the PKTs' PushPacket time (the steady-state reflect loop, ingest timed separately).
    int steady_loops = 0;
    SInt64 steady_warm = 0;
    if (argc == 5 && strcmp(argv[1], "--bench-steady") == 0) {
        steady_loops = atoi(argv[3]);
        steady_warm = atoll(argv[4]);
        if (steady_loops < 1) return 2;
        argv[1] = (char*)"--bench";
        argc = 3;
    }
    const bool udp = argc >= 3 && strcmp(argv[1], "--bench-udp") == 0;
    if (argc >= 3 && (strcmp(argv[1], "--bench") == 0 || udp)) {
        g_bench = true;
        if (udp) {
            const int rx = ::socket(AF_INET, SOCK_DGRAM, 0);
            g_udp_fd = ::socket(AF_INET, SOCK_DGRAM, 0);
            memset(&g_udp_dst, 0, sizeof(g_udp_dst));
            g_udp_dst.sin_family = AF_INET;
            g_udp_dst.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
            socklen_t al = sizeof(g_udp_dst);
            if (rx < 0 || g_udp_fd < 0 || ::bind(rx, (sockaddr*)&g_udp_dst, sizeof(g_udp_dst)) != 0 ||
                ::getsockname(rx, (sockaddr*)&g_udp_dst, &al) != 0) {
                perror("udp sink");
                return 2;
            }
        }
        argv[1] = argv[2];
        if (argc == 4) reps = atoi(argv[3]);
        argc = 3;
    }
    if (argc != 3 || reps < 1) {
        fprintf(stderr, "usage: %s trace.edtr capture.edcp | --bench[-udp] trace.edtr [repeat]\n", argv[0]);
        return 2;
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 2; }
    Reader r;
    fseek(f, 0, SEEK_END); r.d.resize(ftell(f)); fseek(f, 0, SEEK_SET);
    if (fread(r.d.data(), 1, r.d.size(), f) != r.d.size()) { perror("read"); return 2; }
    fclose(f);
    if (memcmp(&r.d[0], "EDTR", 4) != 0) { fprintf(stderr, "bad magic\n"); return 2; }
    r.p = 4;
    UInt32 version = r.get<UInt32>();
    if (version < 1 || version > 4) { fprintf(stderr, "bad version\n"); return 2; }

    static NoopAssert logger;
    SetAssertLogger(&logger);
    g_no_refresh = getenv("EDGPU_REPLAY_NO_REFRESH") && atoi(getenv("EDGPU_REPLAY_NO_REFRESH")) != 0;
    if (const char* lp = getenv("EDGPU_KEEPALIVE_LOG")) {
        if (!(g_ka_log = fopen(lp, "w"))) { perror(lp); return 2; }
    }
    g_gate = getenv("EDTR_SERVER_GATE") && atoi(getenv("EDTR_SERVER_GATE")) != 0;

    static QTSS_Callbacks cbs;
    for (int i = 0; i < kLastCallback; i++) cbs.addr[i] = (QTSS_CallbackProcPtr)cb_fail;
    cbs.addr[kMillisecondsCallback]        = (QTSS_CallbackProcPtr)cb_milliseconds;
    cbs.addr[kAddStaticAttributeCallback]  = (QTSS_CallbackProcPtr)cb_ok;
    cbs.addr[kIDForTagCallback]            = (QTSS_CallbackProcPtr)cb_id_for_tag;
    cbs.addr[kGetAttributePtrByIDCallback] = (QTSS_CallbackProcPtr)cb_get_value_ptr;
    cbs.addr[kGetAttributeByIDCallback]    = (QTSS_CallbackProcPtr)cb_get_value;
    cbs.addr[kSetAttributeByIDCallback]    = (QTSS_CallbackProcPtr)cb_set_value;
    cbs.addr[kWriteCallback]               = (QTSS_CallbackProcPtr)cb_write;
    cbs.addr[kRefreshTimeOutCallback]      = (QTSS_CallbackProcPtr)cb_refresh_timeout;
    cbs.addr[kLockObjectCallback]          = (QTSS_CallbackProcPtr)cb_ok;
    cbs.addr[kUnlockObjectCallback]        = (QTSS_CallbackProcPtr)cb_ok;
    cbs.addr[kTeardownCallback]            = (QTSS_CallbackProcPtr)cb_teardown;
    cbs.addr[kGetAttrInfoByNameCallback]   = (QTSS_CallbackProcPtr)cb_attr_info_by_name;
    cbs.addr[kGetNumValuesCallback]        = (QTSS_CallbackProcPtr)cb_num_values;
    cbs.addr[kGetValueAsStringCallback]    = (QTSS_CallbackProcPtr)cb_value_as_string;
    QTSS_PrivateArgs args;
    memset(&args, 0, sizeof(args));
    args.inServerAPIVersion = QTSS_API_VERSION;
    args.inCallbacks = &cbs;
    extern QTSS_Error _stublibrary_main(void*, QTSS_DispatchFuncPtr);
    _stublibrary_main(&args, NULL);

    // Register role work the module does (QTSSReflectorModule.cpp:265-365 subset).
    ReflectorStream::Register();
    RTPSessionOutput::Register();
    (void)QTSS_IDForAttr(qtssRTPStreamObjectType, "qtssReflectorModuleStreamCookie", &g_cookie_attr);
    g_mod_prefs = new_obj();
    g_srv_prefs = new_obj();
    // the trace's prefs (version 4: after the sessions); peek past the sessions for them
    std::map<std::string, std::string> trace_prefs;
    {
        size_t q = r.p;
        UInt32 ns; memcpy(&ns, &r.d[q], 4); q += 4;
        for (UInt32 s = 0; s < ns; s++) { UInt32 l; memcpy(&l, &r.d[q], 4); q += 4 + l + (version >= 2 ? 1 : 0); }
        if (version >= 4) {
            UInt32 l; memcpy(&l, &r.d[q], 4);
            trace_prefs = parse_prefs(std::string((const char*)&r.d[q + 4], l));
        }
    }
    std::map<std::string, std::string> eff;
    for (auto& d : kPrefDefaults) eff[d[0]] = d[1];
    for (auto& kv : trace_prefs) {
        if (!eff.count(kv.first)) { fprintf(stderr, "unknown pref %s\n", kv.first.c_str()); return 2; }
    }
    // the server's player list is always present (the shipped easydarwin.xml's LIST-PREF);
    // module prefs the trace does not name are missing from the prefs object
    trace_prefs.emplace("player_requires_rtp_header_info", eff["player_requires_rtp_header_info"]);
    load_prefs(trace_prefs);
    ReflectorStream::Initialize((QTSS_ModulePrefsObject)g_mod_prefs);   // ReflectorStream.cpp:87-117
    reread_prefs();

    // The replay; bench mode repeats it with fresh sessions, subscribers and clock each pass.
    const size_t p0 = r.p;
    std::vector<Sub> subs;
    double bench_secs = 0;
    UInt64 pkts_at_warm = 0, bytes_at_warm = 0;        // --bench-steady: the counters when the window began
    for (int rep = 0; rep < reps; rep++) {
    r.p = p0;
    g_now = 0;
    g_rand_calls = 0;
    g_reports.clear();
    g_rtcp_sockets.clear();
    subs.clear();
    // Sessions: every one is set up and has its pusher at time 0.
    UInt32 nsess = r.get<UInt32>();
    std::vector<std::string> sdps(nsess);
    std::vector<UInt8> sflags(nsess, 0);
    for (UInt32 s = 0; s < nsess; s++) {
        UInt32 sdplen = r.get<UInt32>();
        sdps[s].assign((const char*)&r.d[r.p], sdplen);
        r.p += sdplen;
        sflags[s] = version >= 2 ? r.get<UInt8>() : 0;
    }
    if (version >= 4) { const UInt32 l = r.get<UInt32>(); r.p += l; }   // the prefs, read above
    // each track's media (SDPSourceInfo: m= lines in order; qtssRTPStrPayloadType, QRM:1732-1765)
    std::vector<std::vector<bool>> media_video(nsess);
    for (UInt32 s = 0; s < nsess; s++)
        for (size_t q = 0; (q = sdps[s].find("m=", q)) != std::string::npos; q += 2)
            if (q == 0 || sdps[s][q - 1] == '\n') media_video[s].push_back(sdps[s].compare(q, 7, "m=video") == 0);
    OSRefTable sessionMap;                         // sSessionMap (QTSSReflectorModule.cpp:89)
    std::vector<Live> live(nsess);
    // a pusher connection's client session (ordinal live[s].pubs), its `setups` SETUPs' timeout
    auto new_pusher = [&](UInt32 s, UInt32 setups) {
        FakeObj* b = new_obj();
        b->push_s = (int)s;
        b->push_k = live[s].pubs++;
        b->to_ms = (SInt64)g_mp.broadcasterTimeoutSecs * 1000;
        b->deadline = g_now + b->to_ms;
        for (UInt32 k = 0; k < setups; k++) ka_log('S', g_now, b, (" " + std::to_string(b->to_ms)).c_str());
        return b;
    };
    // AddBroadcasterClientSession (QTSSReflectorModule.cpp:1715): the sockets refresh this pusher
    auto name_pusher = [&](ReflectorSession* sess, FakeObj* b) {
        QTSS_StandardRTSP_Params bp;
        memset(&bp, 0, sizeof(bp));
        bp.inClientSession = (QTSS_ClientSessionObject)b;
        sess->AddBroadcasterClientSession(&bp);
    };
    // FindOrCreateSession's create branch for a push (QTSSReflectorModule.cpp:1391-1478):
    // SDPSourceInfo -> ReflectorSession -> SetupReflectorSession(kMarkSetup|kIsPushSession),
    // Register + Resolve (the pusher's reference)
    auto create = [&](UInt32 s) -> bool {
        const std::string& sdp = sdps[s];
        char* sdpbuf = new char[sdp.size() + 1];
        memcpy(sdpbuf, sdp.data(), sdp.size()); sdpbuf[sdp.size()] = 0;
        SDPSourceInfo* info = new SDPSourceInfo(sdpbuf, (UInt32)sdp.size());
        char name[64];
        snprintf(name, sizeof(name), "live/stream%u.sdp", s);
        StrPtrLen nm(name);
        ReflectorSession* sess = new ReflectorSession(&nm, 1, NULL);
        sess->SetHasBufferedStreams(true);
        FakeObj* req = new_obj();
        UInt32 tcp = qtssRTPTransportTypeTCP;
        set_value(req, qtssRTSPReqTransportType, 0, &tcp, sizeof(tcp));
        FakeObj* bcast = new_pusher(s, 0);
        QTSS_StandardRTSP_Params params;
        memset(&params, 0, sizeof(params));
        params.inRTSPRequest = (QTSS_RTSPRequestObject)req;
        params.inClientSession = (QTSS_ClientSessionObject)bcast;
        QTSS_Error err = sess->SetupReflectorSession(info, &params,
            ReflectorSession::kMarkSetup | ReflectorSession::kIsPushSession, g_mp.oneSSRC, g_mp.timeoutSSRC);
        if (err != QTSS_NoErr) { fprintf(stderr, "setup failed %d\n", (int)err); return false; }
        if (sessionMap.Register(sess->GetRef()) != OS_NoErr) { fprintf(stderr, "register failed\n"); return false; }
        if (sessionMap.Resolve(sess->GetRef()->GetString()) != sess->GetRef()) { fprintf(stderr, "resolve failed\n"); return false; }
        for (UInt32 x = 0; x < sess->GetNumStreams(); x++) {
            UDPSocketPair* pr = sess->GetStreamByIndex(x)->GetSocketPair();
            g_rtcp_sockets[pr->GetSocketB()] = std::make_pair(s, (UInt16)x);
            if (!(sflags[s] & 1)) continue;
            // UDP push: bind the pair to an even/odd loopback port pair
            if (pr->GetSocketA()->Open() != OS_NoErr || pr->GetSocketB()->Open() != OS_NoErr) {
                fprintf(stderr, "socket open failed\n"); return false;
            }
            static UInt16 port = 41000;
            bool bound = false;
            for (int tries = 0; tries < 2000 && !bound; tries++, port += 2)
                bound = pr->GetSocketA()->Bind(INADDR_LOOPBACK, port) == OS_NoErr &&
                        pr->GetSocketB()->Bind(INADDR_LOOPBACK, port + 1) == OS_NoErr;
            if (!bound) { fprintf(stderr, "no loopback port pair\n"); return false; }
        }
        live[s].sess = sess;
        live[s].bcast = bcast;
        live[s].published = true;
        live[s].killAttr = g_mp.killClients;       // the pusher's RECORD (:1884)
        for (UInt32 x = 0; x < sess->GetNumStreams(); x++)
            ka_log('S', g_now, bcast, (" " + std::to_string(bcast->to_ms)).c_str());
        name_pusher(sess, bcast);
        return true;
    };
    for (UInt32 s = 0; s < nsess; s++)
        if (!create(s)) return 3;
    // Releases one reference of live[s]'s session; at 0 it is UnRegistered and killed
    // (RemoveOutput, QTSSReflectorModule.cpp:2162-2192; the kill event is a no-op without task
    // threads, the object is simply dropped here)
    auto release = [&](ReflectorSession* sess) {
        OSRef* ref = sess->GetRef();
        if (ref->GetRefCount() > 0) sessionMap.Release(ref);
        if (ref->GetRefCount() == 0) {
            sessionMap.UnRegister(ref);
            sess->Signal(Task::kKillEvent);
            for (Live& l : live)
                if (l.sess == sess) { l.sess = nullptr; l.published = false; }
        }
    };
    // DestroySession's player branch -> RemoveOutput(output, session, false): out of every
    // track's bucket (ReflectorSession::RemoveOutput(output, true)), delete, release
    auto remove_output = [&](Sub& sb) {
        if (sb.output == NULL) return;
        sb.rsess->RemoveOutput(sb.output, true);
        delete sb.output;
        sb.output = NULL;
        release(sb.rsess);
    };

    // the pusher of s leaves (UNPUBLISH, or its timeout): DestroySession, broadcaster branch
    // (QTSSReflectorModule.cpp:2082-2109), then RemoveOutput(NULL, session, kill) (:2133-2196)
    auto unpublish = [&](UInt32 s, bool kill) {
        ReflectorSession* sess = live[s].sess;
        live[s].published = false;
        SourceInfo* info = sess->GetSourceInfo();
        for (UInt32 x = 0; info != NULL && x < info->GetNumStreams(); x++)
            if (info->GetStreamInfo(x) != NULL) info->GetStreamInfo(x)->fSetupToReceive = false;
        sess->RemoveSessionFromOutput((QTSS_ClientSessionObject)live[s].bcast);
        g_torn_down.clear();
        if (kill || live[s].killAttr || g_mp.killClients) sess->TearDownAllOutputs();
        std::vector<void*> closing = g_torn_down;
        release(sess);
        // the server closes every torn-down client session: ClientSessionClosing
        for (auto& sb : subs)
            if (sb.output != NULL && sb.rsess == sess &&
                std::find(closing.begin(), closing.end(), (void*)sb.client) != closing.end())
                remove_output(sb);
    };

    std::vector<char> pktbuf(70000);
    const auto t_start = std::chrono::steady_clock::now();
    const size_t ev0 = r.p;
    SInt64 loop_dur = 0, loop_off = 0;                 // --bench-steady: the trace's span, this loop's offset
    bool warm = steady_loops == 0;
    for (int loop = 0; loop < std::max(1, steady_loops); loop++) {
    r.p = ev0;
    loop_off = (SInt64)loop * loop_dur;
    while (!r.done()) {
        UInt8 type = r.get<UInt8>();
        if (type == 0) break;
        SInt64 t = r.get<SInt64>() + loop_off;
        if (steady_loops) {
            if (loop == 0 && type == 3) loop_dur = std::max(loop_dur, t);
            if (!warm && t >= steady_warm) {
                warm = true;
                pkts_at_warm = g_bench_pkts; bytes_at_warm = g_bench_bytes;
                g_reflect_s = g_push_s = 0; g_ticks = g_pushed = 0;
            }
            if (type != 1 && type != 2 && type != 3) {
                fprintf(stderr, "--bench-steady takes PKT / JOIN / TICK traces only\n");
                return 2;
            }
        }
        // pushers whose deadline the clock reached time out first, earliest first, at their deadline
        for (;;) {
            SInt64 best = INT64_MAX;
            UInt32 bs = 0;
            for (UInt32 s = 0; s < nsess; s++)
                if (live[s].published && live[s].bcast->deadline > 0 && live[s].bcast->deadline <= t &&
                    live[s].bcast->deadline < best) { best = live[s].bcast->deadline; bs = s; }
            if (best == INT64_MAX) break;
            if (best > g_now) g_now = best;
            ka_log('X', best, live[bs].bcast);
            unpublish(bs, false);
        }
        if (t > g_now) g_now = t;
        if (type == 1) {            // PKT
            UInt32 s = r.get<UInt32>();
            UInt8 ch = r.get<UInt8>();
            UInt32 len = r.get<UInt32>();
            memcpy(pktbuf.data(), &r.d[r.p], len);
            r.p += len;
            if (!live[s].published) continue;             // no pusher connection carries it
            ReflectorSession* sess = live[s].sess;
            if (live[s].bcast->deadline) live[s].bcast->deadline = g_now + live[s].bcast->to_ms;   // RTSPSession.cpp:2157
            UInt32 idx = ch / 2;
            if (idx < sess->GetNumStreams()) {
                const auto a = g_bench ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
                sess->GetStreamByIndex(idx)->PushPacket(pktbuf.data(), len, (ch & 1) != 0);
                if (g_bench) {
                    g_push_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
                    g_pushed++;
                }
            }
        } else if (type == 2) {     // JOIN
            UInt32 s = r.get<UInt32>();
            UInt32 sub_id = r.get<UInt32>();
            UInt8 transport = r.get<UInt8>();
            UInt8 uaflags = r.get<UInt8>();
            if (steady_loops && loop > 0) continue;       // the players joined once, in the first loop
            ReflectorSession* sess = live[s].sess;
            if (sess == nullptr) continue;                // no such session: the player's SETUP fails
            // RTP-Info player (ua_flags bit 0: the kRequiresRTPInfoSeqAndTime profile, UA
            // "Android"/"vlc"): DoPlay's rtpInfoEnabled branch (QTSSReflectorModule.cpp:
            // 1971-2004) runs HaveStreamBuffers (:1804-1865) with the reference's own
            // HasFirstRTP / GetFirstPacketInfo; when a stream has nothing buffered the PLAY
            // is deferred (idle-timer retry), which this trace model drops as a join.
            std::vector<UInt16> firstSeq(sess->GetNumStreams(), 0);
            // DoPlay's rtpInfoEnabled (QTSSReflectorModule.cpp:1962-1969) for the player's user agent
            FakeObj* client = new_obj();
            const char* ua = kUserAgents[uaflags & 1];
            set_value(client, qtssCliSesFirstUserAgent, 0, ua, (UInt32)strlen(ua));
            if (g_gate) {
                // the RTPSession's window (RTPSessionInterface.cpp:131), overbuffering off for a
                // player without x-dynamic-rate (QTSSReflectorModule.cpp:1772-1777), the TCP
                // streams' SetWindowSize(kUInt32_Max) (RTPStream.cpp:466-469); PLAY now (RTPSession::Play)
                client->window = new RTPOverbufferWindow(50, kUInt32_Max, 25, 2.0f);
                client->window->TurnOffOverbuffering();
                if (transport) client->window->SetWindowSize(kUInt32_Max);
                client->play_time = g_now;
            }
            QTSS_StandardRTSP_Params pp;
            memset(&pp, 0, sizeof(pp));
            pp.inClientSession = (QTSS_ClientSessionObject)client;
            bool rtpInfo = false;
            if (g_mp.playerCompat)
                rtpInfo = QTSSModuleUtils::HavePlayerProfile((QTSS_PrefsObject)g_srv_prefs, &pp,
                                                             QTSSModuleUtils::kRequiresRTPInfoSeqAndTime);
            if (g_mp.forceRTPInfo) rtpInfo = true;
            if (g_mp.rtpInfoDisabled) rtpInfo = false;
            if (rtpInfo) {
                bool have = true;
                for (UInt32 x = 0; x < sess->GetNumStreams() && have; x++) {
                    ReflectorStream* rs = sess->GetStreamByIndex(x);
                    UInt32 ts = 0; SInt64 arr = 0;
                    have = rs != NULL && rs->HasFirstRTP() &&
                           rs->GetRTPSender()->GetFirstPacketInfo(&firstSeq[x], &ts, &arr);
                }
                if (!have) continue;
            }
            // the player's reference (FindOrCreateSession's Resolve, :1388)
            if (sessionMap.Resolve(sess->GetRef()->GetString()) != sess->GetRef()) {
                fprintf(stderr, "resolve failed\n"); return 3;
            }
            Sub sb;
            sb.id = sub_id; sb.session = s; sb.rsess = sess;
            sb.client = client;
            UInt32 nstreams = sess->GetNumStreams();
            for (UInt32 x = 0; x < nstreams; x++) {
                FakeObj* st = new_obj();
                st->is_stream = true;
                st->sub_id = sub_id; st->session = s; st->track = x;
                st->transport = transport ? qtssRTPTransportTypeTCP : qtssRTPTransportTypeUDP;
                st->rtp_channel = 2 * x; st->rtcp_channel = 2 * x + 1;   // RTPStream.cpp:472-473
                st->client = client;
                st->video = x < media_video[s].size() && media_video[s][x];
                void* cookie = sess->GetStreamByIndex(x)->GetStreamCookie();
                set_value(st, g_cookie_attr, 0, &cookie, sizeof(cookie));
                set_value(st, qtssRTPStrTransportType, 0, &st->transport, sizeof(UInt32));
                set_value(st, qtssRTPStrFirstSeqNumber, 0, &firstSeq[x], sizeof(UInt16));
                QTSS_RTPStreamObject so = (QTSS_RTPStreamObject)st;
                set_value(sb.client, qtssCliSesStreamObjects, x, &so, sizeof(so));
                sb.streams.push_back(st);
            }
            sb.output = new RTPSessionOutput((QTSS_ClientSessionObject)sb.client, sess, NULL, g_cookie_attr);
            sess->AddOutput(sb.output, true);
            sb.output->InitializeStreams();
            QTSS_RTPSessionState playing = qtssPlayingState;
            set_value(sb.client, qtssCliSesState, 0, &playing, sizeof(playing));
            subs.push_back(sb);
        } else if (type == 3) {     // TICK
            const auto a = std::chrono::steady_clock::now();
            const UInt64 before = g_bench_pkts;
            for (UInt32 s = 0; s < nsess; s++) {
                ReflectorSession* sess = live[s].sess;
                if (sess == nullptr) continue;
                for (UInt32 x = 0; x < sess->GetNumStreams(); x++) reflect_stream(sess->GetStreamByIndex(x));
            }
            if (g_bench) {
                g_reflect_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
                g_ticks++;
                (void)before;
            }
            if (!g_bench) for (auto& o : g_objs) o->budget[0] = o->budget[1] = -1;
        } else if (type == 5) {     // UPKT: a datagram read by ReflectorSocket::GetIncomingData
            UInt32 s = r.get<UInt32>();
            UInt8 ch = r.get<UInt8>();
            UInt32 addr = r.get<UInt32>();
            UInt16 port = r.get<UInt16>();
            UInt32 len = r.get<UInt32>();
            memcpy(pktbuf.data(), &r.d[r.p], len);
            r.p += len;
            if (!live[s].published) continue;             // the pusher is gone
            ReflectorSession* sess = live[s].sess;
            UInt32 idx = ch / 2;
            // an empty read is GetIncomingData's "no more data" (ProcessPacket then re-arms the
            // socket's event), not a datagram: traces carry none
            if (idx >= sess->GetNumStreams() || len == 0) continue;
            UDPSocketPair* pr = sess->GetStreamByIndex(idx)->GetSocketPair();
            ReflectorSocket* so = (ReflectorSocket*)((ch & 1) ? pr->GetSocketB() : pr->GetSocketA());
            ReflectorPacket* pk = so->GetPacket();
            if (pk == NULL) continue;
            // RecvFrom into the packet's kMaxReflectorPacketSize (2060, private) buffer
            // truncates the datagram; SetPacketData stores the same bytes (at exactly 2060 it
            // logs its '>' assert, which the harness's logger counts and ignores)
            const UInt32 n = std::min<UInt32>(len, 2060u);
            pk->SetPacketData(pktbuf.data(), n);
            OSMutexLocker locker(so->GetDemuxer()->GetMutex());
            so->ProcessPacket(g_now, pk, addr, port);
        } else if (type == 6) {     // LEAVE
            UInt32 sub_id = r.get<UInt32>();
            for (auto& sb : subs)
                if (sb.id == sub_id && sb.output != NULL) remove_output(sb);
        } else if (type == 7) {     // UNPUBLISH: the pusher's client session closes
            UInt32 s = r.get<UInt32>();
            UInt8 kill = r.get<UInt8>();
            if (!live[s].published) continue;
            unpublish(s, kill != 0);
        } else if (type == 8) {     // PUBLISH: a pusher's ANNOUNCE + SETUPs + RECORD
            UInt32 s = r.get<UInt32>();
            if (live[s].published) {                      // duplicate broadcast: refused at the first
                (void)new_pusher(s, 1);                   // SETUP, after its timeout was set (:1644, 1682)
                continue;
            }
            if (live[s].sess != nullptr) {
                // FindOrCreateSession's Resolve branch: the session is set up already
                ReflectorSession* sess = live[s].sess;
                if (sessionMap.Resolve(sess->GetRef()->GetString()) != sess->GetRef()) {
                    fprintf(stderr, "resolve failed\n"); return 3;
                }
                live[s].published = true;
                live[s].killAttr = g_mp.killClients;
                live[s].bcast = new_pusher(s, sess->GetNumStreams());
                name_pusher(sess, live[s].bcast);
            } else if (!create(s)) {
                return 3;
            }
        } else if (type == 9) {     // PREFS: the server's prefs rewritten, QTSS_RereadPrefs_Role
            const UInt32 l = r.get<UInt32>();
            std::map<std::string, std::string> over = parse_prefs(std::string((const char*)&r.d[r.p], l));
            r.p += l;
            over.emplace("player_requires_rtp_header_info", "Android,vlc");
            load_prefs(over);
            reread_prefs();             // RereadPrefs (ReflectorStream's prefs are not re-read)
        } else if (type == 4) {     // BLOCK
            UInt32 sub_id = r.get<UInt32>();
            UInt16 track = r.get<UInt16>();
            UInt8 kind = r.get<UInt8>();
            UInt32 budget = r.get<UInt32>();
            for (auto& sb : subs)
                if (sb.id == sub_id && track < sb.streams.size()) sb.streams[track]->budget[kind & 1] = budget;
        } else {
            fprintf(stderr, "bad event type %u at %zu\n", type, r.p);
            return 3;
        }
    }

    }   // steady loop
    bench_secs += std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
    }   // rep
    if (g_ka_log) fclose(g_ka_log);

    if (steady_loops) {             // the counted window only
        printf("{\"relayed_packets\": %llu, \"relayed_bytes\": %llu, \"reflect_seconds\": %.6f, \"push_seconds\": %.6f, "
               "\"pushed_packets\": %llu, \"ticks\": %llu, \"window_ms\": [%lld, %lld], \"loops\": %d}\n",
               (unsigned long long)(g_bench_pkts - pkts_at_warm), (unsigned long long)(g_bench_bytes - bytes_at_warm),
               g_reflect_s, g_push_s, (unsigned long long)g_pushed, (unsigned long long)g_ticks, (long long)steady_warm,
               (long long)g_now, steady_loops);
        return 0;
    }
    if (g_bench) {                  // the replays only: PushPacket + ReflectPackets + joins
        // reflect_seconds: the TICKs alone (ReflectPackets and, with --bench-udp, every sendto)
        printf("{\"relayed_packets\": %llu, \"relayed_bytes\": %llu, \"seconds\": %.6f, \"reflect_seconds\": %.6f, "
               "\"repeat\": %d}\n",
               (unsigned long long)g_bench_pkts, (unsigned long long)g_bench_bytes, bench_secs, g_reflect_s, reps);
        return 0;
    }

    // Capture: one record per (subscriber, track, kind), sorted by (sub, track, kind).
    FILE* o = fopen(argv[2], "wb");
    if (!o) { perror(argv[2]); return 2; }
    fwrite("EDCP", 1, 4, o);
    UInt32 nrec = 0;
    for (auto& sb : subs) nrec += (UInt32)sb.streams.size() * 2;
    fwrite(&nrec, 4, 1, o);
    std::sort(subs.begin(), subs.end(), [](const Sub& a, const Sub& b) { return a.id < b.id; });
    for (auto& sb : subs) {
        for (FakeObj* st : sb.streams) {
            for (int k = 0; k < 2; k++) {
                UInt32 u32; UInt16 u16; UInt8 u8; UInt64 u64;
                u32 = st->sub_id; fwrite(&u32, 4, 1, o);
                u32 = st->session; fwrite(&u32, 4, 1, o);
                u16 = (UInt16)st->track; fwrite(&u16, 2, 1, o);
                u8 = (UInt8)k; fwrite(&u8, 1, 1, o);
                u8 = (UInt8)(st->transport == qtssRTPTransportTypeTCP); fwrite(&u8, 1, 1, o);
                u64 = st->npk[k]; fwrite(&u64, 8, 1, o);
                u64 = st->cap[k].size(); fwrite(&u64, 8, 1, o);
                fwrite(st->cap[k].data(), 1, st->cap[k].size(), o);
            }
        }
    }
    if (!g_reports.empty()) {               // EDRR trailer: receiver reports sent to pushers
        fwrite("EDRR", 1, 4, o);
        UInt32 m = (UInt32)g_reports.size();
        fwrite(&m, 4, 1, o);
        for (auto& rr : g_reports) {
            UInt32 ln = (UInt32)rr.bytes.size();
            fwrite(&rr.t, 8, 1, o); fwrite(&rr.session, 4, 1, o); fwrite(&rr.track, 2, 1, o);
            fwrite(&rr.addr, 4, 1, o); fwrite(&rr.port, 2, 1, o); fwrite(&ln, 4, 1, o);
            fwrite(rr.bytes.data(), 1, ln, o);
        }
    }
    fclose(o);
    // EDGPU_TT_OUT=<path>: the transmit time RTPSessionOutput::WritePacket put in every accepted
    // write's QTSS_PacketStruct (RTPSessionOutput.cpp:603-608; the input of the server's
    // thinning, RTPStream::UpdateQualityLevel, and over-buffer window), in capture order:
    // "EDTT" u32 records, per record u32 n + n x i64
    if (const char* ttp = getenv("EDGPU_TT_OUT")) {
        FILE* t = fopen(ttp, "wb");
        if (!t) { perror(ttp); return 2; }
        fwrite("EDTT", 1, 4, t);
        fwrite(&nrec, 4, 1, t);
        for (auto& sb : subs)
            for (FakeObj* st : sb.streams)
                for (int k = 0; k < 2; k++) {
                    const UInt32 n = (UInt32)st->tt[k].size();
                    fwrite(&n, 4, 1, t);
                    fwrite(st->tt[k].data(), 8, n, t);
                }
        fclose(t);
    }
    fprintf(stderr, "ref_harness: %zu subs, %lu asserts logged\n", subs.size(), logger.count);
    if (g_gate) {                              // the write gate's stale drops (fStalePacketsDropped)
        unsigned long long stale = 0;
        for (auto& sb : subs)
            for (FakeObj* st : sb.streams) stale += st->stale_dropped;
        fprintf(stderr, "ref_harness: gate stale_dropped %llu\n", stale);
    }
    return 0;
}
