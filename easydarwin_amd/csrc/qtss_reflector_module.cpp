// qtss_reflector_module.cpp -- QTSSReflectorModule for EasyDarwin, backed by the MI355X relay
// engine: the drop-in for the reference module's live-relay path.
//
// The server loads it like the reference module -- QTSSReflectorModule_Main hands back the
// dispatch function (QTSSReflectorModule.cpp:228-262) -- and drives it through the same roles:
//
//   role                      reference handler (QTSSReflectorModule.cpp)   here
//   Register                  Register (:265-365)                           roles + attributes
//   Initialize / Shutdown     Initialize (:368-409) / Shutdown              engine context, tick thread
//   RTSPPreProcessor          ProcessRTSPRequest (:681-729)                 ANNOUNCE / DESCRIBE / SETUP /
//                                                                           PLAY / RECORD / PAUSE / TEARDOWN
//   RTSPIncomingData          ProcessRTPData (:604-678)                     '$' frame -> PushPacket
//   ClientSessionClosing      DestroySession (:2070-2131)                   RemoveOutput / pusher leave
//
// and writes every relayed packet back through QTSS_Write (callback 10) on the subscriber's
// RTP stream object with qtssWriteFlagsIsRTP / IsRTCP | WriteBurstBegin, exactly as
// RTPSessionOutput::WritePacket does (RTPSessionOutput.cpp:564-662); the server's
// RTPStream::Write then frames it (UDP datagram or '$' ch BE16(len), RTPStream.cpp:1048-1259).
// QTSS_WouldBlock from the server stops that sub-stream for the tick and the engine bookmarks
// the blocked packet (SendPacketsToOutput, ReflectorStream.cpp:1138-1198).
//
// What runs where: every packet-rate step (ingest parse, SSRC latch, keyframe index, fan-out
// planning and the write-many copy) runs on the GPU through the edgpu C ABI (via
// edgpu_reflector::Reflector, reflector_adapter.h); this file is RTSP-session bookkeeping.
// Reflect cadence: the reference reflects from ReflectorSocket tasks on packet arrival and
// sender wakeups (ReflectorStream.cpp:1676-1714); here a tick thread reflects every
// edgpu_tick_msec (default 20 ms), or the host calls EDGPU_QTSSReflectorModule_Tick.
//
// Preferences: read from the server's prefs objects exactly where the reference reads them --
// the QTSSReflectorModule prefs object (QTSSModuleUtils::GetModulePrefsObject) for
// ReflectorStream::Initialize's prefs at Initialize (ReflectorStream.cpp:87-117: bucket delay,
// buffer size -> over-buffer and the new-output window, relocation threshold with its 1000-ms
// floor, RTP-Info offset; they configure the engine context) and for the module prefs at
// Initialize and at every QTSS_RereadPrefs_Role (RereadPrefs, QTSSReflectorModule.cpp:454-537:
// kill_clients_when_broadcast_stops, use_one_SSRC_per_stream and timeout_stream_SSRC_secs for
// sessions set up from then on, the RTP-Info switches, disable_overbuffering), and the server's
// prefs object for the RTP-Info players list at every PLAY (HavePlayerProfile,
// QTSSModuleUtils.cpp:983-1046).  A missing pref, or one of the wrong type, takes the reference's
// default and is added to the prefs object with it, as QTSSModuleUtils::GetAttribute does
// (QTSSModuleUtils.cpp:679-721, 798-862).  Environment variables set only engine capacities and
// the tick (EDGPU_QTSS_*).
//
// Session lifecycle: reference-counted as the reference's session map does it -- the pusher
// holds one reference (FindOrCreateSession's Register + Resolve, :1469-1477), every output one
// (its first SETUP's Resolve, :1388, 1616-1622).  A pusher leaving (DestroySession's broadcaster
// branch, :2082-2109) frees its tracks for a new pusher and, with kill_clients (the client
// session's QTSSReflectorModuleTearDownClients attribute, set from the
// kill_clients_when_broadcast_stops pref at RECORD, :1884),
// tears every output down (TearDownAllOutputs -> QTSS_Teardown, whose ClientSessionClosing then
// removes it); at reference count 0 the session ends (RemoveOutput, :2162-2192): its engine
// session and rings, its UDP socket pairs and its announced SDP (CSdpCache::eraseSdpMap) go.
// A pusher of a session that players kept alive continues it as it is; after the end, the next
// pusher gets a fresh one.  A player's SETUP needs the session to exist (a pusher's SETUP made it,
// :1391-1396: an announced-only stream is not enough).
//
// Locking: `mu` guards the sessions / outputs bookkeeping and is held through a tick (the
// egress callbacks); the pushers' ingest never takes it -- RTSPIncomingData routes through
// one stripe of the route table (module session -> engine session, striped by session id) into
// one stripe of the Reflector's push path, and the UDP reader thread takes only `udpMu` -- so a
// pusher never waits for a tick, and pushers of different sessions rarely share a lock.
//
// Scope (docs/PARITY.md §4.10): RTSP-interleaved pushers (EasyPusher's default transport), UDP
// pushers and UDP / TCP players.  A UDP push SETUP binds the track's even/odd socket pair as
// ReflectorStream::BindSockets does (ReflectorStream.cpp:388-500, UDPSocketPool.cpp:81-150) and
// answers with its port (qtssRTSPReqSetUpServerPort, QTSSReflectorModule.cpp:1686-1688); a
// reader thread hands every datagram with its source address to the engine
// (ReflectorSocket::GetIncomingData -> ProcessPacket, ReflectorStream.cpp:1716-1735, 1769-1875)
// and the receiver reports go out of the track's RTCP socket (SendReceiverReport, :510-527).
// RTSPRoute / RTSPAuthorize / Easy_GetDeviceStream (redirects, access files, the CMS control
// plane) are not registered.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "qtss_module_abi.h"
#include "reflector_adapter.h"

using namespace edqtss;

namespace {

// ---- the module side of the callback table (QTSS_Private.cpp's stubs) ----------------------
QTSS_Callbacks* sCallbacks = nullptr;
QTSS_StreamRef sErrorLog = nullptr;     // the server's error log (QTSS_PrivateArgs.inErrorLogStream)

template <typename... A>
QTSS_Error cb(uint32_t index, A... args) {
    if (!sCallbacks || index >= kLastCallback || !sCallbacks->addr[index]) return QTSS_Unimplemented;
    return (sCallbacks->addr[index])(args...);
}
int64_t Milliseconds() {
    int64_t t = 0;
    if (cb(kMillisecondsCallback, &t) != QTSS_NoErr)
        t = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
    return t;
}
QTSS_Error GetValuePtr(QTSS_Object o, QTSS_AttributeID id, uint32_t idx, void** buf, uint32_t* len) {
    *buf = nullptr;
    *len = 0;
    return cb(kGetAttributePtrByIDCallback, o, id, idx, buf, len);
}
QTSS_Error GetValue(QTSS_Object o, QTSS_AttributeID id, uint32_t idx, void* buf, uint32_t* len) {
    return cb(kGetAttributeByIDCallback, o, id, idx, buf, len);
}
QTSS_Error SetValue(QTSS_Object o, QTSS_AttributeID id, uint32_t idx, const void* buf, uint32_t len) {
    return cb(kSetAttributeByIDCallback, o, id, idx, buf, len);
}
std::string GetString(QTSS_Object o, QTSS_AttributeID id) {
    void* p = nullptr;
    uint32_t n = 0;
    if (GetValuePtr(o, id, 0, &p, &n) != QTSS_NoErr || !p) return std::string();
    return std::string((const char*)p, n);
}
template <typename T>
bool GetPOD(QTSS_Object o, QTSS_AttributeID id, T* out) {
    void* p = nullptr;
    uint32_t n = 0;
    if (GetValuePtr(o, id, 0, &p, &n) != QTSS_NoErr || !p || n != sizeof(T)) return false;
    memcpy(out, p, sizeof(T));
    return true;
}

// ---- preferences (QTSSModuleUtils::GetAttribute, QTSSModuleUtils.cpp:679-721, 781-862) ------
// The attribute ID of pref `name` of type `type` in `prefs`, or false when it is missing or of
// another type (CheckAttributeDataType: the reference then recreates it with the default).
bool PrefID(QTSS_Object prefs, const char* name, uint32_t type, QTSS_AttributeID* id) {
    QTSS_Object info = nullptr;
    if (!prefs || cb(kGetAttrInfoByNameCallback, prefs, name, &info) != QTSS_NoErr || !info) return false;
    uint32_t t = qtssAttrDataTypeUnknown, n = sizeof(t);
    if (GetValue(info, qtssAttrDataType, 0, &t, &n) != QTSS_NoErr || t != type) return false;
    n = sizeof(*id);
    return GetValue(info, qtssAttrID, 0, id, &n) == QTSS_NoErr;
}
// Reads pref `name` into *out; a missing / mistyped / unreadable pref takes the default, which is
// added to the prefs object (CreateAttribute: QTSS_AddInstanceAttribute + QTSS_SetValue).
template <typename T>
void GetPref(QTSS_Object prefs, const char* name, uint32_t type, T* out, T def) {
    QTSS_AttributeID id = 0;
    uint32_t n = sizeof(T);
    if (PrefID(prefs, name, type, &id) && GetValue(prefs, id, 0, out, &n) == QTSS_NoErr && n == sizeof(T)) return;
    *out = def;
    if (!prefs) return;
    (void)cb(kAddInstanceAttributeCallback, prefs, name, (void*)nullptr, type);
    if (PrefID(prefs, name, type, &id)) (void)SetValue(prefs, id, 0, &def, sizeof(T));
}
// A value as a string (QTSS_GetValueAsString: the server new[]s it, the caller deletes it); false
// when the object holds no value there (an empty one included, QTSSDictionary.cpp:144-146).
bool ValueString(QTSS_Object o, QTSS_AttributeID id, uint32_t idx, std::string* out) {
    char* c = nullptr;
    if (!o || cb(kGetValueAsStringCallback, o, id, idx, &c) != QTSS_NoErr || !c) return false;
    out->assign(c);
    delete[] c;
    return true;
}
// A char-array pref (QTSSModuleUtils::GetStringAttribute, QTSSModuleUtils.cpp:723-768): its value,
// else the default, which is added to the prefs object.
std::string GetStringPref(QTSS_Object prefs, const char* name, const char* def) {
    QTSS_AttributeID id = 0;
    std::string v;
    if (PrefID(prefs, name, qtssAttrDataTypeCharArray, &id) && ValueString(prefs, id, 0, &v)) return v;
    if (prefs) {
        (void)cb(kAddInstanceAttributeCallback, prefs, name, (void*)nullptr, (uint32_t)qtssAttrDataTypeCharArray);
        if (PrefID(prefs, name, qtssAttrDataTypeCharArray, &id)) (void)SetValue(prefs, id, 0, def, (uint32_t)strlen(def));
    }
    return def;
}
// Every value of a list pref, as QTSSModuleUtils::AddressInList walks it (QTSSModuleUtils.cpp:956-981)
std::vector<std::string> GetStringListPref(QTSS_Object prefs, const char* name, const char* def) {
    (void)GetStringPref(prefs, name, def);          // created with the default when missing (QRM:537)
    std::vector<std::string> out;
    QTSS_AttributeID id = 0;
    if (!PrefID(prefs, name, qtssAttrDataTypeCharArray, &id)) return {def};
    uint32_t n = 0;
    (void)cb(kGetNumValuesCallback, prefs, id, &n);
    for (uint32_t i = 0; i < n; i++) {
        std::string v;
        if (ValueString(prefs, id, i, &v)) out.push_back(v);
        else out.push_back(std::string());
    }
    return out;
}
// The error response QTSSModuleUtils::SendErrorResponse(WithMessage) sends (QTSSModuleUtils.cpp:
// 369-484) with the server's RTSP_error_message pref off, its default (QTSServerPrefs.cpp:149): the
// status, no keep-alive, the headers, an empty body.
QTSS_Error SendErrorResponse(QTSS_Object req, uint32_t status) {
    (void)SetValue(req, qtssRTSPReqStatusCode, 0, &status, sizeof(status));
    const bool no = false;
    (void)SetValue(req, qtssRTSPReqRespKeepAlive, 0, &no, sizeof(no));
    (void)cb(kSendRTSPHeadersCallback, req);
    (void)cb(kWriteCallback, req, (const void*)"", (uint32_t)0, (uint32_t*)nullptr, (uint32_t)0);
    (void)SetValue(req, qtssRTSPReqRespMsg, 0, "", (uint32_t)0);
    return QTSS_RequestFailed;
}

// ---- module state ---------------------------------------------------------------------------
// attributes the module adds (the reference's names, QTSSReflectorModule.cpp:313-346)
QTSS_AttributeID sOutputAttr, sClientBroadcastSessionAttr, sRTSPBroadcastSessionAttr, sStreamCookieAttr,
    sRequestBodyAttr, sBufferOffsetAttr, sRTPInfoWaitTimeAttr, sKillClientsEnabledAttr;

// The broadcaster keep-alive of one session's sockets (ReflectorSocket::fBroadcasterClientSession /
// fLastBroadcasterTimeOutRefresh, ReflectorStream.h:216-239): every push SETUP names the pusher's
// client session on all of the session's sockets (AddBroadcasterClientSession, ReflectorSession.cpp:
// 193-206), its leaving clears it (RemoveSessionFromOutput, :285-293), and every pushed packet --
// interleaved or a UDP datagram -- calls QTSS_RefreshTimeOut on it when its socket last did so more
// than 10 s ago (ReflectorSocket::ProcessPacket, ReflectorStream.cpp:1779-1786).  The server refreshes
// an RTSP-interleaved pusher itself on every '$' frame (RTSPSession.cpp:2157); a UDP pusher's packets
// land on the module's sockets, so without this the server times its session out.  One socket per
// track x {RTP, RTCP}; `last` is read and written under the lock of the path that carries the packet
// (the route stripe or udpMu), `client` is set under `mu`.
struct Keepalive {
    static constexpr int64_t kIntervalMs = 10000;       // kRefreshBroadcastSessionIntervalMilliSecs
    std::atomic<QTSS_Object> client{nullptr};
    std::vector<std::atomic<int64_t>> last;
    explicit Keepalive(size_t sockets) : last(sockets) { for (auto& l : last) l.store(0); }
};

struct Output;
struct Session {                        // a pushed stream ("<path>-<channel>", QRM:1384)
    uint32_t id = 0;                    // module session id (never reused; client attributes hold it)
    std::string name;
    uint32_t engine = 0;                // edgpu session
    bool udpPush = false;               // pushed over UDP: RTCP on the odd port (Q12/Q14)
    uint32_t pushers = 0;               // pushers attached (each holds a reference; > 1 only with
                                        // allow_duplicate_broadcasts)
    std::shared_ptr<Keepalive> ka;      // the sockets' broadcaster refresh
    uint32_t refs = 0;                  // the session map's reference count: pusher + outputs
    std::vector<uint32_t> trackIDs;     // a=control:trackID=N per m= line, SDP order
    std::vector<uint16_t> sdpPorts;     // the m= lines' ports (StreamInfo::fPort)
    std::vector<int> pair;              // UDP push: the track's socket pair (index into Module::udp)
    std::vector<bool> setupToReceive;   // StreamInfo::fSetupToReceive
    std::string sdp;
    std::vector<Output*> slots;         // the streams' bucket arrays: outputs in bucket order
};

// One track of a UDP push session: RTP on an even port, RTCP on the next (ReflectorSocket A/B)
struct UdpPair {
    int fd[2] = {-1, -1};               // -1 once its session ended
    uint16_t port = 0;
    uint32_t engine = 0, track = 0;     // engine session, track index
    std::shared_ptr<Keepalive> ka;      // its session's (guarded by udpMu)
};

struct Output {                         // one player (RTPSessionOutput)
    QTSS_Object client = nullptr;
    uint32_t session = 0;
    bool tcp = false;
    bool joined = false;                // engine subscriber exists (guarded by mu)
    std::atomic<bool> paused{false};
    uint32_t handle = 0;
    // per track: the RTP stream object SETUP created (or null); read by the write threads
    std::unique_ptr<std::atomic<QTSS_Object>[]> streams;
    uint32_t nstreams = 0;
    int32_t slot = -1;                  // position in the session's buckets (sBucketSize members each)
    int64_t bufferDelayMs = 0;          // RTPSessionOutput::fBufferDelayMSecs (its write thread's, once joined)
    // a teardown while a tick writes (ClientSessionClosing): `closed` stops new writes to it,
    // `writing` is held by the one write thread delivering to it (the reference's RemoveOutput
    // waits for the stream's fBucketMutex, ReflectorStream.cpp:338-362, 1051)
    std::atomic<bool> closed{false}, writing{false};
};

struct Module {
    std::mutex mu;                      // the reference's session-map / bucket mutexes, one lock here
    std::unique_ptr<edgpu_reflector::Reflector> R;
    std::map<std::string, std::string> announced;         // CSdpCache: stream name -> SDP
    std::map<std::string, uint32_t> byName;               // registered sessions: name -> id
    std::map<uint32_t, Session> sessions;                 // by module session id
    uint32_t nextId = 1;
    bool killClients = false;           // kill_clients_when_broadcast_stops (QRM:476-477)
    // the pushers' path (RTSPIncomingData): module session id -> (engine session, tracks) while a
    // pusher is attached; stripe id % kRouteStripes guards its part alone
    static constexpr uint32_t kRouteStripes = 16;
    struct Route { uint32_t engine, tracks; Keepalive* ka; };
    struct alignas(64) RouteStripe {
        std::mutex mu;
        std::map<uint32_t, Route> route;
    } routes[kRouteStripes];
    std::mutex udpMu;                   // guards `udp` (the reader thread takes only this)
    std::vector<std::unique_ptr<Output>> outputs;
    // The tick's writes run without `mu` (and without the engine lock, SetConcurrentDelivery): they
    // find an output by its engine handle in a table read without a lock -- chunks of 4096 entries,
    // set under `mu` -- and an output removed meanwhile stays allocated until every tick that may
    // have read it has ended (graveyard, by the tick sequence at removal).
    static constexpr uint32_t kChunkBits = 12, kChunk = 1u << kChunkBits, kChunks = 1u << 16;
    std::unique_ptr<std::atomic<std::atomic<Output*>*>[]> handleChunks{new std::atomic<std::atomic<Output*>*>[kChunks]};
    uint64_t tickSeq = 0;                                              // ticks started (under mu)
    std::vector<std::pair<uint64_t, std::unique_ptr<Output>>> graveyard;
    std::mutex tickMu;                  // one tick at a time (the ticker and EDGPU_QTSSReflectorModule_Tick)
    int32_t rtpInfoWaitLoops = 10;      // sWaitTimeLoopCount: 100-ms PLAY retries before 404
    uint32_t tickMs = 20;
    // EDGPU_QTSS_REFLECT_ON_ARRIVAL=<ms> (default 2): reflect as soon as packets are waiting, at
    // most every <ms> (the reference reflects a sender when its socket task wakes on new packets,
    // ReflectorStream.cpp:573, 603-618, 1676-1714); tickMs stays the longest interval.  0: a tick
    // every tickMs.  At C2's real rate: 4.3 ms mean RTSPIncomingData -> QTSS_Write latency against
    // 12.9 ms with 20-ms ticks, the same throughput.
    uint32_t arrivalMinMs = 2;
    std::atomic<bool> pending{false};   // a packet arrived since the last tick took the batch
    std::mutex wakeMu;
    std::condition_variable wake;
    // ReflectorStream::Initialize's prefs (read once, at Initialize)
    int64_t overBufferMs = 1000;        // sOverBufferInMsec (reflector_buffer_size_sec x 1000)
    int64_t bucketDelayMs = 73;         // sBucketDelayInMsec (reflector_bucket_offset_delay_msec)
    uint32_t bucketSize = 16;           // ReflectorStream::sBucketSize
    // RereadPrefs' module prefs (Initialize and QTSS_RereadPrefs_Role; guarded by mu)
    bool oneSSRC = true;                // use_one_SSRC_per_stream (sessions set up from now on)
    uint32_t timeoutSSRC = 30;          // timeout_stream_SSRC_secs
    bool rtpInfoDisabled = false;       // disable_rtp_play_info
    bool playerCompat = true;           // enable_player_compatibility
    bool forceRTPInfo = false;          // force_rtp_info_sequence_and_time
    bool disableOverbuffering = false;  // disable_overbuffering
    bool announceEnabled = true;        // enable_broadcast_announce (DoAnnounce, QRM:900)
    std::atomic<bool> pushEnabled{true};   // enable_broadcast_push (ProcessRTPData, QRM:606; read without mu)
    bool allowDuplicates = false;       // allow_duplicate_broadcasts (DoSetup, QRM:1682)
    uint32_t broadcasterTimeoutMs = 30000;  // max(30, timeout_broadcaster_session_secs) x 1000 (QRM:483-487, 541)
    // access (RTSPAuthorize, RTSPRoute, AllowBroadcast; QRM:489-538)
    bool allowBroadcasts = true;        // allow_broadcasts (sReflectBroadcasts)
    bool authLocal = false;             // authenticate_local_broadcast
    bool allowNonSDP = true;            // allow_non_sdp_urls: a player's session by its full path
    std::string broadcasterGroup = "broadcaster";   // BroadcasterGroup
    std::string redirectKeyword;        // redirect_broadcast_keyword, trimmed (GetTrimmedKeyWord)
    std::string redirectDir;            // redirect_broadcasts_dir, movie-folder relative (SetMoviesRelativeDir)
    std::vector<std::string> ipAllowList{"127.0.0.*"};   // ip_allow_list
    QTSS_Object modPrefs = nullptr;     // this module's prefs object
    QTSS_Object serverPrefs = nullptr;  // the server's prefs object (player_requires_rtp_header_info)
    uint64_t rereads = 0;
    bool manualTick = false;
    std::vector<UdpPair> udp;
    std::thread ticker, reader;
    std::atomic<bool> stop{false};
    QTSS_Error tickErr = QTSS_NoErr;
    EDGPU_QTSSTickInfo lastTick{};      // guarded by mu
    std::vector<uint32_t> orphans;      // engine sessions whose removal the engine refused: retried per tick
    // GPU watchdog: a tick the engine's watchdog ended (EDGPU_TIMEOUT) tears every player down and
    // SETUPs are refused (503) until a tick succeeds again; EDGPU_QTSS_WATCHDOG_MS (default 2000)
    std::atomic<bool> gpuStalled{false};
    uint64_t stallTick = 0, stallUs = 0;  // EDGPU_QTSS_TEST_STALL=<tick>:<ms>: a stall before that tick (tests)
};
Module* M = nullptr;

Output* OutputOf(uint32_t h) {
    if ((h >> Module::kChunkBits) >= Module::kChunks) return nullptr;
    std::atomic<Output*>* c = M->handleChunks[h >> Module::kChunkBits].load(std::memory_order_acquire);
    return c ? c[h & (Module::kChunk - 1)].load(std::memory_order_acquire) : nullptr;
}
// Caller holds mu.
void SetOutputOf(uint32_t h, Output* o) {
    if ((h >> Module::kChunkBits) >= Module::kChunks) {
        fprintf(stderr, "QTSSReflectorModule: subscriber handle %u past the handle table\n", h);
        return;
    }
    std::atomic<std::atomic<Output*>*>& slot = M->handleChunks[h >> Module::kChunkBits];
    std::atomic<Output*>* c = slot.load(std::memory_order_acquire);
    if (!c) {
        c = new std::atomic<Output*>[Module::kChunk];
        for (uint32_t i = 0; i < Module::kChunk; i++) c[i].store(nullptr, std::memory_order_relaxed);
        slot.store(c, std::memory_order_release);
    }
    c[h & (Module::kChunk - 1)].store(o, std::memory_order_release);
}

// The channel of a request: the first "channel" parameter (any case) of the URL-decoded query
// string, 1 without one (DoSessionSetup / DoAnnounce, QRM:740-756 / 919-935: EasyUtil::Urldecode,
// '%XX' and '+' -> ' ', then QueryParamList::BulidList's name=value parse, QueryParamList.cpp:64-103,
// and DoFindCGIValueForParam's case-insensitive lookup of EASY_TAG_CHANNEL "Channel")
uint32_t ChannelOf(const std::string& query) {
    std::string q;
    for (size_t i = 0; i < query.size(); i++) {
        if (query[i] == '%' && i + 2 < query.size()) {
            auto hex = [](char c) { return c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10; };
            q += (char)((hex(query[i + 1]) << 4) | hex(query[i + 2]));
            i += 2;
        } else {
            q += query[i] == '+' ? ' ' : query[i];
        }
    }
    for (size_t i = 0; i < q.size();) {
        const size_t eq = q.find('=', i);
        if (eq == std::string::npos) break;                     // a name with no '=': the parse ends
        std::string name = q.substr(i, eq - i), value;
        size_t j = eq + 1;
        if (j < q.size() && q[j] == '"') {                      // a quoted value
            const size_t close = q.find('"', j + 1);
            value = q.substr(j + 1, (close == std::string::npos ? q.size() : close) - j - 1);
            j = close == std::string::npos ? q.size() : q.find('&', close + 1);
        } else {
            const size_t amp = q.find('&', j);
            value = q.substr(j, (amp == std::string::npos ? q.size() : amp) - j);
            j = amp;
        }
        std::string lower = name;
        for (char& c : lower) c = (char)tolower((unsigned char)c);
        if (lower == "channel") return (uint32_t)atoi(value.c_str());
        if (j == std::string::npos) break;
        i = j + 1;
    }
    return 1;
}

// "<file name>-<channel>", the reference's stream name (theStreamName, QRM:937-938 / 1383-1384):
// the server's qtssRTSPReqFileName is the path's FIRST component (RTSPRequestInterface::GetFileName,
// RTSPRequestInterface.cpp:681-711), and the player's lookup path is the same name (GetFullPath with
// EasyDarwin's empty root directory, RTSPRequestInterface.cpp:219-224)
std::string StreamName(QTSS_Object req) {
    return GetString(req, qtssRTSPReqFileName) + "-" + std::to_string(ChannelOf(GetString(req, qtssRTSPReqQueryString)));
}
// A player's stream name (DoSessionSetup with allow_non_sdp_urls, QRM:769-793): the full path,
// QTSSModuleUtils::GetFullPath (QTSSModuleUtils.cpp:228-285) = the request's root directory + its
// file name -- the file name alone unless an RTSPRoute module set a root (RedirectBroadcast)
std::string PlayerStreamName(QTSS_Object req, bool allowNonSDP) {
    if (!allowNonSDP) return StreamName(req);
    std::string root = GetString(req, qtssRTSPReqRootDir), file = GetString(req, qtssRTSPReqFileName);
    if (!root.empty() && root.back() == '/')
        while (!file.empty() && file[0] == '/') file.erase(0, 1);
    return root + file + "-" + std::to_string(ChannelOf(GetString(req, qtssRTSPReqQueryString)));
}

// a first SETUP the reflector does not take: an empty file name, or a ".mov" (DoSessionSetup,
// QRM:758-767, 805-818)
bool NotReflected(QTSS_Object req) {
    const std::string n = GetString(req, qtssRTSPReqFileName);
    return n.empty() || (n.size() > 4 && n.compare(n.size() - 4, 4, ".mov") == 0);
}

uint32_t TrackFromRequest(QTSS_Object req, bool* ok) {
    const std::string digits = GetString(req, qtssRTSPReqFileDigit);
    *ok = !digits.empty();
    return (uint32_t)strtoul(digits.c_str(), nullptr, 10);
}

// each track's trackID as SDPSourceInfo::Parse assigns it (a=control, else the position;
// GetStreamInfoByTrackID, SourceInfo.cpp) -- the engine's parse, edgpu_sdp_parse
std::vector<uint32_t> SdpTrackIDs(const std::string& sdp) {
    std::vector<edgpu_sdp_track> t(64);
    uint32_t n = 0;
    if (edgpu_sdp_parse(sdp.data(), (uint32_t)sdp.size(), t.data(), (uint32_t)t.size(), &n) != 0) return {};
    std::vector<uint32_t> ids(n);
    for (uint32_t i = 0; i < n; i++) ids[i] = t[i].track_id;
    return ids;
}

// each m= line's port (SDPSourceInfo::Parse reads it into StreamInfo::fPort,
// SDPSourceInfo.cpp:260-353); 0 when absent
std::vector<uint16_t> SdpPorts(const std::string& sdp) {
    std::vector<uint16_t> ports;
    for (size_t k = 0; k < sdp.size();) {
        const size_t e = std::min(sdp.find_first_of("\r\n", k), sdp.size());
        if (sdp.compare(k, 2, "m=") == 0) {
            const size_t sp = sdp.find(' ', k);
            ports.push_back(sp < e ? (uint16_t)strtoul(sdp.c_str() + sp + 1, nullptr, 10) : (uint16_t)0);
        }
        k = e + 1;
    }
    return ports;
}

int TrackIndex(const Session& s, uint32_t trackID) {
    for (size_t i = 0; i < s.trackIDs.size(); i++)
        if (s.trackIDs[i] == trackID) return (int)i;
    return -1;
}

// ---- the egress seam: RTPSessionOutput::WritePacket -> QTSS_Write ---------------------------
class QTSSSink : public edgpu_reflector::OutputSink {
public:
    int64_t now = 0;
    std::map<uint32_t, int32_t> firstNewSlot;      // per sender: bucket position of its first new output
    bool WantsArrivals() const override { return true; }
    // ReflectPackets sets `firstPacket` at the first output (in bucket order) without a bookmark
    // and never clears it for the rest of that sender's outputs (ReflectorStream.cpp:1086-1104)
    void BeginTick(const edgpu_substream_out* subs, uint32_t n) override {
        firstNewSlot.clear();
        for (uint32_t i = 0; i < n; i++) {
            if (!(subs[i].flags & EDGPU_SUB_NEW)) continue;
            const Output* o = OutputOf(subs[i].subscriber);
            if (!o || o->slot < 0) continue;
            auto f = firstNewSlot.find(subs[i].sender);
            if (f == firstNewSlot.end() || o->slot < f->second) firstNewSlot[subs[i].sender] = o->slot;
        }
    }
    int WritePacket(uint32_t, uint16_t, bool, bool, const uint8_t*, uint32_t, uint32_t) override {
        return edgpu_reflector::kRequestFailed;                  // Write() below is the entry point
    }
    // A sub-stream's packets come consecutively: the output and first-new slot found for the
    // last write serve the next ones (a tick writes millions of packets at fleet scale).  One
    // cache per write thread; the tables they read are not modified during the write phase.
    struct alignas(64) Cache {
        uint32_t lastHandle = 0xFFFFFFFFu, lastSender = 0xFFFFFFFFu;
        Output* lastOut = nullptr;
        int32_t lastFirst = -1;
        bool lastHasFirst = false;
    };
    Cache cache[64];
    // The write thread moves on from output `c.lastOut` (or ends its writes): the output's teardown
    // may proceed (it waits for `writing` to drop).
    static void Leave(Cache& c) {
        if (c.lastOut) c.lastOut->writing.store(false, std::memory_order_release);
        c.lastOut = nullptr;
        c.lastHandle = 0xFFFFFFFFu;
    }
    void EndWrites(uint32_t worker) override { Leave(cache[worker & 63]); }
    int Write(const edgpu_reflector::PacketWrite& w) override {
        Cache& c = cache[w.worker & 63];
        uint32_t& lastSender = c.lastSender;
        int32_t& lastFirst = c.lastFirst;
        bool& lastHasFirst = c.lastHasFirst;
        if (w.subscriber != c.lastHandle) {
            Leave(c);
            c.lastHandle = w.subscriber;
            Output* o = OutputOf(w.subscriber);
            if (o) {
                // hold it, then check it is still an output (a teardown sets `closed`, then waits)
                o->writing.store(true, std::memory_order_seq_cst);
                if (o->closed.load(std::memory_order_seq_cst)) o->writing.store(false, std::memory_order_release);
                else c.lastOut = o;
            }
        }
        if (!c.lastOut) {
            if (getenv("EDGPU_QTSS_DEBUG")) fprintf(stderr, "QTSSReflectorModule: write for unknown handle %u\n", w.subscriber);
            return edgpu_reflector::kNoErr;
        }
        Output& o = *c.lastOut;
        // not playing (paused): WritePacket returns QTSS_WouldBlock (RTPSessionOutput.cpp:575-579)
        if (o.paused.load(std::memory_order_relaxed)) return edgpu_reflector::kWouldBlock;
        QTSS_Object stream = w.track < o.nstreams ? o.streams[w.track].load(std::memory_order_acquire) : nullptr;
        if (!stream) {                                                                           // track not SETUP
            if (getenv("EDGPU_QTSS_DEBUG")) fprintf(stderr, "QTSSReflectorModule: handle %u track %u not set up\n", w.subscriber, w.track);
            return edgpu_reflector::kNoErr;
        }
        // the server frames interleaved packets itself (RTPStream::Write): hand it the packet
        const uint8_t* pkt = w.interleaved ? w.wire + 4 : w.wire;
        const uint32_t len = w.interleaved ? w.wireLen - 4 : w.wireLen;
        if (w.sender != lastSender) {
            const auto f = firstNewSlot.find(w.sender);
            lastSender = w.sender;
            lastHasFirst = f != firstNewSlot.end();
            lastFirst = lastHasFirst ? f->second : -1;
        }
        const bool firstPacket = lastHasFirst && o.slot >= lastFirst;
        // the transmit time (RTPSessionOutput.cpp:603-608): now - bucket delay, moved to the
        // packet's arrival + the output's buffer delay while that delay is positive
        const int64_t bucketDelay = M->bucketDelayMs * (int64_t)(o.slot < 0 ? 0 : (uint32_t)o.slot / M->bucketSize);
        QTSS_PacketStruct ps;
        ps.packetData = const_cast<uint8_t*>(pkt);
        ps.packetTransmitTime = now - bucketDelay;
        if (o.bufferDelayMs > 0) ps.packetTransmitTime += o.bufferDelayMs - (now - w.arrivalMs);
        ps.suggestedWakeupTime = -1;
        const uint32_t flags = (w.isRTCP ? qtssWriteFlagsIsRTCP : qtssWriteFlagsIsRTP) | qtssWriteFlagsWriteBurstBegin;
        const QTSS_Error err = cb(kWriteCallback, stream, (const void*)&ps, len, (uint32_t*)nullptr, flags);
        // only QTSS_WouldBlock stops SendPacketsToOutput (ReflectorStream.cpp:1158-1190); blocked
        // on a first-packet pass, the output's buffer delay becomes this packet's age (:617-622)
        if (err == QTSS_WouldBlock) {
            if (firstPacket) o.bufferDelayMs = now - w.arrivalMs;
            return edgpu_reflector::kWouldBlock;
        }
        return edgpu_reflector::kNoErr;
    }
    // ReflectorStream::SendReceiverReport (ReflectorStream.cpp:510-527): kept until the tick's
    // engine part is over, then sent by SendReports
    struct RR { uint32_t session; uint16_t track; uint32_t addr; uint16_t port; std::string bytes; };
    std::vector<RR> reports;
    void SendReceiverReport(uint32_t session, uint16_t track, uint32_t addr, uint16_t port, const uint8_t* rr,
                            uint32_t len) override {
        reports.push_back(RR{session, track, addr, port, std::string((const char*)rr, len)});
    }
    // from the track's RTCP socket to the pusher's RTCP address; the send result is ignored, as
    // there.  Caller holds mu.
    void SendReports() {
        for (const RR& r : reports)
            for (const auto& kv : M->sessions) {
                const Session& s = kv.second;
                if (s.engine != r.session || r.track >= s.pair.size() || s.pair[r.track] < 0) continue;
                sockaddr_in to;
                memset(&to, 0, sizeof(to));
                to.sin_family = AF_INET;
                to.sin_addr.s_addr = htonl(r.addr);
                to.sin_port = htons(r.port);
                std::lock_guard<std::mutex> g(M->udpMu);
                const int fd = M->udp[s.pair[r.track]].fd[1];
                if (fd >= 0) (void)sendto(fd, r.bytes.data(), r.bytes.size(), MSG_NOSIGNAL, (const sockaddr*)&to, sizeof(to));
                break;
            }
        reports.clear();
    }
};

// ---- UDP push sockets -----------------------------------------------------------------------
// A socket pair on INADDR_ANY: `port` only when nonzero, else the first free even/odd pair
// from 6970 up (UDPSocketPool::CreateUDPSocketPair, UDPSocketPool.cpp:81-150; BindSockets
// retries a push with port 0 when the SDP's port is taken, ReflectorStream.cpp:432-443).
// 1 MiB receive buffers (:466-472).  Non-blocking: the reader drains each socket to EAGAIN.
bool BindPair(uint16_t port, UdpPair* out) {
    auto open1 = [](uint16_t p) -> int {
        const int fd = socket(AF_INET, SOCK_DGRAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
        if (fd < 0) return -1;
        const int rcv = 1 << 20;
        (void)setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &rcv, sizeof(rcv));
        sockaddr_in a;
        memset(&a, 0, sizeof(a));
        a.sin_family = AF_INET;
        a.sin_addr.s_addr = htonl(INADDR_ANY);
        a.sin_port = htons(p);
        if (bind(fd, (const sockaddr*)&a, sizeof(a)) != 0) { close(fd); return -1; }
        return fd;
    };
    auto try_pair = [&](uint32_t p) {
        const int a = open1((uint16_t)p);
        if (a < 0) return false;
        const int b = open1((uint16_t)(p + 1));
        if (b < 0) { close(a); return false; }
        out->fd[0] = a; out->fd[1] = b; out->port = (uint16_t)p;
        return true;
    };
    if (port != 0 && port < 65535 && try_pair(port)) return true;
    for (uint32_t p = 6970; p + 1 < 65536; p += 2)
        if (try_pair(p)) return true;
    return false;
}

// A packet reached the batch: in reflect-on-arrival mode the first one after a tick wakes the
// ticker (later ones only read the flag: no shared-line writes per packet).
inline void NotifyArrival() {
    if (!M->arrivalMinMs || M->pending.load(std::memory_order_relaxed)) return;
    if (!M->pending.exchange(true, std::memory_order_acq_rel)) {
        std::lock_guard<std::mutex> g(M->wakeMu);
        M->wake.notify_one();
    }
}

// ReflectorSocket::ProcessPacket's broadcaster refresh (ReflectorStream.cpp:1779-1786) for socket
// `sock` (2 x track + RTCP) of a session at `now`; the caller holds the lock of the packet's path.
inline void RefreshBroadcaster(Keepalive* ka, uint32_t sock, int64_t now) {
    if (!ka || sock >= ka->last.size()) return;
    QTSS_Object c = ka->client.load(std::memory_order_acquire);
    if (!c) return;
    std::atomic<int64_t>& last = ka->last[sock];
    if (now - last.load(std::memory_order_relaxed) > Keepalive::kIntervalMs) {
        (void)cb(kRefreshTimeOutCallback, c);
        last.store(now, std::memory_order_relaxed);
    }
}

// ReflectorSocket::GetIncomingData (ReflectorStream.cpp:1716-1735): every datagram waiting on a
// UDP push socket, read like RecvFrom into a kMaxReflectorPacketSize (2060) buffer -- a longer
// datagram is truncated there -- and handed to the engine with its source address (the UDP RTCP
// SR gate, Q14, and the pusher's RTCP address, :1769-1875, are the engine's).  An empty
// datagram is the reference's "no more data" read: nothing to ingest.  Takes udpMu only.
uint32_t DrainUDP() {
    if (!M->R) return 0;
    char buf[2060];
    uint32_t n = 0;
    std::lock_guard<std::mutex> g(M->udpMu);
    for (const UdpPair& u : M->udp) {
        for (int k = 0; k < 2; k++) {
            if (u.fd[k] < 0) continue;
            for (;;) {
                sockaddr_in from;
                socklen_t fl = sizeof(from);
                const ssize_t r = recvfrom(u.fd[k], buf, sizeof(buf), MSG_DONTWAIT, (sockaddr*)&from, &fl);
                if (r < 0) {
                    if (errno == EINTR) continue;
                    break;                                            // EAGAIN: drained
                }
                if (r == 0) continue;
                const int64_t now = Milliseconds();
                RefreshBroadcaster(u.ka.get(), 2 * u.track + (uint32_t)k, now);
                M->R->ProcessUDPPacket(u.engine, u.track, k == 1, buf, (uint32_t)r, ntohl(from.sin_addr.s_addr),
                                       ntohs(from.sin_port), now);
                NotifyArrival();
                n++;
            }
        }
    }
    return n;
}

// the reader thread: poll every UDP push socket, drain what arrived (never waits for a tick)
void ReaderLoop() {
    std::vector<pollfd> pf;
    while (!M->stop.load()) {
        {
            std::lock_guard<std::mutex> g(M->udpMu);
            pf.clear();
            for (const UdpPair& u : M->udp)
                for (int k = 0; k < 2; k++)
                    if (u.fd[k] >= 0) pf.push_back(pollfd{u.fd[k], POLLIN, 0});
        }
        if (pf.empty()) { std::this_thread::sleep_for(std::chrono::milliseconds(5)); continue; }
        if (poll(pf.data(), pf.size(), 10) > 0) (void)DrainUDP();
    }
}

// One reflect tick.  `mu` is held only to start and to end it: the engine part (ingest, fan-out,
// readback) holds the Reflector's engine lock, and the QTSS_Writes hold neither (SetConcurrentDelivery),
// so SETUP / PLAY / TEARDOWN proceed while a tick writes -- as the reference's per-stream
// fBucketMutex lets them (ReflectorStream.cpp:1051); a TEARDOWN waits only for the output it removes.
// The server's error log (QTSSModuleUtils::LogError: QTSS_Write on the error log stream with the
// verbosity as the flags, QTSSModuleUtils.cpp:168-200), and stderr.
void LogError(const std::string& msg) {
    fprintf(stderr, "%s\n", msg.c_str());
    if (sErrorLog) (void)cb(kWriteCallback, sErrorLog, (const void*)msg.data(), (uint32_t)msg.size(), (uint32_t*)nullptr,
                            (uint32_t)1 /* qtssWarningVerbosity */);
}

QTSS_Error Tick() {
    std::lock_guard<std::mutex> tg(M->tickMu);
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t seq;
    double held = 0;                                      // ms this tick held `mu`
    {
        std::lock_guard<std::mutex> g(M->mu);
        if (!M->R) return QTSS_RequestFailed;
        seq = ++M->tickSeq;
        held += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    M->pending.store(false, std::memory_order_release);   // this tick takes what arrived so far
    if (M->stallTick && seq == M->stallTick) (void)M->R->DebugStall((uint32_t)M->stallUs);
    QTSSSink sink;
    sink.now = Milliseconds();
    const int err = M->R->ReflectPackets(sink.now, &sink);
    std::unique_lock<std::mutex> g(M->mu);
    // The GPU watchdog: the engine ended a wait the device did not finish in time (EDGPU_TIMEOUT).
    // Its players get nothing while the device is stuck, so every one is torn down as
    // kill_clients_when_broadcast_stops tears a broadcast's down (QRM:2156-2159, RTPSessionOutput::
    // TearDown), SETUPs are refused (503) and the pushers' packets wait in the batch; the first tick
    // that succeeds again (the stuck work has finished) lifts it.
    std::vector<QTSS_Object> teardown;
    if (err == EDGPU_TIMEOUT) {
        if (!M->gpuStalled.exchange(true)) {
            for (const auto& out : M->outputs)
                if (!out->closed.load()) teardown.push_back(out->client);
            LogError("QTSSReflectorModule: GPU watchdog: the device did not finish a reflect tick in time (" +
                     std::string(edgpu_last_error()) + "); tearing down " + std::to_string(teardown.size()) +
                     " players, refusing SETUP until the device recovers");
        }
    } else if (!err && M->gpuStalled.exchange(false)) {
        LogError("QTSSReflectorModule: GPU watchdog: the device recovered, reflecting again");
    }
    const auto t1 = std::chrono::steady_clock::now();
    sink.SendReports();
    // outputs removed before or during this tick: no tick can reach them any more
    M->graveyard.erase(std::remove_if(M->graveyard.begin(), M->graveyard.end(),
                                      [&](const std::pair<uint64_t, std::unique_ptr<Output>>& e) { return e.first <= seq; }),
                       M->graveyard.end());
    for (size_t i = 0; i < M->orphans.size();)
        if (M->R->RemoveSession(M->orphans[i], true) == 0) M->orphans.erase(M->orphans.begin() + i);
        else i++;
    const edgpu_reflector::Reflector::TickInfo& t = M->R->LastTick();
    EDGPU_QTSSTickInfo& o = M->lastTick;
    o.ingested_packets = t.ingested_packets; o.ingested_bytes = t.ingested_bytes;
    o.readback_bytes = t.readback_bytes; o.arena_bytes = t.arena_bytes; o.writes = t.writes;
    o.ingest_ms = t.ingest_ms; o.fanout_ms = t.fanout_ms; o.readback_ms = t.readback_ms; o.write_ms = t.write_ms;
    o.prestaged_bytes = t.prestaged_bytes;
    o.passes = t.passes;
    o.rereads = M->rereads;
    if (t.stream_errors) {
        // per-stream isolation: name the sessions whose outputs lost packets, and go on
        std::vector<uint32_t> marked;
        if (M->R->StreamErrors(&marked) == 0)
            for (uint32_t e : marked) {
                o.stream_errors++;
                for (const auto& kv : M->sessions)
                    if (kv.second.engine == e)
                        fprintf(stderr, "QTSSReflectorModule: stream %s lost packets its outputs needed (sender ring "
                                        "at its bound: raise EDGPU_QTSS_MAX_RING_MB / _PACKETS)\n", kv.second.name.c_str());
            }
    }
    // the session lock's hold: what SETUP / PLAY / TEARDOWN may wait for (the tick's wall time is
    // ingest + fan-out + readback + writes)
    o.hold_ms = held + std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
    o.hold_max_ms = std::max(o.hold_max_ms, o.hold_ms);
    o.hold_sum_ms += o.hold_ms;
    o.wall_sum_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    o.ingest_sum_ms += t.ingest_ms; o.fanout_sum_ms += t.fanout_ms;
    o.readback_sum_ms += t.readback_ms; o.write_sum_ms += t.write_ms;
    o.ticks++;
    if (err) {
        // the first failure is logged with the engine's message; later ones are counted
        if (o.failed_ticks++ == 0)
            fprintf(stderr, "QTSSReflectorModule: tick failed (%d): %s\n", err,
                    M->R->LastError().empty() ? edgpu_last_error() : M->R->LastError().c_str());
        o.last_error = err;
    }
    g.unlock();
    // outside `mu`: the server may close a client session before QTSS_Teardown returns
    const uint32_t reason = qtssCliSesTearDownBroadcastEnded;
    for (QTSS_Object c : teardown) {
        (void)SetValue(c, qtssCliTeardownReason, 0, &reason, sizeof(reason));
        (void)cb(kTeardownCallback, c);
    }
    return err == 0 ? QTSS_NoErr : QTSS_RequestFailed;
}

// ---- roles ----------------------------------------------------------------------------------
QTSS_Error Register(QTSS_Register_Params* p) {
    // the reference's roles (QRM:268-276) but Easy_GetDeviceStream, EasyCMS's
    for (QTSS_Role r : {QTSS_Initialize_Role, QTSS_Shutdown_Role, QTSS_RTSPPreProcessor_Role,
                        QTSS_ClientSessionClosing_Role, QTSS_RTSPIncomingData_Role, QTSS_RTSPAuthorize_Role,
                        QTSS_RereadPrefs_Role, QTSS_RTSPRoute_Role})
        (void)cb(kAddRoleCallback, r);
    struct { QTSS_ObjectType type; const char* name; QTSS_AttrDataType dt; QTSS_AttributeID* id; } attrs[] = {
        {qtssClientSessionObjectType, "QTSSReflectorModuleRTPInfoWaitTime", qtssAttrDataTypeSInt32, &sRTPInfoWaitTimeAttr},
        {qtssClientSessionObjectType, "QTSSReflectorModuleOutput", qtssAttrDataTypeVoidPointer, &sOutputAttr},
        {qtssRTPStreamObjectType, "QTSSReflectorModuleStreamCookie", qtssAttrDataTypeVoidPointer, &sStreamCookieAttr},
        {qtssRTSPRequestObjectType, "QTSSReflectorModuleRequestBuffer", qtssAttrDataTypeVoidPointer, &sRequestBodyAttr},
        {qtssRTSPRequestObjectType, "QTSSReflectorModuleRequestBufferLen", qtssAttrDataTypeUInt32, &sBufferOffsetAttr},
        {qtssClientSessionObjectType, "QTSSReflectorModuleBroadcasterSession", qtssAttrDataTypeVoidPointer,
         &sClientBroadcastSessionAttr},
        {qtssClientSessionObjectType, "QTSSReflectorModuleTearDownClients", qtssAttrDataTypeBool16,
         &sKillClientsEnabledAttr},
        {qtssRTSPSessionObjectType, "QTSSReflectorModuleBroadcasterSession", qtssAttrDataTypeVoidPointer,
         &sRTSPBroadcastSessionAttr},
    };
    for (auto& a : attrs) {
        (void)cb(kAddStaticAttributeCallback, a.type, a.name, (void*)nullptr, a.dt);
        (void)cb(kIDForTagCallback, a.type, a.name, a.id);
    }
    if (p) snprintf(p->outModuleName, sizeof(p->outModuleName), "%s", "QTSSReflectorModule");
    return QTSS_NoErr;
}

// RereadPrefs' module prefs (QTSSReflectorModule.cpp:454-537: the names, types and defaults of
// :100-166); sessions set up from now on take the SSRC ones (:1457).  Caller holds mu.
void ReadModulePrefsLocked() {
    QTSS_Object o = M->modPrefs;
    GetPref<bool>(o, "disable_rtp_play_info", qtssAttrDataTypeBool16, &M->rtpInfoDisabled, false);
    GetPref<bool>(o, "kill_clients_when_broadcast_stops", qtssAttrDataTypeBool16, &M->killClients, false);
    GetPref<bool>(o, "use_one_SSRC_per_stream", qtssAttrDataTypeBool16, &M->oneSSRC, true);
    GetPref<uint32_t>(o, "timeout_stream_SSRC_secs", qtssAttrDataTypeUInt32, &M->timeoutSSRC, 30u);
    GetPref<bool>(o, "disable_overbuffering", qtssAttrDataTypeBool16, &M->disableOverbuffering, false);
    GetPref<bool>(o, "enable_player_compatibility", qtssAttrDataTypeBool16, &M->playerCompat, true);
    GetPref<bool>(o, "force_rtp_info_sequence_and_time", qtssAttrDataTypeBool16, &M->forceRTPInfo, false);
    GetPref<bool>(o, "enable_broadcast_announce", qtssAttrDataTypeBool16, &M->announceEnabled, true);
    bool push = true;
    GetPref<bool>(o, "enable_broadcast_push", qtssAttrDataTypeBool16, &push, true);
    M->pushEnabled.store(push, std::memory_order_relaxed);
    GetPref<bool>(o, "allow_duplicate_broadcasts", qtssAttrDataTypeBool16, &M->allowDuplicates, false);
    uint32_t bsecs = 30;
    GetPref<uint32_t>(o, "timeout_broadcaster_session_secs", qtssAttrDataTypeUInt32, &bsecs, 30u);
    M->broadcasterTimeoutMs = std::max<uint32_t>(bsecs, 30) * 1000;
    GetPref<bool>(o, "allow_non_sdp_urls", qtssAttrDataTypeBool16, &M->allowNonSDP, true);
    GetPref<bool>(o, "authenticate_local_broadcast", qtssAttrDataTypeBool16, &M->authLocal, false);
    GetPref<bool>(o, "allow_broadcasts", qtssAttrDataTypeBool16, &M->allowBroadcasts, true);
    M->broadcasterGroup = GetStringPref(o, "BroadcasterGroup", "broadcaster");
    // GetTrimmedKeyWord (QRM:411-427): leading '/'s dropped, up to the next '/'
    std::string kw = GetStringPref(o, "redirect_broadcast_keyword", "");
    size_t k0 = 0;
    while (k0 < kw.size() && kw[k0] == '/') k0++;
    const size_t k1 = kw.find('/', k0);
    M->redirectKeyword = kw.substr(k0, k1 == std::string::npos ? std::string::npos : k1 - k0);
    // a directory that does not start at '/' (the empty default too) is under the movie folder
    // (SetMoviesRelativeDir, QRM:429-448, 528-531)
    M->redirectDir = GetStringPref(o, "redirect_broadcasts_dir", "");
    if (M->redirectDir.empty() || M->redirectDir[0] != '/') {
        std::string movies;
        (void)ValueString(M->serverPrefs, qtssPrefsMovieFolder, 0, &movies);
        if (!movies.empty() && movies.back() != '/') movies += '/';
        M->redirectDir = movies + M->redirectDir;
    }
    M->ipAllowList = GetStringListPref(o, "ip_allow_list", "127.0.0.*");
}

QTSS_Error Initialize(QTSS_Initialize_Params* ip) {
    std::lock_guard<std::mutex> g(M->mu);
    if (const char* v = getenv("EDGPU_QTSS_TICK_MSEC")) M->tickMs = (uint32_t)std::max(1, atoi(v));
    if (const char* v = getenv("EDGPU_QTSS_REFLECT_ON_ARRIVAL")) M->arrivalMinMs = (uint32_t)std::max(0, atoi(v));
    if (const char* v = getenv("EDGPU_QTSS_MANUAL_TICK")) M->manualTick = atoi(v) != 0;
    if (M->manualTick) M->arrivalMinMs = 0;         // the host ticks: nobody to wake
    // the prefs objects: the server's (inPrefs) and this module's (GetModulePrefsObject:
    // qtssModPrefs of the module object, QTSSModuleUtils.cpp:634-642)
    M->serverPrefs = ip ? ip->inPrefs : nullptr;
    M->modPrefs = nullptr;
    if (ip && ip->inModule) {
        uint32_t n = sizeof(M->modPrefs);
        if (GetValue(ip->inModule, qtssModPrefs, 0, &M->modPrefs, &n) != QTSS_NoErr) M->modPrefs = nullptr;
    }
    // ReflectorStream::Initialize (ReflectorStream.cpp:87-117), read once
    uint32_t bucket = 73, bufSec = 1, relocate = 2000, rtpInfoOffset = 500;
    GetPref<uint32_t>(M->modPrefs, "reflector_bucket_offset_delay_msec", qtssAttrDataTypeUInt32, &bucket, 73u);
    GetPref<uint32_t>(M->modPrefs, "reflector_buffer_size_sec", qtssAttrDataTypeUInt32, &bufSec, 1u);
    GetPref<uint32_t>(M->modPrefs, "rtp_reflector_threshold_msec", qtssAttrDataTypeUInt32, &relocate, 2000u);
    GetPref<uint32_t>(M->modPrefs, "reflector_rtp_info_offset_msec", qtssAttrDataTypeUInt32, &rtpInfoOffset, 500u);
    bool useReceiveTime = false;
    uint32_t maxFutureSec = 60;
    GetPref<bool>(M->modPrefs, "reflector_use_in_packet_receive_time", qtssAttrDataTypeBool16, &useReceiveTime, false);
    GetPref<uint32_t>(M->modPrefs, "reflector_in_packet_max_receive_sec", qtssAttrDataTypeUInt32, &maxFutureSec, 60u);
    M->bucketDelayMs = bucket;
    M->overBufferMs = (int64_t)bufSec * 1000;
    ReadModulePrefsLocked();
    edgpu_config cfg;
    edgpu_config_default(&cfg);
    // the engine takes the prefs with the reference's meaning (0 in edgpu_config selects its
    // default, so a 0 pref is passed as the smallest value; the threshold's 1000-ms floor is the
    // engine's, as in ReflectorStream::Initialize)
    cfg.reflector_buffer_size_sec = bufSec ? bufSec : 1;
    cfg.rtp_reflector_threshold_msec = relocate ? relocate : 1000;
    cfg.reflector_rtp_info_offset_msec = rtpInfoOffset ? rtpInfoOffset : EDGPU_FALSE;
    cfg.timeout_stream_SSRC_secs = M->timeoutSSRC ? M->timeoutSSRC : 30;
    cfg.use_one_SSRC_per_stream = M->oneSSRC ? 1u : EDGPU_FALSE;
    cfg.reflector_use_in_packet_receive_time = useReceiveTime ? 1u : 0u;
    cfg.reflector_in_packet_max_receive_sec = maxFutureSec ? maxFutureSec : EDGPU_FALSE;
    if (const char* v = getenv("EDGPU_QTSS_DEVICE")) cfg.device = atoi(v);
    // the GPU watchdog: the longest a tick waits for the device (ms; 0: no bound)
    cfg.watchdog_ms = 2000;
    if (const char* v = getenv("EDGPU_QTSS_WATCHDOG_MS")) cfg.watchdog_ms = atoi(v) > 0 ? (uint32_t)atoi(v) : EDGPU_FALSE;
    if (const char* v = getenv("EDGPU_QTSS_TEST_STALL")) {           // tests: <tick>:<ms>
        M->stallTick = strtoull(v, nullptr, 10);
        if (const char* c = strchr(v, ':')) M->stallUs = strtoull(c + 1, nullptr, 10) * 1000;
    }
    // capacities for large fleets (edgpu_config; 0 / unset: the engine defaults): the fan-out
    // arena and descriptors of one tick, the ingest batch of one tick
    if (const char* v = getenv("EDGPU_QTSS_ARENA_MB")) cfg.out_arena_bytes = (uint64_t)atoll(v) << 20;
    if (const char* v = getenv("EDGPU_QTSS_ARENA_BYTES")) cfg.out_arena_bytes = strtoull(v, nullptr, 0);
    if (const char* v = getenv("EDGPU_QTSS_MAX_OUT_PACKETS")) cfg.max_out_packets = (uint32_t)atoll(v);
    if (const char* v = getenv("EDGPU_QTSS_MAX_BATCH_PACKETS")) cfg.max_batch_packets = (uint32_t)atoll(v);
    // sender rings: their starting capacities and the bound of their growth (powers of two; the
    // rings grow to hold what the reference retains, RemoveOldPackets, ReflectorStream.cpp:1233-1289)
    if (const char* v = getenv("EDGPU_QTSS_VIDEO_RING_MB")) cfg.video_ring_bytes = (uint64_t)atoll(v) << 20;
    if (const char* v = getenv("EDGPU_QTSS_VIDEO_RING_PACKETS")) cfg.video_ring_packets = (uint32_t)atoll(v);
    if (const char* v = getenv("EDGPU_QTSS_MAX_RING_MB")) cfg.max_ring_bytes = (uint64_t)atoll(v) << 20;
    if (const char* v = getenv("EDGPU_QTSS_MAX_RING_PACKETS")) cfg.max_ring_packets = (uint32_t)atoll(v);
    if (const char* v = getenv("EDGPU_QTSS_RING_GROWTH")) cfg.ring_growth = atoi(v) ? 0u : EDGPU_FALSE;
    M->R.reset(new edgpu_reflector::Reflector(&cfg));
    if (M->R->Status() != 0) {
        fprintf(stderr, "QTSSReflectorModule: edgpu context: %s\n", edgpu_last_error());
        M->R.reset();
        return QTSS_RequestFailed;          // no gfx950 device: fail loudly, no CPU fallback
    }
    // threads that make a tick's QTSS_Write calls (each player's writes stay on one thread)
    uint32_t writers = 4;
    if (const char* v = getenv("EDGPU_QTSS_WRITE_THREADS")) writers = (uint32_t)std::max(1, atoi(v));
    M->R->SetWriteThreads(writers);
    // the tick's writes run without the engine lock (EDGPU_QTSS_CONCURRENT_DELIVERY=0: held throughout)
    bool concurrent = true;
    if (const char* v = getenv("EDGPU_QTSS_CONCURRENT_DELIVERY")) concurrent = atoi(v) != 0;
    M->R->SetConcurrentDelivery(concurrent);
    if (!M->manualTick) {
        M->stop = false;
        M->reader = std::thread(ReaderLoop);
        M->ticker = std::thread([] {
            // a tick every tickMs from the previous tick's start (not tickMs after its end); in
            // reflect-on-arrival mode as soon as a packet waits, at most every arrivalMinMs
            using Clk = std::chrono::steady_clock;
            Clk::time_point last = Clk::now();
            while (!M->stop.load()) {
                const Clk::time_point longest = last + std::chrono::milliseconds(M->tickMs);
                if (M->arrivalMinMs) {
                    std::unique_lock<std::mutex> lk(M->wakeMu);
                    M->wake.wait_until(lk, longest, [] { return M->stop.load() || M->pending.load(); });
                    lk.unlock();
                    std::this_thread::sleep_until(last + std::chrono::milliseconds(M->arrivalMinMs));
                } else {
                    std::this_thread::sleep_until(longest);
                }
                if (M->stop.load()) break;
                last = Clk::now();
                const QTSS_Error e = Tick();
                if (e) M->tickErr = e;
            }
        });
    }
    return QTSS_NoErr;
}

// QTSS_RereadPrefs_Role (RereadPrefs, QTSSReflectorModule.cpp:454-537): the module prefs again;
// ReflectorStream's are read once, at Initialize, as in the reference.
QTSS_Error RereadPrefs() {
    std::lock_guard<std::mutex> g(M->mu);
    ReadModulePrefsLocked();
    M->rereads++;
    return QTSS_NoErr;
}

QTSS_Error Shutdown() {
    M->stop = true;
    {
        std::lock_guard<std::mutex> w(M->wakeMu);
        M->wake.notify_all();
    }
    if (M->ticker.joinable()) M->ticker.join();
    if (M->reader.joinable()) M->reader.join();
    std::lock_guard<std::mutex> g(M->mu);
    {
        std::lock_guard<std::mutex> u(M->udpMu);
        for (UdpPair& p : M->udp)
            for (int& fd : p.fd)
                if (fd >= 0) { close(fd); fd = -1; }
        M->udp.clear();
    }
    for (Module::RouteStripe& r : M->routes) {
        std::lock_guard<std::mutex> g(r.mu);
        r.route.clear();
    }
    M->R.reset();
    return QTSS_NoErr;
}

// ANNOUNCE (DoAnnounce, QRM:898-1174): read the request body (QTSS_Read, resumable), keep the
// SDP under the stream name for the pusher's SETUPs and the players' DESCRIBE
QTSS_Error DoAnnounce(QTSS_StandardRTSP_Params* p) {
    // any name will do (the reference's SDP suffix is empty, QRM:183, 953-962); an announced
    // "<name>.kill" only looks a session up to kill it (QRM:940-951, 1052-1059) -- by the bare name,
    // which never carries the "-<channel>" every session name has, so here it is refused outright
    {   // enable_broadcast_announce (QRM:900: 412 Precondition Failed, nothing cached)
        std::lock_guard<std::mutex> g(M->mu);
        if (!M->announceEnabled) return SendErrorResponse(p->inRTSPRequest, qtssPreconditionFailed);
    }
    const std::string name = GetString(p->inRTSPRequest, qtssRTSPReqFileName);
    if (name.size() > 5 && name.compare(name.size() - 5, 5, ".kill") == 0) return QTSS_RequestFailed;
    uint32_t clen = 0;
    if (!GetPOD(p->inRTSPRequest, qtssRTSPReqContentLen, &clen)) return SendErrorResponse(p->inRTSPRequest, qtssClientBadRequest);   // QRM:973-978
    std::string* body = nullptr;
    if (!GetPOD(p->inRTSPRequest, sRequestBodyAttr, &body) || !body) {
        body = new std::string();
        (void)SetValue(p->inRTSPRequest, sRequestBodyAttr, 0, &body, sizeof(body));
    }
    if (body->size() < clen) {
        const size_t off = body->size();
        body->resize(clen);
        uint32_t got = 0;
        const QTSS_Error e = cb(kReadCallback, p->inRTSPRequest, (void*)&(*body)[off], (uint32_t)(clen - off), &got);
        if (e != QTSS_NoErr && e != QTSS_WouldBlock) { delete body; (void)SetValue(p->inRTSPRequest, sRequestBodyAttr, 0, nullptr, 0); return QTSS_RequestFailed; }
        body->resize(off + got);
        if (body->size() < clen) {               // the rest arrives later: ask to be called again
            (void)cb(kRequestEventCallback, p->inRTSPRequest, (uint32_t)1 /* QTSS_ReadableEvent */);
            return QTSS_NoErr;
        }
    }
    {
        std::lock_guard<std::mutex> g(M->mu);
        M->announced[StreamName(p->inRTSPRequest)] = *body;
    }
    delete body;
    std::string* none = nullptr;
    (void)SetValue(p->inRTSPRequest, sRequestBodyAttr, 0, &none, sizeof(none));
    return cb(kSendStandardRTSPCallback, p->inRTSPRequest, p->inClientSession, (uint32_t)0);
}

// DESCRIBE (DoDescribe, QRM:1176-1377): the announced SDP
QTSS_Error DoDescribe(QTSS_StandardRTSP_Params* p) {
    std::string sdp;
    {
        std::lock_guard<std::mutex> g(M->mu);
        auto it = M->announced.find(StreamName(p->inRTSPRequest));
        if (it == M->announced.end()) return QTSS_RequestFailed;
        sdp = it->second;
    }
    const std::string n = std::to_string(sdp.size());
    (void)cb(kAppendRTSPHeadersCallback, p->inRTSPRequest, (uint32_t)qtssContentLengthHeader, n.c_str(), (uint32_t)n.size());
    (void)cb(kSendStandardRTSPCallback, p->inRTSPRequest, p->inClientSession, (uint32_t)0);
    return cb(kWriteCallback, p->inRTSPRequest, (const void*)sdp.data(), (uint32_t)sdp.size(), (uint32_t*)nullptr,
              (uint32_t)qtssWriteFlagsNoFlags);
}

Session* FindSession(uint32_t id) {
    auto it = M->sessions.find(id);
    return it == M->sessions.end() ? nullptr : &it->second;
}

// The pushers' route to the engine (RTSPIncomingData reads it without `mu`).
void SetRoute(const Session& s, bool on) {
    Module::RouteStripe& r = M->routes[s.id % Module::kRouteStripes];
    std::lock_guard<std::mutex> g(r.mu);
    if (on) r.route[s.id] = Module::Route{s.engine, (uint32_t)s.trackIDs.size(), s.ka.get()};
    else r.route.erase(s.id);
}

// FindOrCreateSession (QRM:1379-1545).  A player only finds a registered session (:1391-1396);
// a pusher's SETUP registers one from the announced SDP, and its transport decides whether the
// session is pushed over UDP.  A found session is not set up again (:1521-1531).
Session* FindOrCreateSession(const std::string& name, QTSS_Object req, bool isPush, bool udpPush = false) {
    auto it = M->byName.find(name);
    if (it != M->byName.end()) {
        // AllowBroadcast before anything else (QRM:1489-1495, 2293-2304): with allow_broadcasts off
        // every pusher and player SETUP of the session is forbidden
        if (!M->allowBroadcasts) { (void)SendErrorResponse(req, qtssClientForbidden); return nullptr; }
        return FindSession(it->second);
    }
    if (!isPush) return nullptr;
    auto a = M->announced.find(name);
    if (a == M->announced.end() || !M->R) return nullptr;
    if (!M->allowBroadcasts) { (void)SendErrorResponse(req, qtssClientForbidden); return nullptr; }   // QRM:1429-1437
    Session s;
    s.id = M->nextId++;
    s.name = name;
    s.sdp = a->second;
    s.udpPush = udpPush;
    if (M->R->SetupReflectorSession(s.sdp, udpPush, &s.engine) != 0) return nullptr;
    // SetupReflectorSession(..., sOneSSRCPerStream, sTimeoutSSRCSecs) with the prefs of now (:1457)
    if (M->R->SetSSRCFilter(s.engine, M->oneSSRC, M->timeoutSSRC) != 0) {
        (void)M->R->RemoveSession(s.engine, false);
        return nullptr;
    }
    s.trackIDs = SdpTrackIDs(s.sdp);
    s.trackIDs.resize(M->R->GetNumStreams(s.engine));
    s.sdpPorts = SdpPorts(s.sdp);
    s.sdpPorts.resize(s.trackIDs.size(), 0);
    s.pair.assign(s.trackIDs.size(), -1);
    s.setupToReceive.assign(s.trackIDs.size(), false);
    s.ka = std::make_shared<Keepalive>(2 * s.trackIDs.size());
    // each ReflectorStream draws its receiver-report SSRC from rand() and its CNAME from
    // OS::Milliseconds()/1000 when it is built (ReflectorStream.cpp:164-201, RTCPSRPacket.cpp:87-117)
    for (uint32_t t = 0; t < s.trackIDs.size(); t++)
        (void)M->R->SetSourceIdentity(s.engine, t, (uint32_t)rand(), Milliseconds() / 1000);
    const uint32_t id = s.id;
    M->sessions[id] = s;
    M->byName[name] = id;
    return &M->sessions[id];
}

// One reference of `s` released; at 0 the session ends (RemoveOutput, QRM:2162-2192): UnRegister,
// CSdpCache::eraseSdpMap, kill -- the engine session with its rings, and the UDP socket pairs.
void ReleaseLocked(Session* s) {
    if (s->refs > 0) s->refs--;
    if (s->refs > 0) return;
    SetRoute(*s, false);
    // the engine may refuse (a device error): the session is gone from the module either way, and
    // its engine session -- rings and all -- is removed at a later tick instead of leaking
    if (M->R && M->R->RemoveSession(s->engine, false) != 0) {
        fprintf(stderr, "QTSSReflectorModule: session %s: engine removal deferred (%s)\n", s->name.c_str(), edgpu_last_error());
        M->orphans.push_back(s->engine);
    }
    {
        std::lock_guard<std::mutex> g(M->udpMu);
        for (int pi : s->pair)
            if (pi >= 0) {
                for (int& fd : M->udp[pi].fd)
                    if (fd >= 0) { close(fd); fd = -1; }
                M->udp[pi].ka.reset();
            }
    }
    M->byName.erase(s->name);
    M->announced.erase(s->name);
    if (getenv("EDGPU_QTSS_DEBUG")) fprintf(stderr, "QTSSReflectorModule: session %s ended\n", s->name.c_str());
    M->sessions.erase(s->id);
}

// FindOrCreateSession's last step (QRM:1540-1542): the disable_overbuffering pref turns the
// client session's overbuffering off (the server's RTPStream then sends at the transmit times)
void DisableOverbufferingIfPref(QTSS_Object client) {
    if (!M->disableOverbuffering) return;
    const bool off = false;
    (void)SetValue(client, qtssCliSesOverBufferEnabled, 0, &off, sizeof(off));
}

// SETUP (DoSetup, QRM:1597-1800)
QTSS_Error DoSetup(QTSS_StandardRTSP_Params* p) {
    // the device is stuck (GPU watchdog): no new pusher or player until a tick succeeds
    if (M->gpuStalled.load()) return SendErrorResponse(p->inRTSPRequest, qtssServerUnavailable);
    uint32_t mode = qtssRTPTransportModePlay, transport = qtssRTPTransportTypeUDP;
    (void)GetPOD(p->inRTSPRequest, qtssRTSPReqTransportMode, &mode);
    (void)GetPOD(p->inRTSPRequest, qtssRTSPReqTransportType, &transport);
    const bool isPush = mode == qtssRTPTransportModeRecord;
    bool digitOK = false;
    const uint32_t trackID = TrackFromRequest(p->inRTSPRequest, &digitOK);
    std::lock_guard<std::mutex> g(M->mu);
    if (isPush) {
        const bool udp = transport != qtssRTPTransportTypeTCP;
        // the pusher's first SETUP resolves (or registers) the session and holds its reference;
        // its later SETUPs find it on the client session (QRM:1624-1645)
        uintptr_t held = 0;
        Session* s = nullptr;
        if (GetPOD(p->inClientSession, sClientBroadcastSessionAttr, &held) && held) s = FindSession((uint32_t)held);
        const bool first = s == nullptr;
        if (first) s = NotReflected(p->inRTSPRequest) ? nullptr : FindOrCreateSession(StreamName(p->inRTSPRequest), p->inRTSPRequest, true, udp);
        if (!s) return QTSS_RequestFailed;
        if (first) DisableOverbufferingIfPref(p->inClientSession);
        // the pusher's client session times out after timeout_broadcaster_session_secs (at least
        // 30 s) without a refresh; set at every push SETUP once the session resolved (QRM:1644)
        const uint32_t tmo = M->broadcasterTimeoutMs;
        (void)SetValue(p->inClientSession, qtssCliSesTimeoutMsec, 0, &tmo, sizeof(tmo));
        // the reference sets the session up for one transport; a pusher of the other cannot join it
        // (DeleteReflectorPushSession: the reference it took goes back, :1548-1570)
        auto refuse = [&]() { if (first && s->refs == 0) ReleaseLocked(s); return QTSS_RequestFailed; };
        if (s->udpPush != udp) return refuse();
        // no track digit, a bad track: 400; a track another pusher set up: 412 unless
        // allow_duplicate_broadcasts (QRM:1656-1686)
        if (!digitOK) { (void)refuse(); return SendErrorResponse(p->inRTSPRequest, qtssClientBadRequest); }
        const int t = TrackIndex(*s, trackID);
        if (t < 0) { (void)refuse(); return SendErrorResponse(p->inRTSPRequest, qtssClientBadRequest); }
        if (s->setupToReceive[t] && !M->allowDuplicates) { (void)refuse(); return SendErrorResponse(p->inRTSPRequest, qtssPreconditionFailed); }
        if (udp) {
            // the track's socket pair (BindSockets) and its port in the SETUP response
            if (s->pair[t] < 0) {
                UdpPair u;
                if (!BindPair(s->sdpPorts[t], &u)) return refuse();        // sCantBindReflectorSocketErr
                u.engine = s->engine;
                u.track = (uint32_t)t;
                u.ka = s->ka;
                std::lock_guard<std::mutex> ug(M->udpMu);
                // a slot an ended session left (both sockets closed) is reused: the table and the
                // reader's poll set stay as large as the live UDP tracks under churn
                int slot = -1;
                for (size_t i = 0; i < M->udp.size() && slot < 0; i++)
                    if (M->udp[i].fd[0] < 0 && M->udp[i].fd[1] < 0) slot = (int)i;
                if (slot < 0) { M->udp.push_back(u); slot = (int)M->udp.size() - 1; }
                else M->udp[slot] = u;
                s->pair[t] = slot;
            }
            const uint16_t port = M->udp[s->pair[t]].port;
            (void)SetValue(p->inRTSPRequest, qtssRTSPReqSetUpServerPort, 0, &port, sizeof(port));
        }
        QTSS_Object stream = nullptr;
        QTSS_Error e = cb(kAddRTPStreamCallback, p->inClientSession, p->inRTSPRequest, &stream, (uint32_t)0);
        if (e != QTSS_NoErr) { (void)refuse(); return e; }
        s->setupToReceive[t] = true;
        if (first) {                                     // the pusher's reference
            s->refs++;
            s->pushers++;
            SetRoute(*s, true);
        }
        // AddBroadcasterClientSession (QRM:1715): this pusher is the one every socket refreshes
        s->ka->client.store(p->inClientSession, std::memory_order_release);
        const uintptr_t sid = s->id;
        (void)SetValue(p->inClientSession, sClientBroadcastSessionAttr, 0, &sid, sizeof(sid));
        return cb(kSendStandardRTSPCallback, p->inRTSPRequest, stream, (uint32_t)0);
    }
    // a player: the first SETUP creates its output and takes a reference (QRM:1614-1622)
    Output* o = nullptr;
    if (!GetPOD(p->inClientSession, sOutputAttr, &o) || !o) {
        Session* s = NotReflected(p->inRTSPRequest) ? nullptr
                                                    : FindOrCreateSession(PlayerStreamName(p->inRTSPRequest, M->allowNonSDP),
                                                                          p->inRTSPRequest, false);
        if (!s) return QTSS_RequestFailed;
        DisableOverbufferingIfPref(p->inClientSession);
        M->outputs.emplace_back(new Output());
        o = M->outputs.back().get();
        o->client = p->inClientSession;
        o->session = s->id;
        o->tcp = transport == qtssRTPTransportTypeTCP;
        o->nstreams = (uint32_t)s->trackIDs.size();
        o->streams.reset(new std::atomic<QTSS_Object>[o->nstreams]);
        for (uint32_t k = 0; k < o->nstreams; k++) o->streams[k].store(nullptr, std::memory_order_relaxed);
        s->refs++;
        (void)SetValue(p->inClientSession, sOutputAttr, 0, &o, sizeof(o));
    }
    Session* s = FindSession(o->session);
    if (!s) return QTSS_RequestFailed;
    const int t = digitOK ? TrackIndex(*s, trackID) : -1;
    if (t < 0) return SendErrorResponse(p->inRTSPRequest, qtssClientBadRequest);   // no digit / bad track (QRM:1659-1663, 1728-1730)
    QTSS_Object stream = nullptr;
    QTSS_Error e = cb(kAddRTPStreamCallback, p->inClientSession, p->inRTSPRequest, &stream, (uint32_t)0);
    if (e != QTSS_NoErr) return e;
    (void)SetValue(stream, qtssRTPStrTrackID, 0, &trackID, sizeof(trackID));
    const uintptr_t cookie = ((uintptr_t)o->session << 16) | (uint32_t)t;          // the stream cookie
    (void)SetValue(stream, sStreamCookieAttr, 0, &cookie, sizeof(cookie));
    if ((uint32_t)t < o->nstreams) o->streams[t].store(stream, std::memory_order_release);
    return cb(kSendStandardRTSPCallback, p->inRTSPRequest, stream, (uint32_t)qtssSetupRespDontWriteSSRC);
}

// A value of the server's prefs as a string (QTSS_GetValueAsString: the server allocates it with
// new[], the caller deletes it, as StrPtrLenDel does)
bool PrefString(QTSS_Object o, QTSS_AttributeID id, uint32_t idx, std::string* out) {
    char* c = nullptr;
    if (cb(kGetValueAsStringCallback, o, id, idx, &c) != QTSS_NoErr || !c) return false;
    out->assign(c);
    delete[] c;
    return true;
}

// DoPlay's rtpInfoEnabled (QTSSReflectorModule.cpp:1872, 1962-1969): the player profile
// kRequiresRTPInfoSeqAndTime -- HavePlayerProfile, a case-sensitive substring of the first user
// agent in the server's player_requires_rtp_header_info list, "*" matching any
// (QTSSModuleUtils.cpp:983-1046) -- when enable_player_compatibility; forced on by
// force_rtp_info_sequence_and_time, off with disable_rtp_play_info.  Caller holds mu.
bool RequiresRTPInfoLocked(QTSS_Object client) {
    bool on = false;
    if (M->playerCompat) {
        const std::string ua = GetString(client, qtssCliSesFirstUserAgent);
        uint32_t n = 0;
        if (!ua.empty() && M->serverPrefs &&
            cb(kGetNumValuesCallback, M->serverPrefs, (QTSS_AttributeID)qtssPrefsPlayersReqRTPHeader, &n) == QTSS_NoErr)
            for (uint32_t i = 0; i < n; i++) {
                std::string pl;
                if (!PrefString(M->serverPrefs, qtssPrefsPlayersReqRTPHeader, i, &pl)) break;
                if (pl == "*" || ua.find(pl) != std::string::npos) { on = true; break; }
            }
    }
    if (M->forceRTPInfo) on = true;
    if (M->rtpInfoDisabled) on = false;
    return on;
}

// PLAY / RECORD (DoPlay, QRM:1867-2023)
QTSS_Error DoPlay(QTSS_StandardRTSP_Params* p, Output* o) {
    uint32_t flags = 0;
    if (!o) {                                             // the pusher's RECORD / PLAY
        uintptr_t sid = 0;
        if (!GetPOD(p->inClientSession, sClientBroadcastSessionAttr, &sid) || !sid) return QTSS_RequestFailed;
        // the pref decides, per pusher, whether its leaving tears the players down (QRM:1884)
        const bool kill = M->killClients;                 // a C++ bool, as the reference writes it
        (void)SetValue(p->inClientSession, sKillClientsEnabledAttr, 0, &kill, sizeof(kill));
        (void)SetValue(p->inRTSPSession, sRTSPBroadcastSessionAttr, 0, &sid, sizeof(sid));
        const bool keep = true;
        (void)SetValue(p->inRTSPRequest, qtssRTSPReqRespKeepAlive, 0, &keep, sizeof(keep));
    } else {
        std::unique_lock<std::mutex> g(M->mu);
        Session* s = FindSession(o->session);
        if (!s) return QTSS_RequestFailed;
        if (o->joined && o->paused.load()) {              // resume after PAUSE
            o->paused.store(false);
        } else if (!o->joined) {
            const bool tcp = o->tcp;
            uint32_t h = 0;
            int err;
            if (RequiresRTPInfoLocked(o->client)) {
                flags = qtssPlayRespWriteTrackInfo;
                std::vector<edgpu_rtp_info> info;
                err = M->R->PlayRTPInfo(s->engine, tcp, Milliseconds(), &h, &info);
                if (getenv("EDGPU_QTSS_DEBUG"))
                    fprintf(stderr, "QTSSReflectorModule: RTP-Info PLAY session=%u now=%lld err=%d %s\n", o->session,
                            (long long)Milliseconds(), err, err ? edgpu_last_error() : "");
                if (err == edgpu_reflector::kWouldBlock) {
                    // nothing buffered yet: retry the PLAY from the idle timer, then give up (QRM:1985-2003)
                    int32_t loops = 0;
                    uint32_t n = sizeof(loops);
                    if (GetValue(p->inClientSession, sRTPInfoWaitTimeAttr, 0, &loops, &n) != QTSS_NoErr)
                        loops = M->rtpInfoWaitLoops;
                    else if (loops < 1)
                        return QTSS_RequestFailed;
                    else
                        loops--;
                    (void)SetValue(p->inClientSession, sRTPInfoWaitTimeAttr, 0, &loops, sizeof(loops));
                    g.unlock();
                    return cb(kSetIdleTimerCallback, (int64_t)100);
                }
                if (err) return QTSS_RequestFailed;
                for (size_t t = 0; t < o->nstreams && t < info.size(); t++) {
                    QTSS_Object st = o->streams[t].load();
                    if (!st) continue;
                    (void)SetValue(st, qtssRTPStrFirstSeqNumber, 0, &info[t].seq, sizeof(info[t].seq));
                    (void)SetValue(st, qtssRTPStrFirstTimestamp, 0, &info[t].rtptime, sizeof(info[t].rtptime));
                }
            } else if ((err = M->R->AddOutput(s->engine, tcp, &h)) != 0) {
                return QTSS_RequestFailed;
            }
            o->handle = h;
            o->joined = true;
            // ReflectorSession::AddOutput: the first free bucket member (ReflectorStream.cpp:281-336)
            std::vector<Output*>& slots = s->slots;
            size_t k = 0;
            while (k < slots.size() && slots[k]) k++;
            if (k == slots.size()) slots.push_back(nullptr);
            slots[k] = o;
            o->slot = (int32_t)k;
            if (getenv("EDGPU_QTSS_DEBUG"))
                fprintf(stderr, "QTSSReflectorModule: output joined session=%u handle=%u slot=%zu tcp=%d\n", o->session, h, k, (int)tcp);
            o->bufferDelayMs = M->overBufferMs;         // RTPSessionOutput(): fBufferDelayMSecs
            SetOutputOf(h, o);                          // the write threads find it from now on
        }
        g.unlock();
        const QTSS_Error e = cb(kPlayCallback, p->inClientSession, p->inRTSPRequest,
                                (uint32_t)(flags ? qtssPlayRespWriteTrackInfo : qtssPlayFlagsAppendServerInfo));
        if (e != QTSS_NoErr && e != QTSS_Unimplemented) return e;
    }
    return cb(kSendStandardRTSPCallback, p->inRTSPRequest, p->inClientSession, flags);
}

// RemoveOutput(output, session, false) (QRM:2133-2196): out of the buckets, delete, and the
// output's reference on the session goes
// A tick writing to `o` finishes the write it is in; later ones skip it (Output::closed).
void StopWrites(Output* o) {
    o->closed.store(true, std::memory_order_seq_cst);
    while (o->writing.load(std::memory_order_seq_cst)) std::this_thread::yield();
}

void RemoveOutputLocked(Output* o) {
    StopWrites(o);                      // (callers outside a tick's writes find it idle)
    if (o->joined) {                    // an output whose PLAY never succeeded has no handle
        if (M->R) (void)M->R->RemoveOutput(o->handle);
        SetOutputOf(o->handle, nullptr);
    }
    Session* s = FindSession(o->session);
    if (s && o->slot >= 0) s->slots[o->slot] = nullptr;
    for (auto it = M->outputs.begin(); it != M->outputs.end(); ++it)
        if (it->get() == o) {
            // a tick that started before now may still hold it: freed once that tick has ended
            M->graveyard.emplace_back(M->tickSeq, std::move(*it));
            M->outputs.erase(it);
            break;
        }
    if (s) ReleaseLocked(s);
}

QTSS_Error ProcessRTSPRequest(QTSS_StandardRTSP_Params* p) {
    QTSS_RTSPMethod method = 0;
    if (!GetPOD(p->inRTSPRequest, qtssRTSPReqMethod, &method)) return QTSS_RequestFailed;
    if (method == qtssAnnounceMethod) return DoAnnounce(p);
    if (method == qtssDescribeMethod) return DoDescribe(p);
    if (method == qtssSetupMethod) return DoSetup(p);
    Output* o = nullptr;
    if (!GetPOD(p->inClientSession, sOutputAttr, &o) || !o) {     // a broadcaster's session
        if (method == qtssPlayMethod || method == qtssRecordMethod) return DoPlay(p, nullptr);
        return QTSS_RequestFailed;
    }
    switch (method) {
    case qtssPlayMethod:
        return DoPlay(p, o);
    case qtssTeardownMethod:
        (void)cb(kTeardownCallback, p->inClientSession);
        (void)cb(kSendStandardRTSPCallback, p->inRTSPRequest, p->inClientSession, (uint32_t)0);
        break;
    case qtssPauseMethod: {
        o->paused.store(true);
        (void)cb(kPauseCallback, p->inClientSession);
        (void)cb(kSendStandardRTSPCallback, p->inRTSPRequest, p->inClientSession, (uint32_t)0);
        break;
    }
    default:
        break;
    }
    return QTSS_NoErr;
}

// RTSPIncomingData (ProcessRTPData, QRM:604-678): one '$' ch BE16(len) frame of a pusher.  Never
// takes `mu`: one stripe of the route table and one of the Reflector's push path, so it never waits for a tick.
QTSS_Error ProcessRTPData(QTSS_IncomingData_Params* p) {
    if (!M->pushEnabled.load(std::memory_order_relaxed)) return QTSS_NoErr;      // enable_broadcast_push (QRM:606)
    uintptr_t sid = 0;
    if (!GetPOD(p->inRTSPSession, sRTSPBroadcastSessionAttr, &sid) || !sid) return QTSS_NoErr;
    if (!p->inPacketData || p->inPacketLen < 4) return QTSS_NoErr;
    const uint8_t* d = (const uint8_t*)p->inPacketData;
    const uint8_t channel = d[1];
    // the frame's own length, as the reference reads it; never past the buffer the server gave
    const uint32_t len = std::min<uint32_t>((uint32_t)d[2] << 8 | d[3], p->inPacketLen - 4);
    const int64_t now = Milliseconds();
    Module::RouteStripe& r = M->routes[(uint32_t)sid % Module::kRouteStripes];
    std::lock_guard<std::mutex> g(r.mu);
    auto it = r.route.find((uint32_t)sid);
    if (!M->R || it == r.route.end()) return QTSS_NoErr;       // no pusher attached any more
    const uint32_t track = channel / 2;
    if (track >= it->second.tracks) return QTSS_NoErr;
    // ReflectorStream::PushPacket takes only non-empty packets to ProcessPacket (RS.cpp:533), whose
    // first step is the broadcaster refresh
    if (len) RefreshBroadcaster(it->second.ka, channel, now);
    M->R->PushPacket(it->second.engine, track, (const char*)d + 4, len, (channel & 1) != 0, now);
    NotifyArrival();
    return QTSS_NoErr;
}

// ClientSessionClosing (DestroySession, QRM:2070-2131 -> RemoveOutput :2133-2196)
QTSS_Error DestroySession(QTSS_ClientSessionClosing_Params* p) {
    Output* o = nullptr;
    if (GetPOD(p->inClientSession, sOutputAttr, &o) && o) {
        StopWrites(o);                  // waits for a tick's write to it only, not for `mu`
        std::lock_guard<std::mutex> g(M->mu);
        RemoveOutputLocked(o);
        Output* none = nullptr;
        (void)SetValue(p->inClientSession, sOutputAttr, 0, &none, sizeof(none));
        return QTSS_NoErr;
    }
    uintptr_t sid = 0;
    if (GetPOD(p->inClientSession, sClientBroadcastSessionAttr, &sid) && sid) {
        // the pusher left (DestroySession's broadcaster branch, QRM:2082-2109)
        const uintptr_t none = 0;
        (void)SetValue(p->inClientSession, sClientBroadcastSessionAttr, 0, &none, sizeof(none));
        bool kill = false;                                // (QRM:2101-2103: a bool, sizeof 1)
        uint32_t n = sizeof(kill);
        if (GetValue(p->inClientSession, sKillClientsEnabledAttr, 0, &kill, &n) != QTSS_NoErr) kill = false;
        std::vector<QTSS_Object> teardown;
        {
            std::lock_guard<std::mutex> g(M->mu);
            Session* s = FindSession((uint32_t)sid);
            if (!s || !s->pushers) return QTSS_NoErr;
            s->setupToReceive.assign(s->setupToReceive.size(), false);   // a new pusher may set up
            // RemoveSessionFromOutput: the sockets stop refreshing this pusher (another one keeps
            // its own place only if it set up last, ReflectorStream.h:217)
            QTSS_Object me = p->inClientSession;
            s->ka->client.compare_exchange_strong(me, nullptr, std::memory_order_acq_rel);
            if (--s->pushers == 0) SetRoute(*s, false);
            // RemoveOutput(NULL, session, kill): TearDownAllOutputs asks the server to close every
            // output's client session (RTPSessionOutput::TearDown); each then comes back through
            // ClientSessionClosing and releases its reference
            if (kill || M->killClients)
                for (const auto& out : M->outputs)
                    if (out->session == s->id) teardown.push_back(out->client);
            ReleaseLocked(s);
        }
        // outside `mu`: the server may close the client session before QTSS_Teardown returns
        const uint32_t reason = qtssCliSesTearDownBroadcastEnded;
        for (QTSS_Object c : teardown) {
            (void)SetValue(c, qtssCliTeardownReason, 0, &reason, sizeof(reason));
            (void)cb(kTeardownCallback, c);
        }
    }
    return QTSS_NoErr;
}

// ---- access: RTSPAuthorize and RTSPRoute ------------------------------------------------------
// IPComponentStr (QTSSModuleUtils.cpp:1074-1135): an address as four '.'-separated components,
// valid once four non-empty ones are read (anything after the fourth is ignored); a "*" component
// on either side matches any.
struct IPComponents {
    std::string c[4];
    bool valid = false;
    explicit IPComponents(const std::string& s) {
        size_t p = 0;
        for (int k = 0; p < s.size(); k++) {
            size_t e = s.find('.', p);
            if (e == std::string::npos) e = s.size();
            if (e == p) break;                           // an empty component
            c[k] = s.substr(p, e - p);
            p = e + 1;
            if (k == 3) { valid = true; break; }
        }
    }
    bool Equal(const IPComponents& t) const {
        if (!valid || !t.valid) return false;
        for (int k = 0; k < 4; k++)
            if (t.c[k] != "*" && c[k] != "*" && t.c[k] != c[k]) return false;
        return true;
    }
};

// QTSSModuleUtils::UserInGroup (QTSSModuleUtils.cpp:918-953): a named user one of whose groups is
// exactly `group`
bool UserInGroup(QTSS_Object profile, const std::string& group) {
    if (!profile || group.empty()) return false;
    if (GetString(profile, qtssUserName).empty()) return false;
    uint32_t n = 0;
    (void)cb(kGetNumValuesCallback, profile, (QTSS_AttributeID)qtssUserGroups, &n);
    for (uint32_t i = 0; i < n; i++) {
        std::string g;
        if (ValueString(profile, qtssUserGroups, i, &g) && g == group) return true;
    }
    return false;
}

uint32_t RequestActions(QTSS_Object req) {
    uint32_t a = qtssActionFlagsNoFlags;
    (void)GetPOD(req, qtssRTSPReqAction, &a);
    return a;
}

// AcceptSession (QRM:2199-2229): a write request (a push) from a user in BroadcasterGroup, from a
// local address (127.0.0.*) unless authenticate_local_broadcast, or from an address ip_allow_list
// matches.  Caller holds mu.
bool AcceptSession(QTSS_StandardRTSP_Params* p) {
    if (RequestActions(p->inRTSPRequest) != qtssActionFlagsWrite) return false;
    QTSS_Object profile = nullptr;
    (void)GetPOD(p->inRTSPRequest, qtssRTSPReqUserProfile, &profile);
    if (UserInGroup(profile, M->broadcasterGroup)) return true;
    char addr[20] = {0};
    uint32_t len = sizeof(addr);
    if (GetValue(p->inRTSPSession, qtssRTSPSesRemoteAddrStr, 0, addr, &len) != QTSS_NoErr) return false;
    const IPComponents client(std::string(addr, len));
    if (client.Equal(IPComponents("127.0.0.*"))) return !M->authLocal;
    for (const std::string& a : M->ipAllowList)
        if (IPComponents(a).Equal(client)) return true;
    return false;
}

// QTSSModuleUtils::AuthorizeRequest (QTSSModuleUtils.cpp:1049-1068)
void SetAuthorization(QTSS_Object req, bool allowed, bool found, bool handled) {
    (void)SetValue(req, qtssRTSPReqUserAllowed, 0, &allowed, sizeof(allowed));
    (void)SetValue(req, qtssRTSPReqUserFound, 0, &found, sizeof(found));
    (void)SetValue(req, qtssRTSPReqAuthHandled, 0, &handled, sizeof(handled));
}

// QTSS_RTSPAuthorize_Role (ReflectorAuthorizeRTSPRequest, QRM:2231-2257).  An accepted push is
// authorized outright.  Anything else goes to QTAccessFile::AuthorizeRequest (QTAccessFile.cpp:
// 492-609) for the request's action with every action but a write left alone: a read is not
// touched.  For a write it needs the request's local path, root directory and user profile (the
// server sets the root only when a RTSPRoute module does: EasyDarwin's requests carry none, so a
// write stops there), looks for a "qtaccess" file from the request's directory up to the root,
// reads it -- through QTSSModuleUtils::ReadEntireFile, which in EasyDarwin serves the announced-SDP
// cache alone (QTSSModuleUtils.cpp:68-155), so the text is always empty and "require valid-user"
// stands in -- and that rule, outside any <Limit WRITE> block, never admits a write
// (QTAccessFile::AccessAllowed, :187-324).  The user profile's realm becomes the request's; a
// request without a user is marked handled.  The module then refuses the write: not allowed, no
// user, not handled.  (Where no qtaccess file is found the reference reads the cache with a NULL
// path, which throws from std::string; the same empty text is taken here.)
QTSS_Error Authorize(QTSS_StandardRTSP_Params* p) {
    std::lock_guard<std::mutex> g(M->mu);
    QTSS_Object req = p->inRTSPRequest;
    if (AcceptSession(p)) {
        SetAuthorization(req, true, true, true);
        return QTSS_NoErr;
    }
    const uint32_t action = RequestActions(req);
    bool authorized = false;
    do {
        if (action == qtssActionFlagsNoFlags || (action & ~(uint32_t)qtssActionFlagsWrite)) break;
        std::string local, root;
        QTSS_Object profile = nullptr;
        if (!ValueString(req, qtssRTSPReqLocalPath, 0, &local) || !ValueString(req, qtssRTSPReqRootDir, 0, &root)) break;
        if (!GetPOD(req, qtssRTSPReqUserProfile, &profile) || !profile) break;
        // GetAccessFile_Copy (QTAccessFile.cpp:326-379): the directories of the path, deepest first,
        // no higher than the root directory
        {
            const size_t max_len = local.size() + strlen("qtaccess") + 2;
            std::string dir = local;
            const size_t slash = dir.rfind('/');
            if (slash != std::string::npos) dir.resize(slash);
            while (dir.size() + strlen("qtaccess") + 1 < max_len) {
                const std::string f = dir + "/qtaccess";
                QTSS_Object file = nullptr;
                if (cb(kOpenFileObjectCallback, f.c_str(), (uint32_t)0, &file) == QTSS_NoErr) {
                    (void)cb(kCloseFileObjectCallback, file);
                    break;
                }
                const size_t s2 = dir.rfind('/');
                if (s2 == std::string::npos) break;
                dir.resize(s2);
                if (s2 < root.size()) break;
            }
        }
        std::string user;
        (void)ValueString(profile, qtssUserName, 0, &user);
        const bool allow = false;                        // "require valid-user" for a write: see above
        uint32_t scheme = qtssAuthNone;
        uint32_t n = sizeof(scheme);
        if (GetValue(req, qtssRTSPReqAuthScheme, 0, &scheme, &n) != QTSS_NoErr) break;
        std::string realm;
        if (ValueString(profile, qtssUserRealm, 0, &realm))
            (void)SetValue(req, qtssRTSPReqURLRealm, 0, realm.data(), (uint32_t)realm.size());
        authorized = allow;
        if (!allow && user.empty()) SetAuthorization(req, false, false, true);
    } while (false);
    if (!authorized && (action & qtssActionFlagsWrite)) SetAuthorization(req, false, false, false);
    return QTSS_NoErr;
}

// QTSS_RTSPRoute_Role (RedirectBroadcast, QRM:2259-2291): a request whose path starts with
// /<redirect_broadcast_keyword>/ (any case) gets the redirect directory as its root and the path
// without the keyword -- so its file name, the stream's name, is the next path component
QTSS_Error Route(QTSS_StandardRTSP_Params* p) {
    std::string kw, dir;
    {
        std::lock_guard<std::mutex> g(M->mu);
        kw = M->redirectKeyword;
        dir = M->redirectDir;
    }
    if (kw.empty() || dir.empty()) return QTSS_NoErr;
    std::string path;
    (void)ValueString(p->inRTSPRequest, qtssRTSPReqFilePath, 0, &path);
    size_t at = (!path.empty() && path[0] == '/') ? 1 : 0;
    const size_t end = std::min(path.find('/', at), path.size());
    const std::string first = path.substr(at, end - at);
    if (first.size() != kw.size()) return QTSS_NoErr;
    for (size_t i = 0; i < kw.size(); i++)
        if (tolower((unsigned char)first[i]) != tolower((unsigned char)kw[i])) return QTSS_NoErr;
    (void)SetValue(p->inRTSPRequest, qtssRTSPReqRootDir, 0, dir.data(), (uint32_t)dir.size());
    const std::string rest = path.substr(end);
    (void)SetValue(p->inRTSPRequest, qtssRTSPReqFilePath, 0, rest.data(), (uint32_t)rest.size());
    return QTSS_NoErr;
}

QTSS_Error Dispatch(QTSS_Role role, QTSS_RoleParams* p) {
    switch (role) {
    case QTSS_Register_Role: return Register(p ? &p->regParams : nullptr);
    case QTSS_Initialize_Role: return Initialize(p ? &p->initParams : nullptr);
    case QTSS_Shutdown_Role: return Shutdown();
    case QTSS_RereadPrefs_Role: return RereadPrefs();
    case QTSS_RTSPPreProcessor_Role: return ProcessRTSPRequest(&p->rtspRequestParams);
    case QTSS_RTSPIncomingData_Role: return ProcessRTPData(&p->rtspIncomingDataParams);
    case QTSS_ClientSessionClosing_Role: return DestroySession(&p->clientSessionClosingParams);
    case QTSS_RTSPAuthorize_Role: return Authorize(&p->rtspRequestParams);
    case QTSS_RTSPRoute_Role: return Route(&p->rtspRequestParams);
    default: return QTSS_NoErr;
    }
}

}  // namespace

extern "C" QTSS_Error QTSSReflectorModule_Main(void* inPrivateArgs) {
    // _stublibrary_main (QTSS_Private.cpp:44-59)
    QTSS_PrivateArgs* a = (QTSS_PrivateArgs*)inPrivateArgs;
    if (!a) return QTSS_BadArgument;
    sCallbacks = a->inCallbacks;
    sErrorLog = a->inErrorLogStream;
    a->outStubLibraryVersion = kApiVersion;
    a->outDispatchFunction = Dispatch;
    if (!M) {
        M = new Module();
        for (uint32_t k = 0; k < Module::kChunks; k++) M->handleChunks[k].store(nullptr, std::memory_order_relaxed);
    }
    return QTSS_NoErr;
}

extern "C" QTSS_Error EDGPU_QTSSReflectorModule_Tick(void) {
    if (!M) return QTSS_RequestFailed;
    return Tick();
}

// Manual mode (EDGPU_QTSS_MANUAL_TICK=1, no reader thread): read every datagram waiting on the
// UDP push sockets now; returns how many were handed to the engine.
extern "C" QTSS_Error EDGPU_QTSSReflectorModule_LastTick(EDGPU_QTSSTickInfo* out) {
    if (!M || !out) return QTSS_BadArgument;
    std::lock_guard<std::mutex> g(M->mu);
    *out = M->lastTick;
    return QTSS_NoErr;
}

extern "C" uint32_t EDGPU_QTSSReflectorModule_PollUDP(void) {
    if (!M) return 0;
    return DrainUDP();
}
