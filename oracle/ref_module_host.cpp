// oracle/ref_module_host.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured as the
// product).  What the EasyDarwin server process gives the REFERENCE QTSSReflectorModule when the
// module, compiled from the read-only reference sources, is loaded as a QTSS module by the fake
// server tools/qtss_replay (oracle/_ref/Makefile: libQTSSReflectorModule_ref.so):
//
//   * the server object behind QTSServerInterface::GetServer(), of which the module only reads
//     the reflector session map (QTSSReflectorModule.cpp:373 -> QTSServerInterface.h:232), and the
//     server's module tables with zero modules in any role (QTSServerInterface.h:356-357; the
//     Redis roles ReflectorSession calls then do nothing -- as in oracle/ref_harness.cpp);
//   * the socket event machinery the server sets up before loading modules (Socket::Initialize,
//     epollInit): the UDP-push sockets BindSockets binds register with it (RequestEvent); the
//     event thread is not started;
//   * the clock: OS::Milliseconds is link-wrapped onto QTSS_Milliseconds, the fake server's
//     virtual clock (the reference server's OS::Milliseconds is the same clock the callback
//     reads);
//   * the work the server's task threads would do, as manual entry points with the names the
//     drop-in exports (include/qtss_module_abi.h), so one fake server drives both:
//       EDGPU_QTSSReflectorModule_Tick    -- ReflectPackets on every sender of every registered
//                                            session (RTP then RTCP, track order), as
//                                            ReflectorSocket::Run does (ReflectorStream.cpp:
//                                            1709-1714) and oracle/ref_harness.cpp's TICK does;
//       EDGPU_REFHOST_Ticker(on)          -- (--bench real time) the server's task threads: a
//                                            ReflectorSocket task runs ReflectPackets as soon as a
//                                            pushed packet signals it (ReflectorStream.cpp:573,
//                                            1676-1714); here EDGPU_REF_TICK_THREADS threads sweep
//                                            their share of the sessions' senders every
//                                            EDGPU_REF_REFLECT_MSEC (default 1) ms, without the
//                                            session map's mutex (a task holds its session);
//       EDGPU_QTSSReflectorModule_PollUDP -- the datagrams waiting on the UDP-push sockets the
//                                            module bound (UDPSocketPool, BindSockets :388-506),
//                                            each clamped to the 2060-byte packet buffer and
//                                            handed to ReflectorSocket::ProcessPacket(now,
//                                            packet, remote addr, remote port), as
//                                            GetIncomingData does (:2013-2060) and the harness's
//                                            UPKT does; returns the datagrams read.
// Everything else -- ANNOUNCE / SETUP / PLAY / RECORD, the session map and reference counts,
// RTPSessionOutput, prefs, teardown -- is the reference module's own code.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "QTSS.h"
#include "QTSS_Private.h"
#include "OS.h"
#include "OSQueue.h"
#include "OSRef.h"
#include "ReflectorSession.h"
#include "ReflectorStream.h"
#include "QTSServerInterface.h"
#include "MyAssert.h"
#include "Socket.h"
#include "epollEvent.h"

// The server's module tables (no module in any role) and the server object.
QTSSModule** QTSServerInterface::sModuleArray[QTSSModule::kNumRoles];
UInt32       QTSServerInterface::sNumModulesInRole[QTSSModule::kNumRoles];
QTSServerInterface* QTSServerInterface::sServer = NULL;

// fReflectorSessionMap is the one member of the server object the module reads; it (and sServer)
// is reached through a pointer taken by explicit instantiation (which the language exempts from
// access checks) -- the server object here is storage with that member set, its constructor
// (QTSServerInterface.cpp, the whole server) is not run.
namespace {
template <typename Tag, typename Tag::type M> struct Steal { friend typename Tag::type get(Tag) { return M; } };
struct SessionMapMember { typedef OSRefTable* QTSServerInterface::*type; friend type get(SessionMapMember); };
template struct Steal<SessionMapMember, &QTSServerInterface::fReflectorSessionMap>;
struct ServerStatic { typedef QTSServerInterface** type; friend type get(ServerStatic); };
template struct Steal<ServerStatic, &QTSServerInterface::sServer>;
// each ReflectorSocket's own free-packet queue, which ReflectorSocket::Run hands to ReflectPackets
// (ReflectorStream.cpp:1713): the packets RemoveOldPackets frees go back to the socket that GetPacket
// takes them from (:2039-2047), so a long run recycles them as the server does
struct FreeQueueMember { typedef OSQueue ReflectorSocket::*type; friend type get(FreeQueueMember); };
template struct Steal<FreeQueueMember, &ReflectorSocket::fFreeQueue>;

alignas(QTSServerInterface) unsigned char g_server[sizeof(QTSServerInterface)];
OSRefTable* g_sessions = NULL;
bool g_callbacks = false;                 // the stub library has the server's callback table

OSRefTable* session_map() {
    if (g_sessions == NULL) {
        g_sessions = new OSRefTable();
        QTSServerInterface* s = reinterpret_cast<QTSServerInterface*>(g_server);
        s->*get(SessionMapMember()) = g_sessions;
        *get(ServerStatic()) = s;
    }
    return g_sessions;
}

// the registered sessions, in name order (a deterministic tick order)
std::vector<ReflectorSession*> live_sessions() {
    std::vector<std::pair<std::string, ReflectorSession*>> v;
    for (OSRefHashTableIter it(session_map()->GetHashTable()); !it.IsDone(); it.Next()) {
        OSRef* ref = it.GetCurrent();
        if (ref == NULL || ref->GetObject() == NULL) continue;
        v.push_back(std::make_pair(std::string(ref->GetString()->Ptr, ref->GetString()->Len),
                                   (ReflectorSession*)ref->GetObject()));
    }
    std::sort(v.begin(), v.end(), [](const std::pair<std::string, ReflectorSession*>& a,
                                     const std::pair<std::string, ReflectorSession*>& b) { return a.first < b.first; });
    std::vector<ReflectorSession*> out;
    for (auto& e : v) out.push_back(e.second);
    return out;
}
}  // namespace

// The server's assert logger (the reference's MyAssert writes through a null pointer without
// one): asserts are counted, and printed with EDTR_SHOW_ASSERTS, as the reference harness does.
struct HostAssert : public AssertLogger {
    unsigned long count = 0;
    void LogAssert(char* m) override { if (getenv("EDTR_SHOW_ASSERTS")) fprintf(stderr, "assert: %s\n", m); ++count; }
};

// QTSSReflectorModule_Main -> _stublibrary_main: from here on the callbacks are set
extern "C" QTSS_Error __real__stublibrary_main(void*, QTSS_DispatchFuncPtr);
extern "C" QTSS_Error __wrap__stublibrary_main(void* args, QTSS_DispatchFuncPtr fn) {
    static HostAssert logger;
    SetAssertLogger(&logger);
    // the server's socket event machinery, set up before modules load (RunServer): the event
    // thread object the sockets register with and the epoll set; the thread itself is not started --
    // PollUDP reads the sockets
    Socket::Initialize();
    (void)epollInit();
    (void)session_map();
    const QTSS_Error e = __real__stublibrary_main(args, fn);
    g_callbacks = e == QTSS_NoErr;
    return e;
}

extern "C" SInt64 __wrap__ZN2OS12MillisecondsEv() { return g_callbacks ? QTSS_Milliseconds() : 0; }

// EDGPU_QTSSReflectorModule_LastTick's block (include/qtss_module_abi.h EDGPU_QTSSTickInfo, same
// layout): for the fake server's --bench mode, the tick count and each tick's wall time, all of which
// is spent holding the session map's mutex
struct TickInfo {
    uint64_t ingested_packets, ingested_bytes, readback_bytes, arena_bytes, writes;
    double ingest_ms, fanout_ms, readback_ms, write_ms, hold_ms;
    uint64_t ticks, failed_ticks;
    int64_t last_error;
    uint64_t prestaged_bytes, passes, rereads;
    double hold_max_ms, hold_sum_ms;
    uint64_t stream_errors;
    double wall_sum_ms, ingest_sum_ms, fanout_sum_ms, readback_sum_ms, write_sum_ms;
};
static TickInfo g_tick;
extern "C" QTSS_Error EDGPU_QTSSReflectorModule_LastTick(TickInfo* out) {
    *out = g_tick;
    return QTSS_NoErr;
}

// ReflectPackets on a session's senders, RTP then RTCP per track, each under its socket's demuxer
// mutex with its free queue (ReflectorStream.cpp:1676-1714)
static void reflect_session(ReflectorSession* sess) {
    for (UInt32 x = 0; x < sess->GetNumStreams(); x++) {
        ReflectorStream* st = sess->GetStreamByIndex(x);
        if (st == NULL || st->GetSocketPair() == NULL) continue;
        ReflectorSocket* a = (ReflectorSocket*)st->GetSocketPair()->GetSocketA();
        ReflectorSocket* b = (ReflectorSocket*)st->GetSocketPair()->GetSocketB();
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
}

static std::atomic<bool> g_rt_stop{false};
static std::vector<std::thread> g_rt_threads;
extern "C" void EDGPU_REFHOST_Ticker(int on) {
    if (!on) {
        g_rt_stop = true;
        for (std::thread& t : g_rt_threads) t.join();
        g_rt_threads.clear();
        return;
    }
    const unsigned nthreads = getenv("EDGPU_REF_TICK_THREADS") ? std::max(1, atoi(getenv("EDGPU_REF_TICK_THREADS"))) : 1;
    const int every = getenv("EDGPU_REF_REFLECT_MSEC") ? std::max(0, atoi(getenv("EDGPU_REF_REFLECT_MSEC"))) : 1;
    g_rt_stop = false;
    for (unsigned w = 0; w < nthreads; w++)
        g_rt_threads.emplace_back([w, nthreads, every]() {
            while (!g_rt_stop.load()) {
                std::vector<ReflectorSession*> sessions;
                {
                    OSMutexLocker locker(session_map()->GetMutex());
                    sessions = live_sessions();     // (the bench's sessions live until its end)
                }
                const auto a = std::chrono::steady_clock::now();
                for (size_t k = w; k < sessions.size(); k += nthreads) reflect_session(sessions[k]);
                if (w == 0) {
                    g_tick.ticks++;
                    g_tick.wall_sum_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
                }
                std::this_thread::sleep_for(std::chrono::milliseconds(every));
            }
        });
}

extern "C" QTSS_Error EDGPU_QTSSReflectorModule_Tick(void) {
    const auto t0 = std::chrono::steady_clock::now();
    struct Done {
        std::chrono::steady_clock::time_point t0;
        ~Done() {
            g_tick.ticks++;
            g_tick.passes = 1;
            g_tick.hold_ms = g_tick.write_ms =
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            g_tick.hold_max_ms = std::max(g_tick.hold_max_ms, g_tick.hold_ms);
            g_tick.hold_sum_ms += g_tick.hold_ms;
            g_tick.wall_sum_ms += g_tick.hold_ms;
        }
    } done{t0};
    OSMutexLocker locker(session_map()->GetMutex());
    // EDGPU_REF_TICK_THREADS=N (default 1): the sessions' senders reflect on N threads, as the
    // server's task threads run the ReflectorSocket tasks (one socket's senders on one thread at a
    // time, under its demuxer mutex, with its free queue: ReflectorStream.cpp:1676-1714)
    static const unsigned nthreads = getenv("EDGPU_REF_TICK_THREADS") ? (unsigned)atoi(getenv("EDGPU_REF_TICK_THREADS")) : 1;
    const std::vector<ReflectorSession*> sessions = live_sessions();
    auto reflect = [&](unsigned w, unsigned nw) {
        for (size_t k = w; k < sessions.size(); k += nw) reflect_session(sessions[k]);
    };
    if (nthreads <= 1) {
        reflect(0, 1);
    } else {
        std::vector<std::thread> th;
        for (unsigned w = 1; w < nthreads; w++) th.emplace_back(reflect, w, nthreads);
        reflect(0, nthreads);
        for (std::thread& t : th) t.join();
    }
    return QTSS_NoErr;
}

extern "C" UInt32 EDGPU_QTSSReflectorModule_PollUDP(void) {
    OSMutexLocker locker(session_map()->GetMutex());
    UInt32 n = 0;
    char buf[65536];
    for (ReflectorSession* sess : live_sessions())
        for (UInt32 x = 0; x < sess->GetNumStreams(); x++) {
            ReflectorStream* st = sess->GetStreamByIndex(x);
            UDPSocketPair* pr = st == NULL ? NULL : st->GetSocketPair();
            if (pr == NULL) continue;
            for (int k = 0; k < 2; k++) {
                ReflectorSocket* so = (ReflectorSocket*)(k ? pr->GetSocketB() : pr->GetSocketA());
                if (so == NULL || so->GetSocketFD() < 0) continue;
                for (;;) {
                    sockaddr_in from;
                    socklen_t fl = sizeof(from);
                    const ssize_t got = recvfrom(so->GetSocketFD(), buf, sizeof(buf), MSG_DONTWAIT, (sockaddr*)&from, &fl);
                    if (got <= 0) break;
                    ReflectorPacket* pk = so->GetPacket();
                    if (pk == NULL) break;
                    pk->SetPacketData(buf, std::min<UInt32>((UInt32)got, 2060u));
                    OSMutexLocker dl(so->GetDemuxer()->GetMutex());
                    so->ProcessPacket(OS::Milliseconds(), pk, ntohl(from.sin_addr.s_addr), ntohs(from.sin_port));
                    n++;
                }
            }
        }
    return n;
}
