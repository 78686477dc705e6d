// reflector_adapter.h -- C++ module-side seams of QTSSReflectorModule, implemented on top of
// the edgpu C ABI.  A reflector module built against this header keeps the reference's call
// pattern (SURVEY.md §8.b "internal seams"):
//
//   reference                                         here
//   ReflectorSession::SetupReflectorSession           Reflector::SetupReflectorSession
//     (ReflectorSession.cpp:140-188)
//   ReflectorSession::AddOutput / RemoveOutput        Reflector::AddOutput / RemoveOutput
//     (ReflectorSession.cpp:209-279)
//   ReflectorStream::PushPacket(char*, UInt32, bool)  Reflector::PushPacket (same arguments
//     (ReflectorStream.cpp:529-576)                     plus the session/track it belongs to)
//   ReflectorSocket::Run -> ReflectPackets            Reflector::ReflectPackets(now, sink)
//     (ReflectorStream.cpp:1676-1714, 1024-1136)
//   ReflectorSocket::GetIncomingData ->               Reflector::ProcessUDPPacket (a UDP
//     ProcessPacket(now, pkt, addr, port)               pusher's datagram with its source)
//     (ReflectorStream.cpp:1716-1735, 1769-1875)
//   ReflectorStream::SendReceiverReport ->            OutputSink::SendReceiverReport, from
//     UDPSocket::SendTo (ReflectorStream.cpp:510-527)   ReflectPackets on the 5-s timer
//   ReflectorOutput::WritePacket (pure virtual,       OutputSink::WritePacket, called once per
//     ReflectorOutput.h:114) -> QTSS_Write ->           send-ready packet with the bytes already
//     RTPStream::Write framing                           framed for the subscriber's transport
//   CKeyFrameCache (keyframecache.h:45-72)            edgpu_reflector::CKeyFrameCache, same
//                                                        public API + LoadGOP() from HBM
//
// Threading: one Reflector per GPU.  PushPacket / ProcessUDPPacket -- the pushers' ingest
// (RTSPIncomingData, the UDP socket reader) -- may be called from any thread at any time: each
// reserves its slot in the pending batch under a short lock (one of 16 stripes, by session) and
// copies the packet outside it,
// and never waits for a tick (the reference takes only the demuxer / stream mutex per packet,
// ReflectorStream.cpp:529-576, 1769-1875).  Every other call takes the Reflector's engine lock
// (the edgpu context is one device queue and its host tables), so callers on different threads are
// serialised here; ReflectPackets holds it for the tick and takes the push lock only to swap the
// pending batch.  SetConcurrentDelivery(true): the tick gives the engine lock up while its writes
// run (the QTSS_Write half of a tick, most of its time at fleet scale), so AddOutput, RemoveOutput
// and session set-up proceed meanwhile -- the reference serialises only per stream (fBucketMutex,
// ReflectorStream.cpp:1051); PlayRTPInfo and RemoveSession, which ingest what is pending, wait for
// the tick's writes to end (the batch being written from is the one they would refill).  With
// SetWriteThreads(n > 1) ReflectPackets delivers a tick's packets from n threads, split by
// session: all of one subscriber's writes come from one thread, in the order one thread would
// make them, and a session's subscribers -- the same packet bytes -- share that thread's caches
// (the reference's ReflectorSocket tasks also write to different outputs from different task
// threads, ReflectorStream.cpp:1676-1714).
//
// Copies: a pushed packet is copied once, into a pinned slot buffer (two, used alternately),
// and reaches HBM by one asynchronous DMA (edgpu_ingest EDGPU_PTR_PINNED); a tick's output comes
// back as its distinct bytes only (tick_regions.h + edgpu_arena_gather), not the write-many
// arena (the reference copies a pushed packet once, ReflectorStream.h:104-114, and writes each
// relayed packet from that copy).
#pragma once
#include <stdint.h>
#include <atomic>
#include <chrono>
#include <memory>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "edgpu.h"

namespace edgpu_host { struct TickRegions; }

namespace edgpu_reflector {

// QTSS_Error values (QTSS.h:61-76)
enum { kNoErr = 0, kRequestFailed = -1, kBadArgument = -10, kWouldBlock = -14 };

// The egress seam.  `wire` points at the bytes to put on the wire for this subscriber: the
// UDP datagram, or the complete '$' ch BE16(len) + packet frame for an RTSP-interleaved
// subscriber (RTSPSessionInterface.cpp:329-344).  Return kNoErr to continue, kWouldBlock when
// the socket is flow-controlled (EAGAIN): the rest of this sub-stream's packets are not
// offered this tick and the next tick resumes at this packet, as SendPacketsToOutput does.
// One write of a tick, with what RTPSessionOutput::WritePacket needs beyond the bytes to build
// the QTSS_PacketStruct transmit time (RTPSessionOutput.cpp:603-608).
struct PacketWrite {
    uint32_t subscriber;
    uint16_t track;
    bool isRTCP, interleaved;
    const uint8_t* wire;
    uint32_t wireLen;
    uint32_t packetID;
    int64_t arrivalMs;              // the packet's fTimeArrived; -1 unless the sink WantsArrivals()
    uint32_t sender;                // engine sender (the ReflectorSender this write comes from)
    bool newOutput;                 // the output had no bookmark on this sender when the tick began
    uint32_t worker;                // the delivering thread, 0 .. Reflector::WriteThreads() - 1
};

class OutputSink {
public:
    virtual ~OutputSink() {}
    virtual int WritePacket(uint32_t subscriber, uint16_t track, bool isRTCP, bool interleaved,
                            const uint8_t* wire, uint32_t wireLen, uint32_t packetID) = 0;
    // Sinks that model the transmit time override these three: ReflectPackets then reads the
    // tick's arrival times (edgpu_fanout_arrivals), shows the sink the first pass's sub-streams
    // that carry packets or are new outputs first, in table order (the reference walks each
    // sender's outputs in bucket order, so whether an earlier output was new decides
    // `firstPacket` for the later ones, ReflectorStream.cpp:1086-1108),
    // and calls Write for every packet.  Write / WritePacket are called concurrently for
    // different subscribers when the Reflector has more than one write thread (w.worker tells
    // them apart); BeginTick runs before, on the ticking thread.
    virtual bool WantsArrivals() const { return false; }
    virtual void BeginTick(const edgpu_substream_out* subs, uint32_t n) { (void)subs; (void)n; }
    virtual int Write(const PacketWrite& w) {
        return WritePacket(w.subscriber, w.track, w.isRTCP, w.interleaved, w.wire, w.wireLen, w.packetID);
    }
    // A receiver report for a UDP pusher: send `rr` from the track's RTCP socket to
    // (addr, port), both in host order (ReflectorStream::SendReceiverReport's SendTo, whose
    // result the reference ignores).
    virtual void SendReceiverReport(uint32_t session, uint16_t track, uint32_t addr, uint16_t port,
                                    const uint8_t* rr, uint32_t len) {
        (void)session; (void)track; (void)addr; (void)port; (void)rr; (void)len;
    }
    // A write thread has made the last write of a copy pass (on that thread).
    virtual void EndWrites(uint32_t worker) { (void)worker; }
};

class Reflector {
public:
    explicit Reflector(const edgpu_config* cfg = nullptr);
    ~Reflector();
    Reflector(const Reflector&) = delete;
    Reflector& operator=(const Reflector&) = delete;

    int  Status() const { return fStatus; }                 // construction result
    // push session from its SDP; udpPush: RTCP arrives on a bound odd port (Q12/Q14)
    int  SetupReflectorSession(const std::string& sdp, bool udpPush, uint32_t* outSession);
    uint32_t GetNumStreams(uint32_t session) const;
    // the session's SSRC filter settings, from the module prefs when it is set up
    // (SetupReflectorSession's inFilterSSRCs / inTimeout, QTSSReflectorModule.cpp:1457)
    int  SetSSRCFilter(uint32_t session, bool oneSSRCPerStream, uint32_t timeoutSecs);
    // player joins every track of `session`; takes effect at the next ReflectPackets
    int  AddOutput(uint32_t session, bool interleaved, uint32_t* outHandle);
    // PLAY of an RTP-Info player (UA "vlc"/"Android"; DoPlay + HaveStreamBuffers,
    // QTSSReflectorModule.cpp:1804-1865, 1971-2004): first ingests what was pushed so far,
    // then fills outInfo[track] for the RTP-Info header.  kWouldBlock: nothing buffered yet,
    // retry the PLAY later (the reference's 100 ms idle timer); no output was added.
    int  PlayRTPInfo(uint32_t session, bool interleaved, int64_t nowMs, uint32_t* outHandle,
                     std::vector<edgpu_rtp_info>* outInfo);
    int  RemoveOutput(uint32_t handle);
    // the end of a push session (reference count 0, QTSSReflectorModule.cpp:2133-2196):
    // packets still pending for it are ingested first; killOutputs tears its outputs down with it
    int  RemoveSession(uint32_t session, bool killOutputs);
    // one pushed packet, exactly as ProcessRTPData hands it to ReflectorStream::PushPacket
    void PushPacket(uint32_t session, uint32_t track, const char* packet, uint32_t packetLen,
                    bool isRTCP, int64_t nowMs);
    // one datagram read from a UDP push session's socket pair (rtcpPort: the odd port), with
    // the source address GetIncomingData's RecvFrom returns (host order)
    void ProcessUDPPacket(uint32_t session, uint32_t track, bool rtcpPort, const char* packet,
                          uint32_t packetLen, uint32_t remoteAddr, uint16_t remotePort, int64_t nowMs);
    // the receiver-report SSRC / CNAME time a track's ReflectorStream would have drawn
    int  SetSourceIdentity(uint32_t session, uint32_t track, uint32_t ssrc, int64_t cnameSecs);
    // ingest everything pushed since the last call, update the keyframe index, fan out at
    // `nowMs` and deliver every send-ready packet to `sink` (per sub-stream, in order).
    int  ReflectPackets(int64_t nowMs, OutputSink* sink);
    // threads that deliver a tick's writes (default 1; at most 64); call between ticks
    void SetWriteThreads(uint32_t n);
    // the tick's writes run without the engine lock (see Threading above); default off
    void SetConcurrentDelivery(bool on);
    // the engine lock, for code that calls the edgpu ABI on Context() itself (CKeyFrameCache::LoadGOP)
    std::mutex& EngineMutex() { return fEngineMu; }
    uint32_t WriteThreads() const { return fNumWriters; }
    edgpu_ctx* Context() { return fCtx; }

    // per-tick measurements of the last ReflectPackets (tools/bench_module)
    struct TickInfo {
        uint64_t ingested_packets = 0, ingested_bytes = 0;   // batch handed to edgpu_ingest
        uint64_t readback_bytes = 0, arena_bytes = 0;       // PCIe bytes read back vs the arena
        uint64_t writes = 0;                                // OutputSink::Write calls
        uint64_t prestaged_bytes = 0;                       // of the batch, copied ahead while it filled
        uint32_t passes = 0;                                // copy passes (> 1: the tick exceeded the arena)
        uint32_t stream_errors = 0;                         // sessions the tick marked (edgpu_stream_errors)
        double ingest_ms = 0, fanout_ms = 0, readback_ms = 0, write_ms = 0;
    };
    const TickInfo& LastTick() const { return fTick; }
    // the sessions marked with a stream error (a sender ring lost a packet one of their outputs
    // needed) since the last call, and clears them: edgpu_stream_errors
    int StreamErrors(std::vector<uint32_t>* sessions);
    // diagnostics: one wave on the engine stream waits `us` of the device clock (edgpu_debug_stall)
    int DebugStall(uint32_t us);
    // the message of the last ReflectPackets failure that happened on another thread than the
    // caller's (edgpu_last_error() is per thread); empty otherwise
    const std::string& LastError() const { return fLastErr; }

private:
    int  FlushIngest();                                     // edgpu_ingest + keyframe index
    // one copy pass of a tick to the sink (ReflectPackets)
    int  DeliverPass(const edgpu_fanout_result& res, const edgpu_tick_stats& st, OutputSink* sink, bool firstPass,
                     std::vector<edgpu_blocked>* blockedOut);
    // every copy pass of a launched fan-out (ReflectPackets; on failure the caller drains the rest)
    int  DeliverTick(edgpu_fanout_result* res, edgpu_tick_stats* st, OutputSink* sink,
                     std::vector<edgpu_blocked>* blocked, std::chrono::steady_clock::time_point t0);
    int  fail_with(int code, const std::string& msg) { fLastErr = msg; return code; }
    std::string fLastErr;
    // the engine lock and the tick's write phase (SetConcurrentDelivery): fTickLock is the ticking
    // thread's hold of fEngineMu, given up during writes when fConcurrent; fDelivering is true from
    // a tick's first write to its backpressure report (waiters: fIdleCv on fEngineMu)
    std::mutex fEngineMu;
    std::condition_variable fIdleCv;
    bool fDelivering = false;
    bool fConcurrent = false;
    std::unique_lock<std::mutex>* fTickLock = nullptr;
    void WaitIdle(std::unique_lock<std::mutex>& lk) { fIdleCv.wait(lk, [&] { return !fDelivering; }); }
    int  ReflectPacketsLocked(int64_t nowMs, OutputSink* sink);
    // one pushed packet: its slot (16-B aligned, the packet 4 bytes in) in the batch's pinned blob
    struct Pushed { uint32_t session; uint8_t channel, flags; int64_t t; uint64_t slot; uint32_t len; };   // flags: EDGPU_PKT_*
    // The push path is striped by session (session % kStripes): a pusher takes only its stripe's
    // lock, and a stripe carves its slots out of 64-KiB slabs of the batch's pinned blob, so
    // pushers of different sessions share no lock and no counter per packet.
    static constexpr uint32_t kStripes = 16;
    static constexpr uint64_t kSlab = 64 << 10;
    struct alignas(64) Stripe {                             // one stripe's part of a batch (own lines:
                                                            // its counters change per packet)
        std::vector<Pushed> pushed;                         // arrival order (per session)
        std::vector<edgpu_udp_source> sources;              // UDP datagrams' sources, same order
        uint64_t slab = 0, used = 0, cap = 0;               // the current slab: blob offset, used, size
        std::atomic<uint32_t> copying{0};                   // reserved slots still being copied
    };
    struct Batch {
        uint8_t* blob = nullptr;                            // pinned (edgpu_host_alloc)
        uint64_t cap = 0;
        uint64_t next = 0;                                  // slab bump pointer (under a stripe lock + CAS)
        Stripe st[kStripes];
        // pinned descriptor / segment arrays, filled at the flush (grouped by session)
        edgpu_pkt_desc* desc = nullptr; uint32_t* seg = nullptr; uint32_t* segSess = nullptr;
        uint64_t descCap = 0;
        // Streaming the blob to the device while it fills (edgpu_ingest_prestage): per slab, the
        // copies still in flight and whether its stripe has moved on to another slab.  A sealed
        // slab with none in flight is final; the stager thread copies the prefix of final slabs
        // ahead, and the flush copies only the rest.
        struct alignas(64) Pend { std::atomic<uint32_t> n{0}; };   // own line: pushers of different
        std::unique_ptr<Pend[]> slabPend;                   // stripes count on neighbouring slabs
        std::unique_ptr<std::atomic<uint8_t>[]> slabSealed;
        uint64_t nslabs = 0;                                // slabs tracked (max_batch_bytes / kSlab)
        uint64_t staged = 0;                                // slabs copied ahead (under fStageMu)
    };
    struct alignas(64) StripeLock { std::mutex mu; };
    void LockAllStripes();
    void UnlockAllStripes();
    bool GrowBlob(Batch* b, uint64_t need);                 // all stripes quiescent; false: no memory
    void Append(uint32_t session, uint32_t track, const char* packet, uint32_t packetLen, bool isRTCP,
                int64_t nowMs, const edgpu_udp_source* src);
    // the write phase of a tick, for the subscribers of one worker
    struct WriteJob {
        const edgpu_substream_out* subs; uint32_t nsubs;   // the pass's active sub-streams (compact)
        const uint32_t* tabq = nullptr;                     // compact index -> sub-stream table row
        // sub-stream s's i-th write is rows[row_of[s] + i] (edgpu_fanout_rows: identity sub-streams
        // of one sender share their longest one's rows); its bytes are at regions->at(host, s) +
        // row.offset + delta[s]
        const edgpu_packet_row* rows; const uint32_t* row_of; const int64_t* delta;
        bool arrivals = false;                                          // the sink wants row.arrival
        const uint8_t* host; const edgpu_host::TickRegions* regions;   // the tick's bytes
        // identity UDP sub-streams without a region: every packet came with the batch this tick
        // ingested, still in `batch` (the pinned blob), at its row's source slot
        const uint8_t* batch = nullptr;
        OutputSink* sink;
        // the gather's parts: sub-streams [part_q[k-1], part_q[k]) need part k; `ready` counts the
        // parts in the pinned buffer; `failed`: a gather failed (the writers stop)
        uint32_t nparts = 1;
        const uint32_t* part_q = nullptr;
        std::atomic<uint32_t>* ready = nullptr;
        std::atomic<bool>* failed = nullptr;
        // one line per worker: the writers' results must not share a cache line (a per-packet
        // counter in a shared line serialised the write threads)
        struct alignas(64) Result { std::vector<edgpu_blocked> blocked; uint64_t writes = 0; int err = 0; };
        Result out[64];
    };
    void WriteSubscribers(WriteJob& j, uint32_t worker, uint32_t nworkers);
    void StagerLoop();
    // the stager thread (EDGPU_PRESTAGE_BYTES: the least it copies ahead at once, default 1 MiB;
    // 0: no stager, the flush copies the whole blob); fStageMu guards fStageArmed (the batch it
    // streams, -1 none), the batches' `staged` and their blob pointers against GrowBlob
    std::thread fStager;
    std::mutex fStageMu;
    std::condition_variable fStageCv;
    int fStageArmed = -1;
    bool fStageStop = false;
    uint64_t fPrestageBytes = 1ull << 20;
    void WorkerLoop(uint32_t worker);
    edgpu_ctx* fCtx = nullptr;
    int fStatus = kRequestFailed;
    // stripe k guards the fill batch's stripe k and fTracks[s] for s % kStripes == k; fFill and
    // fTracks' size change under all stripe locks
    StripeLock fStripe[kStripes];
    Batch fBatch[2];
    int fFill = 0;
    std::vector<uint32_t> fTracks;                          // per session (0: none)
    std::vector<uint32_t> fSortCount;                       // FlushIngest's counting sort by session
    std::vector<const Pushed*> fSortOrder;
    // readback buffers
    struct PinBuf { void* p = nullptr; uint64_t cap = 0; };  // pinned, grown on demand
    int  EnsurePinned(PinBuf& b, uint64_t bytes);
    PinBuf fPinSubs, fPinQ, fPinRows;                       // active sub-streams, their table rows, rows
    std::vector<uint32_t> fRowSel, fRowOf, fRowRep;         // edgpu_fanout_rows' selection, per sub-stream row start
    std::vector<int64_t> fRowDelta;
    const uint8_t* fIngestedBlob = nullptr;                 // the blob the last FlushIngest ingested (intact
                                                            // until the next one swaps it back in)
    bool fBatchSources = true;                              // EDGPU_BATCH_SOURCES=0: read every byte back
    bool fPushStreaming = true;                             // EDGPU_PUSH_STREAMING=0: cached stores in Append
    std::vector<uint8_t> fSkip;                             // per sub-stream: written from the batch
    uint64_t fGatherSplitBytes = 8ull << 20;               // see ReflectPackets
    uint32_t fGatherParts = 4;                              // EDGPU_GATHER_PARTS (<= TickParts::kMax)
    uint8_t* fHostOut = nullptr; uint64_t fHostOutCap = 0;  // pinned: the tick's gathered bytes (edgpu_arena_gather target)
    TickInfo fTick;
    // write threads (workers 1..n-1; the ticking thread is worker 0)
    uint32_t fNumWriters = 1;
    std::vector<std::thread> fWorkers;
    std::mutex fPoolMu;
    std::condition_variable fPoolCv, fPoolDone;
    WriteJob* fJob = nullptr;
    uint64_t fJobSeq = 0;
    uint32_t fJobsLeft = 0;
    bool fPoolStop = false;
};

// CKeyFrameCache with the reference's public API and TLV record format
// ([0x28][BE16 len][bytes][0x29], keyframecache.cpp:103-143).  PutOnePacket/GetOnePacket/
// SetBuf behave as in the reference, pinned to it by tests/golden/keyframecache_vectors.json
// -- including PutOnePacket's in-place rewrite of the caller's buf[13] (0x67 for an SPS start,
// else 0x41) -- except: no ./data.264 debug dump (keyframecache.cpp:25-50), no write past a
// packet shorter than 14 bytes, and packets over 5116 bytes are refused where the reference
// overruns its 5 KiB scratch.  LoadGOP() fills the cache from the GPU's GOP index (key
// pointer -> newest) instead of per-packet PutOnePacket.
class CKeyFrameCache {
public:
    char* _memory;
    int curdatalen;
    int mem_size;

    explicit CKeyFrameCache(int len);
    ~CKeyFrameCache();
    bool PutOnePacket(char* buf, int len, int nalutype, int start);
    bool GetOnePacket(char* outbuf, int& outLen, int curOffset);
    bool SetBuf(char* frameBuf, int len);
    int  LoadGOP(Reflector& r, uint32_t session, uint32_t track, uint32_t* outPackets = nullptr);
};

}  // namespace edgpu_reflector
