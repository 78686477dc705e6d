// reflector_adapter.cpp -- see reflector_adapter.h.
#include "reflector_adapter.h"
#include "tick_regions.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <emmintrin.h>

namespace edgpu_reflector {

using Clock = std::chrono::steady_clock;
static double ms_since(Clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

Reflector::Reflector(const edgpu_config* cfg) {
    fStatus = edgpu_ctx_create(cfg, &fCtx);
    // ticks with at least this many distinct bytes gather in parts, overlapped with the writes
    // (EDGPU_GATHER_SPLIT_BYTES; tests set 0 to run the pipelined path on small ticks)
    if (const char* v = getenv("EDGPU_GATHER_SPLIT_BYTES")) fGatherSplitBytes = strtoull(v, nullptr, 0);
    if (const char* v = getenv("EDGPU_GATHER_PARTS"))
        fGatherParts = std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)atoi(v), edgpu_host::TickParts::kMax));
    if (const char* v = getenv("EDGPU_PRESTAGE_BYTES")) fPrestageBytes = strtoull(v, nullptr, 0);
    if (const char* v = getenv("EDGPU_BATCH_SOURCES")) fBatchSources = atoi(v) != 0;
    // EDGPU_PUSH_STREAMING=0: the push path copies a slot with cached stores (no fence) instead of
    // streaming ones -- better when the batch being filled stays in the host's cache
    if (const char* v = getenv("EDGPU_PUSH_STREAMING")) fPushStreaming = atoi(v) != 0;
    if (fStatus || !fCtx) return;
    edgpu_config c;
    if (cfg) c = *cfg; else edgpu_config_default(&c);
    if (!c.max_batch_bytes) c.max_batch_bytes = 1ull << 30;      // 0: the engine's default (edgpu_ctx_create)
    for (Batch& b : fBatch) {
        b.nslabs = c.max_batch_bytes / kSlab + 1;
        b.slabPend.reset(new Batch::Pend[b.nslabs]);
        b.slabSealed.reset(new std::atomic<uint8_t>[b.nslabs]);
        for (uint64_t i = 0; i < b.nslabs; i++) { b.slabPend[i].n.store(0); b.slabSealed[i].store(0); }
    }
    if (fPrestageBytes) {
        fStageArmed = fFill;
        fStager = std::thread([this]() { StagerLoop(); });
    }
}

Reflector::~Reflector() {
    SetWriteThreads(1);
    if (fStager.joinable()) {
        { std::lock_guard<std::mutex> g(fStageMu); fStageStop = true; }
        fStageCv.notify_all();
        fStager.join();
    }
    if (!fCtx) return;
    (void)edgpu_sync(fCtx);
    for (Batch& b : fBatch)
        for (void* p : {(void*)b.blob, (void*)b.desc, (void*)b.seg, (void*)b.segSess})
            if (p) (void)edgpu_host_free(fCtx, p);
    if (fHostOut) (void)edgpu_host_free(fCtx, fHostOut);
    for (PinBuf* pb : {&fPinSubs, &fPinQ, &fPinRows})
        if (pb->p) (void)edgpu_host_free(fCtx, pb->p);
    edgpu_ctx_destroy(fCtx);
}

int Reflector::EnsurePinned(PinBuf& b, uint64_t bytes) {
    if (bytes <= b.cap) return kNoErr;
    if (b.p) (void)edgpu_host_free(fCtx, b.p);
    b.p = nullptr; b.cap = 0;
    const uint64_t cap = std::max<uint64_t>(bytes + bytes / 4, 1 << 16);
    const int err = edgpu_host_alloc(fCtx, cap, &b.p);
    if (!err) b.cap = cap;
    return err;
}

int Reflector::SetupReflectorSession(const std::string& sdp, bool udpPush, uint32_t* outSession) {
    if (!fCtx) return kRequestFailed;
    std::lock_guard<std::mutex> eg(fEngineMu);
    uint32_t s = 0, n = 0;
    int err = edgpu_session_add(fCtx, sdp.data(), (uint32_t)sdp.size(), udpPush ? 1 : 0, &s);
    if (err) return err;
    if ((err = edgpu_session_tracks(fCtx, s, &n))) return err;
    LockAllStripes();
    if (fTracks.size() <= s) fTracks.resize(s + 1, 0);
    fTracks[s] = n;
    UnlockAllStripes();
    if (outSession) *outSession = s;
    return kNoErr;
}

int Reflector::SetSSRCFilter(uint32_t session, bool oneSSRCPerStream, uint32_t timeoutSecs) {
    if (!fCtx) return kRequestFailed;
    std::lock_guard<std::mutex> eg(fEngineMu);
    return edgpu_session_ssrc_prefs(fCtx, session, oneSSRCPerStream ? 1 : 0, timeoutSecs);
}

uint32_t Reflector::GetNumStreams(uint32_t session) const {
    std::lock_guard<std::mutex> g(const_cast<std::mutex&>(fStripe[session % kStripes].mu));
    return session < fTracks.size() ? fTracks[session] : 0;
}

void Reflector::LockAllStripes() {
    for (StripeLock& l : fStripe) l.mu.lock();
}

void Reflector::UnlockAllStripes() {
    for (uint32_t k = kStripes; k-- > 0;) fStripe[k].mu.unlock();
}

// A larger pinned blob for batch b (the caller holds every stripe lock): waits for the copies in
// flight, moves the bytes so far over (the slots keep their offsets).
bool Reflector::GrowBlob(Batch* b, uint64_t need) {
    for (Stripe& st : b->st)
        while (st.copying.load(std::memory_order_acquire)) std::this_thread::yield();
    const uint64_t cap = std::max<uint64_t>(b->cap ? b->cap * 2 : (4ull << 20), need);
    void* nb = nullptr;
    if (edgpu_host_alloc(fCtx, cap, &nb) != 0) return false;
    if (b->next) memcpy(nb, b->blob, b->next);
    // the stager reads the blob pointer under fStageMu; edgpu_host_free waits for its copies
    std::lock_guard<std::mutex> g(fStageMu);
    if (b->blob) (void)edgpu_host_free(fCtx, b->blob);
    b->blob = (uint8_t*)nb;
    b->cap = cap;
    return true;
}

// Copies the finished prefix of the batch being filled to the device (edgpu_ingest_prestage)
// whenever it has grown by fPrestageBytes, so that the tick's ingest finds most of its blob there.
void Reflector::StagerLoop() {
    std::unique_lock<std::mutex> lk(fStageMu);
    while (!fStageStop) {
        // idle (no batch armed) until a flush arms one; while armed, a look every 200 us
        if (fStageArmed < 0) fStageCv.wait(lk, [&] { return fStageStop || fStageArmed >= 0; });
        else fStageCv.wait_for(lk, std::chrono::microseconds(200));
        if (fStageStop || fStageArmed < 0) continue;
        Batch& b = fBatch[fStageArmed];
        const uint64_t lim = std::min<uint64_t>(__atomic_load_n(&b.next, __ATOMIC_ACQUIRE) / kSlab, b.nslabs);
        uint64_t e = b.staged;
        while (e < lim && b.slabSealed[e].load(std::memory_order_acquire) &&
               b.slabPend[e].n.load(std::memory_order_acquire) == 0)
            e++;
        if ((e - b.staged) * kSlab < fPrestageBytes) continue;
        if (edgpu_ingest_prestage(fCtx, b.blob, b.staged * kSlab, (e - b.staged) * kSlab) != 0) {
            fStageArmed = -1;                                // the flush copies the rest
            continue;
        }
        b.staged = e;
    }
}

int Reflector::AddOutput(uint32_t session, bool interleaved, uint32_t* outHandle) {
    if (!fCtx) return kRequestFailed;
    std::lock_guard<std::mutex> eg(fEngineMu);
    return edgpu_subscriber_add(fCtx, session, interleaved ? EDGPU_TRANSPORT_TCP : EDGPU_TRANSPORT_UDP, outHandle);
}

int Reflector::PlayRTPInfo(uint32_t session, bool interleaved, int64_t nowMs, uint32_t* outHandle,
                           std::vector<edgpu_rtp_info>* outInfo) {
    if (!fCtx) return kRequestFailed;
    std::unique_lock<std::mutex> eg(fEngineMu);
    WaitIdle(eg);                                           // a tick's writes may read the batch
    int err = FlushIngest();
    if (err) return err;
    std::vector<edgpu_rtp_info> info(std::max<uint32_t>(GetNumStreams(session), 1));
    err = edgpu_subscriber_play(fCtx, session, interleaved ? EDGPU_TRANSPORT_TCP : EDGPU_TRANSPORT_UDP,
                                EDGPU_PLAY_RTP_INFO, nowMs, outHandle, info.data());
    if (!err && outInfo) *outInfo = info;
    return err;
}

int Reflector::RemoveOutput(uint32_t handle) {
    if (!fCtx) return kRequestFailed;
    std::lock_guard<std::mutex> eg(fEngineMu);
    return edgpu_subscriber_remove(fCtx, handle);
}

int Reflector::RemoveSession(uint32_t session, bool killOutputs) {
    if (!fCtx) return kRequestFailed;
    std::unique_lock<std::mutex> eg(fEngineMu);
    WaitIdle(eg);                                           // a tick's writes may read the batch
    // what was pushed to it before the end is ingested (the reference had queued it)
    int err = FlushIngest();
    if (err) return err;
    // the engine first: if it refuses (outputs still attached without killOutputs, a device
    // error), the session lives on and its pushes keep flowing
    if ((err = edgpu_session_remove(fCtx, session, killOutputs ? EDGPU_SESSION_KILL_OUTPUTS : 0))) return err;
    {
        // later pushes to it are dropped, and what another thread pushed since the flush is
        // discarded (its id may be reused by the next session)
        std::lock_guard<std::mutex> g(fStripe[session % kStripes].mu);
        if (session < fTracks.size()) fTracks[session] = 0;
        Stripe& st = fBatch[fFill].st[session % kStripes];
        st.pushed.erase(std::remove_if(st.pushed.begin(), st.pushed.end(),
                                       [&](const Pushed& p) { return p.session == session; }), st.pushed.end());
        st.sources.erase(std::remove_if(st.sources.begin(), st.sources.end(),
                                        [&](const edgpu_udp_source& u) { return u.session == session; }), st.sources.end());
    }
    return kNoErr;
}

// Writes one packet's slot ([4 zero bytes][packet][zero pad to 16], `slot` bytes at the 16-B
// aligned `d`) with streaming stores: the batch leaves by DMA and is never read back by this core,
// so the stores skip the read-for-ownership a cached copy pays per line (about half the push
// path's per-packet time at C2).  The caller fences before publishing the slot.
static void stream_slot(uint8_t* d, const char* p, uint32_t n, uint64_t slot) {
    alignas(16) uint8_t t[16];
    memset(t, 0, sizeof(t));
    const uint32_t h = std::min<uint32_t>(n, 12);
    memcpy(t + 4, p, h);
    _mm_stream_si128(reinterpret_cast<__m128i*>(d), _mm_load_si128(reinterpret_cast<const __m128i*>(t)));
    uint64_t off = 16;
    const char* s = p + h;
    uint32_t left = n - h;
    for (; left >= 16; left -= 16, s += 16, off += 16)
        _mm_stream_si128(reinterpret_cast<__m128i*>(d + off), _mm_loadu_si128(reinterpret_cast<const __m128i*>(s)));
    if (off < slot) {                                      // the last bytes and the zero pad
        memset(t, 0, sizeof(t));
        memcpy(t, s, left);
        _mm_stream_si128(reinterpret_cast<__m128i*>(d + off), _mm_load_si128(reinterpret_cast<const __m128i*>(t)));
    }
}

// The same slot with ordinary (cached) stores: header room zeroed, packet, zero pad.
static void cached_slot(uint8_t* d, const char* p, uint32_t n, uint64_t slot) {
    memset(d, 0, 4);
    memcpy(d + 4, p, n);
    memset(d + 4 + n, 0, slot - 4 - n);
}

// Appends one packet's slot ([4-B interleave header room][packet][pad to 16]) to the batch being
// filled: the only host copy of the packet.  Under its stripe's lock the pusher reserves the slot
// in the stripe's slab (a new 64-KiB slab from the blob when it is full); it copies the packet
// after releasing the lock (`copying` counts copies in flight: a flush or a blob growth waits
// for them).  The pinned blob grows by doubling under every stripe lock (the slots so far
// copied over); the batch being filled is never one whose DMA may be in flight.
void Reflector::Append(uint32_t session, uint32_t track, const char* packet, uint32_t packetLen, bool isRTCP,
                       int64_t nowMs, const edgpu_udp_source* src) {
    const uint32_t clamped = std::min<uint32_t>(packetLen, 2060);   // bytes past 2060 are never read (Q11)
    const uint64_t slot = (clamped + 4 + 15) & ~15ull;
    const uint32_t k = session % kStripes;
    Stripe* sp = nullptr;
    uint8_t* d = nullptr;
    std::atomic<uint32_t>* pend = nullptr;
    for (;;) {
        std::unique_lock<std::mutex> g(fStripe[k].mu);
        if (session >= fTracks.size() || track >= fTracks[session]) return;
        Batch& b = fBatch[fFill];
        Stripe& st = b.st[k];
        if (st.used + slot > st.cap) {                       // a new slab
            // b.next moves by CAS under other stripes' locks: read it atomically
            if (__atomic_load_n(&b.next, __ATOMIC_RELAXED) + kSlab > b.cap) {
                // grow under every stripe lock (taken in order: release ours first), then retry
                g.unlock();
                LockAllStripes();
                Batch& bb = fBatch[fFill];
                const bool ok = bb.next + kSlab <= bb.cap || GrowBlob(&bb, bb.next + kSlab);
                UnlockAllStripes();
                if (!ok) return;                             // out of pinned memory: dropped
                continue;
            }
            // other stripes take slabs under their own locks: the bump pointer is a CAS
            uint64_t off = __atomic_load_n(&b.next, __ATOMIC_RELAXED);
            while (off + kSlab <= b.cap &&
                   !__atomic_compare_exchange_n(&b.next, &off, off + kSlab, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {}
            if (off + kSlab > b.cap) continue;               // lost the race for the last slab: grow
            // the stripe's previous slab is complete once its copies in flight are
            if (st.cap && st.slab / kSlab < b.nslabs) b.slabSealed[st.slab / kSlab].store(1, std::memory_order_release);
            st.slab = off; st.used = 0; st.cap = kSlab;
        }
        d = b.blob + st.slab + st.used;
        if (st.slab / kSlab < b.nslabs) {
            pend = &b.slabPend[st.slab / kSlab].n;
            pend->fetch_add(1, std::memory_order_relaxed);
        }
        // a datagram from an odd source port: GetSSRC(theRemotePort & 1) of the receive-time trailer
        const uint8_t fl = (src && (src->port & 1)) ? (uint8_t)EDGPU_PKT_REMOTE_ODD : (uint8_t)0;
        st.pushed.push_back(Pushed{session, (uint8_t)(2 * track + (isRTCP ? 1 : 0)), fl, nowMs, st.slab + st.used, packetLen});
        if (src) st.sources.push_back(*src);
        st.used += slot;
        st.copying.fetch_add(1, std::memory_order_relaxed);
        sp = &st;
        break;
    }
    if (fPushStreaming) {
        stream_slot(d, packet, clamped, slot);
        _mm_sfence();                                    // the slot is complete before it is published
    } else {
        cached_slot(d, packet, clamped, slot);           // (ordinary stores: ordered by the release below)
    }
    if (pend) pend->fetch_sub(1, std::memory_order_release);
    sp->copying.fetch_sub(1, std::memory_order_release);
}

void Reflector::PushPacket(uint32_t session, uint32_t track, const char* packet, uint32_t packetLen,
                           bool isRTCP, int64_t nowMs) {
    // ReflectorStream::PushPacket ignores empty packets (ReflectorStream.cpp:533); the
    // '$' framing caps a pushed packet at 65535 bytes.
    if (packetLen == 0 || !fCtx) return;
    Append(session, track, packet, std::min<uint32_t>(packetLen, 65535), isRTCP, nowMs, nullptr);
}

void Reflector::ProcessUDPPacket(uint32_t session, uint32_t track, bool rtcpPort, const char* packet,
                                 uint32_t packetLen, uint32_t remoteAddr, uint16_t remotePort, int64_t nowMs) {
    if (packetLen == 0 || !fCtx) return;
    edgpu_udp_source u;
    memset(&u, 0, sizeof(u));
    u.session = session;
    u.channel = (uint8_t)(2 * track + (rtcpPort ? 1 : 0));
    u.port = remotePort;
    u.addr = remoteAddr;
    u.len = packetLen;
    memcpy(u.head, packet, std::min<uint32_t>(packetLen, 4));
    Append(session, track, packet, packetLen, rtcpPort, nowMs, &u);
}

int Reflector::DebugStall(uint32_t us) {
    if (!fCtx) return kRequestFailed;
    std::lock_guard<std::mutex> eg(fEngineMu);
    return edgpu_debug_stall(fCtx, us);
}

int Reflector::SetSourceIdentity(uint32_t session, uint32_t track, uint32_t ssrc, int64_t cnameSecs) {
    if (!fCtx) return kRequestFailed;
    std::lock_guard<std::mutex> eg(fEngineMu);
    return edgpu_source_identity(fCtx, session, track, ssrc, cnameSecs);
}

int Reflector::FlushIngest() {
    const auto t0 = Clock::now();
    fTick.ingested_packets = fTick.ingested_bytes = 0;
    fIngestedBlob = nullptr;
    // The batch to become the fill buffer was handed to edgpu_ingest two flushes ago; every call
    // that flushed has synchronised the stream since (fan-out stats, PLAY, session removal), so its
    // DMA is done -- this sync is the guarantee for error paths (idle stream: microseconds).
    int err = edgpu_sync(fCtx);
    if (err) return err;
    {   // the stager leaves this batch
        std::lock_guard<std::mutex> g(fStageMu);
        fStageArmed = -1;
        fTick.prestaged_bytes = fBatch[fFill].staged * kSlab;
    }
    LockAllStripes();
    Batch& b = fBatch[fFill];
    fFill ^= 1;
    {   // the batch to be filled now starts with no slab sealed and nothing copied ahead
        Batch& nb = fBatch[fFill];
        std::lock_guard<std::mutex> g(fStageMu);
        for (uint64_t i = 0; i < nb.nslabs; i++) nb.slabSealed[i].store(0, std::memory_order_relaxed);
        nb.staged = 0;
    }
    UnlockAllStripes();
    for (Stripe& st : b.st)                                  // pushers mid-copy
        while (st.copying.load(std::memory_order_acquire)) std::this_thread::yield();
    uint32_t n = 0;
    for (const Stripe& st : b.st) n += (uint32_t)st.pushed.size();
    // slabs of this batch the stager copied ahead: if no pinned ingest consumes them (nothing
    // left to ingest, e.g. RemoveSession dropped the only session's packets, or an error below),
    // the engine must drop them, or the next batch would keep this one's prefix
    bool ingested = false;
    auto drop_prestage = [&]() { if (fTick.prestaged_bytes && !ingested) (void)edgpu_ingest_prestage(fCtx, nullptr, 0, 0); };
    if (n) {
        // descriptors grouped by session (a session's packets are all in one stripe, in arrival
        // order): a stable counting sort by session id; the slots stay where the pushers wrote them
        uint32_t nsess = 0;
        for (const Stripe& st : b.st)
            for (const Pushed& p : st.pushed) nsess = std::max(nsess, p.session + 1);
        fSortCount.assign((size_t)nsess + 1, 0);
        for (const Stripe& st : b.st)
            for (const Pushed& p : st.pushed) fSortCount[p.session + 1]++;
        for (uint32_t s = 0; s < nsess; s++) fSortCount[s + 1] += fSortCount[s];
        fSortOrder.resize(n);
        std::vector<const Pushed*>& order = fSortOrder;
        for (const Stripe& st : b.st)
            for (const Pushed& p : st.pushed) order[fSortCount[p.session]++] = &p;
        if (b.descCap < n) {
            for (void* p : {(void*)b.desc, (void*)b.seg, (void*)b.segSess})
                if (p) (void)edgpu_host_free(fCtx, p);
            b.desc = nullptr; b.seg = b.segSess = nullptr; b.descCap = 0;
            const uint64_t cap = std::max<uint64_t>(n, 4096);
            void *d = nullptr, *sg = nullptr, *ss = nullptr;
            if ((err = edgpu_host_alloc(fCtx, cap * sizeof(edgpu_pkt_desc), &d)) ||
                (err = edgpu_host_alloc(fCtx, (cap + 1) * sizeof(uint32_t), &sg)) ||
                (err = edgpu_host_alloc(fCtx, cap * sizeof(uint32_t), &ss))) {
                for (void* p : {d, sg, ss}) if (p) (void)edgpu_host_free(fCtx, p);
                drop_prestage();
                return err;
            }
            b.desc = (edgpu_pkt_desc*)d; b.seg = (uint32_t*)sg; b.segSess = (uint32_t*)ss; b.descCap = cap;
        }
        uint32_t nseg = 0;
        for (uint32_t k = 0; k < n; k++) {
            const Pushed& p = *order[k];
            if (nseg == 0 || b.segSess[nseg - 1] != p.session) { b.seg[nseg] = k; b.segSess[nseg] = p.session; nseg++; }
            b.desc[k].slot = (uint32_t)(p.slot / 16);
            b.desc[k].len = (uint16_t)p.len;
            b.desc[k].channel = p.channel;
            b.desc[k].flags = p.flags;
            b.desc[k].arrival_ms = p.t;
            fTick.ingested_bytes += p.len;
        }
        b.seg[nseg] = n;
        fTick.ingested_packets = n;
        err = edgpu_ingest(fCtx, b.desc, n, b.seg, b.segSess, nseg, b.blob, b.next, EDGPU_PTR_PINNED);
        ingested = true;                                     // (a refused batch drops the prestage itself)
        if (!err) fIngestedBlob = b.blob;                    // intact until the next flush swaps it back in
        if (!err) err = edgpu_keyframe_index(fCtx);
    }
    drop_prestage();
    std::vector<edgpu_udp_source> sources;
    for (const Stripe& st : b.st) sources.insert(sources.end(), st.sources.begin(), st.sources.end());
    for (Stripe& st : b.st) { st.pushed.clear(); st.sources.clear(); st.slab = st.used = st.cap = 0; }
    b.next = 0;
    if (fStager.joinable() && !err) {   // the stager streams the batch being filled into the
        {                               // staging set the next ingest uses
            std::lock_guard<std::mutex> g(fStageMu);
            fStageArmed = fFill;
        }
        fStageCv.notify_one();
    }
    if (err) return err;
    if (!sources.empty() && (err = edgpu_udp_sources(fCtx, sources.data(), (uint32_t)sources.size()))) return err;
    fTick.ingest_ms = ms_since(t0);
    return kNoErr;
}

int Reflector::StreamErrors(std::vector<uint32_t>* sessions) {
    if (!fCtx || !sessions) return kBadArgument;
    std::lock_guard<std::mutex> eg(fEngineMu);
    sessions->clear();
    uint32_t n = 0;
    int err = edgpu_stream_errors(fCtx, nullptr, nullptr, 0, &n);
    if (err || !n) return err;
    std::vector<int32_t> codes(n);
    sessions->resize(n);
    if ((err = edgpu_stream_errors(fCtx, sessions->data(), codes.data(), n, &n))) return err;
    sessions->resize(std::min<size_t>(n, sessions->size()));
    return kNoErr;
}

int Reflector::ReflectPackets(int64_t nowMs, OutputSink* sink) {
    if (!fCtx) return kRequestFailed;
    std::unique_lock<std::mutex> eg(fEngineMu);
    fTickLock = &eg;
    const int err = ReflectPacketsLocked(nowMs, sink);
    fTickLock = nullptr;
    if (fDelivering) {                                      // the tick is over: waiters may ingest
        fDelivering = false;
        fIdleCv.notify_all();
    }
    return err;
}

void Reflector::SetConcurrentDelivery(bool on) {
    std::unique_lock<std::mutex> eg(fEngineMu);
    WaitIdle(eg);
    fConcurrent = on;
}

int Reflector::ReflectPacketsLocked(int64_t nowMs, OutputSink* sink) {
    fLastErr.clear();
    int err = FlushIngest();
    if (err) return err;
    auto t0 = Clock::now();
    fTick.readback_bytes = fTick.arena_bytes = fTick.writes = 0;
    fTick.fanout_ms = fTick.readback_ms = fTick.write_ms = 0;
    fTick.passes = 0;
    fTick.stream_errors = 0;
    edgpu_fanout_result res;
    if ((err = edgpu_fanout(fCtx, nowMs, &res))) return err;
    uint32_t nrr = 0;
    err = edgpu_source_reports(fCtx, nullptr, 0, &nrr);
    if (err && nrr) err = kNoErr;
    if (!err && nrr && sink) {
        std::vector<edgpu_source_report> rr(nrr);
        if (!(err = edgpu_source_reports(fCtx, rr.data(), nrr, &nrr)))
            for (const edgpu_source_report& r : rr)
                sink->SendReceiverReport(r.session, r.track, r.addr, r.port, r.bytes, r.len);
    }
    edgpu_tick_stats st;
    std::vector<edgpu_blocked> blocked;
    if (!err) err = DeliverTick(&res, &st, sink, &blocked, t0);
    if (err) {
        // A pass that failed must not leave the context owing the rest of the tick: every later
        // ingest, fan-out and session removal would be refused for good.  The remaining passes are
        // launched without delivery (the engine counts them in lost_passes) and the blocked
        // sub-streams of the passes delivered so far are still reported; the first error stands.
        for (uint32_t guard = 0; guard < (1u << 20); guard++) {
            uint32_t launched = 0;
            if (edgpu_fanout_next(fCtx, &res, &launched) != 0 || !launched) break;
        }
    }
    if (blocked.empty()) return err;
    std::sort(blocked.begin(), blocked.end(),
              [](const edgpu_blocked& a, const edgpu_blocked& b) { return a.substream < b.substream; });
    const int berr = edgpu_fanout_blocked(fCtx, blocked.data(), (uint32_t)blocked.size());
    return err ? err : berr;
}

// Every copy pass of the tick fan-out launched (its first pass): a tick over the arena comes in
// copy passes of consecutive sub-stream rows (edgpu_fanout_next), each delivered before the next is
// copied, so every output gets the whole tick, in the order one pass would have written it.
// Backpressure reports cover the whole tick (appended to *blocked, reported by the caller).
int Reflector::DeliverTick(edgpu_fanout_result* res, edgpu_tick_stats* stp, OutputSink* sink,
                           std::vector<edgpu_blocked>* blocked, Clock::time_point t0) {
    edgpu_tick_stats& st = *stp;
    int err;
    if ((err = edgpu_tick_stats_get(fCtx, &st))) return err;
    fTick.fanout_ms = ms_since(t0);
    if (st.status) return st.status;
    fTick.stream_errors = st.stream_errors;             // the tick went on for every other session
    fTick.arena_bytes = st.arena_bytes;
    for (uint32_t pass = 0;; pass++) {
        fTick.passes++;
        if (sink && st.pass_packets) {
            if ((err = DeliverPass(*res, st, sink, pass == 0, blocked))) return err;
        }
        if (!st.more_passes) break;
        uint32_t launched = 0;
        if ((err = edgpu_fanout_next(fCtx, res, &launched))) return err;
        if (!launched) break;
        if ((err = edgpu_tick_stats_get(fCtx, &st))) return err;
        if (st.status) return st.status;
    }
    return kNoErr;
}

// One copy pass: its sub-stream table, descriptors (and arrivals) and distinct bytes come to pinned
// memory, and the write threads deliver its sub-streams; the ones that blocked are appended.
int Reflector::DeliverPass(const edgpu_fanout_result& res, const edgpu_tick_stats& st, OutputSink* sink,
                           bool firstPass, std::vector<edgpu_blocked>* blockedOut) {
    int err;
    auto t0 = Clock::now();
    // the pass's sub-streams with packets (and the new outputs), compacted in table order into
    // pinned buffers (edgpu_fanout_active: at 2-ms ticks a few % of the table -- every host loop
    // below and every write thread walks only them), then the rows of the writes: one per
    // descriptor of a sub-stream that is not an identity one, one per packet of each sender's
    // identity sub-streams (its longest one's rows serve the others, edgpu_fanout_rows).  Below,
    // a sub-stream is its compact index; fActiveQ maps it to its table row.
    const uint32_t ntab = res.n_substreams;
    if ((err = EnsurePinned(fPinSubs, (uint64_t)std::max<uint32_t>(ntab, 1) * sizeof(edgpu_substream_out))) ||
        (err = EnsurePinned(fPinQ, (uint64_t)std::max<uint32_t>(ntab, 1) * sizeof(uint32_t))))
        return err;
    const edgpu_substream_out* subs = (const edgpu_substream_out*)fPinSubs.p;
    const uint32_t* tabq = (const uint32_t*)fPinQ.p;
    uint32_t nq = 0;
    if ((err = edgpu_fanout_active(fCtx, (edgpu_substream_out*)fPinSubs.p, (uint32_t*)fPinQ.p, ntab, &nq, EDGPU_PTR_HOST)))
        return err;
    if (nq > ntab) return fail_with(kRequestFailed, "active sub-streams exceed the table");
    fRowOf.assign(nq, 0);
    fRowDelta.assign(nq, 0);
    uint64_t nrows = 0;
    // the representative tick_regions gathers (the longest by bytes): its rows serve the
    // sender's other identity sub-streams, each a suffix of it in bytes and in packets
    fRowRep = edgpu_host::identity_reps(subs, nq);
    fRowSel.clear();
    for (uint32_t q = 0; q < nq; q++) {
        const edgpu_substream_out& s = subs[q];
        if (!s.desc_count || ((s.flags & EDGPU_SUB_IDENTITY) && fRowRep[s.sender] != q)) continue;
        fRowSel.push_back(tabq[q]);
        fRowSel.push_back((uint32_t)nrows);
        fRowOf[q] = (uint32_t)nrows;
        fRowDelta[q] = -(int64_t)s.out_base;
        nrows += s.desc_count;
    }
    for (uint32_t q = 0; q < nq; q++) {             // the others of a sender: a suffix of its rows
        const edgpu_substream_out& s = subs[q];
        if (!s.desc_count || !(s.flags & EDGPU_SUB_IDENTITY) || fRowRep[s.sender] == q) continue;
        const edgpu_substream_out& R = subs[fRowRep[s.sender]];
        fRowOf[q] = fRowOf[fRowRep[s.sender]] + (R.desc_count - s.desc_count);
        fRowDelta[q] = -(int64_t)R.out_base - (int64_t)(R.out_bytes - s.out_bytes);
    }
    if (nrows > 0xFFFFFFFFull) return fail_with(kRequestFailed, "tick rows exceed 2^32");
    if ((err = EnsurePinned(fPinRows, nrows * sizeof(edgpu_packet_row)))) return err;
    if ((err = edgpu_fanout_rows(fCtx, fRowSel.data(), (uint32_t)(fRowSel.size() / 2), (edgpu_packet_row*)fPinRows.p,
                                 nrows, EDGPU_PTR_HOST)))
        return err;
    // the suffix sharing holds only if every sub-stream's first row is where its bytes start in
    // the representative's region (a UDP datagram 4 bytes into its slot, after the interleave
    // header room); a plan that broke it would write wrong bytes silently
    const edgpu_packet_row* rw = (const edgpu_packet_row*)fPinRows.p;
    for (uint32_t q = 0; q < nq; q++) {
        const edgpu_substream_out& s = subs[q];
        if (!s.desc_count || !(s.flags & EDGPU_SUB_IDENTITY) || fRowRep[s.sender] == q) continue;
        const edgpu_substream_out& R = subs[fRowRep[s.sender]];
        if (R.desc_count < s.desc_count || R.out_bytes < s.out_bytes ||
            rw[fRowOf[q]].offset != R.out_base + (R.out_bytes - s.out_bytes) +
                                        (s.transport == EDGPU_TRANSPORT_TCP ? 0u : 4u))
            return fail_with(kRequestFailed, "identity sub-stream is not a suffix of its sender's longest");
    }
    const edgpu_packet_row* rows = (const edgpu_packet_row*)fPinRows.p;
    // Packets that came with the batch this tick ingested are still in its pinned blob: an identity
    // UDP sub-stream made only of them is written from there (its wire bytes are the packets') and
    // needs no readback.  The rest -- GOP replays of new outputs, earlier batches, interleaved or
    // rewritten sub-streams -- is gathered.
    const bool useSrc = fBatchSources && fIngestedBlob != nullptr;
    fSkip.assign(useSrc ? nq : 0, 0);
    if (useSrc)
        for (uint32_t q = 0; q < nq; q++) {
            const edgpu_substream_out& s = subs[q];
            if (!s.desc_count || !(s.flags & EDGPU_SUB_IDENTITY)) continue;
            // a sub-stream is a range of its sender's queue and the batch is the queue's newest
            // part: all its packets came with the batch iff its first one did
            fSkip[q] = rows[fRowOf[q]].source != EDGPU_NO_SOURCE ? 1 : 0;
        }
    // the pass's distinct bytes only: one region per identity sender + the other sub-streams
    const edgpu_host::TickRegions tr = edgpu_host::tick_regions(subs, nq, useSrc ? fSkip.data() : nullptr);
    if (tr.bytes > fHostOutCap) {            // grown geometrically: pinning costs ~40 ms per call
        if (fHostOut) (void)edgpu_host_free(fCtx, fHostOut);
        fHostOut = nullptr; fHostOutCap = 0;
        void* h = nullptr;
        const uint64_t cap = std::max<uint64_t>(tr.bytes + tr.bytes / 2, 1 << 20);
        if ((err = edgpu_host_alloc(fCtx, cap, &h))) return err;
        fHostOut = (uint8_t*)h;
        fHostOutCap = cap;
    }
    fTick.readback_bytes += tr.bytes + (uint64_t)nq * (sizeof(edgpu_substream_out) + sizeof(uint32_t)) +
                            nrows * sizeof(edgpu_packet_row);
    // The distinct bytes are gathered straight into the pinned buffer (the kernel's stores cross
    // PCIe, one pass) in up to TickParts::kMax parts of the sub-stream table, each part's regions after the
    // previous part's: with several write threads a gather thread brings part k + 1 over while the
    // writers deliver part k (a sub-stream only uses regions created at or before its own index).
    const edgpu_host::TickParts parts =
        edgpu_host::tick_parts(tr, nq, fNumWriters > 1 && tr.bytes >= fGatherSplitBytes ? fGatherParts : 1);
    const uint32_t nparts = parts.n;
    const uint32_t* part_q = parts.q;
    const uint32_t* part_r = parts.r;
    // with concurrent delivery the engine lock is given up while the writes run: the gatherer's
    // later parts then take it per part, as any other engine call does
    const bool release = fConcurrent && fTickLock != nullptr;
    auto gather = [&](uint32_t k) -> int {
        const uint32_t r0 = part_r[k], r1 = part_r[k + 1];
        if (r1 <= r0) return kNoErr;
        std::unique_lock<std::mutex> gl(fEngineMu, std::defer_lock);
        if (release && k > 0) gl.lock();
        return edgpu_arena_gather(fCtx, &res, tr.reg.data() + r0, r1 - r0, fHostOut + tr.reg_off[r0],
                                  fHostOutCap - tr.reg_off[r0]);
    };
    if ((err = gather(0))) return err;
    std::atomic<uint32_t> ready{1};
    std::atomic<bool> failed{false};
    int gatherErr = kNoErr;
    std::string gatherMsg;
    std::thread gatherer;
    if (nparts > 1)
        gatherer = std::thread([&] {
            for (uint32_t k = 1; k < nparts; k++) {
                if ((gatherErr = gather(k))) {
                    gatherMsg = edgpu_last_error();          // per thread: keep it for the tick thread
                    failed.store(true, std::memory_order_relaxed);
                    ready.store(nparts, std::memory_order_release);   // release the waiting writers
                    return;
                }
                ready.store(k + 1, std::memory_order_release);
            }
        });
    fTick.readback_ms += ms_since(t0);
    t0 = Clock::now();
    fDelivering = true;                                     // until the tick's end (ReflectPackets)
    if (release) fTickLock->unlock();
    struct Relock {                                         // the engine lock back for what follows
        std::unique_lock<std::mutex>* l;
        ~Relock() { if (l) l->lock(); }
    } relock{release ? fTickLock : nullptr};
    if (firstPass) sink->BeginTick(subs, nq);               // every row carries its flags in every pass
    WriteJob job;
    job.subs = subs; job.nsubs = nq; job.tabq = tabq;
    job.rows = rows; job.row_of = fRowOf.data(); job.delta = fRowDelta.data();
    job.arrivals = sink->WantsArrivals();
    job.batch = useSrc ? fIngestedBlob : nullptr;
    job.sink = sink;
    job.host = fHostOut;
    job.regions = &tr;
    job.nparts = nparts; job.part_q = part_q; job.ready = &ready; job.failed = &failed;
    const uint32_t nw = fNumWriters;
    if (nw == 1) {
        WriteSubscribers(job, 0, 1);
    } else {
        {
            std::lock_guard<std::mutex> g(fPoolMu);
            fJob = &job;
            fJobsLeft = nw - 1;
            fJobSeq++;
        }
        fPoolCv.notify_all();
        WriteSubscribers(job, 0, nw);
        std::unique_lock<std::mutex> g(fPoolMu);
        fPoolDone.wait(g, [&] { return fJobsLeft == 0; });
        fJob = nullptr;
    }
    if (gatherer.joinable()) gatherer.join();
    if (gatherErr) return fail_with(gatherErr, gatherMsg);
    // SendPacketsToOutput (ReflectorStream.cpp:1138-1198): a write that would block stopped its
    // sub-stream for the tick; the engine bookmarks the blocked packet
    for (uint32_t k = 0; k < nw; k++) {
        const WriteJob::Result& r = job.out[k];
        fTick.writes += r.writes;
        if (r.err) return r.err;
        blockedOut->insert(blockedOut->end(), r.blocked.begin(), r.blocked.end());
    }
    fTick.write_ms += ms_since(t0);
    return kNoErr;
}

// The worker of a sub-stream: by its session (the sender of track t, kind k is the session's first
// sender + 2t + k), so all of one subscriber's sub-streams -- and every subscriber of a session,
// which read the same packet bytes -- go to one thread.
static inline uint32_t writer_of(const edgpu_substream_out& q, uint32_t nworkers) {
    const uint32_t session_key = q.sender - (2u * q.track + q.kind);
    return (uint32_t)(((uint64_t)(session_key * 0x9E3779B1u) * nworkers) >> 32);
}

// The writes of the subscribers of one worker, sub-stream by sub-stream in table order (the order
// one thread takes): a write that would block stops that sub-stream.
void Reflector::WriteSubscribers(WriteJob& j, uint32_t worker, uint32_t nworkers) {
    struct End {
        OutputSink* s; uint32_t w;
        ~End() { s->EndWrites(w); }
    } end{j.sink, worker};
    WriteJob::Result& r = j.out[worker];
    r.err = kNoErr;
    r.blocked.clear();
    uint64_t writes = 0;
    uint32_t part = 0;
    for (uint32_t s = 0; s < j.nsubs; s++) {
        const edgpu_substream_out& q = j.subs[s];
        if (!q.desc_count || (nworkers > 1 && writer_of(q, nworkers) != worker)) continue;
        while (part + 1 < j.nparts && s >= j.part_q[part]) part++;
        // its packets all in the ingested batch: read them there; else its bytes are in part
        // `part` of the gather: wait for it (a failed gather also ends the wait; the tick then
        // returns its error)
        const bool fromBatch = j.regions->src[s].first == edgpu_host::TickRegions::kNone;
        if (!fromBatch) {
            while (j.ready->load(std::memory_order_acquire) <= part) std::this_thread::yield();
            if (j.failed->load(std::memory_order_relaxed)) { r.writes = writes; return; }
        }
        const uint8_t* base = fromBatch ? nullptr : j.regions->at(j.host, s);
        const int64_t delta = j.delta[s];
        const edgpu_packet_row* row = j.rows + j.row_of[s];
        for (uint32_t i = 0; i < q.desc_count; i++) {
            const edgpu_packet_row& o = row[i];
            PacketWrite w;
            w.subscriber = q.subscriber;
            w.track = q.track;
            w.isRTCP = q.kind != 0;
            w.interleaved = q.transport == EDGPU_TRANSPORT_TCP;
            // (a batch slot holds 4 bytes of interleave-header room, then the packet)
            w.wire = fromBatch ? j.batch + (uint64_t)o.source * 16 + 4 : base + ((int64_t)o.offset + delta);
            w.wireLen = o.len;
            w.packetID = o.packet_id;
            w.arrivalMs = j.arrivals ? o.arrival : -1;
            w.sender = q.sender;
            w.newOutput = (q.flags & EDGPU_SUB_NEW) != 0;
            w.worker = worker;
            writes++;
            const int err = j.sink->Write(w);
            if (err == kWouldBlock) { r.blocked.push_back(edgpu_blocked{j.tabq[s], i}); break; }
            if (err) { r.err = err; r.writes = writes; return; }
        }
    }
    r.writes = writes;
}

void Reflector::WorkerLoop(uint32_t worker) {
    uint64_t seen = 0;
    for (;;) {
        WriteJob* job;
        uint32_t nw;
        {
            std::unique_lock<std::mutex> g(fPoolMu);
            fPoolCv.wait(g, [&] { return fPoolStop || fJobSeq != seen; });
            if (fPoolStop) return;
            seen = fJobSeq;
            job = fJob;
            nw = fNumWriters;
        }
        WriteSubscribers(*job, worker, nw);
        {
            std::lock_guard<std::mutex> g(fPoolMu);
            if (--fJobsLeft == 0) fPoolDone.notify_all();
        }
    }
}

void Reflector::SetWriteThreads(uint32_t n) {
    std::unique_lock<std::mutex> eg(fEngineMu);
    WaitIdle(eg);
    n = std::max<uint32_t>(1, std::min<uint32_t>(n, 64));
    if (n == fNumWriters && fWorkers.size() + 1 == n) return;
    {
        std::lock_guard<std::mutex> g(fPoolMu);
        fPoolStop = true;
    }
    fPoolCv.notify_all();
    for (std::thread& t : fWorkers) t.join();
    fWorkers.clear();
    fPoolStop = false;
    fNumWriters = n;
    for (uint32_t k = 1; k < n; k++) fWorkers.emplace_back([this, k] { WorkerLoop(k); });
}

// ---------------------------------------------------------------------------------------
static const unsigned char kSTX = 0x28, kETX = 0x29;   // BUF_STX / BUF_ETX

CKeyFrameCache::CKeyFrameCache(int len) : mem_size(len) {
    _memory = (char*)malloc(mem_size);
    curdatalen = 0;
}

CKeyFrameCache::~CKeyFrameCache() {
    free(_memory);
    _memory = nullptr;
    mem_size = 0;
    curdatalen = 0;
}

bool CKeyFrameCache::PutOnePacket(char* buf, int len, int nalutype, int start) {
    if (buf == nullptr || len == 0) return false;
    if (nalutype == 7 && start == 1) curdatalen = 0;          // a new SPS starts a new GOP
    // the caller's packet is rewritten in place: byte 13 (the NAL header of an FU-A start
    // fragment after a 12-byte RTP header) becomes 0x67 (SPS) or 0x41 (keyframecache.cpp:
    // 27-40); the reference does it for any length (past the packet when len < 14) -- here
    // only inside the packet.  The reference's ./data.264 debug dump is not reproduced.
    if (start == 1 && len >= 14) buf[13] = (char)(nalutype == 7 ? 0x67 : 0x41);
    // the reference's 5 KiB TLV scratch: it overruns it for len > 5116 (FrameBuffer::Encode
    // ignores the capacity, keyframecache.h:24-45); refused here
    if (len < 0 || len + 4 > 5 * 1024) return false;
    unsigned char rec[5 * 1024];
    rec[0] = kSTX;
    rec[1] = (unsigned char)((unsigned)len >> 8);
    rec[2] = (unsigned char)len;
    memcpy(rec + 3, buf, len);
    rec[3 + len] = kETX;
    return SetBuf((char*)rec, len + 4);
}

bool CKeyFrameCache::GetOnePacket(char* outbuf, int& outLen, int curOffset) {
    if (curOffset >= curdatalen) return false;
    if ((unsigned char)_memory[curOffset] != kSTX) return false;
    const int pkgLen = ((unsigned char)_memory[curOffset + 1] << 8) | (unsigned char)_memory[curOffset + 2];
    if (pkgLen >= curdatalen) return false;
    if ((unsigned char)_memory[curOffset + 3 + pkgLen] != kETX) return false;
    memcpy(outbuf, _memory + curOffset + 3, pkgLen);
    outLen = pkgLen;
    return true;
}

bool CKeyFrameCache::SetBuf(char* frameBuf, int len) {
    if (frameBuf == nullptr || len == 0) return false;
    if (len + curdatalen > mem_size) return false;
    memcpy(_memory + curdatalen, frameBuf, len);
    curdatalen += len;
    return true;
}

int CKeyFrameCache::LoadGOP(Reflector& r, uint32_t session, uint32_t track, uint32_t* outPackets) {
    uint64_t n = 0;
    uint32_t k = 0;
    std::lock_guard<std::mutex> eg(r.EngineMutex());
    const int err = edgpu_gop_copy(r.Context(), session, track, (uint8_t*)_memory, (uint64_t)mem_size, &n, &k);
    if (err) return err;
    curdatalen = (int)n;
    if (outPackets) *outPackets = k;
    return kNoErr;
}

}  // namespace edgpu_reflector
