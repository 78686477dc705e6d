// edgpu_engine.cpp -- host side of the relay engine behind the C ABI (include/edgpu.h).
//
// Owns the per-GPU context: HIP stream and events, the device tables of edgpu_device.h, the
// per-sender HBM rings, ingest staging, the fan-out arena, and the session / subscriber
// bookkeeping the reflector keeps on the CPU (ReflectorSession / ReflectorStream /
// ReflectorOutput membership).  Every packet-rate decision runs on the GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include <sched.h>

#include "edgpu.h"
#include "edgpu_device.h"

#include "edgpu_params.h"

namespace edgpu {
hipError_t launch_ingest(const IngestParams& p, uint32_t nseg, hipStream_t st);
hipError_t launch_blocked(const BlockedParams& p, hipStream_t st);
hipError_t launch_first_packet_info(const FirstInfoQuery* q, FirstInfoResult* r, const SenderDev* senders,
                                    uint32_t n, hipStream_t st);
hipError_t launch_image(const ImageParams& p, int phase, hipStream_t st);
hipError_t launch_plan(const PlanParams& p, hipStream_t st);
hipError_t launch_ring_move(int kind, const void* src, uint64_t smask, void* dst, uint64_t dmask, uint64_t lo, uint64_t n,
                            hipStream_t st);
hipError_t launch_plan_pass(const PlanParams& p, hipStream_t st);
hipError_t launch_fanout(const FanoutParams& p, int variant, int num_cus, hipStream_t st);
hipError_t launch_deframe(const TcpParams& p, hipStream_t st);
hipError_t launch_desc_source(const SubDev* subs, const SenderDev* senders, uint32_t nsubs, uint32_t pass,
                              uint32_t epoch, uint32_t* out, hipStream_t st);
hipError_t launch_sub_rows(const SubDev* subs, const SenderDev* senders, const edgpu_out_desc* desc, const uint32_t* sel,
                           uint32_t nsel, uint32_t nsubs, uint32_t pass, uint32_t epoch, edgpu_packet_row* rows,
                           uint64_t nrows, hipStream_t st);
hipError_t launch_desc_arrival(const SubDev* subs, const SenderDev* senders, uint32_t nsubs, uint32_t pass,
                               int64_t* out, hipStream_t st);
hipError_t launch_arena_gather(const uint8_t* arena, const edgpu_region* reg, const uint64_t* dst_off, uint32_t n,
                               uint8_t* dst, hipStream_t st);
hipError_t launch_copy_to_pinned(void* dst, const void* src, uint64_t bytes, hipStream_t st);
hipError_t launch_sub_active(const edgpu_substream_out* sub, uint32_t n, uint32_t* blk, edgpu_substream_out* rows,
                             uint32_t* q, uint32_t cap, uint32_t* total, hipStream_t st);
hipError_t launch_stall(uint64_t ticks, hipStream_t st);
int fanout_chunk(int variant);
int fanout_default(bool patching);
bool fanout_rewrites(int variant);
const char* fanout_name(int variant);
}  // namespace edgpu

using namespace edgpu;

static thread_local std::string g_err;
static int fail(int code, const std::string& msg) { g_err = msg; return code; }
// hipErrorLaunchTimeOut from a bounded wait is the GPU watchdog's (wsync): EDGPU_TIMEOUT
#define HIP_CHECK(expr)                                                                   \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e == hipErrorLaunchTimeOut)                                                  \
            return fail(EDGPU_TIMEOUT, std::string(#expr) + ": GPU watchdog: the device did not finish " \
                                       "the context's work within watchdog_ms");          \
        if (_e != hipSuccess)                                                             \
            return fail(EDGPU_NO_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

// Device allocations.  EDGPU_POISON=1 (debugging) fills every new allocation with 0xA5 so a
// read of memory the engine never wrote shows up deterministically instead of depending on
// what a previous process left in HBM.
static bool poison_on() {
    static const int v = getenv("EDGPU_POISON") ? atoi(getenv("EDGPU_POISON")) : 0;
    return v != 0;
}
template <typename T>
static hipError_t dmalloc(T** p, size_t n) {
    hipError_t e = hipMalloc((void**)p, n);
    if (e == hipSuccess && poison_on()) {
        e = hipMemset(*p, 0xA5, n);
        if (e == hipSuccess) e = hipDeviceSynchronize();
    }
    return e;
}

// Growable device array of POD T.
template <typename T>
struct DevVec {
    T* ptr = nullptr;
    size_t cap = 0;
    hipError_t reserve(size_t n, hipStream_t st) {
        if (n <= cap) return hipSuccess;
        size_t nc = std::max<size_t>(n, cap ? cap * 2 : 64);
        T* np = nullptr;
        hipError_t e = dmalloc(&np, nc * sizeof(T));
        if (e != hipSuccess) return e;
        if (ptr) {
            e = hipMemcpyAsync(np, ptr, cap * sizeof(T), hipMemcpyDeviceToDevice, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            (void)hipFree(ptr);
            if (e != hipSuccess) { (void)hipFree(np); return e; }
        }
        ptr = np;
        cap = nc;
        return hipSuccess;
    }
    void release() { if (ptr) (void)hipFree(ptr); ptr = nullptr; cap = 0; }
};

struct TrackHost { uint32_t type = 0; std::string name; uint32_t track_id = 0; };   // type: 1 video, 2 audio

// A track's receiver-report state toward a UDP pusher (ReflectorStream fields
// fReceiverReportBuffer / fDestRTCPAddr / fDestRTCPPort and the RTCP sender's fLastRRTime).
struct SourceHost {
    uint32_t rr_ssrc = 0;
    std::vector<uint8_t> cname;     // RTCPSRPacket::GetACName, padded
    uint32_t addr = 0;              // 0: unknown (SendReceiverReport returns early)
    uint16_t port = 0;
    int64_t last_rr = 0;
};

// Sender rings come from a pool: chunks from hipMalloc carved by a bump pointer, and a free list per
// size (ring sizes are powers of two: meta rings packets x 36 B, byte rings 2^k B), so ring growth,
// session add / remove and session churn allocate and free no device memory once the pool holds
// enough (hipMalloc + hipFree of a ring cost ~0.2 ms: a burst of 1000 growths stalled a tick for
// a quarter of a second).  Chunk memory stays with the pool until the context is destroyed; a
// ring of kOwn bytes or more has an allocation of its own, freed when the ring is returned (a
// grown sender's old big rings and a removed session's would otherwise sit on the free lists).
// A failed hipMalloc leaves HIP's last error set; it is cleared here, so the next kernel launch's
// check does not report it.
struct RingPool {
    static constexpr size_t kChunk = 512ull << 20, kAlign = 4096, kOwn = 128ull << 20;
    std::vector<void*> chunks;                     // every chunk allocation (freed at destroy)
    std::map<void*, size_t> own;                   // the rings with an allocation of their own
    std::map<size_t, std::vector<void*>> freed;    // by (aligned) size
    char* cur = nullptr;
    size_t left = 0, held = 0;                     // held: device bytes the pool has allocated now
    // EDGPU_RING_POOL_LIMIT=<bytes> (tests): allocations past it fail as an exhausted device would
    size_t limit = getenv("EDGPU_RING_POOL_LIMIT") ? strtoull(getenv("EDGPU_RING_POOL_LIMIT"), nullptr, 0) : 0;
    template <typename T>
    hipError_t alloc(T** p, size_t n) {
        if (limit && held + n > limit) return hipErrorOutOfMemory;
        return dmalloc(p, n);
    }
    static size_t align(size_t b) { return (b + kAlign - 1) & ~(kAlign - 1); }
    hipError_t get(void** out, size_t bytes) {
        bytes = align(bytes);
        auto it = freed.find(bytes);
        if (it != freed.end() && !it->second.empty()) {
            *out = it->second.back();
            it->second.pop_back();
            return poison(*out, bytes);
        }
        void* p = nullptr;
        if (bytes >= kOwn) {                       // a big ring: its own allocation
            hipError_t e = alloc(&p, bytes);
            if (e != hipSuccess) { (void)hipGetLastError(); return e; }
            own[p] = bytes;
            held += bytes;
            *out = p;
            return hipSuccess;
        }
        if (bytes > left) {
            hipError_t e = alloc(&p, kChunk);
            if (e != hipSuccess) {                 // no room for a whole chunk: this ring alone
                (void)hipGetLastError();
                if ((e = alloc(&p, bytes)) != hipSuccess) { (void)hipGetLastError(); return e; }
                own[p] = bytes;
                held += bytes;
                *out = p;
                return hipSuccess;
            }
            chunks.push_back(p);
            held += kChunk;
            cur = (char*)p;
            left = kChunk;
        }
        *out = cur;
        cur += bytes;
        left -= bytes;
        return poison(*out, bytes);
    }
    void put(void* p, size_t bytes) {
        if (!p) return;
        auto o = own.find(p);
        if (o != own.end()) {                      // its own allocation: back to HIP
            (void)hipFree(p);
            held -= o->second;
            own.erase(o);
            return;
        }
        freed[align(bytes)].push_back(p);
    }
    static hipError_t poison(void* p, size_t n) {  // EDGPU_POISON: as a fresh allocation
        if (!poison_on()) return hipSuccess;
        hipError_t e = hipMemset(p, 0xA5, n);
        return e == hipSuccess ? hipDeviceSynchronize() : e;
    }
    void release() {
        for (void* p : chunks) (void)hipFree(p);
        for (auto& o : own) (void)hipFree(o.first);
        chunks.clear(); own.clear(); freed.clear(); cur = nullptr; left = held = 0;
    }
};

// Bucket-array entries besides a subscriber handle (SessionHost::slots)
constexpr int32_t kPlaceFree = -1, kPlaceRemote = -2;
constexpr uint32_t kMaxPlaces = 1u << 20;

struct SessionHost {
    uint32_t first_sender, ntracks, first_stream;
    bool udp_push;
    uint32_t span = 0;              // tracks' worth of rows it holds (>= ntracks after a reuse)
    uint32_t eyes = 0;              // client outputs (ReflectorStream::fEyeCount, every track)
    std::vector<int32_t> slots;     // the streams' bucket arrays: subscriber per slot, kPlaceFree
                                    // empty, kPlaceRemote a replica's output (remote_join)
    std::vector<SourceHost> src;    // per track
    bool alive = true;              // false after edgpu_session_remove (its id may be reused)
    std::vector<uint32_t> subs;     // attached subscriber handles
};

// RTCPSRPacket::GetACName (RTCPSRPacket.cpp:87-117): item type 1, length byte, "QTSS<secs>",
// a NUL, zero padding to the next multiple of 4 -- at least one more byte.
static std::vector<uint8_t> source_cname(int64_t secs) {
    char b[48];
    const int n = snprintf(b + 1, sizeof(b) - 1, " QTSS%lld", (long long)secs) + 1;
    b[0] = 1;
    b[1] = (char)(n - 2);
    uint32_t len = (uint32_t)n + 1;
    len += 4 - (len % 4);
    std::vector<uint8_t> c(len, 0);
    memcpy(c.data(), b, (size_t)n);
    return c;
}

struct SubscriberHost {
    uint32_t session;
    uint32_t first_sub;         // first SubDev index
    uint32_t nsub;
    bool active;
    int transport;
    uint32_t span;              // SubDev rows it holds (>= nsub in a larger free range)
    int32_t slot;               // its place in the session's bucket arrays
};

struct edgpu_ctx {
    edgpu_config cfg;
    int device = 0;
    int num_cus = 256;
    int fanout_variant = -1;        // EDGPU_FANOUT (A/B measurement); -1 = default kernel
    uint64_t joined_rows = 0;       // sub-stream rows of the outputs added since the last tick
    bool deframe_serial = false;    // EDGPU_DEFRAME_SERIAL (measurement): no deframe / fan-out overlap
    uint32_t tcp_walk = 2;          // EDGPU_TCP_WALK: 0 parallel chunk walk + resolve, 1 serial chain,
                                    // 2 segments of tcp_seg chunks (TcpParams.walk)
    uint32_t tcp_seg = 4;           // EDGPU_TCP_SEG
    uint32_t ablate = 0;
    int timing = EDGPU_TIMING_ALL;  // edgpu_set_timing: which per-launch event pairs are recorded
    uint32_t ingest_mode = 0;       // EDGPU_INGEST: 0 copy in k_ingest, 1 separate copy kernel
    uint32_t tcp_copy = 3;          // EDGPU_INGEST_TCP: 3 frame state in SGPRs, DPP neighbour word, two
                                    // frames per wave round; 2 the same with per-lane frame state;
                                    // 1 one frame per round; 0 two loads per word
    hipStream_t stream = nullptr;
    // the RTSP-interleaved deframe (k_tcp_*) runs on `aux`: it reads only the call's TCP bytes
    // and writes deframe scratch, so it overlaps the previous tick's fan-out still on `stream`;
    // the host reads its report, then enqueues k_ingest (no cross-stream wait left on `stream`)
    hipStream_t aux = nullptr;
    hipEvent_t ev_serial = nullptr;       // EDGPU_DEFRAME_SERIAL
    // the last keyframe index (it reads the segment tables the next deframe rewrites)
    hipEvent_t ev_kf = nullptr;
    bool kf_recorded = false;
    // per-launch timing history: [which][slot][start,end]
    static const int kHist = 256;
    hipEvent_t hist[4][kHist][2] = {};
    uint32_t hist_n[4] = {0, 0, 0, 0};      // pairs recorded (monotonic sequence numbers)
    uint32_t hist_rd[4] = {0, 0, 0, 0};     // pairs already returned by edgpu_kernel_times
    // Borrowed end points.  A whole-tick entry (ring 1) ends at its copy kernel's end event
    // (ring 0 sequence number in tick_end[slot]); a keyframe entry (ring 3) starts at the end
    // event of the ingest it indexes (ring 2 sequence number in kf_from[slot]) when nothing ran
    // on the host between the two, else at its own start event (kf_from[slot] = kOwnStart).
    // A borrowed event is valid while its ring has not recorded kHist more pairs since.
    static const uint32_t kOwnStart = 0xFFFFFFFFu;
    uint32_t tick_end[kHist] = {};
    uint32_t kf_from[kHist] = {};
    uint32_t last_seq[4] = {0, 0, 0, 0};    // each ring's newest complete pair (edgpu_last_timings)
    bool kf_share = false;                  // the last ingest's end event may start the keyframe entry
    uint64_t fanout_launches = 0;
    int64_t last_now = 0;               // clock of the last edgpu_fanout (backpressure reports)
    bool timed_fanout = false, timed_ingest = false, timed_keyframe = false;

    std::vector<SessionHost> sessions;
    std::vector<SubscriberHost> subscribers;
    std::vector<edgpu_source_report> source_reports;   // queued by the last edgpu_fanout
    std::vector<uint32_t> sub_sender;   // host mirror: SubDev index -> sender
    std::vector<uint8_t> sub_active;
    std::vector<uint8_t> sub_rw;        // host mirror: SubDev has a non-identity rewrite
    uint32_t n_rw = 0;                  // active sub-streams with a rewrite
    uint32_t n_tcp = 0;                 // active RTSP-interleaved sub-streams (channel-byte patch)
    uint32_t nsenders = 0, nstreams = 0;
    std::vector<void*> snd_meta, snd_ring;   // per sender: its rings (null once its session is removed)
    std::vector<uint32_t> dead_sessions;     // removed session ids, reused by edgpu_session_add
    std::map<uint32_t, std::vector<uint32_t>> free_subs;   // SubDev ranges of removed subscribers, by size
    // ranges freed since the last edgpu_fanout: their rows still hold that tick's plan (its later
    // copy passes and backpressure reports read them), so they are reused only from the next tick
    std::vector<std::pair<uint32_t, uint32_t>> free_pending;   // (size, first row)
    uint32_t tick_nsubs = 0;                     // sub-stream rows of the last edgpu_fanout's table
    uint64_t work_cap_needed = 0;
    void* d_null = nullptr;                  // zeroed 4 KiB: the rings of a removed session's senders

    DevVec<SessionDev> d_sessions;
    DevVec<SenderDev> d_senders;
    DevVec<StreamDev> d_streams;
    DevVec<SubDev> d_subs;
    DevVec<uint32_t> d_sub_index;
    DevVec<uint32_t> d_sub_range;
    DevVec<uint32_t> d_sub_pos;
    DevVec<FanSub> d_fansub;
    DevVec<edgpu_substream_out> d_sub_out;
    DevVec<FanWork> d_work;
    DevVec<uint64_t> d_blk_bytes;
    DevVec<uint32_t> d_blk_count;
    DevVec<uint64_t> d_blk_maxb;
    DevVec<uint32_t> d_blk_maxc;
    bool index_dirty = true;
    // copy passes of the last tick (edgpu_fanout_next): the current pass's ordinal and id, the
    // kernel and buffers of the tick, and what the host knows of a further pass (-1: not read
    // back since the last launch, 0: none, 1: one is owed)
    uint32_t pass_ord = 0, pass_id = 0;
    int passes_more = 0;
    int tick_variant = 0;
    uint64_t fanout_passes = 0;

    // ingest staging
    edgpu_pkt_desc* d_desc = nullptr;
    uint32_t* d_seg = nullptr;
    uint32_t* d_seg_sess = nullptr;
    uint8_t* d_blob = nullptr;
    CopyJob* d_jobs = nullptr;
    // pinned-host ingest (EDGPU_PTR_PINNED): two device staging sets filled on `h2d`
    struct PinStage {
        edgpu_pkt_desc* desc = nullptr;
        uint32_t* seg = nullptr;
        uint32_t* sess = nullptr;
        uint8_t* blob = nullptr;
        hipEvent_t copied = nullptr;        // its H2D copy is done (h2d stream)
        hipEvent_t consumed = nullptr;      // k_ingest + keyframe index read it (main stream)
        bool issued = false;
        uint64_t prestaged = 0;             // blob prefix copied ahead (edgpu_ingest_prestage)
    } pin[2];
    hipStream_t h2d = nullptr;
    int pin_next = 0;
    // edgpu_ingest_prestage may run on another thread than the other calls: it and stage_pinned
    // share the staging sets, pin_next and the h2d stream under pin_mu
    std::mutex pin_mu;
    int pend_stage = -1;                    // staging set of the batch pending a keyframe index
    // pending batch for keyframe_index
    const uint32_t* pend_seg = nullptr;
    const uint32_t* pend_seg_sess = nullptr;
    uint32_t pend_nseg = 0;
    bool pending = false;

    uint8_t* d_arena = nullptr;                 // the tick's (pass's) send-ready bytes
    edgpu_out_desc* d_out_desc = nullptr;       // and descriptors
    // RTSP-interleaved ingest: per-session carried partial frame (device) and its length
    // (host mirror, read back with every call's results), per-call walk tables
    std::vector<uint32_t> carry_len;
    DevVec<uint8_t> d_carry;
    DevVec<TcpGroup> d_tcp_groups;
    DevVec<TcpRead> d_tcp_reads;
    DevVec<uint32_t> d_tcp_chunk_group, d_tcp_ncand;
    DevVec<TcpCand> d_tcp_cands;
    DevVec<uint16_t> d_tcp_offs;
    DevVec<uint8_t> d_tcp_links, d_tcp_stage;
    uint64_t* d_tcp_src = nullptr;      // per frame source address (max_batch_packets)
    DevVec<TcpChunkRes> d_tcp_chunkres;
    DevVec<edgpu_tcp_result> d_tcp_results;
    TcpTotals* d_tcp_tot = nullptr;
    uint8_t* d_tcp_raw = nullptr;
    // RTP-Info PLAY query (kMaxTracks entries) and backpressure reports
    FirstInfoQuery* d_fpi_q = nullptr;
    FirstInfoResult* d_fpi_r = nullptr;
    FirstInfoQuery* h_fpi_q = nullptr;          // pinned
    FirstInfoResult* h_fpi_r = nullptr;         // pinned
    uint8_t* h_stage = nullptr;                 // pinned bounce buffer of Readback (kStageBytes)
    DevVec<edgpu_blocked> d_blocked;
    DevVec<edgpu_region> d_gather_reg;          // edgpu_arena_gather
    DevVec<int64_t> d_arrivals;                 // edgpu_fanout_arrivals
    DevVec<uint32_t> d_sources;                 // edgpu_fanout_packet_info
    DevVec<uint32_t> d_row_sel;                 // edgpu_fanout_rows
    DevVec<edgpu_packet_row> d_rows;
    DevVec<uint32_t> d_act_blk, d_act_q;        // edgpu_fanout_active: per-workgroup counts, staging
    DevVec<edgpu_substream_out> d_act_rows;
    uint32_t ingest_epoch = 0;                  // ingests so far
    uint32_t host_epoch_last = 0;               // the last ingest's epoch if it was a host batch, else 0
    DevVec<uint64_t> d_gather_off;
    // session images
    DevVec<ImgPlan> d_img_plan;
    int* d_img_status = nullptr;
    TickTotals* d_totals = nullptr;
    // ring growth (edgpu_config.ring_growth): the plan's requests, how many the host has learnt
    // of since (grown before the next ingest), which fan-out launch they were read for
    GrowReq* d_grow = nullptr;
    uint32_t* h_grow_flag = nullptr;            // pinned, mapped: the plan sets it with a request
    uint32_t* d_grow_flag = nullptr;            // its device address
    uint32_t grow_pending = 0;
    uint64_t grow_seen_launch = 0;
    uint64_t ring_grows = 0;
    uint64_t grow_deferred = 0;     // growth requests left to a later call (the per-call budget)
    uint64_t grow_failures = 0;     // growths the device memory could not hold (best effort: skipped)
    // per sender, the ring sizes whose allocation failed (and the meta ring they were asked for):
    // requests for those or larger are not retried until the sender's rings change
    struct GrowFail { uint64_t meta, pk, bytes; };
    std::map<uint32_t, GrowFail> grow_failed;
    RingPool rings;                 // every sender's meta and byte rings
    // GPU watchdog (wsync): the event a bounded wait polls; wedged while the work it timed out on runs
    hipEvent_t wd_ev = nullptr;
    bool wedged = false;
    uint64_t watchdog_timeouts = 0;
    uint32_t ing_slot = 0;          // the last ingest's counter slot (TickTotals.ing_pk)
    uint64_t kernel_launches = 0;   // edgpu_counters (LaunchScope)
    uint64_t host_syncs = 0;        // host waits on the GPU (wsync / wsync_event)
    uint64_t ring_bytes = 0;                    // device bytes of the live senders' rings
};

// ---- GPU watchdog (per-stream error isolation and a GPU watchdog) ----
// Every wait of the engine on the device (stream and event synchronisation, the readbacks) is
// bounded by edgpu_config.watchdog_ms: an event is recorded behind the work and polled against
// the deadline.  When it passes, the wait returns hipErrorLaunchTimeOut (HIP_CHECK: EDGPU_TIMEOUT)
// and the context is wedged on that event: every call that would enqueue work or wait returns
// EDGPU_TIMEOUT at once, enqueueing nothing, until the event completes -- then the context is
// itself again (the work it timed out on has finished; its results were never read).  The host
// decides what a wedge means (the QTSS module tears the players down and refuses SETUPs until a
// tick succeeds).  edgpu_ctx_destroy waits without a bound.  watchdog_ms = EDGPU_FALSE: unbounded
// waits (hipStreamSynchronize), as before.
static hipError_t wsync_event(edgpu_ctx* x, hipEvent_t ev) {
    x->host_syncs++;
    if (!x->cfg.watchdog_ms) return hipEventSynchronize(ev);
    using Clk = std::chrono::steady_clock;
    const Clk::time_point t0 = Clk::now(), deadline = t0 + std::chrono::milliseconds(x->cfg.watchdog_ms);
    for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e != hipErrorNotReady) return e;
        const Clk::time_point now = Clk::now();
        if (now >= deadline) return hipErrorLaunchTimeOut;
        // a tick's waits are short: spin (yielding) for the first 100 us, then poll every 20 us
        if (now - t0 < std::chrono::microseconds(100)) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}
static hipError_t wsync(edgpu_ctx* x, hipStream_t st) {
    if (x->wedged) {
        if (hipEventQuery(x->wd_ev) == hipErrorNotReady) return hipErrorLaunchTimeOut;
        x->wedged = false;
    }
    if (!x->cfg.watchdog_ms) { x->host_syncs++; return hipStreamSynchronize(st); }
    hipError_t e = hipEventRecord(x->wd_ev, st);
    if (e != hipSuccess) return e;
    e = wsync_event(x, x->wd_ev);
    if (e == hipErrorLaunchTimeOut) { x->wedged = true; x->watchdog_timeouts++; }
    return e;
}
// The device entry of every call: its device current, and no wedge left (see above)
static int device_enter(edgpu_ctx* x) {
    if (hipSetDevice(x->device) != hipSuccess) return fail(EDGPU_NO_DEVICE, "hipSetDevice failed");
    if (x->wedged) {
        if (hipEventQuery(x->wd_ev) == hipErrorNotReady)
            return fail(EDGPU_TIMEOUT, "GPU watchdog: the work the context timed out on is still running");
        x->wedged = false;
    }
    return EDGPU_OK;
}
// Adds the kernels an API call launched (on this thread, EDGPU_LAUNCH) to the context's count;
// only the outermost call of the thread counts (API functions call each other)
struct LaunchScope {
    static thread_local int depth;
    edgpu_ctx* x;
    uint64_t start;
    explicit LaunchScope(edgpu_ctx* c) : x(c), start(tl_launches) { depth++; }
    ~LaunchScope() {
        if (--depth == 0) x->kernel_launches += tl_launches - start;
    }
};
thread_local int LaunchScope::depth = 0;
#define DEVICE_ENTER(x)                                   \
    LaunchScope _edgpu_launch_scope(x);                   \
    do {                                                  \
        if (int _r = device_enter(x)) return _r;          \
    } while (0)

static bool live_session(const edgpu_ctx* x, uint32_t s) { return s < x->sessions.size() && x->sessions[s].alive; }

// Calls that move the rings or the sub-stream table on are refused while the context knows the
// last tick still owes a copy pass (edgpu_fanout_next).
static int owed_pass(const edgpu_ctx* x, const char* what) {
    if (x->passes_more == 1)
        return fail(EDGPU_ERR, std::string(what) + ": the last fan-out tick has a copy pass not yet delivered "
                                                   "(edgpu_fanout_next)");
    return EDGPU_OK;
}
static int read_totals(edgpu_ctx* x, TickTotals* t);
// The same for calls that free what a later copy pass reads (a session's rings and rows): when the
// host has not read the last tick's stats yet, whether a pass is owed is read from the device.
static int owed_pass_known(edgpu_ctx* x, const char* what) {
    if (x->passes_more == -1 && x->fanout_launches) {
        TickTotals t;
        if (int r = read_totals(x, &t)) return r;
        x->passes_more = t.pass_next[x->pass_ord & 1u] != kNoPass ? 1 : 0;
    }
    return owed_pass(x, what);
}

extern "C" {

const char* edgpu_version(void) { return "edgpu 0.1 (gfx950)"; }
const char* edgpu_last_error(void) { return g_err.c_str(); }

void edgpu_config_default(edgpu_config* c) {
    memset(c, 0, sizeof(*c));
}

static void fill_defaults(edgpu_config& c) {
    if (!c.reflector_buffer_size_sec) c.reflector_buffer_size_sec = 1;
    if (!c.rtp_reflector_threshold_msec) c.rtp_reflector_threshold_msec = 2000;
    if (c.rtp_reflector_threshold_msec < 1000) c.rtp_reflector_threshold_msec = 1000;
    if (!c.timeout_stream_SSRC_secs) c.timeout_stream_SSRC_secs = 30;
    c.use_one_SSRC_per_stream = (c.use_one_SSRC_per_stream == EDGPU_FALSE) ? 0 : 1;
    if (!c.video_ring_packets) c.video_ring_packets = 8192;
    if (!c.video_ring_bytes) c.video_ring_bytes = 8ull << 20;
    if (!c.other_ring_packets) c.other_ring_packets = 2048;
    if (!c.other_ring_bytes) c.other_ring_bytes = 1ull << 20;
    if (!c.out_arena_bytes) c.out_arena_bytes = 256ull << 20;
    if (!c.max_out_packets) c.max_out_packets = 1u << 20;
    if (!c.max_batch_packets) c.max_batch_packets = 1u << 20;
    if (!c.max_batch_bytes) c.max_batch_bytes = 1ull << 30;
    if (!c.reflector_rtp_info_offset_msec) c.reflector_rtp_info_offset_msec = 500;
    else if (c.reflector_rtp_info_offset_msec == EDGPU_FALSE) c.reflector_rtp_info_offset_msec = 0;
    c.ring_growth = (c.ring_growth == EDGPU_FALSE) ? 0 : 1;
    if (!c.max_ring_packets) c.max_ring_packets = 1u << 20;
    if (!c.max_ring_bytes) c.max_ring_bytes = 1ull << 30;
    c.reflector_use_in_packet_receive_time = (c.reflector_use_in_packet_receive_time &&
                                              c.reflector_use_in_packet_receive_time != EDGPU_FALSE) ? 1u : 0u;
    if (!c.reflector_in_packet_max_receive_sec) c.reflector_in_packet_max_receive_sec = 60;
    else if (c.reflector_in_packet_max_receive_sec == EDGPU_FALSE) c.reflector_in_packet_max_receive_sec = 0;
    if (!c.ingest_spec_min) c.ingest_spec_min = 128;
    else if (c.ingest_spec_min == EDGPU_FALSE) c.ingest_spec_min = 0;   // never
    if (!c.watchdog_ms) c.watchdog_ms = 10000;
    else if (c.watchdog_ms == EDGPU_FALSE) c.watchdog_ms = 0;   // unbounded waits
}

static bool pow2(uint64_t x) { return x && !(x & (x - 1)); }

int edgpu_ctx_create(const edgpu_config* cfg_in, edgpu_ctx** out) {
    if (!out) return fail(EDGPU_BAD_ARGUMENT, "out is NULL");
    *out = nullptr;
    edgpu_config c;
    if (cfg_in) c = *cfg_in; else edgpu_config_default(&c);
    fill_defaults(c);
    if (!pow2(c.video_ring_packets) || !pow2(c.other_ring_packets) || !pow2(c.video_ring_bytes) ||
        !pow2(c.other_ring_bytes) || c.video_ring_bytes < 4096 || c.other_ring_bytes < 4096 ||
        !pow2(c.max_ring_packets) || !pow2(c.max_ring_bytes))
        return fail(EDGPU_BAD_ARGUMENT, "ring capacities must be powers of two (bytes >= 4096)");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(EDGPU_NO_DEVICE, "no HIP device visible (libedgpu needs an MI355X / gfx950)");
    if (c.device < 0 || c.device >= ndev) return fail(EDGPU_BAD_ARGUMENT, "bad device ordinal");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, c.device) != hipSuccess)
        return fail(EDGPU_NO_DEVICE, "hipGetDeviceProperties failed");
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
        return fail(EDGPU_NO_DEVICE, std::string("libedgpu is built for gfx950, device is ") + prop.gcnArchName);
    edgpu_ctx* x = new edgpu_ctx();
    x->cfg = c;
    x->device = c.device;
    x->num_cus = prop.multiProcessorCount;
    if (hipSetDevice(c.device) != hipSuccess) { delete x; return fail(EDGPU_NO_DEVICE, "hipSetDevice failed"); }
    auto bad = [&](const char* what) { edgpu_ctx_destroy(x); return fail(EDGPU_OUT_OF_MEMORY, what); };
    if (hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking) != hipSuccess) return bad("stream");
    if (hipEventCreateWithFlags(&x->wd_ev, hipEventDisableTiming) != hipSuccess) return bad("watchdog event");
    for (auto& w : x->hist) for (auto& s : w) for (auto& e : s) if (hipEventCreate(&e) != hipSuccess) return bad("event");
    if (dmalloc(&x->d_desc, sizeof(edgpu_pkt_desc) * (size_t)c.max_batch_packets) != hipSuccess) return bad("desc staging");
    if (dmalloc(&x->d_seg, sizeof(uint32_t) * ((size_t)c.max_batch_packets + 1)) != hipSuccess) return bad("seg staging");
    if (dmalloc(&x->d_seg_sess, sizeof(uint32_t) * (size_t)c.max_batch_packets) != hipSuccess) return bad("seg staging");
    if (dmalloc(&x->d_jobs, sizeof(CopyJob) * (size_t)c.max_batch_packets) != hipSuccess) return bad("jobs");
    if (dmalloc(&x->d_arena, c.out_arena_bytes) != hipSuccess) return bad("fan-out arena");
    if (dmalloc(&x->d_out_desc, sizeof(edgpu_out_desc) * (size_t)c.max_out_packets) != hipSuccess) return bad("descriptors");
    if (dmalloc(&x->d_totals, sizeof(TickTotals)) != hipSuccess) return bad("totals");
    if (dmalloc(&x->d_grow, sizeof(GrowReq) * kMaxGrow) != hipSuccess) return bad("ring growth requests");
    if (hipHostMalloc((void**)&x->h_grow_flag, 64, hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void**)&x->d_grow_flag, x->h_grow_flag, 0) != hipSuccess)
        return bad("ring growth flag");
    *x->h_grow_flag = 0;
    if (hipMalloc(&x->d_null, 4096) != hipSuccess || hipMemset(x->d_null, 0, 4096) != hipSuccess) return bad("null ring");
    {
        TickTotals t0;
        memset(&t0, 0, sizeof(t0));
        t0.pass_next[0] = t0.pass_next[1] = kNoPass;
        if (hipMemcpy(x->d_totals, &t0, sizeof(t0), hipMemcpyHostToDevice) != hipSuccess) return bad("totals");
    }
    if (const char* v = getenv("EDGPU_FANOUT")) x->fanout_variant = atoi(v);
#ifdef EDGPU_AB_VARIANTS                         // measurement builds only (edgpu_params.h)
    if (const char* v = getenv("EDGPU_ABLATE")) x->ablate = (uint32_t)atoi(v);
    if (const char* v = getenv("EDGPU_INGEST")) x->ingest_mode = (uint32_t)atoi(v) == 1 ? 1u : 0u;
    if (const char* v = getenv("EDGPU_INGEST_TCP")) x->tcp_copy = (uint32_t)std::min(std::max(atoi(v), 0), 3);
    // measurement: the deframe waits for everything enqueued before it (no overlap with the last fan-out)
    if (const char* v = getenv("EDGPU_DEFRAME_SERIAL")) x->deframe_serial = atoi(v) != 0;
#endif
    // the deframe walk (TcpParams.walk): "serial" / "parallel"
    if (const char* v = getenv("EDGPU_TCP_WALK"))
        x->tcp_walk = !strcmp(v, "serial") || !strcmp(v, "1") ? 1u : !strcmp(v, "seg") || !strcmp(v, "2") ? 2u : 0u;
    if (const char* v = getenv("EDGPU_TCP_SEG")) x->tcp_seg = (uint32_t)std::max(atoi(v), 1);
    *out = x;
    return EDGPU_OK;
}

int edgpu_ctx_destroy(edgpu_ctx* x) {
    if (!x) return EDGPU_OK;
    (void)hipSetDevice(x->device);
    if (x->stream) (void)hipStreamSynchronize(x->stream);
    x->rings.release();                          // (every sender's rings)
    if (x->d_null) (void)hipFree(x->d_null);
    x->d_sessions.release(); x->d_senders.release(); x->d_streams.release(); x->d_subs.release();
    x->d_sub_index.release(); x->d_sub_range.release(); x->d_sub_pos.release(); x->d_fansub.release(); x->d_sub_out.release(); x->d_work.release();
    x->d_blk_bytes.release(); x->d_blk_count.release(); x->d_blk_maxb.release(); x->d_blk_maxc.release();
    x->d_img_plan.release();
    x->d_carry.release(); x->d_tcp_groups.release(); x->d_tcp_reads.release(); x->d_tcp_chunk_group.release();
    x->d_tcp_ncand.release(); x->d_tcp_cands.release(); x->d_tcp_links.release(); x->d_tcp_chunkres.release();
    x->d_tcp_results.release(); x->d_tcp_offs.release(); x->d_tcp_stage.release(); x->d_blocked.release();
    x->d_gather_reg.release(); x->d_gather_off.release(); x->d_arrivals.release(); x->d_sources.release(); x->d_row_sel.release(); x->d_rows.release();
    x->d_act_blk.release(); x->d_act_q.release(); x->d_act_rows.release();
    if (x->d_fpi_q) (void)hipFree(x->d_fpi_q);
    if (x->d_fpi_r) (void)hipFree(x->d_fpi_r);
    if (x->h_fpi_q) (void)hipHostFree(x->h_fpi_q);
    if (x->h_fpi_r) (void)hipHostFree(x->h_fpi_r);
    if (x->h_stage) (void)hipHostFree(x->h_stage);
    if (x->h_grow_flag) (void)hipHostFree(x->h_grow_flag);
    if (x->d_tcp_src) (void)hipFree(x->d_tcp_src);
    if (x->d_tcp_tot) (void)hipFree(x->d_tcp_tot);
    if (x->d_tcp_raw) (void)hipFree(x->d_tcp_raw);
    if (x->d_img_status) (void)hipFree(x->d_img_status);
    for (void* p : {(void*)x->d_desc, (void*)x->d_seg, (void*)x->d_seg_sess, (void*)x->d_jobs,
                    (void*)x->d_blob, (void*)x->d_arena, (void*)x->d_out_desc, (void*)x->d_totals, (void*)x->d_grow})
        if (p) (void)hipFree(p);
    for (auto& w : x->hist) for (auto& s : w) for (auto& e : s) if (e) (void)hipEventDestroy(e);
    if (x->h2d) (void)hipStreamSynchronize(x->h2d);
    for (auto& st : x->pin) {
        for (void* p : {(void*)st.desc, (void*)st.seg, (void*)st.sess, (void*)st.blob}) if (p) (void)hipFree(p);
        if (st.copied) (void)hipEventDestroy(st.copied);
        if (st.consumed) (void)hipEventDestroy(st.consumed);
    }
    if (x->h2d) (void)hipStreamDestroy(x->h2d);
    if (x->aux) (void)hipStreamSynchronize(x->aux);
    if (x->ev_serial) (void)hipEventDestroy(x->ev_serial);
    if (x->ev_kf) (void)hipEventDestroy(x->ev_kf);
    if (x->aux) (void)hipStreamDestroy(x->aux);
    if (x->stream) (void)hipStreamDestroy(x->stream);
    if (x->wd_ev) (void)hipEventDestroy(x->wd_ev);
    delete x;
    return EDGPU_OK;
}

// Waits for everything the context has enqueued (the context stream and the deframe's).
static hipError_t sync_all(edgpu_ctx* x) {
    hipError_t e = wsync(x, x->stream);
    if (e == hipSuccess && x->aux) e = wsync(x, x->aux);
    return e;
}

// Device -> host reads.  Every read of the engine is enqueued on the context stream after the
// work that produces it and completes at one hipStreamSynchronize before the host looks at the
// destination.  Reads that fit go through a pinned bounce buffer, so no small read (a totals
// record, a sender header, per-read reports) is a pageable async copy into the caller's or the
// stack's memory; larger ones (GOP bytes, whole ticks) copy straight into the destination, which
// HIP completes through its own staging before the synchronize returns.
static constexpr size_t kStageBytes = 64 << 10;
struct Readback {
    edgpu_ctx* x;
    hipStream_t st;         // the stream the reads follow (the context stream unless given)
    struct Item { void* dst; size_t off, bytes; };
    std::vector<Item> staged;
    size_t used = 0;
    explicit Readback(edgpu_ctx* c, hipStream_t s = nullptr) : x(c), st(s ? s : c->stream) {}
    hipError_t add(void* dst, const void* src, size_t bytes) {
        if (!bytes) return hipSuccess;
        if (!x->h_stage) {
            hipError_t e = hipHostMalloc((void**)&x->h_stage, kStageBytes, hipHostMallocDefault);
            if (e != hipSuccess) { x->h_stage = nullptr; return e; }
        }
        if (bytes <= kStageBytes - used) {
            staged.push_back({dst, used, bytes});
            hipError_t e = hipMemcpyAsync(x->h_stage + used, src, bytes, hipMemcpyDeviceToHost, st);
            used += (bytes + 15) & ~size_t(15);
            return e;
        }
        // a large read into pinned memory: a copy kernel storing over PCIe beats the DMA copy
        if (bytes >= kKernelCopyBytes && !(((uintptr_t)dst | (uintptr_t)src) & 15) && is_pinned(dst))
            return launch_copy_to_pinned(dst, src, bytes, st);
        return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st);
    }
    static constexpr size_t kKernelCopyBytes = 256 << 10;
    static bool is_pinned(const void* p) {
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, p) != hipSuccess) { (void)hipGetLastError(); return false; }
        return a.type == hipMemoryTypeHost;
    }
    hipError_t run() {
        hipError_t e = wsync(x, st);
        if (e != hipSuccess) return e;
        for (const Item& it : staged) memcpy(it.dst, x->h_stage + it.off, it.bytes);
        staged.clear();
        used = 0;
        return hipSuccess;
    }
};

// The tick totals, after every stream of the context has drained.
static int read_totals(edgpu_ctx* x, TickTotals* t) {
    DEVICE_ENTER(x);
    HIP_CHECK(sync_all(x));
    Readback rb(x);
    HIP_CHECK(rb.add(t, x->d_totals, sizeof(*t)));
    HIP_CHECK(rb.run());
    return EDGPU_OK;
}

// The plan's ring-growth requests of the tick read back in `t` (once per fan-out launch): grown
// before the next ingest (grow_rings).
static void note_grow(edgpu_ctx* x, const TickTotals& t) {
    if (!x->fanout_launches || x->grow_seen_launch == x->fanout_launches) return;
    x->grow_seen_launch = x->fanout_launches;
    if (t.grow_count) x->grow_pending = std::min<uint32_t>(t.grow_count, kMaxGrow);
    if (x->h_grow_flag) __atomic_store_n(x->h_grow_flag, 0u, __ATOMIC_RELEASE);
}

// One sender's rings replaced by ones of (at least) `want_pk` packets / `want_by` bytes, powers of
// two within the configured bounds; its entries move to their places under the new masks (the rings
// are addressed by monotonic index / virtual byte, so an entry's new place is its index & new mask).
// The sender's floor becomes `tail`, the oldest entry intact in the old rings: older ones were lost
// already and must not look intact in the larger rings.  Nothing may be in flight (the caller synced).
static int grow_sender(edgpu_ctx* x, uint32_t sender, uint64_t want_pk, uint64_t want_by, uint64_t tail,
                       const uint64_t* expect_head, bool* grown, const SenderDev* now = nullptr) {
    *grown = false;
    if (sender >= x->nsenders || !x->snd_meta[sender]) return EDGPU_OK;
    SenderDev D;
    if (now) {
        D = *now;                               // read by the caller, nothing ran since
    } else {
        Readback rb(x);
        HIP_CHECK(rb.add(&D, x->d_senders.ptr + sender, sizeof(D)));
        HIP_CHECK(rb.run());
    }
    if ((expect_head && D.head != *expect_head) || D.meta != (uint64_t)(uintptr_t)x->snd_meta[sender]) return EDGPU_OK;
    const uint64_t old_pk = (uint64_t)D.pk_mask + 1, old_by = ((uint64_t)D.word_mask + 1) * 16;
    // the power of two at least v, capped at the bound (itself a power of two)
    auto pow2_at_least = [](uint64_t v, uint64_t bound) { uint64_t p = 1; while (p < v && p < bound) p <<= 1; return p; };
    const uint64_t new_pk = std::max(old_pk, pow2_at_least(want_pk, x->cfg.max_ring_packets));
    const uint64_t new_by = std::max(old_by, pow2_at_least(want_by, x->cfg.max_ring_bytes));
    if (new_pk <= old_pk && new_by <= old_by) return EDGPU_OK;
    void* meta = x->snd_meta[sender];
    void* ring = x->snd_ring[sender];
    void* nmeta = meta;
    void* nring = ring;
    if (new_pk > old_pk) {
        if (x->rings.get(&nmeta, new_pk * (sizeof(PktMeta) + sizeof(uint32_t))) != hipSuccess)
            return fail(EDGPU_OUT_OF_MEMORY, "ring growth: sender meta ring");
        const uint64_t lo = D.head > old_pk ? D.head - old_pk : 0;
        HIP_CHECK(launch_ring_move(0, meta, old_pk - 1, nmeta, new_pk - 1, lo, D.head - lo, x->stream));
        HIP_CHECK(launch_ring_move(1, (const uint8_t*)meta + old_pk * sizeof(PktMeta), old_pk - 1,
                                   (uint8_t*)nmeta + new_pk * sizeof(PktMeta), new_pk - 1, lo, D.head - lo, x->stream));
    }
    if (new_by > old_by) {
        if (x->rings.get(&nring, new_by) != hipSuccess) {
            if (nmeta != meta) x->rings.put(nmeta, new_pk * (sizeof(PktMeta) + sizeof(uint32_t)));
            return fail(EDGPU_OUT_OF_MEMORY, "ring growth: sender byte ring");
        }
        const uint64_t wend = D.vbyte_end / 16, wlo = wend > old_by / 16 ? wend - old_by / 16 : 0;
        HIP_CHECK(launch_ring_move(2, ring, old_by / 16 - 1, nring, new_by / 16 - 1, wlo, wend - wlo, x->stream));
    }
    D.meta = (uint64_t)(uintptr_t)nmeta;
    D.ring = (uint64_t)(uintptr_t)nring;
    D.pk_mask = (uint32_t)(new_pk - 1);
    D.word_mask = (uint32_t)(new_by / 16 - 1);
    D.floor = std::max(D.floor, tail);
    HIP_CHECK(hipMemcpyAsync(x->d_senders.ptr + sender, &D, sizeof(D), hipMemcpyHostToDevice, x->stream));
    HIP_CHECK(wsync(x, x->stream));
    if (nmeta != meta) x->rings.put(meta, old_pk * (sizeof(PktMeta) + sizeof(uint32_t)));
    if (nring != ring) x->rings.put(ring, old_by);
    x->snd_meta[sender] = nmeta;
    x->snd_ring[sender] = nring;
    x->work_cap_needed += new_pk / 16 - old_pk / 16;
    x->ring_bytes += (new_pk - old_pk) * (sizeof(PktMeta) + sizeof(uint32_t)) + (new_by - old_by);
    x->ring_grows++;
    x->index_dirty = true;                      // the work list is sized from the rings
    *grown = true;
    return EDGPU_OK;
}

// Ring growth (edgpu_config.ring_growth), at a tick boundary -- before an ingest or an image import,
// nothing in flight: every sender the last plan found holding more than half of a ring's capacity
// of what the reference would retain gets that ring grown to the requested size (grow_sender), its
// floor raised to the tail the plan measured.  A request made before the sender's head moved on (a
// replica's image apply in between) is dropped; the next plan makes it again.
// Ring growth per call (grow_rings), counted -- not timed, so which senders grow in which call
// follows from the trace alone: at most this many senders and this many new ring bytes (at least
// one sender).  A C2 burst (1024 video senders passing half of their 8-MiB rings within a tick or
// two) then grows in four calls of ~4 ms (~17 us per 16-MiB ring moved).
static constexpr size_t kGrowSendersPerCall = 256;
static constexpr uint64_t kGrowBytesPerCall = 8ull << 30;
static int grow_rings(edgpu_ctx* x) {
    uint32_t n = x->grow_pending;
    x->grow_pending = 0;
    if (x->h_grow_flag && __atomic_load_n(x->h_grow_flag, __ATOMIC_ACQUIRE)) {
        // a plan asked (the host did not read that tick's stats): its request count
        __atomic_store_n(x->h_grow_flag, 0u, __ATOMIC_RELEASE);
        HIP_CHECK(sync_all(x));
        TickTotals t;
        if (int r = read_totals(x, &t)) return r;
        n = std::max(n, std::min<uint32_t>(t.grow_count, kMaxGrow));
    }
    if (!n) return EDGPU_OK;
    HIP_CHECK(sync_all(x));
    std::vector<GrowReq> req(n);
    {
        Readback rb(x);
        HIP_CHECK(rb.add(req.data(), x->d_grow, n * sizeof(GrowReq)));
        HIP_CHECK(rb.run());
    }
    std::sort(req.begin(), req.end(), [](const GrowReq& a, const GrowReq& b) { return a.sender < b.sender; });
    req.erase(std::unique(req.begin(), req.end(), [](const GrowReq& a, const GrowReq& b) { return a.sender == b.sender; }),
              req.end());
    std::vector<SenderDev> cur(req.size());
    const auto tr = std::chrono::steady_clock::now();
    {   // the sender table in one copy (one small copy per sender costs ~10 us each)
        std::vector<SenderDev> all(x->nsenders);
        Readback rb(x);
        HIP_CHECK(rb.add(all.data(), x->d_senders.ptr, all.size() * sizeof(SenderDev)));
        HIP_CHECK(rb.run());
        for (size_t k = 0; k < req.size(); k++)
            if (req[k].sender < x->nsenders) cur[k] = all[req[k].sender];
    }
    const double read_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr).count();
    // A burst of requests (every C2 video sender passes half its ring within a tick or two) is spread
    // over ticks: each call grows at most kGrowSendersPerCall senders / kGrowBytesPerCall new bytes;
    // the next plan re-measures the rest and asks again -- a request means the ring still has half
    // its capacity left.  Growth is best effort: a ring the device memory cannot hold is skipped and
    // counted (grow_failures), the sender keeps its rings (a packet that later falls out of them
    // marks its session in edgpu_stream_errors, as past the configured bounds), the call goes on,
    // and the ingest that follows is not refused for it.
    const auto t0 = std::chrono::steady_clock::now();
    size_t k = 0, grown_n = 0;
    uint64_t new_bytes = 0;
    for (; k < req.size(); k++) {
        const GrowReq& R = req[k];
        const uint64_t want_pk = 1ull << R.pk_log2, want_by = 1ull << R.bytes_log2;
        auto f = x->grow_failed.find(R.sender);
        if (f != x->grow_failed.end() && cur[k].meta == f->second.meta && want_pk >= f->second.pk && want_by >= f->second.bytes)
            continue;                                  // failed before at this size: not retried
        if (grown_n && (grown_n >= kGrowSendersPerCall || new_bytes >= kGrowBytesPerCall)) {
            x->grow_deferred += req.size() - k;
            break;
        }
        bool grown = false;
        const int r = grow_sender(x, R.sender, want_pk, want_by, R.tail, &R.head, &grown, &cur[k]);
        if (r == EDGPU_OUT_OF_MEMORY) {
            x->grow_failures++;
            x->grow_failed[R.sender] = edgpu_ctx::GrowFail{cur[k].meta, want_pk, want_by};
            continue;
        }
        if (r) return r;
        if (grown) {
            grown_n++;
            new_bytes += want_pk * (sizeof(PktMeta) + sizeof(uint32_t)) + want_by;
            x->grow_failed.erase(R.sender);
        }
    }
    static const bool dbg = getenv("EDGPU_DEBUG_GROW") != nullptr;
    if (dbg)
        fprintf(stderr, "edgpu: ring growth: %zu of %zu requests in %.3f ms (read %.3f ms)\n", k, req.size(),
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), read_ms);
    return EDGPU_OK;
}

int edgpu_sync(edgpu_ctx* x) {
    if (!x) return fail(EDGPU_BAD_ARGUMENT, "ctx is NULL");
    HIP_CHECK(sync_all(x));
    return EDGPU_OK;
}

// SDP restatement of SDPSourceInfo::Parse (SDPSourceInfo.cpp:172-420), pinned byte for byte
// to the reference by tests/golden/sdp_vectors.json (tests/test_cold_parsers.py):
//   * lines end at CR or LF; empty lines are skipped;
//   * every line whose first byte is 'm' is a track (trackID = its 1-based position); two
//     bytes in, a StringParser "word" (letters, '-', '_') names the media: exactly "video"
//     or "audio", else unknown -- so "m=video2" is video and "m=VIDEO" is not;
//   * 'a' lines before the first track are ignored; "a=" + word "rtpmap": the first such line of
//     a track that has a space after the word names the track with the REST of the line after
//     that space (trailing blanks included: the H.264 gate, Q3, is an exact compare), later
//     rtpmap lines are ignored; word "control": after the ':' and the first '=', the first
//     run of digits is the trackID (0 when there is none).
static bool sdp_word_char(char c) {
    return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '-' || c == '_';
}
static std::vector<TrackHost> parse_sdp(const char* sdp, uint32_t n) {
    std::vector<TrackHost> t;
    const std::string s(sdp, n);
    size_t p = 0;
    while (p < s.size()) {
        size_t e = s.find_first_of("\r\n", p);
        if (e == std::string::npos) e = s.size();
        const std::string line = s.substr(p, e - p);
        p = e < s.size() ? e + 1 : e;
        if (line.empty()) continue;
        size_t w = std::min<size_t>(2, line.size()), we = w;
        while (we < line.size() && sdp_word_char(line[we])) we++;
        const std::string word = line.substr(w, we - w);
        if (line[0] == 'm') {
            TrackHost th;
            th.type = word == "video" ? 1 : word == "audio" ? 2 : 0;
            th.track_id = (uint32_t)t.size() + 1;
            t.push_back(th);
        } else if (line[0] == 'a' && !t.empty()) {
            if (word == "rtpmap") {
                const size_t sp = line.find(' ', we);
                if (t.back().name.empty() && sp != std::string::npos) t.back().name = line.substr(sp + 1);
            } else if (word == "control") {
                uint32_t id = 0;
                const size_t colon = line.find(':', we);
                const size_t eq = colon == std::string::npos ? std::string::npos : line.find('=', colon + 1);
                if (eq != std::string::npos) {
                    size_t d = eq + 1;
                    while (d < line.size() && !(line[d] >= '0' && line[d] <= '9')) d++;
                    for (; d < line.size() && line[d] >= '0' && line[d] <= '9'; d++) id = id * 10 + (uint32_t)(line[d] - '0');
                }
                t.back().track_id = id;
            }
        }
    }
    return t;
}

int edgpu_sdp_parse(const char* sdp, uint32_t sdp_len, edgpu_sdp_track* out, uint32_t cap, uint32_t* n_tracks) {
    if ((!sdp && sdp_len) || !n_tracks || (cap && !out)) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    const std::vector<TrackHost> t = parse_sdp(sdp ? sdp : "", sdp_len);
    *n_tracks = (uint32_t)t.size();
    if (t.size() > cap) return fail(EDGPU_BAD_ARGUMENT, "track buffer too small");
    for (size_t i = 0; i < t.size(); i++) {
        memset(&out[i], 0, sizeof(out[i]));
        out[i].payload_type = t[i].type;
        out[i].track_id = t[i].track_id;
        out[i].name_len = (uint32_t)std::min<size_t>(t[i].name.size(), sizeof(out[i].name));
        memcpy(out[i].name, t[i].name.data(), out[i].name_len);
    }
    return EDGPU_OK;
}

// A removed session's sender records: rings point at the zeroed null buffer (a one-packet,
// one-word ring), nothing enqueued, so every per-sender kernel finds an empty sender.
static SenderDev dead_sender(const edgpu_ctx* x, uint32_t sid) {
    SenderDev D;
    memset(&D, 0, sizeof(D));
    D.meta = D.ring = (uint64_t)(uintptr_t)x->d_null;
    D.session = sid;
    D.key = -1;
    D.last_nonzero = -1;
    D.new_start = -1;
    return D;
}

int edgpu_session_add(edgpu_ctx* x, const char* sdp, uint32_t sdp_len, int udp_push, uint32_t* out_session) {
    if (!x || !sdp) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    DEVICE_ENTER(x);
    std::vector<TrackHost> tracks = parse_sdp(sdp, sdp_len);
    if (tracks.empty() || tracks.size() > kMaxTracks)
        return fail(EDGPU_BAD_ARGUMENT, "SDP must describe 1..16 tracks");
    // a removed session whose rows fit gives its id and table rows (senders, streams): the
    // smallest such, so the tables stay as large as the most sessions / tracks live at once under
    // churn with mixed track counts (rows it does not use stay dead senders)
    uint32_t sid = (uint32_t)x->sessions.size();
    bool reuse = false;
    size_t best = x->dead_sessions.size();
    for (size_t k = 0; k < x->dead_sessions.size(); k++) {
        const uint32_t sp = x->sessions[x->dead_sessions[k]].span;
        if (sp >= tracks.size() && (best == x->dead_sessions.size() || sp < x->sessions[x->dead_sessions[best]].span))
            best = k;
    }
    uint32_t span = (uint32_t)tracks.size();
    if (best < x->dead_sessions.size()) {
        sid = x->dead_sessions[best];
        span = x->sessions[sid].span;
        x->dead_sessions.erase(x->dead_sessions.begin() + (long)best);
        reuse = true;
    }
    const uint32_t ntracks = (uint32_t)tracks.size();
    const uint32_t first_sender = reuse ? x->sessions[sid].first_sender : x->nsenders;
    const uint32_t first_stream = reuse ? x->sessions[sid].first_stream : x->nstreams;
    SessionHost sh{first_sender, ntracks, first_stream, udp_push != 0};
    sh.span = span;
    // receiver-report identity, as the ReflectorStream constructor draws it (:164-201)
    const int64_t wall_ms = std::chrono::duration_cast<std::chrono::milliseconds>(
        std::chrono::system_clock::now().time_since_epoch()).count();
    sh.src.resize(sh.ntracks);
    for (auto& h : sh.src) { h.rr_ssrc = (uint32_t)::rand(); h.cname = source_cname(wall_ms / 1000); }
    const uint32_t nsnd = 2 * sh.ntracks;
    if (!reuse) {
        HIP_CHECK(x->d_sessions.reserve(sid + 1, x->stream));
        HIP_CHECK(x->d_senders.reserve(x->nsenders + nsnd, x->stream));
        HIP_CHECK(x->d_streams.reserve(x->nstreams + sh.ntracks, x->stream));
        HIP_CHECK(x->d_sub_range.reserve(2 * (x->nsenders + nsnd), x->stream));
        x->snd_meta.resize(x->nsenders + nsnd, nullptr);
        x->snd_ring.resize(x->nsenders + nsnd, nullptr);
    }
    std::vector<SenderDev> snd(nsnd);
    std::vector<StreamDev> str(sh.ntracks);
    std::vector<std::pair<uint64_t, uint64_t>> sizes(nsnd);   // (packets, bytes) per sender
    auto undo = [&](uint32_t upto) {            // returns the rings allocated so far
        for (uint32_t i = 0; i < upto; i++) {
            void*& m = x->snd_meta[first_sender + i];
            void*& r = x->snd_ring[first_sender + i];
            x->rings.put(m, sizes[i].first * (sizeof(PktMeta) + sizeof(uint32_t)));
            x->rings.put(r, sizes[i].second);
            m = r = nullptr;
        }
    };
    for (uint32_t t = 0; t < sh.ntracks; t++) {
        uint32_t base = 0;
        if (tracks[t].type == 1) base |= kSndVideo;
        if (tracks[t].type == 2) base |= kSndAudio;
        if (tracks[t].name == "H264/90000") base |= kSndH264;    // exact, case-sensitive (Q3)
        for (uint32_t k = 0; k < 2; k++) {
            SenderDev& D = snd[2 * t + k];
            memset(&D, 0, sizeof(D));
            const bool big = (k == 0 && tracks[t].type == 1);
            const uint64_t pk = big ? x->cfg.video_ring_packets : x->cfg.other_ring_packets;
            const uint64_t by = big ? x->cfg.video_ring_bytes : x->cfg.other_ring_bytes;
            void* meta = nullptr; void* ring = nullptr;
            const uint32_t gs = first_sender + 2 * t + k;
            // the meta ring, then a uint32 blob slot per entry (edgpu_fanout_packet_info)
            sizes[2 * t + k] = {pk, by};
            if (x->rings.get(&meta, pk * (sizeof(PktMeta) + sizeof(uint32_t))) != hipSuccess) { undo(2 * t + k); return fail(EDGPU_OUT_OF_MEMORY, "sender meta ring"); }
            x->snd_meta[gs] = meta;
            if (x->rings.get(&ring, by) != hipSuccess) { undo(2 * t + k + 1); return fail(EDGPU_OUT_OF_MEMORY, "sender byte ring"); }
            x->snd_ring[gs] = ring;
            D.meta = (uint64_t)(uintptr_t)meta;
            D.ring = (uint64_t)(uintptr_t)ring;
            D.pk_mask = (uint32_t)(pk - 1);
            D.word_mask = (uint32_t)(by / 16 - 1);
            D.flags = base | (k ? kSndRtcpKind : 0u) | ((k && sh.udp_push) ? kSndRtcpPort : 0u);
            D.session = sid;
            D.stream = first_stream + t;
            D.track = t;
            D.key = -1;
            D.last_nonzero = -1;
            D.new_start = -1;
            x->work_cap_needed += pk / 16 + 1;          // smallest chunk of any variant
            x->ring_bytes += pk * (sizeof(PktMeta) + sizeof(uint32_t)) + by;
        }
        str[t].packet_count = 0;
    }
    SessionDev sd{sh.first_sender, sh.ntracks, 0u, sh.first_stream, x->cfg.use_one_SSRC_per_stream,
                  x->cfg.timeout_stream_SSRC_secs};
    HIP_CHECK(hipMemcpyAsync(x->d_senders.ptr + first_sender, snd.data(), nsnd * sizeof(SenderDev), hipMemcpyHostToDevice, x->stream));
    HIP_CHECK(hipMemcpyAsync(x->d_streams.ptr + first_stream, str.data(), sh.ntracks * sizeof(StreamDev), hipMemcpyHostToDevice, x->stream));
    HIP_CHECK(hipMemcpyAsync(x->d_sessions.ptr + sid, &sd, sizeof(sd), hipMemcpyHostToDevice, x->stream));
    HIP_CHECK(wsync(x, x->stream));
    if (reuse) {
        x->sessions[sid] = sh;
    } else {
        x->sessions.push_back(sh);
        x->nsenders += nsnd;
        x->nstreams += sh.ntracks;
    }
    if (sid < x->carry_len.size()) x->carry_len[sid] = 0;     // no interleaved frame carried over
    x->index_dirty = true;
    if (out_session) *out_session = sid;
    return EDGPU_OK;
}

// Deactivates subscriber `handle`'s sub-streams (host mirror + device flag, enqueued; the caller
// synchronises) and returns its SubDev range to the free list.
static int detach_subscriber(edgpu_ctx* x, uint32_t handle) {
    SubscriberHost& s = x->subscribers[handle];
    static const uint8_t zero = 0;              // the copies are enqueued: static storage
    for (uint32_t i = 0; i < s.nsub; i++) {
        x->sub_active[s.first_sub + i] = 0;
        if (x->sub_rw[s.first_sub + i]) { x->sub_rw[s.first_sub + i] = 0; x->n_rw--; }
        HIP_CHECK(hipMemcpyAsync(reinterpret_cast<uint8_t*>(x->d_subs.ptr + s.first_sub + i) + offsetof(SubDev, active),
                                 &zero, 1, hipMemcpyHostToDevice, x->stream));
    }
    s.active = false;
    if (s.transport == EDGPU_TRANSPORT_TCP) x->n_tcp -= s.nsub;
    SessionHost& sh = x->sessions[s.session];
    sh.eyes--;                                   // RemoveOutput(..., isClient) -> DecEyeCount
    sh.subs.erase(std::find(sh.subs.begin(), sh.subs.end(), handle));
    if (s.slot >= 0 && (size_t)s.slot < sh.slots.size() && sh.slots[s.slot] == (int32_t)handle)
        sh.slots[s.slot] = kPlaceFree;           // ReflectorStream::RemoveOutput
    x->free_pending.emplace_back(s.span, s.first_sub);
    x->index_dirty = true;
    return EDGPU_OK;
}

int edgpu_session_remove(edgpu_ctx* x, uint32_t session, uint32_t flags) {
    if (!x || !live_session(x, session)) return fail(EDGPU_BAD_ARGUMENT, "bad session");
    if (flags & ~EDGPU_SESSION_KILL_OUTPUTS) return fail(EDGPU_BAD_ARGUMENT, "bad flags");
    if (x->pending) return fail(EDGPU_ERR, "edgpu_keyframe_index must run after edgpu_ingest");
    if (int r = owed_pass_known(x, "edgpu_session_remove")) return r;
    SessionHost& sh = x->sessions[session];
    if (!sh.subs.empty() && !(flags & EDGPU_SESSION_KILL_OUTPUTS))
        return fail(EDGPU_ERR, "session still has outputs (the reference keeps a ReflectorSession while outputs "
                               "hold references to it; pass EDGPU_SESSION_KILL_OUTPUTS to tear them down)");
    DEVICE_ENTER(x);
    // TearDownAllOutputs: every attached subscriber goes with it
    while (!sh.subs.empty()) { int r = detach_subscriber(x, sh.subs.back()); if (r) return r; }
    // the rings may still be read by a fan-out copy in flight or a pinned batch
    HIP_CHECK(sync_all(x));
    if (x->h2d) HIP_CHECK(wsync(x, x->h2d));
    const uint32_t nsnd = 2 * sh.ntracks;
    std::vector<SenderDev> old(nsnd), snd(nsnd, dead_sender(x, session));
    {
        Readback rb(x);
        HIP_CHECK(rb.add(old.data(), x->d_senders.ptr + sh.first_sender, nsnd * sizeof(SenderDev)));
        HIP_CHECK(rb.run());
    }
    for (uint32_t i = 0; i < nsnd; i++) {
        const uint32_t gs = sh.first_sender + i;
        x->work_cap_needed -= ((uint64_t)old[i].pk_mask + 1) / 16 + 1;
        x->ring_bytes -= ((uint64_t)old[i].pk_mask + 1) * (sizeof(PktMeta) + sizeof(uint32_t)) +
                         ((uint64_t)old[i].word_mask + 1) * 16;
        snd[i].stream = old[i].stream;
        snd[i].track = old[i].track;
        // the rings go back to the pool (a later session or growth takes them)
        x->rings.put(x->snd_meta[gs], ((uint64_t)old[i].pk_mask + 1) * (sizeof(PktMeta) + sizeof(uint32_t)));
        x->rings.put(x->snd_ring[gs], ((uint64_t)old[i].word_mask + 1) * 16);
        x->snd_meta[gs] = x->snd_ring[gs] = nullptr;
        x->grow_failed.erase(gs);
    }
    std::vector<StreamDev> str(sh.ntracks);
    for (auto& st : str) st.packet_count = 0;
    SessionDev sd{sh.first_sender, sh.ntracks, 0u, sh.first_stream, 0u, 0u};
    HIP_CHECK(hipMemcpyAsync(x->d_senders.ptr + sh.first_sender, snd.data(), nsnd * sizeof(SenderDev), hipMemcpyHostToDevice, x->stream));
    HIP_CHECK(hipMemcpyAsync(x->d_streams.ptr + sh.first_stream, str.data(), sh.ntracks * sizeof(StreamDev), hipMemcpyHostToDevice, x->stream));
    HIP_CHECK(hipMemcpyAsync(x->d_sessions.ptr + session, &sd, sizeof(sd), hipMemcpyHostToDevice, x->stream));
    HIP_CHECK(wsync(x, x->stream));
    sh.alive = false;
    sh.eyes = 0;
    sh.slots.clear();                            // (remote places too)
    for (auto& h : sh.src) h = SourceHost();
    if (session < x->carry_len.size()) x->carry_len[session] = 0;
    x->dead_sessions.push_back(session);
    x->index_dirty = true;
    return EDGPU_OK;
}

int edgpu_session_ssrc_prefs(edgpu_ctx* x, uint32_t session, uint32_t use_one_SSRC_per_stream,
                             uint32_t timeout_stream_SSRC_secs) {
    if (!x || !live_session(x, session)) return fail(EDGPU_BAD_ARGUMENT, "bad session");
    if (x->pending) return fail(EDGPU_ERR, "edgpu_keyframe_index must run after edgpu_ingest");
    DEVICE_ENTER(x);
    const uint32_t v[2] = {use_one_SSRC_per_stream ? 1u : 0u, timeout_stream_SSRC_secs};
    // stream-ordered before the next ingest, which reads them
    HIP_CHECK(hipMemcpyAsync(&x->d_sessions.ptr[session].ssrc_filter, v, sizeof(v), hipMemcpyHostToDevice, x->stream));
    HIP_CHECK(wsync(x, x->stream));   // `v` is on the stack
    return EDGPU_OK;
}

int edgpu_session_tracks(edgpu_ctx* x, uint32_t session, uint32_t* out_tracks) {
    if (!x || !live_session(x, session) || !out_tracks) return fail(EDGPU_BAD_ARGUMENT, "bad session");
    *out_tracks = x->sessions[session].ntracks;
    return EDGPU_OK;
}

// Adds one subscriber's sub-streams (RTPSessionOutput + ReflectorSession::AddOutput) to the
// host tables -- in a removed subscriber's SubDev range of the same size when there is one,
// else at the end -- and its records to `v` as (SubDev index, record) for upload_subs; returns
// its handle (handles are never reused).
static uint32_t append_subscriber(edgpu_ctx* x, uint32_t session, int transport, uint32_t flags,
                                  const uint16_t* first_seq, std::vector<std::pair<uint32_t, SubDev>>& v) {
    SessionHost& sh = x->sessions[session];
    const uint32_t handle = (uint32_t)x->subscribers.size();
    const uint32_t nsub = 2 * sh.ntracks;
    x->joined_rows += nsub;
    uint32_t first = (uint32_t)x->sub_sender.size(), span = nsub;
    auto fr = x->free_subs.lower_bound(nsub);      // the smallest free range that fits
    while (fr != x->free_subs.end() && fr->second.empty()) ++fr;
    if (fr != x->free_subs.end()) {
        first = fr->second.back();
        span = fr->first;                          // rows past nsub stay inactive
        fr->second.pop_back();
    } else {
        x->sub_sender.resize(first + nsub, 0);
        x->sub_active.resize(first + nsub, 0);
        x->sub_rw.resize(first + nsub, 0);
    }
    for (uint32_t t = 0; t < sh.ntracks; t++)
        for (uint32_t k = 0; k < 2; k++) {
            SubDev Q;
            memset(&Q, 0, sizeof(Q));
            Q.handle = handle;
            Q.sender = sh.first_sender + 2 * t + k;
            Q.track = (uint16_t)t;
            Q.kind = (uint8_t)k;
            Q.transport = (uint8_t)transport;
            Q.channel = (uint8_t)(2 * t + k);        // GetTwoChannelNumbers in SETUP order
            Q.active = 1;
            Q.bookmark = -1;
            Q.first_seq = (k == 0 && first_seq) ? first_seq[t] : 0;
            Q.rtp_info = (k == 0 && (flags & EDGPU_PLAY_RTP_INFO)) ? 1 : 0;
            const uint32_t q = first + 2 * t + k;
            x->sub_sender[q] = Q.sender;
            x->sub_active[q] = 1;
            x->sub_rw[q] = 0;
            v.emplace_back(q, Q);
        }
    // ReflectorStream::AddOutput + FindBucket (RS.cpp:281-334): the first empty place in bucket
    // order (bucket = slot / 16, each holding 16); every track's array holds the output there
    int32_t slot = 0;
    while ((size_t)slot < sh.slots.size() && sh.slots[slot] != kPlaceFree) slot++;
    if ((size_t)slot == sh.slots.size()) sh.slots.push_back(kPlaceFree);
    sh.slots[slot] = (int32_t)handle;
    x->subscribers.push_back(SubscriberHost{session, first, nsub, true, transport, span, slot});
    if (transport == EDGPU_TRANSPORT_TCP) x->n_tcp += nsub;
    sh.eyes++;                                   // AddOutput(..., isClient) -> IncEyeCount
    sh.subs.push_back(handle);
    x->index_dirty = true;
    return handle;
}

// Uploads SubDev records (index, record) -- consecutive indices in one copy each run.
static int upload_subs(edgpu_ctx* x, const std::vector<std::pair<uint32_t, SubDev>>& v) {
    if (v.empty()) return EDGPU_OK;
    HIP_CHECK(x->d_subs.reserve(x->sub_sender.size(), x->stream));
    std::vector<SubDev> run;
    for (size_t i = 0; i < v.size();) {
        size_t j = i;
        run.clear();
        while (j < v.size() && v[j].first == v[i].first + (j - i)) run.push_back(v[j++].second);
        HIP_CHECK(hipMemcpyAsync(x->d_subs.ptr + v[i].first, run.data(), run.size() * sizeof(SubDev),
                                 hipMemcpyHostToDevice, x->stream));
        HIP_CHECK(wsync(x, x->stream));     // `run` is reused
        i = j;
    }
    return EDGPU_OK;
}

// HaveStreamBuffers for an RTP-Info PLAY (QTSSReflectorModule.cpp:1804-1865), every track
// at once on the device: first_seq[t] / info[t] on success, EDGPU_WOULD_BLOCK when a track
// has nothing buffered.
static int first_packet_info(edgpu_ctx* x, const SessionHost& sh, int64_t now_ms, std::vector<uint16_t>& first_seq,
                             edgpu_rtp_info* info) {
    std::vector<FirstInfoQuery> q(sh.ntracks);
    const int64_t over = (int64_t)x->cfg.reflector_buffer_size_sec * 1000;
    const int64_t window = over - std::min<int64_t>(x->cfg.reflector_rtp_info_offset_msec, over);
    for (uint32_t t = 0; t < sh.ntracks; t++) {
        q[t].rtp_sender = sh.first_sender + 2 * t;
        q[t].rtcp_sender = sh.udp_push ? 0xFFFFFFFFu : sh.first_sender + 2 * t + 1;
        q[t].cutoff = now_ms - window;                  // age <= window  <=>  arrival >= cutoff
    }
    // Persistent device buffers and pinned host staging (kMaxTracks entries).  Round 1 took
    // per-call buffers from the stream-ordered pool: the query copy into a recycled block was
    // sometimes lost and the kernel answered the previous PLAY's query.
    if (!x->d_fpi_q) {
        if (dmalloc(&x->d_fpi_q, kMaxTracks * sizeof(FirstInfoQuery)) != hipSuccess ||
            dmalloc(&x->d_fpi_r, kMaxTracks * sizeof(FirstInfoResult)) != hipSuccess ||
            hipHostMalloc((void**)&x->h_fpi_q, kMaxTracks * sizeof(FirstInfoQuery), hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void**)&x->h_fpi_r, kMaxTracks * sizeof(FirstInfoResult), hipHostMallocDefault) != hipSuccess)
            return fail(EDGPU_OUT_OF_MEMORY, "RTP-Info query buffers");
    }
    memcpy(x->h_fpi_q, q.data(), q.size() * sizeof(FirstInfoQuery));
    HIP_CHECK(hipMemcpyAsync(x->d_fpi_q, x->h_fpi_q, q.size() * sizeof(FirstInfoQuery), hipMemcpyHostToDevice, x->stream));
    HIP_CHECK(launch_first_packet_info(x->d_fpi_q, x->d_fpi_r, x->d_senders.ptr, sh.ntracks, x->stream));
    HIP_CHECK(hipMemcpyAsync(x->h_fpi_r, x->d_fpi_r, q.size() * sizeof(FirstInfoResult), hipMemcpyDeviceToHost, x->stream));
    HIP_CHECK(wsync(x, x->stream));
    std::vector<FirstInfoResult> r(x->h_fpi_r, x->h_fpi_r + sh.ntracks);
    if (getenv("EDGPU_DEBUG_PLAY")) {                    // debugging: the PLAY's inputs and results
        for (uint32_t t = 0; t < sh.ntracks; t++) {
            SenderDev d[2];
            Readback rb(x);
            HIP_CHECK(rb.add(d, x->d_senders.ptr + q[t].rtp_sender, 2 * sizeof(SenderDev)));
            HIP_CHECK(rb.run());
            fprintf(stderr, "play now=%lld track=%u cutoff=%lld head=%llu/%llu found=%u seq=%u key=%lld new_start=%lld "
                    "tail=%llu floor=%llu\n", (long long)now_ms, t, (long long)q[t].cutoff, (unsigned long long)d[0].head,
                    (unsigned long long)d[1].head, r[t].found, r[t].seq, (long long)d[0].key, (long long)d[0].new_start,
                    (unsigned long long)d[0].tail, (unsigned long long)d[0].floor);
        }
    }
    for (uint32_t t = 0; t < sh.ntracks; t++) {
        if (r[t].found != 1)
            return fail(EDGPU_WOULD_BLOCK, r[t].found == 0 ? "RTP-Info PLAY: no RTP packet received yet (retry)"
                                                           : "RTP-Info PLAY: nothing buffered in the window (retry)");
        first_seq[t] = (uint16_t)r[t].seq;
        if (info) { info[t].seq = (uint16_t)r[t].seq; info[t]._pad = 0; info[t].rtptime = r[t].rtptime; }
    }
    return EDGPU_OK;
}

int edgpu_subscriber_add(edgpu_ctx* x, uint32_t session, int transport, uint32_t* out_handle) {
    return edgpu_subscriber_play(x, session, transport, 0, 0, out_handle, nullptr);
}

int edgpu_subscriber_play(edgpu_ctx* x, uint32_t session, int transport, uint32_t flags, int64_t now_ms,
                          uint32_t* out_handle, edgpu_rtp_info* out_info) {
    if (!x || !live_session(x, session)) return fail(EDGPU_BAD_ARGUMENT, "bad session");
    if (transport != EDGPU_TRANSPORT_UDP && transport != EDGPU_TRANSPORT_TCP)
        return fail(EDGPU_BAD_ARGUMENT, "bad transport");
    if (flags & ~EDGPU_PLAY_RTP_INFO) return fail(EDGPU_BAD_ARGUMENT, "bad play flags");
    if (x->pending) return fail(EDGPU_ERR, "edgpu_keyframe_index must run after edgpu_ingest");
    DEVICE_ENTER(x);
    const SessionHost& sh = x->sessions[session];
    std::vector<uint16_t> first_seq(sh.ntracks, 0);
    if (flags & EDGPU_PLAY_RTP_INFO) {
        const int r = first_packet_info(x, sh, now_ms, first_seq, out_info);
        if (r) return r;
    }
    std::vector<std::pair<uint32_t, SubDev>> v;
    const uint32_t handle = append_subscriber(x, session, transport, flags, first_seq.data(), v);
    const int r = upload_subs(x, v);
    if (r) return r;
    if (out_handle) *out_handle = handle;
    return EDGPU_OK;
}

int edgpu_subscribers_add(edgpu_ctx* x, uint32_t n, const uint32_t* sessions, const int32_t* transports,
                          uint32_t* out_handles) {
    if (!x || (n && (!sessions || !transports))) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    for (uint32_t i = 0; i < n; i++) {
        if (!live_session(x, sessions[i])) return fail(EDGPU_BAD_ARGUMENT, "bad session");
        if (transports[i] != EDGPU_TRANSPORT_UDP && transports[i] != EDGPU_TRANSPORT_TCP)
            return fail(EDGPU_BAD_ARGUMENT, "bad transport");
    }
    if (!n) return EDGPU_OK;
    DEVICE_ENTER(x);
    std::vector<std::pair<uint32_t, SubDev>> v;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t h = append_subscriber(x, sessions[i], transports[i], 0, nullptr, v);
        if (out_handles) out_handles[i] = h;
    }
    return upload_subs(x, v);
}

int edgpu_subscriber_slot(edgpu_ctx* x, uint32_t handle, int32_t* out_slot) {
    if (!x || !out_slot || handle >= x->subscribers.size() || !x->subscribers[handle].active)
        return fail(EDGPU_BAD_ARGUMENT, "bad subscriber handle");
    *out_slot = x->subscribers[handle].slot;
    return EDGPU_OK;
}

int edgpu_subscriber_remove(edgpu_ctx* x, uint32_t handle) {
    if (!x || handle >= x->subscribers.size() || !x->subscribers[handle].active)
        return fail(EDGPU_BAD_ARGUMENT, "bad subscriber handle");
    DEVICE_ENTER(x);
    const int r = detach_subscriber(x, handle);
    if (r) return r;
    HIP_CHECK(wsync(x, x->stream));
    return EDGPU_OK;
}

int edgpu_subscriber_rewrite(edgpu_ctx* x, uint32_t handle, uint32_t track, const edgpu_rewrite* rw) {
    if (!x || handle >= x->subscribers.size() || !x->subscribers[handle].active)
        return fail(EDGPU_BAD_ARGUMENT, "bad subscriber handle");
    SubscriberHost& s = x->subscribers[handle];
    if (track >= s.nsub / 2) return fail(EDGPU_BAD_ARGUMENT, "bad track");
    if (rw && (rw->flags & ~EDGPU_REWRITE_SSRC)) return fail(EDGPU_BAD_ARGUMENT, "bad rewrite flags");
    const bool on = rw && (rw->seq_delta || rw->ts_delta || (rw->flags & EDGPU_REWRITE_SSRC));
    if (on && !fanout_rewrites(x->fanout_variant))
        return fail(EDGPU_ERR, "the selected fan-out variant (EDGPU_FANOUT) has no rewrite stage");
    if (x->pending) return fail(EDGPU_ERR, "edgpu_keyframe_index must run after edgpu_ingest");
    DEVICE_ENTER(x);
    for (uint32_t k = 0; k < 2; k++) {
        const uint32_t q = s.first_sub + 2 * track + k;
        uint32_t v[3] = {0, 0, 0};
        if (on) {
            v[0] = kRwActive | (k ? kRwRtcp : 0u) | ((rw->flags & EDGPU_REWRITE_SSRC) ? kRwSsrc : 0u) |
                   (uint32_t)rw->seq_delta << 16;
            v[1] = rw->ts_delta;
            v[2] = rw->ssrc;
        }
        HIP_CHECK(hipMemcpyAsync(reinterpret_cast<uint8_t*>(x->d_subs.ptr + q) + offsetof(SubDev, rw), v, sizeof(v),
                                 hipMemcpyHostToDevice, x->stream));
        if (on != (bool)x->sub_rw[q]) { x->sub_rw[q] = on; x->n_rw += on ? 1 : -1; }
    }
    HIP_CHECK(wsync(x, x->stream));     // `v` is stack memory
    return EDGPU_OK;
}

// ---- UDP pushers: source addresses and receiver reports ------------------------------------
// RTCPPacket::ParsePacket (RTCPPacket.cpp:40-63) + the SR-first test of ProcessPacket
// (ReflectorStream.cpp:1799-1815) from a datagram's length and first 4 bytes.
static bool rtcp_sr_first(const uint8_t* h, uint32_t len) {
    if (len < 8) return false;
    const uint32_t words = (uint32_t)h[2] << 8 | h[3];
    return len >= words * 4 + 4 && (h[0] >> 6) == 2 && h[1] == 200;
}

int edgpu_udp_sources(edgpu_ctx* x, const edgpu_udp_source* src, uint32_t n) {
    if (!x || (n && !src)) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    for (uint32_t i = 0; i < n; i++)
        if (!live_session(x, src[i].session)) return fail(EDGPU_BAD_ARGUMENT, "bad session");
    for (uint32_t i = 0; i < n; i++) {
        const edgpu_udp_source& d = src[i];
        SessionHost& sh = x->sessions[d.session];
        const uint32_t track = d.channel >> 1;
        if (track >= sh.ntracks || d.len == 0 || d.addr == 0) continue;
        // fIsRTCP by local-port parity: only a UDP push binds an odd RTCP port (Q12)
        const bool rtcp = sh.udp_push && (d.channel & 1);
        if (rtcp && !rtcp_sr_first(d.head, d.len)) continue;      // dropped before the update
        SourceHost& h = sh.src[track];
        if (h.addr == 0 || rtcp) {                                // NAT_WORKAROUND
            h.addr = d.addr;
            h.port = (uint16_t)(d.port + ((!rtcp && !(d.port & 1)) ? 1 : 0));
        }
    }
    return EDGPU_OK;
}

// The RTCP senders' report timers of one tick (ReflectorStream.cpp:1039-1047, 510-527).
static void queue_source_reports(edgpu_ctx* x, int64_t now) {
    x->source_reports.clear();
    for (uint32_t si = 0; si < x->sessions.size(); si++) {
        SessionHost& sh = x->sessions[si];
        if (!sh.alive) continue;
        for (uint32_t t = 0; t < sh.ntracks; t++) {
            SourceHost& h = sh.src[t];
            if (!(now > h.last_rr + 5000)) continue;              // kRRInterval
            h.last_rr = now;
            if (h.addr == 0) continue;
            edgpu_source_report r;
            memset(&r, 0, sizeof(r));
            r.session = si; r.track = (uint16_t)t; r.addr = h.addr; r.port = h.port;
            uint32_t n = 0;
            auto w32 = [&](uint32_t v) {
                r.bytes[n] = (uint8_t)(v >> 24); r.bytes[n + 1] = (uint8_t)(v >> 16);
                r.bytes[n + 2] = (uint8_t)(v >> 8); r.bytes[n + 3] = (uint8_t)v; n += 4;
            };
            // htonl(eye) & 0x7fffffff on the little-endian host masks bit 31 of the swapped
            // word, i.e. bit 7 of the count's low byte on the wire (:519-521)
            const uint32_t eye = sh.eyes & 0xFFFFFF7Fu;
            w32(0x80c90001u); w32(h.rr_ssrc);                                  // RR, no blocks
            w32(0x81ca0000u + (uint32_t)(h.cname.size() >> 2) + 1); w32(h.rr_ssrc);   // SDES
            memcpy(r.bytes + n, h.cname.data(), h.cname.size()); n += (uint32_t)h.cname.size();
            w32(0x80cc0008u); w32(h.rr_ssrc); w32(0x51545353u); w32(0);        // APP 'QTSS'
            w32(4); w32(0x6579000cu); w32(eye); w32(eye); w32(0);              // eye count
            r.len = n;
            x->source_reports.push_back(r);
        }
    }
}

int edgpu_source_reports(edgpu_ctx* x, edgpu_source_report* out, uint32_t cap, uint32_t* n_out) {
    if (!x || !n_out || (cap && !out)) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    const uint32_t n = (uint32_t)x->source_reports.size();
    *n_out = n;
    if (n > cap) return fail(EDGPU_BAD_ARGUMENT, "report buffer too small");
    if (n) memcpy(out, x->source_reports.data(), n * sizeof(edgpu_source_report));
    return EDGPU_OK;
}

int edgpu_session_eyes_add(edgpu_ctx* x, uint32_t session, int32_t delta) {
    if (!x || !live_session(x, session)) return fail(EDGPU_BAD_ARGUMENT, "bad session");
    SessionHost& sh = x->sessions[session];
    if (delta < 0 && (uint32_t)(-(int64_t)delta) > sh.eyes) return fail(EDGPU_BAD_ARGUMENT, "eye count below zero");
    sh.eyes = (uint32_t)((int64_t)sh.eyes + delta);
    return EDGPU_OK;
}

// A remote output (a replica session's subscriber on another context) in the owner's bucket
// arrays: ReflectorStream::AddOutput's first empty place (RS.cpp:281-334) and its eye
// (IncEyeCount), so that owner and replica subscribers of one session are numbered in one
// array, as the reference's one process numbers them.
int edgpu_session_remote_join(edgpu_ctx* x, uint32_t session, int32_t* out_place) {
    if (!x || !out_place || !live_session(x, session)) return fail(EDGPU_BAD_ARGUMENT, "bad session");
    SessionHost& sh = x->sessions[session];
    int32_t slot = 0;
    while ((size_t)slot < sh.slots.size() && sh.slots[slot] != kPlaceFree) slot++;
    if ((size_t)slot == sh.slots.size()) sh.slots.push_back(kPlaceFree);
    sh.slots[slot] = kPlaceRemote;
    sh.eyes++;
    *out_place = slot;
    return EDGPU_OK;
}

int edgpu_session_remote_leave(edgpu_ctx* x, uint32_t session, int32_t place) {
    if (!x || !live_session(x, session)) return fail(EDGPU_BAD_ARGUMENT, "bad session");
    SessionHost& sh = x->sessions[session];
    if (place < 0 || (size_t)place >= sh.slots.size() || sh.slots[place] != kPlaceRemote)
        return fail(EDGPU_BAD_ARGUMENT, "no remote output at that place");
    if (sh.eyes == 0) return fail(EDGPU_BAD_ARGUMENT, "eye count below zero");
    sh.slots[place] = kPlaceFree;
    sh.eyes--;
    return EDGPU_OK;
}

int edgpu_subscriber_set_slot(edgpu_ctx* x, uint32_t handle, int32_t slot) {
    if (!x || handle >= x->subscribers.size() || !x->subscribers[handle].active)
        return fail(EDGPU_BAD_ARGUMENT, "bad subscriber handle");
    if (slot < 0 || slot >= (int32_t)kMaxPlaces) return fail(EDGPU_BAD_ARGUMENT, "bad place");
    SubscriberHost& s = x->subscribers[handle];
    SessionHost& sh = x->sessions[s.session];
    if ((size_t)slot < sh.slots.size() && sh.slots[slot] != kPlaceFree && sh.slots[slot] != (int32_t)handle)
        return fail(EDGPU_BAD_ARGUMENT, "place taken by another output of the session");
    if (s.slot >= 0 && (size_t)s.slot < sh.slots.size() && sh.slots[s.slot] == (int32_t)handle)
        sh.slots[s.slot] = kPlaceFree;
    if ((size_t)slot >= sh.slots.size()) sh.slots.resize((size_t)slot + 1, kPlaceFree);
    sh.slots[slot] = (int32_t)handle;
    s.slot = slot;
    return EDGPU_OK;
}

int edgpu_source_identity(edgpu_ctx* x, uint32_t session, uint32_t track, uint32_t ssrc, int64_t cname_secs) {
    if (!x || !live_session(x, session) || track >= x->sessions[session].ntracks)
        return fail(EDGPU_BAD_ARGUMENT, "bad session / track");
    SourceHost& h = x->sessions[session].src[track];
    h.rr_ssrc = ssrc;
    h.cname = source_cname(cname_secs);
    return EDGPU_OK;
}

// Records the start / end event of launch kind `w` into the history ring.  A pair counts (its
// sequence number advances) only once its end event is recorded.
static hipError_t hist_mark(edgpu_ctx* x, int w, int end, hipStream_t st = nullptr) {
    if (x->timing < (w == 0 ? EDGPU_TIMING_FANOUT : EDGPU_TIMING_ALL)) return hipSuccess;
    const uint32_t seq = x->hist_n[w];
    hipError_t e = hipEventRecord(x->hist[w][seq % edgpu_ctx::kHist][end], st ? st : x->stream);
    if (e == hipSuccess && end) { x->last_seq[w] = seq; x->hist_n[w] = seq + 1; }
    return e;
}

// Whether ring `w`'s pair `seq` still holds its events (not overwritten since).
static bool hist_live(const edgpu_ctx* x, int w, uint32_t seq) {
    return x->hist_n[w] - seq <= (uint32_t)edgpu_ctx::kHist && x->hist_n[w] != seq;
}

// Start / end events of pair `seq` of ring `w`, resolving the borrowed end points; false when a
// borrowed pair has been overwritten (the entry is skipped).
static bool hist_pair(const edgpu_ctx* x, int w, uint32_t seq, hipEvent_t* a, hipEvent_t* b) {
    const uint32_t slot = seq % edgpu_ctx::kHist;
    *a = x->hist[w][slot][0];
    *b = x->hist[w][slot][1];
    if (w == 1) {
        const uint32_t s0 = x->tick_end[slot];
        if (!hist_live(x, 0, s0)) return false;
        *b = x->hist[0][s0 % edgpu_ctx::kHist][1];
    } else if (w == 3 && x->kf_from[slot] != edgpu_ctx::kOwnStart) {
        const uint32_t s2 = x->kf_from[slot];
        if (!hist_live(x, 2, s2)) return false;
        *a = x->hist[2][s2 % edgpu_ctx::kHist][1];
    }
    return true;
}

// The active sub-stream rows grouped by sender, each sender's in row order (sub_index), every
// sender's [begin, end) into it (sub_range) and each row's position (sub_pos): a counting sort by
// sender, linear in rows + senders (a subscriber joining or leaving rebuilds it before the next
// fan-out: at 2-ms ticks with players coming and going that is most ticks).
static int rebuild_index(edgpu_ctx* x) {
    const uint32_t nsub = (uint32_t)x->sub_sender.size();
    std::vector<uint32_t> range(2 * (size_t)x->nsenders, 0);
    for (uint32_t i = 0; i < nsub; i++)                     // rows per sender (in range[2s + 1])
        if (x->sub_active[i]) range[2 * (size_t)x->sub_sender[i] + 1]++;
    uint32_t total = 0;
    for (uint32_t s = 0; s < x->nsenders; s++) {
        const uint32_t c = range[2 * (size_t)s + 1];
        range[2 * (size_t)s] = total;
        range[2 * (size_t)s + 1] = total;                   // the fill cursor; ends at begin + count
        total += c;
    }
    std::vector<uint32_t> idx(total);
    std::vector<uint32_t> pos(nsub, 0xFFFFFFFFu);
    for (uint32_t i = 0; i < nsub; i++)
        if (x->sub_active[i]) {
            const uint32_t k = range[2 * (size_t)x->sub_sender[i] + 1]++;
            idx[k] = i;
            pos[i] = k;
        }
    HIP_CHECK(x->d_sub_index.reserve(std::max<size_t>(idx.size(), 1), x->stream));
    HIP_CHECK(x->d_fansub.reserve(std::max<size_t>(idx.size(), 1), x->stream));
    HIP_CHECK(x->d_sub_pos.reserve(std::max<size_t>(nsub, 1), x->stream));
    if (nsub) HIP_CHECK(hipMemcpyAsync(x->d_sub_pos.ptr, pos.data(), nsub * 4, hipMemcpyHostToDevice, x->stream));
    HIP_CHECK(x->d_sub_range.reserve(std::max<size_t>(range.size(), 2), x->stream));
    if (!idx.empty()) HIP_CHECK(hipMemcpyAsync(x->d_sub_index.ptr, idx.data(), idx.size() * 4, hipMemcpyHostToDevice, x->stream));
    if (!range.empty()) HIP_CHECK(hipMemcpyAsync(x->d_sub_range.ptr, range.data(), range.size() * 4, hipMemcpyHostToDevice, x->stream));
    const uint32_t nblk = (nsub + 255) / 256;
    HIP_CHECK(x->d_sub_out.reserve(std::max<uint32_t>(nsub, 1), x->stream));
    HIP_CHECK(x->d_blk_bytes.reserve(std::max<uint32_t>(nblk, 1), x->stream));
    HIP_CHECK(x->d_blk_count.reserve(std::max<uint32_t>(nblk, 1), x->stream));
    HIP_CHECK(x->d_blk_maxb.reserve(std::max<uint32_t>(nblk, 1), x->stream));
    HIP_CHECK(x->d_blk_maxc.reserve(std::max<uint32_t>(nblk, 1), x->stream));
    HIP_CHECK(x->d_work.reserve(std::max<uint64_t>(x->work_cap_needed, 1), x->stream));
    HIP_CHECK(wsync(x, x->stream));
    x->index_dirty = false;
    return EDGPU_OK;
}

// Enqueues k_ingest over a staged batch (device pointers) and marks it pending for
// edgpu_keyframe_index.  With `tcp` (edgpu_ingest_interleaved) the deframe kernels have run
// (`deframed`: on aux, observed by the host) or run first, inside the ingest timing events.
static int enqueue_ingest(edgpu_ctx* x, const edgpu_pkt_desc* dd, uint32_t n, const uint32_t* ds, const uint32_t* dss,
                          uint32_t nseg, const uint8_t* db, uint32_t copy_mode, bool host_src, const TcpParams* tcp = nullptr,
                          bool deframed = false) {
    IngestParams p;
    // a host batch: k_ingest records each packet's blob slot (edgpu_fanout_packet_info)
    p.host_epoch = host_src ? ++x->ingest_epoch : 0u;
    if (!host_src) ++x->ingest_epoch;
    x->host_epoch_last = p.host_epoch;
    p.desc = dd; p.seg_off = ds; p.seg_sess = dss; p.blob = db;
    p.src_addr = tcp ? tcp->src_addr : nullptr;
    p.sessions = x->d_sessions.ptr; p.senders = x->d_senders.ptr; p.streams = x->d_streams.ptr;
    p.jobs = x->d_jobs; p.npk = n; p.spec_min = x->cfg.ingest_spec_min; p.ablate = x->ablate; p.copy_mode = copy_mode; p.tcp_copy = x->tcp_copy;
    p.totals = x->d_totals;
    x->ing_slot ^= 1u;
    p.ing_slot = x->ing_slot;
    p.recv_time = x->cfg.reflector_use_in_packet_receive_time;
    // sMaxFuturePacketMSec = sMaxFuturePacketSec * 1000 in UInt32 (ReflectorStream.cpp:113)
    p.max_future_ms = (int64_t)(uint32_t)(x->cfg.reflector_in_packet_max_receive_sec * 1000u);
    p.tcp_groups = tcp ? tcp->groups : nullptr;
    p.tcp_chunkres = tcp ? tcp->chunkres : nullptr;
    p.tcp_offs = tcp ? tcp->offs : nullptr;
    p.tcp_reads = tcp ? tcp->reads : nullptr;
    p.tcp_raw = tcp ? tcp->raw : nullptr;
    p.tcp_stage = tcp ? tcp->stage : nullptr;
    HIP_CHECK(hist_mark(x, 2, 0));
    if (tcp && !deframed) HIP_CHECK(launch_deframe(*tcp, x->stream));
    HIP_CHECK(launch_ingest(p, nseg, x->stream));
    HIP_CHECK(hist_mark(x, 2, 1));
    x->timed_ingest = true;
    x->kf_share = true;                 // (the interleaved path reads its report on aux)
    x->pend_seg = ds; x->pend_seg_sess = dss; x->pend_nseg = nseg; x->pending = true;
    return EDGPU_OK;
}

// A host batch's structure: segment bounds, session ids, slots inside the blob.
static int validate_host_batch(edgpu_ctx* x, const edgpu_pkt_desc* desc, uint32_t n, const uint32_t* seg_off,
                               const uint32_t* seg_sess, uint32_t nseg, uint64_t blob_bytes) {
    if (nseg && seg_off[nseg] != n) return fail(EDGPU_BAD_ARGUMENT, "seg_offsets[n_segments] != n_packets");
    for (uint32_t s = 0; s < nseg; s++) {
        if (seg_off[s] > seg_off[s + 1]) return fail(EDGPU_BAD_ARGUMENT, "segments not monotone");
        if (!live_session(x, seg_sess[s])) return fail(EDGPU_BAD_ARGUMENT, "unknown session in batch");
    }
    for (uint32_t i = 0; i < n; i++)
        if ((uint64_t)desc[i].slot * 16 + ((std::min<uint32_t>(desc[i].len, kMaxPacket) + 4 + 15) & ~15u) > blob_bytes)
            return fail(EDGPU_BAD_ARGUMENT, "packet slot outside blob");
    return EDGPU_OK;
}

int edgpu_host_alloc(edgpu_ctx* x, uint64_t bytes, void** out) {
    if (!x || !out) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    DEVICE_ENTER(x);
    *out = nullptr;
    if (hipHostMalloc(out, std::max<uint64_t>(bytes, 16), hipHostMallocDefault) != hipSuccess)
        return fail(EDGPU_OUT_OF_MEMORY, "pinned host buffer");
    return EDGPU_OK;
}

int edgpu_host_free(edgpu_ctx* x, void* p) {
    if (!x) return fail(EDGPU_BAD_ARGUMENT, "ctx is NULL");
    if (!p) return EDGPU_OK;
    DEVICE_ENTER(x);
    // any thread may free (a pusher growing its blob): the copy stream is created under pin_mu
    hipStream_t h2d;
    {
        std::lock_guard<std::mutex> g(x->pin_mu);
        h2d = x->h2d;
    }
    if (h2d) HIP_CHECK(wsync(x, h2d));
    HIP_CHECK(hipHostFree(p));
    return EDGPU_OK;
}

// The caller may rewrite a pinned batch once the next ingest call has returned: every ingest
// entry point first waits for the outstanding pinned copies (normally long done).
static int wait_pinned_copies(edgpu_ctx* x) {
    for (auto& st : x->pin)
        if (st.issued) HIP_CHECK(wsync_event(x, st.copied));
    return EDGPU_OK;
}

// EDGPU_PTR_PINNED: copies the batch into staging set k on the copy stream; the context stream
// waits for it.  Returns the device pointers of the set.
// The staging set the next pinned batch goes to, allocated (callers hold pin_mu).
static int pin_set(edgpu_ctx* x, edgpu_ctx::PinStage** out) {
    if (!x->h2d) HIP_CHECK(hipStreamCreateWithFlags(&x->h2d, hipStreamNonBlocking));
    edgpu_ctx::PinStage& S = x->pin[x->pin_next];
    if (!S.desc) {
        const size_t np = x->cfg.max_batch_packets;
        if (dmalloc(&S.desc, sizeof(edgpu_pkt_desc) * np) != hipSuccess || dmalloc(&S.seg, 4 * (np + 1)) != hipSuccess ||
            dmalloc(&S.sess, 4 * np) != hipSuccess || dmalloc(&S.blob, x->cfg.max_batch_bytes) != hipSuccess)
            return fail(EDGPU_OUT_OF_MEMORY, "pinned-ingest staging");
        HIP_CHECK(hipEventCreateWithFlags(&S.copied, hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&S.consumed, hipEventDisableTiming));
    }
    *out = &S;
    return EDGPU_OK;
}

static int stage_pinned(edgpu_ctx* x, const edgpu_pkt_desc* desc, uint32_t n, const uint32_t* seg_off,
                        const uint32_t* seg_sess, uint32_t nseg, const uint8_t* blob, uint64_t blob_bytes, int* out_k) {
    std::lock_guard<std::mutex> g(x->pin_mu);
    const int k = x->pin_next;
    edgpu_ctx::PinStage* Sp = nullptr;
    { int r = pin_set(x, &Sp); if (r) return r; }
    edgpu_ctx::PinStage& S = *Sp;
    // the previous batch's copy must be done before its host buffers are handed back (contract),
    // and this set's previous batch must have been read by its ingest + keyframe index
    edgpu_ctx::PinStage& P = x->pin[k ^ 1];
    if (P.issued) HIP_CHECK(wsync_event(x, P.copied));
    if (S.issued && S.prestaged == 0) HIP_CHECK(hipStreamWaitEvent(x->h2d, S.consumed, 0));   // (a prestage waited)
    HIP_CHECK(hipMemcpyAsync(S.desc, desc, (size_t)n * sizeof(edgpu_pkt_desc), hipMemcpyHostToDevice, x->h2d));
    HIP_CHECK(hipMemcpyAsync(S.seg, seg_off, ((size_t)nseg + 1) * 4, hipMemcpyHostToDevice, x->h2d));
    HIP_CHECK(hipMemcpyAsync(S.sess, seg_sess, (size_t)nseg * 4, hipMemcpyHostToDevice, x->h2d));
    if (blob_bytes > S.prestaged)           // the part of the blob not copied ahead
        HIP_CHECK(hipMemcpyAsync(S.blob + S.prestaged, blob + S.prestaged, blob_bytes - S.prestaged,
                                 hipMemcpyHostToDevice, x->h2d));
    S.prestaged = 0;
    HIP_CHECK(hipEventRecord(S.copied, x->h2d));
    HIP_CHECK(hipStreamWaitEvent(x->stream, S.copied, 0));
    S.issued = true;
    x->pin_next = k ^ 1;
    *out_k = k;
    return EDGPU_OK;
}

int edgpu_ingest_prestage(edgpu_ctx* x, const uint8_t* blob, uint64_t offset, uint64_t bytes) {
    if (!x) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    if (!bytes && !offset) {                // discard: the next pinned batch is copied whole
        std::lock_guard<std::mutex> g(x->pin_mu);
        x->pin[x->pin_next].prestaged = 0;
        return EDGPU_OK;
    }
    if (!blob) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    if (!bytes) return EDGPU_OK;
    std::lock_guard<std::mutex> g(x->pin_mu);
    edgpu_ctx::PinStage& N = x->pin[x->pin_next];
    if (offset != N.prestaged) return fail(EDGPU_BAD_ARGUMENT, "a prestaged range must extend the staged prefix");
    if (offset + bytes > x->cfg.max_batch_bytes) return fail(EDGPU_BAD_ARGUMENT, "prestaged bytes exceed max_batch_bytes");
    DEVICE_ENTER(x);
    edgpu_ctx::PinStage* Sp = nullptr;
    { int r = pin_set(x, &Sp); if (r) return r; }
    edgpu_ctx::PinStage& S = *Sp;
    if (S.prestaged == 0 && S.issued) HIP_CHECK(hipStreamWaitEvent(x->h2d, S.consumed, 0));   // its last batch was read
    HIP_CHECK(hipMemcpyAsync(S.blob + offset, blob + offset, bytes, hipMemcpyHostToDevice, x->h2d));
    S.prestaged = offset + bytes;
    return EDGPU_OK;
}

int edgpu_ingest(edgpu_ctx* x, const edgpu_pkt_desc* desc, uint32_t n, const uint32_t* seg_off,
                 const uint32_t* seg_sess, uint32_t nseg, const uint8_t* blob, uint64_t blob_bytes, int where) {
    if (!x) return fail(EDGPU_BAD_ARGUMENT, "ctx is NULL");
    if (x->pending) return fail(EDGPU_ERR, "edgpu_keyframe_index must run after edgpu_ingest");
    // (a pass the host has not learnt of yet is guarded on the device: k_ingest checks the batch
    // against the tick's window while one is owed)
    const int owed = owed_pass(x, "edgpu_ingest");
    if (owed || n > x->cfg.max_batch_packets || nseg > x->cfg.max_batch_packets ||
        (where != EDGPU_PTR_DEVICE && blob_bytes > x->cfg.max_batch_bytes)) {
        if (where == EDGPU_PTR_PINNED) {    // the batch can never go in: drop what was copied ahead
            std::lock_guard<std::mutex> g(x->pin_mu);
            x->pin[x->pin_next].prestaged = 0;
        }
        return owed ? owed : fail(EDGPU_BAD_ARGUMENT, "batch exceeds configured capacity");
    }
    if (n && (!desc || !seg_off || !seg_sess || !blob)) return fail(EDGPU_BAD_ARGUMENT, "NULL batch array");
    DEVICE_ENTER(x);
    if (x->grow_pending || __atomic_load_n(x->h_grow_flag, __ATOMIC_ACQUIRE)) { int r = grow_rings(x); if (r) return r; }
    const edgpu_pkt_desc* dd = desc;
    const uint32_t* ds = seg_off;
    const uint32_t* dss = seg_sess;
    const uint8_t* db = blob;
    if (where == EDGPU_PTR_PINNED) {
        int r = validate_host_batch(x, desc, n, seg_off, seg_sess, nseg, blob_bytes);
        if (r) {                            // nothing will use what was copied ahead
            std::lock_guard<std::mutex> g(x->pin_mu);
            x->pin[x->pin_next].prestaged = 0;
            return r;
        }
        int k = 0;
        if ((r = stage_pinned(x, desc, n, seg_off, seg_sess, nseg, blob, blob_bytes, &k))) return r;
        const edgpu_ctx::PinStage& S = x->pin[k];
        r = enqueue_ingest(x, S.desc, n, S.seg, S.sess, nseg, S.blob, x->ingest_mode, true);
        if (!r) x->pend_stage = k;
        else (void)hipEventRecord(S.consumed, x->stream);   // nothing will read the set: free it
        return r;
    }
    { int r = wait_pinned_copies(x); if (r) return r; }
    if (where == EDGPU_PTR_HOST) {
        // validate on the host (segment bounds, session ids, slot bounds) before any launch
        int r = validate_host_batch(x, desc, n, seg_off, seg_sess, nseg, blob_bytes);
        if (r) return r;
        if (!x->d_blob && dmalloc(&x->d_blob, x->cfg.max_batch_bytes) != hipSuccess)
            return fail(EDGPU_OUT_OF_MEMORY, "blob staging");
        HIP_CHECK(hipMemcpyAsync(x->d_desc, desc, (size_t)n * sizeof(edgpu_pkt_desc), hipMemcpyHostToDevice, x->stream));
        HIP_CHECK(hipMemcpyAsync(x->d_seg, seg_off, ((size_t)nseg + 1) * 4, hipMemcpyHostToDevice, x->stream));
        HIP_CHECK(hipMemcpyAsync(x->d_seg_sess, seg_sess, (size_t)nseg * 4, hipMemcpyHostToDevice, x->stream));
        HIP_CHECK(hipMemcpyAsync(x->d_blob, blob, blob_bytes, hipMemcpyHostToDevice, x->stream));
        // The caller's buffers are pageable host memory it may free or reuse as soon as this
        // returns, and an async copy from pageable memory may still be reading them: wait.
        HIP_CHECK(wsync(x, x->stream));
        dd = x->d_desc; ds = x->d_seg; dss = x->d_seg_sess; db = x->d_blob;
    } else if (where != EDGPU_PTR_DEVICE) {
        return fail(EDGPU_BAD_ARGUMENT, "bad pointer location");
    }
    return enqueue_ingest(x, dd, n, ds, dss, nseg, db, x->ingest_mode, where == EDGPU_PTR_HOST);
}

int edgpu_ingest_interleaved(edgpu_ctx* x, const edgpu_tcp_read* reads, uint32_t n, const uint8_t* bytes,
                             uint64_t nbytes, int where, edgpu_tcp_result* results) {
    if (!x) return fail(EDGPU_BAD_ARGUMENT, "ctx is NULL");
    if (n && (!reads || !bytes || !results)) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    if (where != EDGPU_PTR_HOST && where != EDGPU_PTR_DEVICE) return fail(EDGPU_BAD_ARGUMENT, "bad pointer location");
    if (where == EDGPU_PTR_DEVICE && ((uintptr_t)bytes & 15)) return fail(EDGPU_BAD_ARGUMENT, "device bytes must be 16-B aligned");
    if (where == EDGPU_PTR_HOST && nbytes > x->cfg.max_batch_bytes) return fail(EDGPU_BAD_ARGUMENT, "reads exceed max_batch_bytes");
    if (x->pending) return fail(EDGPU_ERR, "edgpu_keyframe_index must run after edgpu_ingest");
    if (int r = owed_pass(x, "edgpu_ingest_interleaved")) return r;
    if (!n) return EDGPU_OK;
    DEVICE_ENTER(x);
    if (x->grow_pending || __atomic_load_n(x->h_grow_flag, __ATOMIC_ACQUIRE)) { int r = grow_rings(x); if (r) return r; }
    { int r = wait_pinned_copies(x); if (r) return r; }
    x->carry_len.resize(x->sessions.size(), 0);
    // one group per session: its reads are a run of consecutive entries, contiguous in `bytes`
    std::vector<TcpGroup> groups;
    std::vector<TcpRead> rd(n);
    std::vector<uint32_t> chunk_group;
    std::vector<uint8_t> seen(x->sessions.size(), 0);
    for (uint32_t i = 0; i < n;) {
        const uint32_t s = reads[i].session;
        if (!live_session(x, s)) return fail(EDGPU_BAD_ARGUMENT, "unknown session in reads");
        if (x->sessions[s].udp_push) return fail(EDGPU_BAD_ARGUMENT, "interleaved reads for a UDP-push session");
        if (seen[s]) return fail(EDGPU_BAD_ARGUMENT, "a session's reads must be consecutive entries");
        seen[s] = 1;
        uint64_t pos = x->carry_len[s];
        uint32_t j = i;
        for (; j < n && reads[j].session == s; j++) {
            if (reads[j].offset > nbytes || reads[j].len > nbytes - reads[j].offset)
                return fail(EDGPU_BAD_ARGUMENT, "read outside bytes");
            if (j > i && reads[j].offset != reads[j - 1].offset + reads[j - 1].len)
                return fail(EDGPU_BAD_ARGUMENT, "a session's reads must be contiguous in bytes");
            rd[j].start = pos; rd[j].arrival = reads[j].arrival_ms; rd[j].len = reads[j].len; rd[j]._pad = 0;
            pos += reads[j].len;
        }
        TcpGroup G;
        memset(&G, 0, sizeof(G));
        G.session = s; G.first_read = i; G.nreads = j - i;
        G.first_chunk = (uint32_t)chunk_group.size();
        G.carry_len = x->carry_len[s];
        G.raw_off = reads[i].offset;
        G.len = pos;
        G.nchunks = (uint32_t)((pos + kTcpChunk - 1) / kTcpChunk);
        chunk_group.insert(chunk_group.end(), G.nchunks, (uint32_t)groups.size());
        groups.push_back(G);
        i = j;
    }
    const uint32_t ng = (uint32_t)groups.size(), nc = (uint32_t)chunk_group.size();
    HIP_CHECK(x->d_carry.reserve((size_t)x->sessions.size() * kTcpCarry, x->stream));
    HIP_CHECK(x->d_tcp_groups.reserve(ng, x->stream));
    HIP_CHECK(x->d_tcp_reads.reserve(n, x->stream));
    HIP_CHECK(x->d_tcp_results.reserve(n, x->stream));
    HIP_CHECK(x->d_tcp_chunk_group.reserve(std::max<uint32_t>(nc, 1), x->stream));
    HIP_CHECK(x->d_tcp_ncand.reserve(std::max<uint32_t>(nc, 1), x->stream));
    HIP_CHECK(x->d_tcp_chunkres.reserve(std::max<uint32_t>(nc, 1), x->stream));
    HIP_CHECK(x->d_tcp_cands.reserve((size_t)std::max<uint32_t>(nc, 1) * kTcpCands, x->stream));
    HIP_CHECK(x->d_tcp_links.reserve((size_t)std::max<uint32_t>(nc, 1) * kTcpCands, x->stream));
    HIP_CHECK(x->d_tcp_offs.reserve((size_t)std::max<uint32_t>(nc, 1) * kTcpCands * kTcpFrames, x->stream));
    HIP_CHECK(x->d_tcp_stage.reserve((size_t)ng * kTcpCarry, x->stream));
    if (!x->d_tcp_tot && dmalloc(&x->d_tcp_tot, sizeof(TcpTotals)) != hipSuccess) return fail(EDGPU_OUT_OF_MEMORY, "tcp totals");
    if (!x->d_tcp_src && dmalloc(&x->d_tcp_src, sizeof(uint64_t) * (size_t)x->cfg.max_batch_packets) != hipSuccess)
        return fail(EDGPU_OUT_OF_MEMORY, "frame addresses");
    if (!x->aux) {
        HIP_CHECK(hipStreamCreateWithFlags(&x->aux, hipStreamNonBlocking));
        // from now on every keyframe index records ev_kf; the first deframe follows all work so far
        HIP_CHECK(hipEventCreateWithFlags(&x->ev_kf, hipEventDisableTiming));
        HIP_CHECK(hipEventRecord(x->ev_kf, x->stream));
        x->kf_recorded = true;
    }
    // the deframe rewrites the segment tables the last keyframe index reads (a reserve above that
    // grew has synchronised `stream`); the fan-out after that index keeps running
    if (x->kf_recorded) HIP_CHECK(hipStreamWaitEvent(x->aux, x->ev_kf, 0));
    if (x->deframe_serial) {
        if (!x->ev_serial) HIP_CHECK(hipEventCreateWithFlags(&x->ev_serial, hipEventDisableTiming));
        HIP_CHECK(hipEventRecord(x->ev_serial, x->stream));
        HIP_CHECK(hipStreamWaitEvent(x->aux, x->ev_serial, 0));
    }
    const uint8_t* raw = bytes;
    if (where == EDGPU_PTR_HOST) {
        if (!x->d_tcp_raw && dmalloc(&x->d_tcp_raw, x->cfg.max_batch_bytes) != hipSuccess)
            return fail(EDGPU_OUT_OF_MEMORY, "read staging");
        HIP_CHECK(hipMemcpyAsync(x->d_tcp_raw, bytes, nbytes, hipMemcpyHostToDevice, x->aux));
        raw = x->d_tcp_raw;
    }
    HIP_CHECK(hipMemcpyAsync(x->d_tcp_groups.ptr, groups.data(), ng * sizeof(TcpGroup), hipMemcpyHostToDevice, x->aux));
    HIP_CHECK(hipMemcpyAsync(x->d_tcp_reads.ptr, rd.data(), n * sizeof(TcpRead), hipMemcpyHostToDevice, x->aux));
    if (nc) HIP_CHECK(hipMemcpyAsync(x->d_tcp_chunk_group.ptr, chunk_group.data(), nc * 4, hipMemcpyHostToDevice, x->aux));
    HIP_CHECK(hipMemsetAsync(x->d_tcp_results.ptr, 0, n * sizeof(edgpu_tcp_result), x->aux));
    TcpParams p;
    p.groups = x->d_tcp_groups.ptr; p.ngroups = ng; p.nchunks = nc;
    p.reads = x->d_tcp_reads.ptr; p.chunk_group = x->d_tcp_chunk_group.ptr;
    p.cands = x->d_tcp_cands.ptr; p.links = x->d_tcp_links.ptr; p.ncand = x->d_tcp_ncand.ptr;
    p.chunkres = x->d_tcp_chunkres.ptr;
    p.raw = raw; p.raw_bytes = nbytes;
    p.carry = x->d_carry.ptr;
    p.offs = x->d_tcp_offs.ptr; p.stage = x->d_tcp_stage.ptr;
    p.desc = x->d_desc; p.src_addr = x->d_tcp_src; p.max_desc = x->cfg.max_batch_packets;
    p.seg_off = x->d_seg; p.seg_sess = x->d_seg_sess;
    p.results = x->d_tcp_results.ptr; p.tot = x->d_tcp_tot;
    p.walk = x->tcp_walk;
    p.seg = x->tcp_seg;
    HIP_CHECK(launch_deframe(p, x->aux));
    // The report is the deframe's alone (k_tcp_finish counts the frames too): read on aux, it
    // waits for the deframe only, which runs beside the previous tick's fan-out.  k_ingest is
    // enqueued after it, behind that fan-out on `stream`, with nothing to wait for there: the
    // call returns while the fan-out still runs, and the host enqueues the keyframe index and
    // the next fan-out without leaving the device idle.
    TcpTotals tot;
    Readback rb(x, x->aux);
    HIP_CHECK(rb.add(&tot, x->d_tcp_tot, sizeof(tot)));
    HIP_CHECK(rb.add(results, x->d_tcp_results.ptr, n * sizeof(edgpu_tcp_result)));
    HIP_CHECK(rb.run());
    if (tot.status) return fail(EDGPU_OUT_OVERFLOW, "interleaved frames exceed max_batch_packets");
    int r = enqueue_ingest(x, x->d_desc, 0, x->d_seg, x->d_seg_sess, ng, nullptr, 0, false, &p, true);
    if (r) return r;
    for (const TcpGroup& G : groups) x->carry_len[G.session] = results[G.first_read + G.nreads - 1].carry;
    return EDGPU_OK;
}

int edgpu_fanout_blocked(edgpu_ctx* x, const edgpu_blocked* reports, uint32_t n) {
    if (!x || (n && !reports)) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    if (!n) return EDGPU_OK;
    if (x->fanout_launches == 0) return fail(EDGPU_ERR, "no fan-out tick to report on");
    if (x->pending) return fail(EDGPU_ERR, "backpressure reports must precede the next edgpu_ingest");
    const uint32_t nsub = x->tick_nsubs;             // rows of the tick reported on
    for (uint32_t i = 0; i < n; i++)
        if (reports[i].substream >= nsub) return fail(EDGPU_BAD_ARGUMENT, "bad sub-stream index");
    DEVICE_ENTER(x);
    HIP_CHECK(x->d_blocked.reserve(n, x->stream));
    edgpu_blocked* d = x->d_blocked.ptr;
    HIP_CHECK(hipMemcpyAsync(d, reports, n * sizeof(edgpu_blocked), hipMemcpyHostToDevice, x->stream));
    BlockedParams p;
    p.reports = d; p.n = n;
    p.subs = x->d_subs.ptr; p.senders = x->d_senders.ptr; p.sessions = x->d_sessions.ptr;
    p.now = x->last_now;
    p.relocate_ms = x->cfg.rtp_reflector_threshold_msec;
    p.totals = x->d_totals;
    HIP_CHECK(launch_blocked(p, x->stream));
    HIP_CHECK(wsync(x, x->stream));   // `reports` is the caller's host memory
    return EDGPU_OK;
}

int edgpu_keyframe_index(edgpu_ctx* x) {
    if (!x) return fail(EDGPU_BAD_ARGUMENT, "ctx is NULL");
    if (!x->pending) return fail(EDGPU_ERR, "no ingested batch pending a keyframe index");
    DEVICE_ENTER(x);
    // The index itself ran inside k_ingest (each workgroup walks its segment's packets through it
    // in arrival order once they are enqueued): this call only closes the batch -- one kernel
    // launch and its ~5 us of dependent-launch gap less per tick than a separate k_keyframe.
    x->kf_share = false;
    if (x->aux) {       // the next deframe (on aux) rewrites the segment tables this index reads
        HIP_CHECK(hipEventRecord(x->ev_kf, x->stream));
        x->kf_recorded = true;
    }
    if (x->pend_stage >= 0) {                   // the pinned staging set may be refilled now
        HIP_CHECK(hipEventRecord(x->pin[x->pend_stage].consumed, x->stream));
        x->pend_stage = -1;
    }
    x->pending = false;
    return EDGPU_OK;
}

// The copy kernel for this tick: EDGPU_FANOUT when set, else the default for whether any active
// sub-stream needs a per-output patch (TCP channel byte or rewrite).
static int pick_fanout_variant(const edgpu_ctx* x) {
    if (x->fanout_variant >= 0) return x->fanout_variant;
    // A tick whose new outputs hold a quarter or more of its sub-stream rows, and at least
    // kBurstRows of them, replays a GOP to each (C4's join burst): long runs per sub-stream, which
    // the patching kernel's 32-packet chunks move ~3 % faster than the 16-packet ones
    // (profiles/r05zi_c4_variants/); the steady ticks keep the 16-packet kernel.
    constexpr uint64_t kBurstRows = 4096;
    const bool burst = x->joined_rows >= kBurstRows && x->joined_rows * 4 >= x->sub_sender.size();
    return fanout_default(x->n_rw + x->n_tcp > 0 || burst);
}

// The plan parameters of the context's current tick.
static PlanParams plan_params(edgpu_ctx* x, int64_t now_ms) {
    const uint32_t nsub = x->tick_nsubs;            // rows added since are not the tick's
    PlanParams p;
    p.senders = x->d_senders.ptr; p.subs = x->d_subs.ptr; p.sub_index = x->d_sub_index.ptr;
    p.sub_pos = x->d_sub_pos.ptr; p.sub_range = x->d_sub_range.ptr; p.fansub = x->d_fansub.ptr;
    p.sub_out = x->d_sub_out.ptr;
    p.work = x->d_work.ptr;
    p.blk_bytes = x->d_blk_bytes.ptr; p.blk_count = x->d_blk_count.ptr;
    p.blk_maxb = x->d_blk_maxb.ptr; p.blk_maxc = x->d_blk_maxc.ptr;
    p.sessions = x->d_sessions.ptr;
    p.totals = x->d_totals;
    p.T.now = now_ms;
    p.T.over_buffer_ms = (int64_t)x->cfg.reflector_buffer_size_sec * 1000;
    p.T.arena_bytes = x->cfg.out_arena_bytes;
    p.T.max_desc = x->cfg.max_out_packets;
    p.T.nsenders = x->nsenders;
    p.T.nsubs = nsub;
    p.T.nsub_blocks = (nsub + 255) / 256;
    p.T.chunk = (uint32_t)fanout_chunk(x->tick_variant);
    p.T.pass_ord = x->pass_ord;
    p.T.pass_id = x->pass_id;
    p.grow = x->d_grow;
    p.T.grow_on = x->cfg.ring_growth;
    p.T.grow_max_pk = x->cfg.max_ring_packets;
    p.T.grow_max_bytes = x->cfg.max_ring_bytes;
    p.T.grow_flag = x->d_grow_flag;
    return p;
}

// The copy kernel of the current pass (after the plan, on the context stream).
static int launch_copy_pass(edgpu_ctx* x, edgpu_fanout_result* out) {
    FanoutParams f;
    f.senders = x->d_senders.ptr; f.sub_range = x->d_sub_range.ptr; f.subs = x->d_subs.ptr;
    f.sub_index = x->d_sub_index.ptr; f.work = x->d_work.ptr; f.fansub = x->d_fansub.ptr;
    f.arena = x->d_arena; f.desc = x->d_out_desc;
    f.arena_words = x->cfg.out_arena_bytes / 16;
    f.max_desc = x->cfg.max_out_packets;
    f.totals = x->d_totals;
    f.ablate = x->ablate;
    hipStream_t cs = x->stream;
    HIP_CHECK(hist_mark(x, 0, 0, cs));
    HIP_CHECK(launch_fanout(f, x->tick_variant, x->num_cus, cs));
    HIP_CHECK(hist_mark(x, 0, 1, cs));
    x->fanout_passes++;
    x->passes_more = -1;
    if (out) {
        out->arena = f.arena;
        out->desc = f.desc;
        out->substreams = x->d_sub_out.ptr;
        out->n_substreams = x->tick_nsubs;
    }
    return EDGPU_OK;
}

int edgpu_fanout(edgpu_ctx* x, int64_t now_ms, edgpu_fanout_result* out) {
    if (!x) return fail(EDGPU_BAD_ARGUMENT, "ctx is NULL");
    if (x->pending) return fail(EDGPU_ERR, "edgpu_keyframe_index must run after edgpu_ingest");
    if (int r = owed_pass(x, "edgpu_fanout")) return r;
    DEVICE_ENTER(x);
    // rows freed during the last tick may be reused from now on (its passes are delivered)
    for (const auto& f : x->free_pending) x->free_subs[f.first].push_back(f.second);
    x->free_pending.clear();
    if (x->index_dirty) { int r = rebuild_index(x); if (r) return r; }
    x->tick_nsubs = (uint32_t)x->sub_sender.size();     // this tick's table: later passes keep it
    x->last_now = now_ms;
    queue_source_reports(x, now_ms);
    x->tick_variant = pick_fanout_variant(x);
    x->joined_rows = 0;
    x->pass_ord = 0;
    x->pass_id = 0;
    const PlanParams p = plan_params(x, now_ms);
    // the per-tick totals (relayed_*, arena, status, nwork, passes) are reset by the plan's first kernel
    HIP_CHECK(hist_mark(x, 1, 0));
    HIP_CHECK(launch_plan(p, x->stream));
    if (int r = launch_copy_pass(x, out)) return r;
    if (x->timing >= EDGPU_TIMING_ALL) {   // the whole-tick pair (ring 1) ends at this copy kernel's end event
        const uint32_t s1 = x->hist_n[1];
        x->tick_end[s1 % edgpu_ctx::kHist] = x->last_seq[0];
        x->last_seq[1] = s1;
        x->hist_n[1] = s1 + 1;
    }
    x->fanout_launches++;
    x->timed_fanout = true;
    return EDGPU_OK;
}

int edgpu_fanout_next(edgpu_ctx* x, edgpu_fanout_result* out, uint32_t* launched) {
    if (!x || !launched) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    *launched = 0;
    if (x->fanout_launches == 0) return fail(EDGPU_ERR, "no fan-out tick");
    DEVICE_ENTER(x);
    TickTotals t;
    HIP_CHECK(sync_all(x));                  // the host has consumed the current pass
    {
        Readback rb(x);
        HIP_CHECK(rb.add(&t, x->d_totals, sizeof(t)));
        HIP_CHECK(rb.run());
    }
    note_grow(x, t);
    if (t.status) {
        // a failed tick owes nothing: its remaining passes are dropped (the next fan-out counts
        // them in lost_passes), so the context does not refuse every later call
        x->passes_more = 0;
        return fail(t.status, "the tick failed");
    }
    const uint32_t next = t.pass_next[x->pass_ord & 1u];
    if (next == kNoPass) {
        x->passes_more = 0;
        return EDGPU_OK;
    }
    x->pass_ord++;
    x->pass_id = next;
    const PlanParams p = plan_params(x, x->last_now);
    HIP_CHECK(launch_plan_pass(p, x->stream));
    if (int r = launch_copy_pass(x, out)) return r;
    *launched = 1;
    return EDGPU_OK;
}

const char* edgpu_fanout_kernel(edgpu_ctx* x) {
    if (!x) return "";
    return fanout_name(x->fanout_launches ? x->tick_variant : pick_fanout_variant(x));
}

int edgpu_tick_stats_get(edgpu_ctx* x, edgpu_tick_stats* out) {
    if (!x || !out) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    if (x->pending) return fail(EDGPU_ERR, "edgpu_keyframe_index must run after edgpu_ingest (the ingest counters "
                                           "of a batch are set by its index)");
    DEVICE_ENTER(x);
    TickTotals t;
    HIP_CHECK(sync_all(x));
    {
        Readback rb(x);
        HIP_CHECK(rb.add(&t, x->d_totals, sizeof(t)));
        HIP_CHECK(rb.run());
    }
    note_grow(x, t);
    out->relayed_packets = t.relayed_packets;
    out->relayed_bytes = t.relayed_bytes;
    out->arena_bytes = t.arena_bytes;
    out->ingested_packets = t.ing_pk[x->ing_slot];
    out->ingested_bytes = t.ing_b[x->ing_slot];
    out->status = t.status ? t.status : t.ingest_status;
    out->_pad = t.nwork;
    const uint32_t slot = x->pass_ord & 1u;
    out->pass_arena_bytes = t.pass_bytes[slot];
    out->pass_packets = t.pass_desc[slot];
    out->pass = x->pass_ord;
    out->more_passes = (x->fanout_launches && t.pass_next[slot] != kNoPass) ? 1u : 0u;
    out->stream_errors = t.stream_errors;
    if (x->fanout_launches) x->passes_more = t.status ? 0 : (int)out->more_passes;
#ifdef EDGPU_AB_VARIANTS
    if (getenv("EDGPU_FAN_TAIL") && t.fan_done_max > t.fan_t0_min)   // 100-MHz s_memrealtime ticks
        fprintf(stderr, "fan tail: span %.1f us, first exit at %.1f us, items %u; ingest span %.1f us, first exit at %.1f us\n",
                (t.fan_done_max - t.fan_t0_min) / 100.0, (t.fan_done_min - t.fan_t0_min) / 100.0, t.nwork,
                t.ing_last_span / 100.0, t.ing_last_first / 100.0);
    if (getenv("EDGPU_FAN_TAIL") && t.ing_last_ph[0]) {
        fprintf(stderr, "ingest phases (us per segment, %llu segments):", (unsigned long long)t.ing_last_ph[0]);
        for (int k = 1; k < 7; k++) fprintf(stderr, " %.2f", t.ing_last_ph[k] / 100.0 / t.ing_last_ph[0]);
        fprintf(stderr, "\n");
    }
#endif
    return EDGPU_OK;
}

int edgpu_fanout_arrivals(edgpu_ctx* x, int64_t* out, uint32_t n, int kind) {
    if (!x || !out) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    return edgpu_fanout_packet_info(x, out, nullptr, n, kind);
}

// Per descriptor of the current pass: its packet's arrival and/or its blob slot in the last host
// batch (kNoSource when it came with an earlier batch, or the last one was not a host batch).
int edgpu_fanout_packet_info(edgpu_ctx* x, int64_t* arrivals, uint32_t* sources, uint32_t n, int kind) {
    if (!x || (!arrivals && !sources)) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    if (kind != EDGPU_PTR_HOST && kind != EDGPU_PTR_DEVICE) return fail(EDGPU_BAD_ARGUMENT, "bad ptr_kind");
    DEVICE_ENTER(x);
    TickTotals t;
    HIP_CHECK(sync_all(x));
    {
        Readback rb(x);
        HIP_CHECK(rb.add(&t, x->d_totals, sizeof(t)));
        HIP_CHECK(rb.run());
    }
    if (t.status) return fail(t.status, "the last tick failed");
    const uint32_t npass = t.pass_desc[x->pass_ord & 1u];      // the current copy pass's descriptors
    if (n < npass) return fail(EDGPU_OUT_OVERFLOW, "array smaller than the pass's descriptors");
    if (!npass) return EDGPU_OK;
    int64_t* da = arrivals;
    uint32_t* dsrc = sources;
    if (kind == EDGPU_PTR_HOST) {
        if (arrivals) { HIP_CHECK(x->d_arrivals.reserve(npass, x->stream)); da = x->d_arrivals.ptr; }
        if (sources) { HIP_CHECK(x->d_sources.reserve(npass, x->stream)); dsrc = x->d_sources.ptr; }
    }
    if (arrivals) HIP_CHECK(launch_desc_arrival(x->d_subs.ptr, x->d_senders.ptr, x->tick_nsubs, x->pass_id, da, x->stream));
    if (sources) {
        HIP_CHECK(hipMemsetAsync(dsrc, 0xFF, (size_t)npass * sizeof(uint32_t), x->stream));
        if (x->host_epoch_last)
            HIP_CHECK(launch_desc_source(x->d_subs.ptr, x->d_senders.ptr, x->tick_nsubs, x->pass_id, x->host_epoch_last,
                                         dsrc, x->stream));
    }
    Readback rb(x);
    if (kind == EDGPU_PTR_HOST) {
        if (arrivals) HIP_CHECK(rb.add(arrivals, da, (size_t)npass * sizeof(int64_t)));
        if (sources) HIP_CHECK(rb.add(sources, dsrc, (size_t)npass * sizeof(uint32_t)));
    }
    HIP_CHECK(rb.run());
    return EDGPU_OK;
}

int edgpu_fanout_active(edgpu_ctx* x, edgpu_substream_out* rows, uint32_t* q, uint32_t cap, uint32_t* n_out, int kind) {
    if (!x || !n_out || (cap && (!rows || !q))) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    if (kind != EDGPU_PTR_HOST && kind != EDGPU_PTR_DEVICE) return fail(EDGPU_BAD_ARGUMENT, "bad ptr_kind");
    *n_out = 0;
    if (x->fanout_launches == 0) return fail(EDGPU_ERR, "no fan-out tick");
    DEVICE_ENTER(x);
    const uint32_t n = x->tick_nsubs;
    if (!n) return EDGPU_OK;
    const uint32_t nb = (n + 255) / 256;
    HIP_CHECK(x->d_act_blk.reserve((size_t)nb + 1, x->stream));
    uint32_t* total = x->d_act_blk.ptr + nb;
    // pinned host destinations are stored into by the kernel over PCIe; others through a staging copy
    const bool direct = kind == EDGPU_PTR_DEVICE || (!cap || (Readback::is_pinned(rows) && Readback::is_pinned(q)));
    edgpu_substream_out* dr = rows;
    uint32_t* dq = q;
    if (!direct) {
        HIP_CHECK(x->d_act_rows.reserve(std::max<uint32_t>(cap, 1), x->stream));
        HIP_CHECK(x->d_act_q.reserve(std::max<uint32_t>(cap, 1), x->stream));
        dr = x->d_act_rows.ptr; dq = x->d_act_q.ptr;
    }
    HIP_CHECK(launch_sub_active(x->d_sub_out.ptr, n, x->d_act_blk.ptr, dr, dq, cap, total, x->stream));
    uint32_t tot = 0;
    {
        Readback rb(x);
        HIP_CHECK(rb.add(&tot, total, sizeof(tot)));
        HIP_CHECK(rb.run());
    }
    if (!direct && tot && cap) {
        const uint32_t k = std::min(tot, cap);
        Readback rb(x);
        HIP_CHECK(rb.add(rows, dr, (size_t)k * sizeof(edgpu_substream_out)));
        HIP_CHECK(rb.add(q, dq, (size_t)k * sizeof(uint32_t)));
        HIP_CHECK(rb.run());
    }
    *n_out = tot;
    return EDGPU_OK;
}

int edgpu_fanout_rows(edgpu_ctx* x, const uint32_t* sel, uint32_t nsel, edgpu_packet_row* rows, uint64_t nrows, int kind) {
    if (!x || (nsel && (!sel || !rows))) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    if (kind != EDGPU_PTR_HOST && kind != EDGPU_PTR_DEVICE) return fail(EDGPU_BAD_ARGUMENT, "bad ptr_kind");
    if (!nsel || !nrows) return EDGPU_OK;
    DEVICE_ENTER(x);
    TickTotals t;
    HIP_CHECK(sync_all(x));
    {
        Readback rb(x);
        HIP_CHECK(rb.add(&t, x->d_totals, sizeof(t)));
        HIP_CHECK(rb.run());
    }
    if (t.status) return fail(t.status, "the last tick failed");
    edgpu_packet_row* dr = rows;
    if (kind == EDGPU_PTR_HOST) { HIP_CHECK(x->d_rows.reserve(nrows, x->stream)); dr = x->d_rows.ptr; }
    HIP_CHECK(x->d_row_sel.reserve(2 * (uint64_t)nsel, x->stream));
    HIP_CHECK(hipMemcpyAsync(x->d_row_sel.ptr, sel, 2 * (size_t)nsel * sizeof(uint32_t), hipMemcpyHostToDevice, x->stream));
    HIP_CHECK(launch_sub_rows(x->d_subs.ptr, x->d_senders.ptr, x->d_out_desc, x->d_row_sel.ptr, nsel,
                              x->tick_nsubs, x->pass_id, x->host_epoch_last, dr, nrows, x->stream));
    if (kind == EDGPU_PTR_HOST) {
        Readback rb(x);
        HIP_CHECK(rb.add(rows, dr, (size_t)nrows * sizeof(edgpu_packet_row)));
        HIP_CHECK(rb.run());
    } else {
        HIP_CHECK(wsync(x, x->stream));      // `sel` is host memory
    }
    return EDGPU_OK;
}

int edgpu_arena_gather(edgpu_ctx* x, const edgpu_fanout_result* r, const edgpu_region* reg, uint32_t n, void* dst,
                       uint64_t cap) {
    if (!x || !r || (n && (!reg || !dst))) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    if (!n) return EDGPU_OK;
    std::vector<uint64_t> off(n);
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; i++) {
        if ((reg[i].offset | reg[i].bytes) & 15) return fail(EDGPU_BAD_ARGUMENT, "regions must be 16-B aligned");
        if (reg[i].offset + reg[i].bytes > x->cfg.out_arena_bytes) return fail(EDGPU_BAD_ARGUMENT, "region outside the arena");
        off[i] = total;
        total += reg[i].bytes;
    }
    if (total > cap) return fail(EDGPU_OUT_OVERFLOW, "gather destination too small");
    DEVICE_ENTER(x);
    HIP_CHECK(sync_all(x));                      // the tick's copy is done
    HIP_CHECK(x->d_gather_reg.reserve(n, x->stream));
    HIP_CHECK(x->d_gather_off.reserve(n, x->stream));
    HIP_CHECK(hipMemcpyAsync(x->d_gather_reg.ptr, reg, n * sizeof(edgpu_region), hipMemcpyHostToDevice, x->stream));
    HIP_CHECK(hipMemcpyAsync(x->d_gather_off.ptr, off.data(), n * sizeof(uint64_t), hipMemcpyHostToDevice, x->stream));
    HIP_CHECK(launch_arena_gather(r->arena, x->d_gather_reg.ptr, x->d_gather_off.ptr, n, (uint8_t*)dst, x->stream));
    HIP_CHECK(wsync(x, x->stream));  // `reg` and `off` are host memory
    return EDGPU_OK;
}

int edgpu_counters_get(edgpu_ctx* x, edgpu_counters* out) {
    if (!x || !out) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    DEVICE_ENTER(x);
    TickTotals t;
    HIP_CHECK(sync_all(x));
    {
        Readback rb(x);
        HIP_CHECK(rb.add(&t, x->d_totals, sizeof(t)));
        HIP_CHECK(rb.run());
    }
    out->relayed_packets = t.cum_relayed_packets;
    out->relayed_bytes = t.cum_relayed_bytes;
    out->fanout_in_bytes = t.cum_fanout_in_bytes;
    out->fanout_launches = x->fanout_launches;
    out->ingested_packets = t.cum_ingested_packets;
    out->ingested_bytes = t.cum_ingested_bytes;
    out->fanout_passes = x->fanout_passes;
    out->lost_passes = t.cum_lost_passes;
    out->ring_grows = x->ring_grows;
    out->ring_pool_bytes = x->rings.held;
    out->watchdog_timeouts = x->watchdog_timeouts;
    out->kernel_launches = x->kernel_launches;
    out->host_syncs = x->host_syncs;
    out->ring_grow_failures = x->grow_failures;
    out->ring_bytes = x->ring_bytes;
    out->senders = x->nsenders;
    out->substream_rows = (uint32_t)x->sub_sender.size();
    return EDGPU_OK;
}

int edgpu_kernel_times(edgpu_ctx* x, int which, float* out_ms, uint32_t max_n, uint32_t* out_n) {
    if (!x || which < 0 || which > 3 || (!out_ms && max_n)) return fail(EDGPU_BAD_ARGUMENT, "bad argument");
    DEVICE_ENTER(x);
    HIP_CHECK(sync_all(x));
    const uint32_t n = std::min<uint32_t>(x->hist_n[which] - x->hist_rd[which], edgpu_ctx::kHist);
    const uint32_t first = x->hist_n[which] - n;
    uint32_t k = 0;
    for (uint32_t i = 0; i < n && k < max_n; i++) {
        hipEvent_t a, b;
        if (!hist_pair(x, which, first + i, &a, &b)) continue;     // a borrowed event was reused
        HIP_CHECK(hipEventElapsedTime(&out_ms[k], a, b));
        k++;
    }
    x->hist_rd[which] = x->hist_n[which];
    if (out_n) *out_n = k;
    return EDGPU_OK;
}

int edgpu_copy_to_host(edgpu_ctx* x, void* dst, const void* src, uint64_t bytes) {
    if (!x || (!dst && bytes) || (!src && bytes)) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    if (!bytes) return EDGPU_OK;
    DEVICE_ENTER(x);
    HIP_CHECK(sync_all(x));
    Readback rb(x);
    HIP_CHECK(rb.add(dst, src, bytes));
    HIP_CHECK(rb.run());
    return EDGPU_OK;
}

int edgpu_set_timing(edgpu_ctx* x, int level) {
    if (!x || level < EDGPU_TIMING_NONE || level > EDGPU_TIMING_ALL) return fail(EDGPU_BAD_ARGUMENT, "bad timing level");
    x->timing = level;
    return EDGPU_OK;
}

int edgpu_last_timings(edgpu_ctx* x, float out_ms[4]) {
    if (!x || !out_ms) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    DEVICE_ENTER(x);
    HIP_CHECK(sync_all(x));
    out_ms[0] = out_ms[1] = out_ms[2] = out_ms[3] = 0.f;
    // the newest pair of each history ring: every timed point is recorded once per tick (an
    // event record costs the GPU ~5 us of idle between the kernels around it)
    auto last = [&](int w, float* o) {
        hipEvent_t a, b;
        if (x->hist_n[w] == 0) return hipSuccess;          // nothing recorded (edgpu_set_timing)
        if (!hist_pair(x, w, x->last_seq[w], &a, &b)) return hipSuccess;
        return hipEventElapsedTime(o, a, b);
    };
    if (x->timed_fanout) {
        HIP_CHECK(last(0, &out_ms[0]));
        HIP_CHECK(last(1, &out_ms[1]));
    }
    if (x->timed_ingest) HIP_CHECK(last(2, &out_ms[2]));
    if (x->timed_keyframe) HIP_CHECK(last(3, &out_ms[3]));
    return EDGPU_OK;
}

int edgpu_gop_span(edgpu_ctx* x, uint32_t session, uint32_t track, uint64_t* out_packets, uint64_t* out_bytes) {
    if (!x || !live_session(x, session) || track >= x->sessions[session].ntracks)
        return fail(EDGPU_BAD_ARGUMENT, "bad session/track");
    DEVICE_ENTER(x);
    SenderDev D;
    Readback rb(x);
    HIP_CHECK(rb.add(&D, x->d_senders.ptr + x->sessions[session].first_sender + 2 * track, sizeof(D)));
    HIP_CHECK(rb.run());
    uint64_t pk = 0, by = 0;
    if (D.key >= 0) {
        PktMeta m;
        HIP_CHECK(rb.add(&m, reinterpret_cast<PktMeta*>(D.meta) + ((uint64_t)D.key & D.pk_mask), sizeof(m)));
        HIP_CHECK(rb.run());
        pk = D.head - (uint64_t)D.key;
        by = D.vbyte_end - m.vbyte;
    }
    if (out_packets) *out_packets = pk;
    if (out_bytes) *out_bytes = by;
    return EDGPU_OK;
}

int edgpu_gop_copy(edgpu_ctx* x, uint32_t session, uint32_t track, uint8_t* dst, uint64_t cap,
                   uint64_t* out_len, uint32_t* out_packets) {
    if (!x || !live_session(x, session) || track >= x->sessions[session].ntracks || (!dst && cap))
        return fail(EDGPU_BAD_ARGUMENT, "bad argument");
    DEVICE_ENTER(x);
    SenderDev D;
    Readback rb(x);
    HIP_CHECK(rb.add(&D, x->d_senders.ptr + x->sessions[session].first_sender + 2 * track, sizeof(D)));
    HIP_CHECK(rb.run());
    if (out_len) *out_len = 0;
    if (out_packets) *out_packets = 0;
    if (D.key < 0 || (uint64_t)D.key >= D.head) return EDGPU_OK;
    const uint64_t k = (uint64_t)D.key, n = D.head - k, pkcap = (uint64_t)D.pk_mask + 1;
    const uint64_t bcap = ((uint64_t)D.word_mask + 1) * 16;
    if (n > pkcap) return fail(EDGPU_RING_OVERFLOW, "GOP no longer in the packet ring");
    std::vector<PktMeta> meta(n);
    const PktMeta* dmeta = reinterpret_cast<const PktMeta*>(D.meta);
    for (uint64_t i = 0; i < n;) {            // ring segments
        const uint64_t pos = (k + i) & D.pk_mask, run = std::min(n - i, pkcap - pos);
        HIP_CHECK(rb.add(&meta[i], dmeta + pos, run * sizeof(PktMeta)));
        i += run;
    }
    HIP_CHECK(rb.run());
    const uint64_t vb0 = meta[0].vbyte, span = D.vbyte_end - vb0;
    if (std::max(D.vbyte_end, D.vclob) - vb0 > bcap) return fail(EDGPU_RING_OVERFLOW, "GOP no longer in the byte ring");
    std::vector<uint8_t> bytes(span);
    const uint8_t* ring = reinterpret_cast<const uint8_t*>(D.ring);
    for (uint64_t i = 0; i < span;) {
        const uint64_t pos = (vb0 + i) & (bcap - 1), run = std::min(span - i, bcap - pos);
        HIP_CHECK(rb.add(&bytes[i], ring + pos, run));
        i += run;
    }
    HIP_CHECK(rb.run());
    uint64_t len = 0; uint32_t np = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (meta[i].len == 0) continue;
        const uint64_t need = (uint64_t)meta[i].len + 4;
        if (len + need > cap) return fail(EDGPU_OUT_OVERFLOW, "destination too small for the GOP");
        dst[len] = 0x28;                                  // BUF_STX
        dst[len + 1] = (uint8_t)(meta[i].len >> 8);
        dst[len + 2] = (uint8_t)meta[i].len;
        memcpy(dst + len + 3, &bytes[meta[i].vbyte - vb0 + 4], meta[i].len);
        dst[len + 3 + meta[i].len] = 0x29;                // BUF_ETX
        len += need;
        np++;
    }
    if (out_len) *out_len = len;
    if (out_packets) *out_packets = np;
    return EDGPU_OK;
}

// ---------------------------------------------------------------------------------------
// Session images (cross-GPU keyframe fast start)

static int image_launch(edgpu_ctx* x, std::vector<ImgPlan>& plan, int64_t now_ms, uint8_t* buf, int phase) {
    if (!x->d_img_status && dmalloc(&x->d_img_status, sizeof(int)) != hipSuccess)
        return fail(EDGPU_OUT_OF_MEMORY, "image status");
    HIP_CHECK(x->d_img_plan.reserve(std::max<size_t>(plan.size(), 1), x->stream));
    HIP_CHECK(hipMemcpyAsync(x->d_img_plan.ptr, plan.data(), plan.size() * sizeof(ImgPlan), hipMemcpyHostToDevice, x->stream));
    HIP_CHECK(hipMemsetAsync(x->d_img_status, 0, sizeof(int), x->stream));
    ImageParams p;
    p.senders = x->d_senders.ptr; p.sessions = x->d_sessions.ptr; p.streams = x->d_streams.ptr;
    p.plan = x->d_img_plan.ptr; p.nplan = (uint32_t)plan.size();
    p.now = now_ms; p.over_buffer_ms = (int64_t)x->cfg.reflector_buffer_size_sec * 1000;
    p.buf = buf; p.status = x->d_img_status;
    HIP_CHECK(launch_image(p, phase, x->stream));
    int status = 0;
    Readback rb(x);
    HIP_CHECK(rb.add(&status, x->d_img_status, sizeof(int)));
    if (phase == 0 || phase == 3) HIP_CHECK(rb.add(plan.data(), x->d_img_plan.ptr, plan.size() * sizeof(ImgPlan)));
    HIP_CHECK(rb.run());
    if (status) return fail(status, phase == 2 ? "session image rejected by the replica" : "session image export");
    return EDGPU_OK;
}

int edgpu_session_export(edgpu_ctx* x, const uint32_t* sessions, uint32_t n, int64_t now_ms,
                         const uint64_t* from, void* dst, uint64_t cap, uint64_t* offsets, uint64_t* heads) {
    if (!x || (n && (!sessions || !offsets))) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    if (x->pending) return fail(EDGPU_ERR, "edgpu_keyframe_index must run after edgpu_ingest");
    DEVICE_ENTER(x);
    std::vector<ImgPlan> plan;
    for (uint32_t i = 0; i < n; i++) {
        if (!live_session(x, sessions[i])) return fail(EDGPU_BAD_ARGUMENT, "bad session");
        const SessionHost& sh = x->sessions[sessions[i]];
        for (uint32_t ls = 0; ls < 2 * sh.ntracks; ls++) {
            ImgPlan E;
            memset(&E, 0, sizeof(E));
            E.sender = sh.first_sender + ls; E.session = sessions[i]; E.ls = ls; E.first = ls == 0;
            E.from = from ? from[plan.size()] : kImageFull;
            plan.push_back(E);
        }
    }
    offsets[0] = 0;
    if (plan.empty()) return EDGPU_OK;
    int r = image_launch(x, plan, now_ms, nullptr, 0);
    if (r) return r;
    uint64_t base = 0;
    for (uint32_t i = 0, k = 0; i < n; i++) {
        const uint32_t nt = x->sessions[sessions[i]].ntracks, ns = 2 * nt;
        uint64_t cur = sizeof(ImgHeader) + nt * sizeof(ImgStream) + ns * sizeof(ImgSender);
        for (uint32_t ls = 0; ls < ns; ls++) {
            ImgPlan& E = plan[k + ls];
            E.image_base = base;
            E.meta_off = cur; cur += E.nmeta * sizeof(PktMeta);
            E.bytes_off = cur; cur += E.nbytes;
            if (heads) heads[k + ls] = E.floor + E.nmeta;
        }
        cur = (cur + 15) & ~15ull;
        for (uint32_t ls = 0; ls < ns; ls++) plan[k + ls].image_bytes = cur;
        offsets[i] = base;
        base += cur;
        k += ns;
    }
    offsets[n] = base;
    if (!dst) return EDGPU_OK;                         // size query
    if (base > cap) return fail(EDGPU_OUT_OVERFLOW, "image buffer too small");
    r = image_launch(x, plan, now_ms, (uint8_t*)dst, 1);
    if (!r && getenv("EDGPU_DEBUG_PLAY")) {              // debugging: the exported senders' key pointers
        for (const ImgPlan& E : plan) {
            SenderDev d;
            Readback rb(x);
            HIP_CHECK(rb.add(&d, x->d_senders.ptr + E.sender, sizeof(SenderDev)));
            HIP_CHECK(rb.run());
            fprintf(stderr, "export now=%lld session=%u ls=%u from=%lld floor=%llu head=%llu key=%lld\n", (long long)now_ms,
                    E.session, E.ls, (long long)E.from, (unsigned long long)E.floor, (unsigned long long)d.head,
                    (long long)d.key);
        }
    }
    return r;
}

int edgpu_session_import(edgpu_ctx* x, const void* images, const uint64_t* offsets, uint32_t n,
                         const uint32_t* sessions) {
    if (!x || (n && (!images || !offsets || !sessions))) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    if (x->pending) return fail(EDGPU_ERR, "edgpu_keyframe_index must run after edgpu_ingest");
    DEVICE_ENTER(x);
    std::vector<ImgPlan> plan;
    for (uint32_t i = 0; i < n; i++) {
        if (!live_session(x, sessions[i])) return fail(EDGPU_BAD_ARGUMENT, "bad session");
        if (offsets[i] % 16 || offsets[i + 1] < offsets[i] + sizeof(ImgHeader))
            return fail(EDGPU_BAD_ARGUMENT, "bad image offsets");
        const SessionHost& sh = x->sessions[sessions[i]];
        for (uint32_t ls = 0; ls < 2 * sh.ntracks; ls++) {
            ImgPlan E;
            memset(&E, 0, sizeof(E));
            E.sender = sh.first_sender + ls; E.session = sessions[i]; E.ls = ls; E.first = ls == 0;
            E.image_base = offsets[i];
            plan.push_back(E);
        }
    }
    if (plan.empty()) return EDGPU_OK;
    if (x->grow_pending || __atomic_load_n(x->h_grow_flag, __ATOMIC_ACQUIRE)) { int r = grow_rings(x); if (r) return r; }
    if (x->cfg.ring_growth) {
        // a replica's rings must hold what its owner's image carries (a full image: the key packet's
        // GOP, say): a sender whose image part exceeds a ring gets it grown first (k_image_fit
        // measures every sender at once; one readback)
        HIP_CHECK(sync_all(x));
        std::vector<ImgPlan> fit(plan);
        for (size_t k = 0, i = 0; k < fit.size(); k++) {
            while (i + 1 < n && fit[k].image_base != offsets[i]) i++;
            fit[k].image_bytes = offsets[i + 1] - offsets[i];
        }
        if (int r = image_launch(x, fit, 0, (uint8_t*)const_cast<void*>(images), 3)) return r;
        for (const ImgPlan& f : fit) {
            if (!f.nmeta && !f.nbytes) continue;
            // (what the ring keeps beyond the image is the replica plan's growth requests' concern)
            bool grown = false;
            if (int e = grow_sender(x, f.sender, 2 * f.nmeta, 2 * f.nbytes, f.floor, nullptr, &grown)) return e;
        }
    }
    return image_launch(x, plan, 0, (uint8_t*)const_cast<void*>(images), 2);
}

// Per-stream isolation: the sessions a tick marked, read and cleared.
int edgpu_stream_errors(edgpu_ctx* x, uint32_t* sessions, int32_t* codes, uint32_t cap, uint32_t* n) {
    if (!x || !n || (cap && (!sessions || !codes))) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    *n = 0;
    const uint32_t ns = (uint32_t)x->sessions.size();
    if (!ns) return EDGPU_OK;
    DEVICE_ENTER(x);
    HIP_CHECK(sync_all(x));
    std::vector<SessionDev> sd(ns);
    {
        Readback rb(x);
        HIP_CHECK(rb.add(sd.data(), x->d_sessions.ptr, ns * sizeof(SessionDev)));
        HIP_CHECK(rb.run());
    }
    uint32_t k = 0;
    for (uint32_t s = 0; s < ns; s++) {
        if (!sd[s].errors || !x->sessions[s].alive) continue;
        if (k < cap) {
            sessions[k] = s;
            codes[k] = EDGPU_RING_OVERFLOW;
            HIP_CHECK(hipMemsetAsync(&x->d_sessions.ptr[s].errors, 0, sizeof(uint32_t), x->stream));
        }
        k++;
    }
    HIP_CHECK(wsync(x, x->stream));
    *n = k;
    return EDGPU_OK;
}

// Replica feedback: relocations made on this context's sessions since the last call (read and
// cleared), and the owner's side, ReflectorSession::SetHasVideoKeyFrameUpdate(true).
int edgpu_session_relocations(edgpu_ctx* x, const uint32_t* sessions, uint32_t n, uint8_t* out) {
    if (!x || (n && (!sessions || !out))) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    for (uint32_t i = 0; i < n; i++)
        if (!live_session(x, sessions[i])) return fail(EDGPU_BAD_ARGUMENT, "bad session");
    if (!n) return EDGPU_OK;
    DEVICE_ENTER(x);
    std::vector<uint32_t> v(n, 0);
    {
        Readback rb(x);                               // after the backpressure reports (same stream)
        for (uint32_t i = 0; i < n; i++) HIP_CHECK(rb.add(&v[i], &x->d_sessions.ptr[sessions[i]].relocated, sizeof(uint32_t)));
        HIP_CHECK(rb.run());
    }
    for (uint32_t i = 0; i < n; i++) {
        out[i] = v[i] ? 1 : 0;
        if (v[i]) HIP_CHECK(hipMemsetAsync(&x->d_sessions.ptr[sessions[i]].relocated, 0, sizeof(uint32_t), x->stream));
    }
    HIP_CHECK(wsync(x, x->stream));
    return EDGPU_OK;
}

int edgpu_session_key_update(edgpu_ctx* x, const uint32_t* sessions, uint32_t n) {
    if (!x || (n && !sessions)) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    if (x->pending) return fail(EDGPU_ERR, "edgpu_keyframe_index must run after edgpu_ingest");
    for (uint32_t i = 0; i < n; i++)
        if (!live_session(x, sessions[i])) return fail(EDGPU_BAD_ARGUMENT, "bad session");
    if (!n) return EDGPU_OK;
    DEVICE_ENTER(x);
    static const uint32_t one = 1;
    // on the context stream: the next batch's k_ingest reads it
    for (uint32_t i = 0; i < n; i++)
        HIP_CHECK(hipMemcpyAsync(&x->d_sessions.ptr[sessions[i]].video_key_flag, &one, sizeof(one), hipMemcpyHostToDevice,
                                 x->stream));
    HIP_CHECK(wsync(x, x->stream));
    return EDGPU_OK;
}

int edgpu_device_alloc(edgpu_ctx* x, uint64_t bytes, void** out) {
    if (!x || !out) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    DEVICE_ENTER(x);
    *out = nullptr;
    if (dmalloc(out, std::max<uint64_t>(bytes, 16)) != hipSuccess) return fail(EDGPU_OUT_OF_MEMORY, "device buffer");
    return EDGPU_OK;
}

int edgpu_ipc_export(edgpu_ctx* x, const void* p, uint8_t handle[EDGPU_IPC_HANDLE_BYTES]) {
    if (!x || !p || !handle) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    static_assert(sizeof(hipIpcMemHandle_t) == EDGPU_IPC_HANDLE_BYTES, "IPC handle size");
    DEVICE_ENTER(x);
    hipIpcMemHandle_t h;
    HIP_CHECK(hipIpcGetMemHandle(&h, const_cast<void*>(p)));
    memcpy(handle, &h, sizeof(h));
    return EDGPU_OK;
}

int edgpu_ipc_open(edgpu_ctx* x, const uint8_t handle[EDGPU_IPC_HANDLE_BYTES], void** out) {
    if (!x || !handle || !out) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    DEVICE_ENTER(x);
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof(h));
    *out = nullptr;
    HIP_CHECK(hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess));
    return EDGPU_OK;
}

int edgpu_ipc_close(edgpu_ctx* x, void* p) {
    if (!x || !p) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    DEVICE_ENTER(x);
    HIP_CHECK(sync_all(x));                     // nothing enqueued may still read it
    HIP_CHECK(hipIpcCloseMemHandle(p));
    return EDGPU_OK;
}

int edgpu_copy_to_device(edgpu_ctx* x, void* dst, const void* src, uint64_t bytes) {
    if (!x || (bytes && (!dst || !src))) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    if (!bytes) return EDGPU_OK;
    DEVICE_ENTER(x);
    HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, x->stream));
    HIP_CHECK(wsync(x, x->stream));            // `src` is the caller's
    return EDGPU_OK;
}

// The host CPUs of the device's NUMA node (its PCI function's sysfs local_cpulist) that the
// calling thread may run on: where a server's host threads belong next to this GPU.
int edgpu_device_local_cpus(int device, uint32_t* cpus, uint32_t cap, uint32_t* n_out) {
    if (!n_out || (cap && !cpus)) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    *n_out = 0;
    char bdf[64] = {0};
    HIP_CHECK(hipDeviceGetPCIBusId(bdf, (int)sizeof(bdf) - 1, device));
    for (char* c = bdf; *c; c++) *c = (char)tolower((unsigned char)*c);
    const std::string path = std::string("/sys/bus/pci/devices/") + bdf + "/local_cpulist";
    FILE* f = fopen(path.c_str(), "r");
    if (!f) return fail(EDGPU_ERR, "no " + path);
    char buf[4096];
    const size_t len = fread(buf, 1, sizeof(buf) - 1, f);
    fclose(f);
    buf[len] = 0;
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return fail(EDGPU_ERR, "sched_getaffinity");
    uint32_t n = 0;
    for (const char* q = buf; *q >= '0' && *q <= '9';) {          // "a-b,c,d-e\n"
        char* e;
        const long a = strtol(q, &e, 10);
        long b = a;
        if (*e == '-') b = strtol(e + 1, &e, 10);
        for (long c = a; c <= b && c < CPU_SETSIZE; c++)
            if (CPU_ISSET(c, &allowed)) {
                if (n < cap) cpus[n] = (uint32_t)c;
                n++;
            }
        q = *e == ',' ? e + 1 : e;
    }
    *n_out = n;
    return EDGPU_OK;
}

int edgpu_debug_stall(edgpu_ctx* x, uint32_t us) {
    if (!x) return fail(EDGPU_BAD_ARGUMENT, "ctx is NULL");
    DEVICE_ENTER(x);
    int khz = 0;                                      // the s_memrealtime clock
    HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, x->device));
    if (khz <= 0) khz = 100000;
    HIP_CHECK(launch_stall((uint64_t)us * (uint64_t)khz / 1000ull, x->stream));
    return EDGPU_OK;
}

int edgpu_device_free(edgpu_ctx* x, void* p) {
    if (!x) return fail(EDGPU_BAD_ARGUMENT, "ctx is NULL");
    if (!p) return EDGPU_OK;
    DEVICE_ENTER(x);
    HIP_CHECK(wsync(x, x->stream));
    HIP_CHECK(hipFree(p));
    return EDGPU_OK;
}

int edgpu_memcpy_peer(edgpu_ctx* x, void* dst, int src_device, const void* src, uint64_t bytes) {
    if (!x || (bytes && (!dst || !src))) return fail(EDGPU_BAD_ARGUMENT, "NULL argument");
    if (!bytes) return EDGPU_OK;
    DEVICE_ENTER(x);
    if (src_device == x->device)
        HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, x->stream));
    else
        HIP_CHECK(hipMemcpyPeerAsync(dst, x->device, src, src_device, bytes, x->stream));
    return EDGPU_OK;
}

}  // extern "C"
