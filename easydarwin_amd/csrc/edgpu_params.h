// edgpu_params.h -- kernel argument blocks (shared by edgpu_kernels.hip and edgpu_engine.cpp).
#pragma once
#include <stdint.h>
#include "edgpu.h"
#include "edgpu_device.h"

// Measurement builds (-DEDGPU_AB_VARIANTS: `make -C easydarwin_amd/csrc ab` ->
// easydarwin_amd/ab/libedgpu_ab.so, loaded with EDGPU_LIB) carry every fan-out variant ever
// measured, the EDGPU_ABLATE skip-work bits and the alternative ingest copy paths
// (EDGPU_INGEST, EDGPU_INGEST_TCP).  The shipped libedgpu.so has the two default fan-out
// kernels and no skip-work branch: these knobs are compile-time constants there.
#ifdef EDGPU_AB_VARIANTS
#define EDGPU_ABL(P) ((P).ablate)
#define EDGPU_COPY_MODE(P) ((P).copy_mode)
#define EDGPU_TCP_COPY(P) ((P).tcp_copy)
#else
#define EDGPU_ABL(P) 0u
#define EDGPU_COPY_MODE(P) 0u
#define EDGPU_TCP_COPY(P) 3u
#endif

namespace edgpu {

// Kernel launches made on this thread (edgpu_counters.kernel_launches: the engine adds what each
// API call launched).  Every launch goes through EDGPU_LAUNCH.
extern thread_local uint64_t tl_launches;
#define EDGPU_LAUNCH(...)                          \
    do {                                           \
        ++::edgpu::tl_launches;                    \
        hipLaunchKernelGGL(__VA_ARGS__);           \
    } while (0)

// Interleaved frames a k_ingest wave copies per round (all their loads before the first
// store): 4 since the copy is specialised on the frame's word offset (128 VGPRs, 4 waves per
// SIMD); it was 2 (tools/build_ingest_ab.sh builds others)
#ifndef EDGPU_TCP_TD
#define EDGPU_TCP_TD 4
#endif
constexpr uint32_t kTcpFramesPerRound = EDGPU_TCP_TD;

struct TcpGroup;
struct TcpChunkRes;
struct TcpRead;

struct IngestParams {
    const edgpu_pkt_desc* desc;
    const uint32_t* seg_off;
    const uint32_t* seg_sess;
    const uint8_t* blob;
    const uint64_t* src_addr;   // per desc: device address of the frame ('$' header first, any
                                // alignment) instead of blob + slot * 16 (interleaved ingest); or null
    SessionDev* sessions;
    SenderDev* senders;
    StreamDev* streams;
    CopyJob* jobs;          // per desc: slot copy for k_ingest_copy
    uint32_t npk;           // descriptors in the batch
    uint32_t spec_min;      // the speculative copy from this many packets per segment on (0: never)
    uint32_t copy_mode;     // 0: copy inside k_ingest, 1: k_ingest_copy (EDGPU_INGEST)
    uint32_t tcp_copy;      // frames in the TCP byte stream: 1 one aligned load per word + the
                            // neighbour word by DPP, 2 the same with two frames per wave round
                            // (default); 0 two aligned loads per word (EDGPU_INGEST_TCP)
    uint32_t ablate;        // timing experiments only (EDGPU_ABLATE bits 4-7: 16 no totals, 32 no slot
                            // copy, 64 no per-sender scans)
    uint32_t host_epoch;    // != 0: the blob is a host batch the host keeps for the tick; record each
                            // packet's slot and the batch (edgpu_fanout_sources)
    TickTotals* totals;
    uint32_t ing_slot;      // this batch's ingest counters: TickTotals.ing_pk / ing_b [ing_slot]
    // reflector_use_in_packet_receive_time / reflector_in_packet_max_receive_sec
    // (ReflectorStream.cpp:103-107, 113): strip a 12-byte "aktt" BE64 receive-time trailer and
    // rebase the packet's arrival on it (:1960-1994)
    uint32_t recv_time;
    int64_t max_future_ms;  // sMaxFuturePacketMSec
    // Interleaved ingest (null otherwise): segment g is deframe group g, and k_ingest finds each
    // frame itself -- its chunk from the per-chunk results, its start from the walk's recorded
    // starts, its length and channel from its own '$' header, its arrival from the reads --
    // instead of reading a per-frame descriptor.  Frames of chunks the walk did not record
    // (cand kTcpNone, or more than kTcpFrames frames) come from desc / src_addr (k_tcp_finish).
    const TcpGroup* tcp_groups;
    const TcpChunkRes* tcp_chunkres;
    const uint16_t* tcp_offs;
    const TcpRead* tcp_reads;
    const uint8_t* tcp_raw;
    const uint8_t* tcp_stage;
};

struct PlanParams {
    SenderDev* senders;
    SubDev* subs;
    const uint32_t* sub_index;
    const uint32_t* sub_pos;    // SubDev index -> position in sub_index order (~0: inactive)
    const uint32_t* sub_range;  // per sender [begin, end) into sub_index
    edgpu_substream_out* sub_out;
    FanWork* work;
    FanSub* fansub;             // per sub_index position
    uint64_t* blk_bytes;        // per K2 block partials
    uint32_t* blk_count;
    uint64_t* blk_maxb;         // per K2 block: the largest sub-stream (bytes, descriptors)
    uint32_t* blk_maxc;
    SessionDev* sessions;       // stream errors (per-session isolation)
    TickTotals* totals;
    GrowReq* grow;              // ring growth requests (kMaxGrow)
    TickParams T;
};

struct FanoutParams {
    const SenderDev* senders;
    const uint32_t* sub_range;  // per sender [begin, end) into sub_index
    const SubDev* subs;
    const uint32_t* sub_index;
    const FanWork* work;
    const FanSub* fansub;
    uint8_t* arena;
    edgpu_out_desc* desc;
    uint64_t arena_words;       // capacities: stores outside them are dropped and flagged
    uint32_t max_desc;
    TickTotals* totals;
    uint32_t ablate;            // timing-only builds: bit0 skip descriptors, bit1 skip arena stores
};

// ---- RTSP-interleaved ingest ('$'-deframe of pusher TCP reads, edgpu_ingest_interleaved) ----
// A session's stream in one call = its carried bytes (a partial frame from the previous call)
// followed by its reads.  The stream is cut into kTcpChunk-byte chunks walked in parallel from
// every '$' that can start a frame in the chunk's first kTcpMaxFrame bytes; the true walk is
// then stitched chunk to chunk (k_tcp_resolve).
#ifndef EDGPU_TCP_CHUNK
#define EDGPU_TCP_CHUNK 32768                // 32 KiB: ingest incl. deframe 0.405 vs 0.421 ms at 16 KiB,
                                             // 0.479 at 8 KiB (profiles/r02z28_tcp_chunk_ab/)
#endif
constexpr uint32_t kTcpChunk = EDGPU_TCP_CHUNK;   // stream bytes per walk chunk
#ifndef EDGPU_TCP_SPEC
#define EDGPU_TCP_SPEC 0                     // frame headers guessed per burst of the walk (0: none);
                                             // 4 / 8 / 16 measured slower (profiles/r02z30_tcp_spec_ab/,
                                             // r02z33_tcp_walk_spec_ab/)
#endif
constexpr uint32_t kTcpSpec = EDGPU_TCP_SPEC;
#ifndef EDGPU_TCP_CAND_FUSED
#define EDGPU_TCP_CAND_FUSED 0               // 1: a chunk's two candidate windows loaded at once (A/B)
#endif
#ifndef EDGPU_TCP_WALK_CPW
#define EDGPU_TCP_WALK_CPW 2                 // chunks walked side by side per wave (1, 2 or 4): walk
                                             // ~100 -> 60 us (profiles/r02z32_tcp_walk_ab/); four
                                             // (16 / 24 / 32 KiB chunks) slower: 0.289 / 0.285 /
                                             // 0.289 vs 0.281 ms (profiles/r03t_walk_shape_ab/)
#endif
constexpr int kTcpWalkCpw = EDGPU_TCP_WALK_CPW;
#ifndef EDGPU_TCP_WALK_WPE
#define EDGPU_TCP_WALK_WPE 8                 // waves per SIMD asked of k_tcp_walk's registers (63 VGPRs, no spill)
#endif
static_assert(kTcpChunk >= 4096 && kTcpChunk + 2 * 2051 <= 65536, "chunk offsets are 16-bit");
constexpr uint32_t kTcpCands = 64;         // candidates kept per chunk (more: sequential walk)
constexpr uint32_t kTcpFrames = 32;        // frame starts recorded per candidate walk
constexpr uint32_t kTcpMaxFrame = 2047;    // usable request-buffer bytes (QTSS_MAX_REQUEST_BUFFER_SIZE - 1)
constexpr uint32_t kTcpCarry = 2048;       // per-session carry buffer / staged frame
constexpr uint32_t kTcpNone = 0xFFFFFFFFu;

// walk outcome codes (TcpCand.code, TcpGroup.code)
constexpr uint32_t kWalkRun = 0;           // reached the chunk end / the stream end
constexpr uint32_t kWalkPartial = 1;       // incomplete frame at `exit`: carried
constexpr uint32_t kWalkMessage = 2;       // non-'$' byte at a frame boundary: an RTSP message
constexpr uint32_t kWalkDropped = 3;       // frame longer than the request buffer: connection dropped

struct TcpGroup {           // one pusher connection's reads in this call
    uint32_t session, first_read, nreads, first_chunk;
    uint32_t nchunks, carry_len;
    uint64_t raw_off;       // raw-buffer offset of the first read
    uint64_t len;           // stream bytes: carry_len + the reads' bytes
    // k_tcp_resolve
    uint32_t nframes, code;
    uint64_t stop;          // stream position where the walk ended (len: everything framed)
    // k_tcp_scan
    uint32_t frame_base, _pad;
};

struct TcpRead { uint64_t start; int64_t arrival; uint32_t len, _pad; };   // start: stream position
struct TcpCand { uint32_t q, exit, nframes, code; };                        // q / exit: chunk offsets
struct TcpChunkRes { uint32_t entry, fbase, nframes, cand; };   // entry kTcpNone: idle; cand kTcpNone: re-walk
struct TcpTotals { uint32_t frames; int32_t status; };

struct TcpParams {
    TcpGroup* groups;
    uint32_t ngroups, nchunks;
    const TcpRead* reads;
    const uint32_t* chunk_group;
    TcpCand* cands;         // nchunks x kTcpCands
    uint16_t* offs;         // nchunks x kTcpCands x kTcpFrames: frame starts of each candidate walk
    uint8_t* links;         // nchunks x kTcpCands: next chunk's candidate, 0xFE terminal, 0xFF search
    uint32_t* ncand;
    TcpChunkRes* chunkres;
    const uint8_t* raw;
    uint64_t raw_bytes;
    uint8_t* carry;         // per session kTcpCarry bytes
    uint8_t* stage;         // per group kTcpCarry bytes: a frame that starts in the carried bytes
    edgpu_pkt_desc* desc;
    uint64_t* src_addr;     // per frame: its address for k_ingest (IngestParams.src_addr)
    uint32_t max_desc;
    uint32_t* seg_off;      // ngroups + 1
    uint32_t* seg_sess;
    edgpu_tcp_result* results;
    TcpTotals* tot;
    uint32_t walk;          // 0: k_tcp_walk + k_tcp_resolve (candidate windows, every chunk at once);
                            // 1: k_tcp_chain (each stream walked in order, one lane per session);
                            // 2: k_tcp_walk_seg + k_tcp_resolve (candidate windows every `seg` chunks)
    uint32_t seg;           // walk 2: chunks per segment
};

struct BlockedParams {
    const edgpu_blocked* reports;
    uint32_t n;
    SubDev* subs;
    const SenderDev* senders;
    SessionDev* sessions;
    int64_t now;                // the tick's clock
    int64_t relocate_ms;        // sRelocatePacketAgeMSec (rtp_reflector_threshold_msec)
    TickTotals* totals;
};

struct ImageParams {
    SenderDev* senders;
    SessionDev* sessions;
    StreamDev* streams;
    ImgPlan* plan;
    uint32_t nplan;
    int64_t now;
    int64_t over_buffer_ms;
    uint8_t* buf;           // export: destination images; import: source images
    int* status;            // first error wins
};

}  // namespace edgpu
