// edgpu_kernels.hip -- CDNA4 (gfx950) kernels of the relay engine.
//
//   k_ingest        ReflectorStream::PushPacket + ReflectorSocket::ProcessPacket
//                   (ReflectorStream.cpp:529-576, 1769-2010): clamp (Q11), UDP-RTCP SR gate
//                   (Q14), SSRC latch filter (Q13, ReflectorStream.cpp:1732-1767), per-stream
//                   packet ids, enqueue into the sender's HBM rings, key-frame candidate parse
//                   (IsKeyFrameFirstPacket, ReflectorStream.cpp:1403-1513), and the key
//                   pointer update + session-wide audio anchor (ReflectorStream.cpp:1876-1934:
//                   wave 0 of the workgroup, 64 packets per step, ballot + last-set-bit instead
//                   of the reference's per-packet branch chain; it was a kernel of its own,
//                   k_keyframe, until round 6).
//                   One 256-thread workgroup per session segment, one packet per lane.
//   k_plan_*        ReflectPackets' per-tick decisions (ReflectorStream.cpp:1024-1136):
//                   new-output start (key pointer, else GetClientBufferStartPacketOffset),
//                   per-sub-stream range, bookmark and last-id commit, output offsets.
//   k_fanout        SendPacketsToOutput -> WritePacket -> RTPStream::Write framing for every
//                   (sub-stream, packet): each workgroup owns 32 consecutive packets of one
//                   sender, loads their slots from HBM once into registers and writes them
//                   to every sub-stream of that sender (16-B stores), patching the
//                   interleaved channel byte for TCP subscribers, plus one 16-B descriptor
//                   per output packet.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "edgpu.h"
#include "edgpu_device.h"
#include "edgpu_params.h"
#include "edgpu_bytes.h"

namespace edgpu {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// k_ingest's slot-copy policy: bit 0 the copy's source loads non-temporal, bit 1 its ring stores
// (so the copy's stream is the XCD L2's first victim and each packet's first line, read by the
// header phase with the default policy, can still be there when the copy reads it again).
#ifndef EDGPU_INGEST_NT
#define EDGPU_INGEST_NT 0
#endif
__device__ __forceinline__ u32x4 ing_ld(const u32x4* p) {
    if constexpr ((EDGPU_INGEST_NT & 1) != 0) return __builtin_nontemporal_load(p);
    else return *p;
}
__device__ __forceinline__ void ing_st(u32x4* p, u32x4 v) {
    if constexpr ((EDGPU_INGEST_NT & 2) != 0) __builtin_nontemporal_store(v, p);
    else *p = v;
}

__device__ __forceinline__ uint32_t be16(const uint8_t* p) { return (uint32_t)p[0] << 8 | p[1]; }
__device__ __forceinline__ uint32_t be32(const uint8_t* p) {
    return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

// RTSP-interleaved header dword stored at the start of every slot: '$', channel 0, BE16(len)
// (RTSPSessionInterface.cpp:329-336), as a little-endian u32.
__device__ __forceinline__ uint32_t slot_header(uint32_t len) {
    return 0x24u | ((len >> 8) & 0xFF) << 16 | (len & 0xFF) << 24;
}

// H.264 "first packet of a key frame" rule (Q4): length >= 20, header size 12 + 4*CC
// (the X bit and padding are ignored), aggregation units peek at their first NAL, FU-A/B
// only on the start fragment; key iff NAL type 5, 7 or 8.  Bytes at or past `len` read 0.
__device__ bool key_frame_first_packet(const uint8_t* p, uint32_t len) {
    if (len < 20) return false;
    const uint32_t h = 12 + 4u * (p[0] & 0x0F);
    auto at = [&](uint32_t i) -> uint32_t { return i < len ? p[i] : 0u; };
    uint32_t t = at(h) & 0x1F;
    if (t == 24) { if (len > h + 3) t = at(h + 3) & 0x1F; }
    else if (t == 25) { if (len > h + 5) t = at(h + 5) & 0x1F; }
    else if (t == 26) { if (len > h + 8) t = at(h + 8) & 0x1F; }
    else if (t == 27) { if (len > h + 9) t = at(h + 9) & 0x1F; }
    else if (t == 28 || t == 29) { if (len > h + 1 && (at(h + 1) & 0x80)) t = at(h + 1) & 0x1F; }
    return t == 5 || t == 7 || t == 8;
}

__device__ __forceinline__ void set_status(int* st, int code) { atomicCAS(st, 0, code); }

// Header bytes held in registers: hdr[k] holds packet bytes 4k..4k+3 (little-endian).
__device__ __forceinline__ uint32_t hbyte(const uint32_t* h, int i) { return (h[i >> 2] >> (8 * (i & 3))) & 0xFF; }
__device__ __forceinline__ uint32_t hbe16(const uint32_t* h, int i) { return hbyte(h, i) << 8 | hbyte(h, i + 1); }
__device__ __forceinline__ uint32_t hbe32(const uint32_t* h, int i) { return __builtin_bswap32(h[i >> 2]); }

// key_frame_first_packet for the CSRC-free header (h = 12): every byte the rule can read
// (12..21) is already in registers; reads past `len` are excluded by its own length guards
// (len >= 20 here).
__device__ __forceinline__ bool key_frame_first_packet_cc0(const uint32_t* h, uint32_t len) {
    uint32_t t = hbyte(h, 12) & 0x1F;
    if (t == 24) { if (len > 15) t = hbyte(h, 15) & 0x1F; }
    else if (t == 25) { if (len > 17) t = hbyte(h, 17) & 0x1F; }
    else if (t == 26) { if (len > 20) t = hbyte(h, 20) & 0x1F; }
    else if (t == 27) { if (len > 21) t = hbyte(h, 21) & 0x1F; }
    else if (t == 28 || t == 29) { if (len > 13 && (hbyte(h, 13) & 0x80)) t = hbyte(h, 13) & 0x1F; }
    return t == 5 || t == 7 || t == 8;
}

// ReflectorPacket::GetSSRC (ReflectorStream.h:145-158)
__device__ __forceinline__ uint32_t packet_ssrc(const uint8_t* p, uint32_t len, bool rtcp) {
    if (len < 8) return 0;
    if (rtcp) return be32(p + 4);
    if (len < 12) return 0;
    return be32(p + 8);
}

// Inclusive scan of a 64-bit value across the wave, in registers: DPP row shifts (1, 2, 4, 8)
// give each row of 16 lanes its own prefix, then every lane adds the totals of the rows before its
// own (lanes 15, 31, 47, read as scalars).  Call with every lane active.
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, CTRL, 0xF, 0xF, true);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), CTRL, 0xF, 0xF, true);
    return (uint64_t)hi << 32 | lo;
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t x, int l) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l) << 32 |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
}
__device__ __forceinline__ uint64_t wave_inclusive_scan_u64(uint64_t x) {
    x += dpp_u64<0x111>(x);                 // row_shr:1 (a row's first lanes read 0)
    x += dpp_u64<0x112>(x);                 // row_shr:2
    x += dpp_u64<0x114>(x);                 // row_shr:4
    x += dpp_u64<0x118>(x);                 // row_shr:8
    const uint64_t r0 = readlane_u64(x, 15), r1 = readlane_u64(x, 31), r2 = readlane_u64(x, 47);
    const int row = (threadIdx.x & 63) >> 4;
    return x + (row >= 1 ? r0 : 0ull) + (row >= 2 ? r1 : 0ull) + (row >= 3 ? r2 : 0ull);
}

// Exclusive scan over a workgroup of NW waves of 64 (256 threads by default).  `scratch` holds
// NW entries.
template <typename T, int NW = 4>
__device__ __forceinline__ T block_exclusive_scan(T v, T* scratch, T& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    T x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        T y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) scratch[wid] = x;
    __syncthreads();
    T base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
        T t = scratch[w];
        if (w < wid) base += t;
        tot += t;
    }
    __syncthreads();
    total = tot;
    return base + x - v;
}

// Reduction over a workgroup of NW waves of 64 (every thread gets the result); `scratch` holds
// NW entries and may be reused right after.
struct OpSum { template <typename T> __device__ T operator()(T a, T b) const { return a + b; } };
struct OpMax { template <typename T> __device__ T operator()(T a, T b) const { return a > b ? a : b; } };
struct OpMin { template <typename T> __device__ T operator()(T a, T b) const { return a < b ? a : b; } };
template <typename T, typename Op, int NW = 4>
__device__ __forceinline__ T block_reduce(T v, T* scratch) {
    const Op op;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = op(v, (T)__shfl_xor(v, o, 64));
    if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = v;
    __syncthreads();
    T r = scratch[0];
#pragma unroll
    for (int w = 1; w < NW; w++) r = op(r, scratch[w]);
    __syncthreads();
    return r;
}

// =========================================================================================
// Ingest
// =========================================================================================

// Slot copy of RTSP-interleaved frames inside the TCP byte stream (k_ingest, copy_mode 0).  The
// frame's bytes [sp, lim) are misaligned by sh = sp & 15.  Each lane loads ONE aligned block
// (blocks holding a byte of the frame only); slot word w is blocks w and w + 1 funnelled by sh,
// and block w + 1 comes from the next lane by DPP (lane 63 takes the next round's lane 0 by
// readlane).  A wave takes TD frames per round (EDGPU_INGEST_TCP=1 / 2: one / two)
// and issues all their loads before its first store.  Four frames per round (162 VGPRs, 3 waves
// per SIMD) measured slower: ingest incl. deframe 0.563 vs 0.435 ms (profiles/r02z21_*).
template <uint32_t TD, int THREADS>
__device__ __forceinline__ void tcp_slot_copy(uint32_t n, const uint32_t* p_slotb, const uint64_t* p_src,
                                              const uint16_t* p_len, const uint8_t* p_snd, const uint64_t* p_vb,
                                              const uint64_t* s_ring, const uint32_t* s_wmask) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr uint32_t kW = THREADS / 64;
    auto lane0 = [](u32x4 v) {
        return u32x4{(uint32_t)__builtin_amdgcn_readlane((int)v.x, 0), (uint32_t)__builtin_amdgcn_readlane((int)v.y, 0),
                     (uint32_t)__builtin_amdgcn_readlane((int)v.z, 0), (uint32_t)__builtin_amdgcn_readlane((int)v.w, 0)};
    };
    for (uint32_t p = wid; p < n; p += TD * kW) {
        u32x4 b[TD][4];
        uint32_t sb[TD], fl[TD], sh[TD];
#pragma unroll
        for (uint32_t d = 0; d < TD; d++) {
            const uint32_t pd = p + d * kW;
            sb[d] = pd < n ? p_slotb[pd] : 0u;
            const uint8_t* sp = reinterpret_cast<const uint8_t*>(sb[d] ? p_src[pd] : 0ull);
            fl[d] = sb[d] ? 4u + p_len[pd] : 0u;                          // frame bytes
            const uintptr_t a0 = (uintptr_t)sp & ~(uintptr_t)15;
            sh[d] = (uint32_t)((uintptr_t)sp & 15);
            const uint32_t nblk = sb[d] ? (uint32_t)(((uintptr_t)sp + fl[d] - 1 - a0) >> 4) + 1 : 0u;
            const u32x4* ab = reinterpret_cast<const u32x4*>(a0);
            const u32x4 z = u32x4{0u, 0u, 0u, 0u};
            b[d][0] = (uint32_t)lane < nblk ? ab[lane] : z;
            b[d][1] = (uint32_t)lane + 64 < nblk ? ab[lane + 64] : z;
            b[d][2] = (uint32_t)lane + 128 < nblk ? ab[lane + 128] : z;
            b[d][3] = lane == 0 && 192u < nblk ? ab[192] : z;           // lane 63 of round 2's neighbour
        }
#pragma unroll
        for (uint32_t d = 0; d < TD; d++) {
            if (sb[d] == 0) continue;                                    // uniform
            const uint32_t pd = p + d * kW;
            const uint32_t s = p_snd[pd];
            u32x4* ring = reinterpret_cast<u32x4*>(s_ring[s]);
            const uint64_t w0 = p_vb[pd] >> 4;
            const uint32_t wm = s_wmask[s];
            const uint32_t nw = sb[d] / 16;
            u32x4 v0 = funnel16(b[d][0], wave_next(b[d][0], lane0(b[d][1])), sh[d]);
            const u32x4 v1 = funnel16(b[d][1], wave_next(b[d][1], lane0(b[d][2])), sh[d]);
            const u32x4 v2 = funnel16(b[d][2], wave_next(b[d][2], lane0(b[d][3])), sh[d]);
            const int rem = (int)fl[d] - 16 * lane;                         // frame bytes from word `lane`
            if (lane == 0) v0.x = slot_header(p_len[pd]);
            if ((uint32_t)lane < nw) ring[(w0 + lane) & wm] = keep16(v0, rem);
            if ((uint32_t)lane + 64 < nw) ring[(w0 + lane + 64) & wm] = keep16(v1, rem - 1024);
            if ((uint32_t)lane + 128 < nw) ring[(w0 + lane + 128) & wm] = keep16(v2, rem - 2048);
        }
    }
}

// Lane l's 16 frame bytes at offset 4Q + r of (its aligned block `a`, lane l + 1's block);
// lane 63 takes the next round's first block `last`.  The word offset Q is a template argument
// (the caller branches on it once per frame: it is wave-uniform), so only the Q + 1 dwords that
// cross into the next lane move by DPP (wave_shl:1) and each output dword is one alignbyte --
// no per-dword select among the four word offsets.
template <uint32_t Q>
__device__ __forceinline__ u32x4 funnel_next(u32x4 a, u32x4 last, uint32_t r) {
    const uint32_t aa[4] = {a.x, a.y, a.z, a.w}, la[4] = {last.x, last.y, last.z, last.w};
    uint32_t d[8] = {a.x, a.y, a.z, a.w, 0u, 0u, 0u, 0u};
#pragma unroll
    for (uint32_t k = 0; k <= Q; k++)
        d[4 + k] = (uint32_t)__builtin_amdgcn_update_dpp((int)la[k], (int)aa[k], 0x130, 0xF, 0xF, false);
    return u32x4{__builtin_amdgcn_alignbyte(d[Q + 1], d[Q], r), __builtin_amdgcn_alignbyte(d[Q + 2], d[Q + 1], r),
                 __builtin_amdgcn_alignbyte(d[Q + 3], d[Q + 2], r), __builtin_amdgcn_alignbyte(d[Q + 4], d[Q + 3], r)};
}

// One frame's slot words out of its aligned blocks b[k] (block lane + 64k; b3 = block 192):
// rounds past the slot are skipped (uniform), and only the round holding the frame's end clears
// the bytes past it.  Slot word w goes to ring word (w0 + w) & wm.
template <uint32_t Q>
__device__ __forceinline__ void tcp_frame_store(const u32x4 (&b)[3], u32x4 b3, uint32_t r, uint32_t fl, uint32_t nw,
                                                u32x4* ring, uint64_t w0, uint32_t wm, int lane) {
    auto lane0 = [](u32x4 v) {
        return u32x4{(uint32_t)__builtin_amdgcn_readlane((int)v.x, 0), (uint32_t)__builtin_amdgcn_readlane((int)v.y, 0),
                     (uint32_t)__builtin_amdgcn_readlane((int)v.z, 0), (uint32_t)__builtin_amdgcn_readlane((int)v.w, 0)};
    };
    const uint32_t lastk = (nw - 1) >> 6;                      // the round holding the slot's end
    const uint32_t base = (uint32_t)w0 + (uint32_t)lane;      // wm < 2^32: low words suffice
    const int rem = (int)fl - 16 * lane;                        // frame bytes from word `lane`
    u32x4 v0 = funnel_next<Q>(b[0], lane0(b[1]), r);
    if (lane == 0) v0.x = slot_header(fl - 4u);
    if (lastk == 0) v0 = keep16(v0, rem);
    if ((uint32_t)lane < nw) ing_st(ring + (base & wm), v0);
    if (lastk >= 1) {
        u32x4 v1 = funnel_next<Q>(b[1], lane0(b[2]), r);
        if (lastk == 1) v1 = keep16(v1, rem - 1024);
        if ((uint32_t)lane + 64 < nw) ing_st(ring + ((base + 64) & wm), v1);
    }
    if (lastk >= 2) {
        const u32x4 v2 = keep16(funnel_next<Q>(b[2], b3, r), rem - 2048);
        if ((uint32_t)lane + 128 < nw) ing_st(ring + ((base + 128) & wm), v2);
    }
}

// tcp_slot_copy with the per-frame state in SGPRs: a frame's slot size, length and source
// address are uniform across the wave (readfirstlane), and the one block past lane 63's second
// round (block 192, needed by lane 63 of round 2 only) is a scalar load.  Fewer VGPRs per frame
// in flight (12 instead of 16 + 3), so more frames per round fit the occupancy.  The stores go
// through tcp_frame_store, specialised on the frame's word offset.
// (EDGPU_INGEST_TCP=3: two frames per round, 4: four.)
template <uint32_t TD, int THREADS>
__device__ __forceinline__ void tcp_slot_copy_s(uint32_t n, const uint32_t* p_slotb, const uint64_t* p_src,
                                                const uint16_t* p_len, const uint8_t* p_snd, const uint64_t* p_vb,
                                                const uint64_t* s_ring, const uint32_t* s_wmask) {
    typedef __attribute__((address_space(4))) const u32x4 cu32x4;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr uint32_t kW = THREADS / 64;
    auto uni64 = [](uint64_t x) {
        return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x) |
               (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32)) << 32;
    };
    for (uint32_t p = wid; p < n; p += TD * kW) {
        u32x4 b[TD][3], b3[TD];
        uint32_t sb[TD], fl[TD], sh[TD];
#pragma unroll
        for (uint32_t d = 0; d < TD; d++) {
            const uint32_t pd = p + d * kW;                              // uniform
            sb[d] = pd < n ? (uint32_t)__builtin_amdgcn_readfirstlane((int)p_slotb[pd]) : 0u;
            const uint64_t sp = sb[d] ? uni64(p_src[pd]) : 0ull;
            fl[d] = sb[d] ? 4u + (uint32_t)__builtin_amdgcn_readfirstlane((int)p_len[pd]) : 0u;
            const uint64_t a0 = sp & ~15ull;
            sh[d] = (uint32_t)(sp & 15);
            const uint32_t nblk = sb[d] ? (uint32_t)((sp + fl[d] - 1 - a0) >> 4) + 1 : 0u;
            const u32x4* ab = reinterpret_cast<const u32x4*>(a0);
            const u32x4 z = u32x4{0u, 0u, 0u, 0u};
            b[d][0] = (uint32_t)lane < nblk ? ing_ld(ab + lane) : z;
            b[d][1] = (uint32_t)lane + 64 < nblk ? ing_ld(ab + lane + 64) : z;
            b[d][2] = (uint32_t)lane + 128 < nblk ? ing_ld(ab + lane + 128) : z;
            b3[d] = 192u < nblk ? *(cu32x4*)(ab + 192) : z;              // scalar
        }
#pragma unroll
        for (uint32_t d = 0; d < TD; d++) {
            if (sb[d] == 0) continue;                                    // uniform
            const uint32_t pd = p + d * kW;
            const uint32_t s = p_snd[pd];
            u32x4* ring = reinterpret_cast<u32x4*>(s_ring[s]);
            const uint64_t w0 = p_vb[pd] >> 4;
            const uint32_t wm = s_wmask[s];
            const uint32_t nw = sb[d] / 16, r = sh[d] & 3;
            switch (sh[d] >> 2) {                                        // uniform: one scalar branch
            case 0: tcp_frame_store<0>(b[d], b3[d], r, fl[d], nw, ring, w0, wm, lane); break;
            case 1: tcp_frame_store<1>(b[d], b3[d], r, fl[d], nw, ring, w0, wm, lane); break;
            case 2: tcp_frame_store<2>(b[d], b3[d], r, fl[d], nw, ring, w0, wm, lane); break;
            default: tcp_frame_store<3>(b[d], b3[d], r, fl[d], nw, ring, w0, wm, lane); break;
            }
        }
    }
}

// DEPTH: packets per wave per slot-copy round; 4 by default (125 VGPRs, still 4 waves/SIMD),
// EDGPU_INGEST_DEPTH=2 for A/B runs
// THREADS: workgroup size, one packet per lane per round (256 by default; EDGPU_INGEST_THREADS=512
// for A/B: one round for a C2 session's ~375 packets per tick)

// SPEC (descriptor batches in the blob): the slot copy runs FIRST, at each packet's speculative
// ring place -- every packet that passes the track / length test is taken to be enqueued with its
// full length -- and the header words the reflector reads (packet bytes 0..27) are taken from the
// copy's own registers, so each packet's first line is fetched once and one dependent load per
// round is gone.  What the header then decides changes no byte offset: a packet the RTCP-port or
// SSRC test refuses keeps its bytes as a hole in the ring (nothing points into it), a stripped
// receive-time trailer stays as slack at its slot's end and its slot header is rewritten.  Ranks and
// non-empty counts are scanned again only in a round where a decision differed from the guess.
template <uint32_t DEPTH, int THREADS = kIngestThreads, bool SPEC = false>
// waves_per_eu(4): the kernel needs 4 waves per SIMD (4 resident 256-thread sessions per CU), and
// the interleaved copy's four frames in flight fit 128 VGPRs that way
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(4))) void k_ingest(IngestParams P) {
    constexpr int NW = THREADS / 64;
    const uint32_t seg = blockIdx.x;
    const int tid = threadIdx.x;
    const uint32_t b = P.seg_off[seg], e = P.seg_off[seg + 1];
    const SessionDev S = P.sessions[P.seg_sess[seg]];
    const uint32_t nsnd = 2 * S.ntracks;
    // a copy pass the last tick still owes (edgpu_fanout_next): read now, checked at the end
    const bool pass_owed = P.totals->pass_next[P.totals->pass_slot & 1u] != kNoPass;

    __shared__ uint64_t s_head[kMaxSendersPerSession], s_vbyte[kMaxSendersPerSession];
    __shared__ uint32_t s_vcount[kMaxSendersPerSession], s_valid[kMaxSendersPerSession];
    __shared__ int64_t s_lastv[kMaxSendersPerSession], s_lastnz[kMaxSendersPerSession];
    __shared__ uint32_t s_flags[kMaxSendersPerSession], s_pkmask[kMaxSendersPerSession], s_wmask[kMaxSendersPerSession];
    __shared__ uint64_t s_meta[kMaxSendersPerSession], s_ring[kMaxSendersPerSession];
    __shared__ uint64_t s_vclob[kMaxSendersPerSession];     // SPEC: the ring's write high-water mark
    __shared__ uint64_t s_count[kMaxTracks];
    __shared__ uint64_t c_tot[kMaxSendersPerSession];
    __shared__ uint64_t s_wsum[kMaxSendersPerSession][NW];    // per sender, each wave's total
    __shared__ int c_last[kMaxSendersPerSession];   // (tid << 10 | rank) of the chunk's newest non-empty packet
    __shared__ int c_lastacc[kMaxSendersPerSession];  // lane of the chunk's newest accepted packet, per socket
    // per packet of the current chunk
    __shared__ uint8_t p_snd[THREADS];
    __shared__ uint8_t p_acc[THREADS];
    __shared__ uint16_t p_len[THREADS];
    __shared__ uint32_t p_ssrc[THREADS];
    __shared__ int64_t p_ts[THREADS];
    __shared__ uint64_t p_src[THREADS];     // slot / frame start address
    __shared__ uint32_t p_slotb[THREADS];
    __shared__ uint64_t p_vb[THREADS];
    __shared__ int64_t p_arr[THREADS];      // receive-time trailer: the packet's arrival
    __shared__ u32x4 p_hdr[SPEC ? THREADS : 1][2];   // SPEC: slot words 0 and 1, from the copy
    __shared__ uint64_t scan64[NW];
    // ReflectorSocket receive-time state per socket (reflector_use_in_packet_receive_time)
    __shared__ uint32_t s_rth[kMaxSendersPerSession], s_rts[kMaxSendersPerSession];
    __shared__ int64_t s_rta[kMaxSendersPerSession];
    __shared__ uint64_t s_rtr[kMaxSendersPerSession];
    __shared__ uint32_t s_rtn;
    // the keyframe index (ReflectorSocket::ProcessPacket's key and audio-anchor steps,
    // ReflectorStream.cpp:1876-1934), folded in: each sender's key pointer; per chunk each wave's
    // last key / audio event (bit0 any, bit1 it was a key) and, per sender, the newest packet that
    // sets its key pointer as (lane + 1) << 52 | queue index (0: none)
    __shared__ int64_t s_key[kMaxSendersPerSession];
    __shared__ uint32_t s_wev[NW];
    __shared__ unsigned long long s_klast[kMaxSendersPerSession];
    // interleaved ingest: the session's chunk table (frame end of each chunk, the recorded
    // candidate or kTcpNone) and its reads, for every lane's frame lookup
    constexpr uint32_t kLdsChunks = 256, kLdsReads = 64;
    __shared__ uint32_t t_cend[kLdsChunks], t_crec[kLdsChunks];
    __shared__ uint64_t t_rstart[kLdsReads];
    __shared__ int64_t t_rarr[kLdsReads];
    TcpGroup G{};
    if (P.tcp_groups) {
        G = P.tcp_groups[seg];
        for (uint32_t c = tid; c < min(G.nchunks, kLdsChunks); c += THREADS) {
            const TcpChunkRes R = P.tcp_chunkres[G.first_chunk + c];
            t_cend[c] = R.fbase + R.nframes;
            t_crec[c] = R.entry != kTcpNone && R.nframes <= kTcpFrames ? R.cand : kTcpNone;
        }
        if (tid < (int)min(G.nreads, kLdsReads)) {
            t_rstart[tid] = P.tcp_reads[G.first_read + tid].start;
            t_rarr[tid] = P.tcp_reads[G.first_read + tid].arrival;
        }
    }

    if (tid < (int)nsnd) {
        const SenderDev& D = P.senders[S.first_sender + tid];
        s_head[tid] = D.head; s_vbyte[tid] = D.vbyte_end; s_vcount[tid] = D.vcount_end;
        s_valid[tid] = D.valid_ssrc; s_lastv[tid] = D.last_valid_s; s_lastnz[tid] = D.last_nonzero;
        s_flags[tid] = D.flags; s_pkmask[tid] = D.pk_mask; s_wmask[tid] = D.word_mask;
        s_meta[tid] = D.meta; s_ring[tid] = D.ring;
        s_key[tid] = D.key;
        s_vclob[tid] = D.vclob;
        s_klast[tid] = 0ull;
        if (P.recv_time) { s_rth[tid] = D.rt_has; s_rts[tid] = D.rt_ssrc; s_rta[tid] = D.rt_first_arrival; s_rtr[tid] = D.rt_first_receive; }
    }
    if (tid == 0) s_rtn = 0;
    if (tid < (int)S.ntracks) s_count[tid] = P.streams[S.first_stream + tid].packet_count;
    if (tid < (int)nsnd) c_lastacc[tid] = -1;
#ifdef EDGPU_AB_VARIANTS
    if (tid == 0) atomicMin(&P.totals->ing_t0_min, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    // measurement builds: thread 0's time per phase (s_memrealtime, 100 MHz), summed over the
    // non-empty segments (EDGPU_FAN_TAIL prints the means): 1 session / sender state, 2 descriptor
    // + header + SSRC filter, 3 rank scans, 4 meta stores + keyframe ballots, 5 slot copy, 6 tail
    unsigned long long ph_t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long ph_last = __builtin_amdgcn_s_memrealtime();
#define EDGPU_ING_T(k)                                                                   \
    do {                                                                                 \
        if (tid == 0) {                                                                  \
            const unsigned long long ph_now = __builtin_amdgcn_s_memrealtime();          \
            ph_t[k] += ph_now - ph_last;                                                 \
            ph_last = ph_now;                                                            \
        }                                                                                \
    } while (0)
#else
#define EDGPU_ING_T(k) do {} while (0)
#endif
    __syncthreads();
    EDGPU_ING_T(1);

    uint32_t in_pk = 0, in_bytes = 0;          // (a segment: < 2^21 packets, < 2^32 bytes)
    // ReflectorSession::fHasVideoKeyFrameUpdate before the chunk (every thread keeps the same)
    bool kflag = S.video_key_flag != 0;
    constexpr unsigned long long kQiMask = (1ull << 52) - 1;
    for (uint32_t base = b; base < e; base += THREADS) {
        // the last chunk's newest key-pointer packets (its atomics are behind the last barrier)
        if (tid < (int)nsnd && s_klast[tid]) { s_key[tid] = (int64_t)(s_klast[tid] & kQiMask); s_klast[tid] = 0ull; }
        const uint32_t n = min((uint32_t)THREADS, e - base);
        const uint32_t i = base + tid;
        const bool valid = (uint32_t)tid < n;
        if (tid < (int)nsnd) c_last[tid] = -1;
        uint32_t len = 0, track = 0, ls = 0, fl = 0, slot = 0, remote_odd = 0;
        uint64_t src = 0;
        int64_t arrival = 0;
        bool acc = false;
        uint32_t hdr[7] = {0u, 0u, 0u, 0u, 0u, 0u, 0u};   // packet bytes 0..27, little-endian words
        bool direct = false;            // an interleaved frame found here
        if (valid && P.tcp_groups) {
            // the frame's chunk: the first whose frame end passes the frame's session index
            const uint32_t j = i - b;
            uint32_t lo = 0, hi = G.nchunks - 1;
            const bool lds = G.nchunks <= kLdsChunks;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                uint32_t ce;
                if (lds) ce = t_cend[mid];
                else { const TcpChunkRes R = P.tcp_chunkres[G.first_chunk + mid]; ce = R.fbase + R.nframes; }
                if (ce > j) hi = mid; else lo = mid + 1;
            }
            uint32_t rec, fbase;
            if (lds) { rec = t_crec[lo]; fbase = lo ? t_cend[lo - 1] : 0u; }
            else {
                const TcpChunkRes R = P.tcp_chunkres[G.first_chunk + lo];
                rec = R.entry != kTcpNone && R.nframes <= kTcpFrames ? R.cand : kTcpNone;
                fbase = R.fbase;
            }
            if (rec != kTcpNone) {
                direct = true;
                const uint64_t pos = (uint64_t)lo * kTcpChunk +
                                     P.tcp_offs[((size_t)(G.first_chunk + lo) * kTcpCands + rec) * kTcpFrames + (j - fbase)];
                const uint8_t* sp;
                uintptr_t end;                                 // the stream's (or the stage's) end
                if (pos >= G.carry_len) {
                    sp = P.tcp_raw + G.raw_off + (pos - G.carry_len);
                    end = (uintptr_t)(P.tcp_raw + G.raw_off + (G.len - G.carry_len));
                } else {                                        // starts in the carried bytes: staged
                    sp = P.tcp_stage + (uint64_t)seg * kTcpCarry;
                    end = (uintptr_t)(sp + kTcpCarry);
                }
                // the frame's first 48 aligned bytes at once: '$' ch BE16(len) and packet bytes 0..27
                const uintptr_t al = (uintptr_t)sp & ~(uintptr_t)15;
                const uint32_t sh = (uint32_t)((uintptr_t)sp & 15);
                const u32x4 z = u32x4{0u, 0u, 0u, 0u};
                const u32x4 k0 = *reinterpret_cast<const u32x4*>(al);
                const u32x4 k1 = al + 16 < end ? *reinterpret_cast<const u32x4*>(al + 16) : z;
                const u32x4 k2 = sh && al + 32 < end ? *reinterpret_cast<const u32x4*>(al + 32) : z;
                const u32x4 f0 = funnel16(k0, k1, sh);       // frame bytes 0..15
                const uint32_t flen = (f0.x >> 16 & 0xFFu) << 8 | f0.x >> 24;
                len = min(flen, (uint32_t)kMaxPacket);
                const uint32_t ch = f0.x >> 8 & 0xFFu;
                track = ch >> 1;
                ls = 2 * track + (ch & 1);
                // the reads: the frame belongs to the read holding its last byte
                const uint64_t last = pos + 4 + flen - 1;
                uint32_t rl = 0, rh = G.nreads - 1;
                while (rl < rh) {
                    const uint32_t mid = (rl + rh + 1) >> 1;
                    const uint64_t st = G.nreads <= kLdsReads ? t_rstart[mid] : P.tcp_reads[G.first_read + mid].start;
                    if (st <= last) rl = mid; else rh = mid - 1;
                }
                arrival = G.nreads <= kLdsReads ? t_rarr[rl] : P.tcp_reads[G.first_read + rl].arrival;
                slot = 0;
                acc = track < S.ntracks && len > 0;
                src = (uint64_t)(uintptr_t)sp;
                // as load16_unaligned(sp, lim) / (sp + 16, lim) with lim = sp + 4 + len: a block
                // past lim is not read (the word keeps the previous block's bytes)
                const uintptr_t lim = (uintptr_t)sp + 4 + len;
                const u32x4 w0 = sh && al + 16 < lim ? f0 : funnel16(k0, k0, sh);
                const u32x4 w1 = len > 12 ? funnel16(k1, sh && al + 32 < lim ? k2 : k1, sh) : z;
                hdr[0] = w0.y; hdr[1] = w0.z; hdr[2] = w0.w; hdr[3] = w1.x;
                hdr[4] = w1.y; hdr[5] = w1.z; hdr[6] = w1.w;
                if (acc) fl = s_flags[ls];
                if (acc && (fl & kSndRtcpPort))
                    acc = len >= 8 && len >= 4 * hbe16(hdr, 2) + 4 && (hbyte(hdr, 0) >> 6) == 2 && hbyte(hdr, 1) == 200;
                in_pk += 1;
                in_bytes += len;
            }
        }
        if (valid && !direct) {
            const edgpu_pkt_desc d = P.desc[i];
            len = min((uint32_t)d.len, (uint32_t)kMaxPacket);
            track = d.channel >> 1;
            ls = 2 * track + (d.channel & 1);
            arrival = d.arrival_ms;
            slot = d.slot;
            remote_odd = d.flags & EDGPU_PKT_REMOTE_ODD;
            acc = track < S.ntracks && len > 0;       // ProcessRTPData: inIndex < numStreams
            const uint8_t* sp = P.src_addr ? reinterpret_cast<const uint8_t*>(P.src_addr[i])
                                           : P.blob + (uint64_t)slot * 16;
            src = (uint64_t)(uintptr_t)sp;
            in_pk += 1;
            in_bytes += len;
        }
        // ---- SPEC: the speculative ranks / ring places, the slot copy, then the header words ----
        uint32_t my_rank = 0, my_nzpre = 0, my_trank = 0;
        uint64_t my_slotpre = 0;
        // every sender of the session in one pass: each wave scans (count | non-empty << 10 | slot
        // bytes << 20) per sender in registers (wave_inclusive_scan_u64), the wave totals meet in
        // LDS across one barrier.  A packet keeps the prefixes of its own sender and of its track's
        // other one (RTP / RTCP, ls ^ 1): its rank in the track (fStreamCountID order) is their sum.
        // (a packet refused after SPEC's guess, !a with sbytes > 0, still counts its hole's bytes)
        auto rank_scan = [&](bool a, bool z, uint32_t sbytes) {
            const int lane = tid & 63, wid = tid >> 6;
            const uint64_t mx = (a ? 1ull | (uint64_t)(z ? 1 : 0) << 10 : 0ull) | (uint64_t)sbytes << 20;
            const uint32_t ns = (EDGPU_ABL(P) & 64u) ? 0u : nsnd;
            uint64_t my_incl = 0, sib_incl = 0;
            for (uint32_t s = 0; s < ns; s++) {                      // uniform
                const uint64_t incl = wave_inclusive_scan_u64((a || sbytes) && ls == s ? mx : 0ull);
                if (lane == 63) s_wsum[s][wid] = incl;
                if (ls == s) my_incl = incl;
                if ((ls ^ 1u) == s) sib_incl = incl;
            }
            __syncthreads();
            EDGPU_ING_T(3);
            if (tid < (int)ns) {
                uint64_t t = 0;
                for (int w = 0; w < NW; w++) t += s_wsum[tid][w];
                c_tot[tid] = t;
            }
            if ((a || sbytes) && ns) {                               // (then ls < nsnd)
                uint64_t mb = 0, sb = 0;
                for (int w = 0; w < wid; w++) { mb += s_wsum[ls][w]; sb += s_wsum[ls ^ 1u][w]; }
                const uint64_t pre = mb + my_incl - mx;
                my_rank = pre & 1023; my_nzpre = (pre >> 10) & 1023; my_slotpre = pre >> 20;
                my_trank = my_rank + (uint32_t)((sb + sib_incl) & 1023);
            }
        };
        // the slot copy of the round's packets with p_slotb > 0 from p_src to ring place p_vb (as
        // copy_mode 0 below); with `capture`, lanes 0 and 1 leave slot words 0 and 1 for the header
        auto slot_copy = [&](bool capture) {
            constexpr uint32_t kDepth = DEPTH, kW = THREADS / 64;
            const uint32_t lane = tid & 63, wid = tid >> 6;
            for (uint32_t p = wid; p < n; p += kDepth * kW) {
                uint32_t nw[kDepth];
                u32x4 v[kDepth][3];
#pragma unroll
                for (uint32_t d = 0; d < kDepth; d++) {
                    const uint32_t pd = p + d * kW;
                    nw[d] = pd < n ? p_slotb[pd] / 16 : 0u;
                    const u32x4* sp = reinterpret_cast<const u32x4*>(pd < n ? p_src[pd] : 0ull);
#pragma unroll
                    for (uint32_t k = 0; k < 3; k++) {
                        v[d][k] = u32x4{0u, 0u, 0u, 0u};
                        if (lane + 64 * k < nw[d]) v[d][k] = ing_ld(sp + lane + 64 * k);
                    }
                }
#pragma unroll
                for (uint32_t d = 0; d < kDepth; d++) {
                    if (nw[d] == 0) continue;
                    const uint32_t pd = p + d * kW;
                    if (capture && lane < 2) p_hdr[pd][lane] = v[d][0];
                    u32x4* ring = reinterpret_cast<u32x4*>(s_ring[p_snd[pd]]);
                    const uint64_t w0 = p_vb[pd] >> 4;
                    const uint32_t wm = s_wmask[p_snd[pd]];
                    if (lane == 0) v[d][0].x = slot_header(p_len[pd]);
#pragma unroll
                    for (uint32_t k = 0; k < 3; k++)
                        if (lane + 64 * k < nw[d]) ing_st(ring + ((w0 + lane + 64 * k) & wm), v[d][k]);
                }
            }
        };
        const bool acc0 = acc;                 // SPEC's guess: enqueued, non-empty, full length
        const uint32_t len_d = len;
        const uint32_t slotb_s = SPEC && acc ? ((len + 4 + 15) & ~15u) : 0u;
        if constexpr (SPEC) {
            rank_scan(acc0, acc0, slotb_s);
            p_snd[tid] = (uint8_t)ls;
            p_len[tid] = (uint16_t)len;
            p_src[tid] = src;
            p_slotb[tid] = slotb_s;
            p_vb[tid] = acc0 ? s_vbyte[ls] + my_slotpre : 0ull;
            p_arr[tid] = arrival;                     // (kept in LDS across the copy)
            __syncthreads();
            slot_copy(true);
            __syncthreads();
            arrival = p_arr[tid];                     // (and these, rather than held across it)
            src = p_src[tid];
            len = p_len[tid];
            track = ls >> 1;
            if (acc0) {
                const u32x4 w0 = p_hdr[tid][0];
                const u32x4 w1 = len > 12 ? p_hdr[tid][1] : u32x4{0u, 0u, 0u, 0u};
                hdr[0] = w0.y; hdr[1] = w0.z; hdr[2] = w0.w; hdr[3] = w1.x;
                hdr[4] = w1.y; hdr[5] = w1.z; hdr[6] = w1.w;
                fl = s_flags[ls];
                // UDP push: socket B is the odd port, so only SRs survive (Q14)
                if (fl & kSndRtcpPort)
                    acc = len >= 8 && len >= 4 * hbe16(hdr, 2) + 4 && (hbyte(hdr, 0) >> 6) == 2 && hbyte(hdr, 1) == 200;
            }
        }
        if (valid && !direct && !SPEC) {
            const uint8_t* sp = reinterpret_cast<const uint8_t*>(src);
            // the slot's first 32 bytes (packet bytes 0..27) in two 16-B loads: every header
            // field the reflector reads for a CSRC-free packet comes from these registers
            u32x4 w0 = u32x4{0u, 0u, 0u, 0u}, w1 = w0;
            if (P.src_addr) {                              // a frame inside the TCP byte stream
                const uint8_t* lim = sp + 4 + len;
                if (len > 0) w0 = load16_unaligned(sp, lim);
                if (len > 12) w1 = load16_unaligned(sp + 16, lim);
            } else {
                const u32x4* sw = reinterpret_cast<const u32x4*>(sp);
                if (len > 0) w0 = sw[0];
                if (len > 12) w1 = sw[1];
            }
            hdr[0] = w0.y; hdr[1] = w0.z; hdr[2] = w0.w; hdr[3] = w1.x;
            hdr[4] = w1.y; hdr[5] = w1.z; hdr[6] = w1.w;
            if (acc) fl = s_flags[ls];
            // UDP push: socket B is the odd port, so only SRs survive (Q14)
            if (acc && (fl & kSndRtcpPort))
                acc = len >= 8 && len >= 4 * hbe16(hdr, 2) + 4 && (hbyte(hdr, 0) >> 6) == 2 && hbyte(hdr, 1) == 200;
        }
        p_snd[tid] = (uint8_t)ls;
        p_acc[tid] = acc;
        p_len[tid] = (uint16_t)len;
        p_src[tid] = src;
        p_ssrc[tid] = !acc ? 0u : (len < 8 ? 0u : (fl & kSndRtcpPort) ? hbe32(hdr, 4) : (len < 12 ? 0u : hbe32(hdr, 8)));
        p_ts[tid] = arrival / 1000;          // OS::Milliseconds() / 1000, truncating
        // ---- SSRC latch filter (sequential per socket; fast path when nothing changes) ----
        if (S.ssrc_filter) {
            const bool ok = !acc || (s_valid[ls] != 0 && p_ssrc[tid] == s_valid[ls]);
            if (acc) atomicMax(&c_lastacc[ls], tid);       // newest accepted packet per socket
            const int allok = __syncthreads_and(ok ? 1 : 0);
            if (allok) {
                if (tid < (int)nsnd && c_lastacc[tid] >= 0) s_lastv[tid] = p_ts[c_lastacc[tid]];
            } else if (tid == 0) {
                for (uint32_t p = 0; p < n; p++) {
                    if (!p_acc[p]) continue;
                    const uint32_t s = p_snd[p];
                    const uint32_t ssrc = p_ssrc[p];
                    const int64_t now_s = p_ts[p];
                    if (s_valid[s] == 0) { s_valid[s] = ssrc; s_lastv[s] = now_s; continue; }
                    if (ssrc != 0) {
                        if (ssrc == s_valid[s]) { s_lastv[s] = now_s; continue; }
                        p_len[p] = 0;                      // wrong SSRC: stays queued, length 0
                    }
                    if (s_lastv[s] + (int64_t)S.ssrc_timeout_s < now_s) s_valid[s] = 0;
                }
            }
            __syncthreads();
            EDGPU_ING_T(2);
            len = p_len[tid];
        }
        // ---- receive-time trailer (ReflectorSocket::ProcessPacket, ReflectorStream.cpp:1960-1994):
        // after the SSRC filter, a packet longer than 12 bytes whose last 12 are "aktt" + BE64
        // receive time loses them, and its arrival becomes the socket's anchor arrival plus its
        // receive time's offset from the anchor's -- the anchor being the socket's first tagged
        // packet since its SSRC (GetSSRC by the REMOTE port's parity: 0 for a push over RTSP)
        // last changed -- clamped to now + sMaxFuturePacketMSec.  Sequential per socket, so one
        // lane walks a chunk that holds a tagged packet.  The key-frame test saw the whole packet
        // (it ran first, :1876-1909) ----
        const uint32_t len0 = len;
        if (P.recv_time) {                                        // uniform
            bool tag = false;
            if (acc && len > 12) {
                const uint8_t* t = reinterpret_cast<const uint8_t*>(src) + 4 + len - 12;
                tag = t[0] == 'a' && t[1] == 'k' && t[2] == 't' && t[3] == 't';
                if (tag) {
                    uint64_t rt = 0;
                    for (int k = 4; k < 12; k++) rt = rt << 8 | t[k];
                    p_ts[tid] = (int64_t)rt;                      // (the SSRC filter is done with p_ts / p_ssrc)
                    p_ssrc[tid] = remote_odd ? hbe32(hdr, 4) : hbe32(hdr, 8);
                }
            }
            p_arr[tid] = arrival;
            p_acc[tid] = tag ? 2u : 0u;
            if (__syncthreads_or(tag ? 1 : 0)) {
                if (tid == 0) {
                    s_rtn = 1u;
                    for (uint32_t p = 0; p < n; p++) {
                        if (!(p_acc[p] & 2u)) continue;
                        const uint32_t s = p_snd[p];
                        const uint64_t rt = (uint64_t)p_ts[p];
                        const int64_t now_p = p_arr[p];
                        if (!s_rth[s] || s_rts[s] != p_ssrc[p]) {
                            s_rts[s] = p_ssrc[p]; s_rta[s] = now_p; s_rtr[s] = rt; s_rth[s] = 1u;
                        }
                        int64_t a = s_rta[s] + (int64_t)(rt - s_rtr[s]);
                        if (a - now_p > P.max_future_ms) a = now_p + P.max_future_ms;
                        p_arr[p] = a;
                    }
                }
                __syncthreads();
                if (tag) { arrival = p_arr[tid]; len -= 12; p_len[tid] = (uint16_t)len; }   // (the copy's header / bound)
            }
        }
        const bool nz = acc && len > 0;
        const uint32_t slotb = nz ? ((len + 4 + 15) & ~15u) : 0;
        // ---- per-sender queue index / slot offset / non-empty count (rank_scan above).  SPEC:
        // the slot bytes stay the guessed ones (a refused packet's bytes become a hole), and the
        // ranks are scanned again only if a packet's enqueue / non-empty state differs from the guess
        bool recopied = false;
        if constexpr (SPEC) {
            if (__syncthreads_or(acc != acc0 || nz != acc0 ? 1 : 0)) {
                // a refusal: the round is laid out again without the refused packets' bytes and its
                // enqueued packets copied again to their final places (from the batch, so the two
                // copies never read each other).  The guessed layout's end stays as the sender's
                // write high-water mark (vclob): ring slots it reached are no longer intact.
                if (tid < (int)nsnd) s_vclob[tid] = max(s_vclob[tid], s_vbyte[tid] + (c_tot[tid] >> 20));
                const uint32_t fb = nz ? slotb_s : 0u;
                rank_scan(acc, nz, fb);
                p_slotb[tid] = fb;
                p_vb[tid] = nz ? s_vbyte[ls] + my_slotpre : 0ull;
                p_len[tid] = (uint16_t)len;
                __syncthreads();
                slot_copy(false);
                recopied = true;
                // (the header words and the arrival from LDS again, rather than held across the copy)
                const u32x4 z4 = u32x4{0u, 0u, 0u, 0u};
                const u32x4 w0 = acc0 ? p_hdr[tid][0] : z4, w1 = acc0 && len_d > 12 ? p_hdr[tid][1] : z4;
                hdr[0] = w0.y; hdr[1] = w0.z; hdr[2] = w0.w; hdr[3] = w1.x;
                hdr[4] = w1.y; hdr[5] = w1.z; hdr[6] = w1.w;
                arrival = p_arr[tid];
            }
            if (!recopied && nz && len != len_d)         // a stripped trailer: the slot header's length
                reinterpret_cast<uint32_t*>(s_ring[ls])[(((s_vbyte[ls] + my_slotpre) >> 4) & s_wmask[ls]) * 4] =
                    slot_header(len);
        } else {
            rank_scan(acc, nz, slotb);
        }
        if (nz) atomicMax(&c_last[ls], tid << 10 | (int)my_rank);
        uint64_t idx = 0, vb = 0;
        bool kev_key = false, kev_aud = false;
        if (acc) {
            idx = s_head[ls] + my_rank;
            vb = s_vbyte[ls] + my_slotpre;
            PktMeta m;
            m.vbyte = vb;
            m.id = s_count[track] + my_trank + 1;        // fStreamCountID = ++fPacketCount
            m.arrival = arrival;
            m.len = (uint16_t)len;
            m.seq = len >= 4 ? (uint16_t)hbe16(hdr, 2) : (uint16_t)0;
            m.vcount = s_vcount[ls] + my_nzpre;
            reinterpret_cast<PktMeta*>(s_meta[ls])[idx & s_pkmask[ls]] = m;
            if (P.host_epoch)                            // its blob slot, for edgpu_fanout_sources
                reinterpret_cast<uint32_t*>(s_meta[ls] + ((uint64_t)s_pkmask[ls] + 1) * sizeof(PktMeta))[idx & s_pkmask[ls]] = slot;
            const bool by_port_rtp = !(fl & kSndRtcpPort);
            const bool key = by_port_rtp && (fl & kSndVideo) && (fl & kSndH264) && len0 >= 20 &&
                             ((hbyte(hdr, 0) & 0x0F) == 0 ? key_frame_first_packet_cc0(hdr, len0)
                                                          : key_frame_first_packet(reinterpret_cast<const uint8_t*>(src) + 4, len0));
            kev_key = key;
            kev_aud = by_port_rtp && (fl & kSndAudio);
        }
        // ---- keyframe index, part 1: each wave's key / audio events in arrival order (ballots) ----
        const uint64_t kK = __ballot(kev_key), kE = kK | __ballot(kev_aud);
        if ((tid & 63) == 0)
            s_wev[tid >> 6] = kE ? 1u | (uint32_t)((kK >> (63 - __clzll((long long)kE))) & 1ull) << 1 : 0u;
        if constexpr (!SPEC) {
            p_slotb[tid] = slotb;
            p_vb[tid] = vb;
        }
        __syncthreads();
        EDGPU_ING_T(4);
        // ---- keyframe index, part 2: a video key packet moves its sender's key pointer; an audio
        // packet anchors its sender's when the last key / audio event before it was a key packet
        // (none in the chunk before it: the session's flag); the newest such packet per sender wins
        // (Q5).  A lane's previous event: its wave's lower lanes, else the earlier waves' last ----
        {
            const int lane = tid & 63, wid = tid >> 6;
            bool fin = kflag;
            for (int w = 0; w < wid; w++)
                if (s_wev[w] & 1u) fin = (s_wev[w] >> 1) & 1u;
            const uint64_t below = lane ? (kE & ((1ull << lane) - 1)) : 0ull;
            const bool anchor = kev_aud && (below ? ((kK >> (63 - __clzll((long long)below))) & 1ull) != 0 : fin);
            if (kev_key || anchor)
                atomicMax(&s_klast[ls], (unsigned long long)(tid + 1) << 52 | (idx & kQiMask));
            for (int w = 0; w < NW; w++)                              // the flag after the chunk
                if (s_wev[w] & 1u) kflag = (s_wev[w] >> 1) & 1u;
        }
        // ---- slot copy: here, one wave per packet (copy_mode 0), or as a job for
        // k_ingest_copy's flat grid over packets (copy_mode 1) ----
        if (SPEC || (EDGPU_ABL(P) & 32u)) {
            // SPEC: copied above; or a timing ablation: no slot copy
        } else if (EDGPU_COPY_MODE(P) == 0 && P.src_addr && EDGPU_TCP_COPY(P) >= 1) {   // frames inside the TCP byte stream
            if (EDGPU_TCP_COPY(P) == 3) tcp_slot_copy_s<kTcpFramesPerRound, THREADS>(n, p_slotb, p_src, p_len, p_snd, p_vb, s_ring, s_wmask);
            else if (EDGPU_TCP_COPY(P) >= 2) tcp_slot_copy<2, THREADS>(n, p_slotb, p_src, p_len, p_snd, p_vb, s_ring, s_wmask);
            else tcp_slot_copy<1, THREADS>(n, p_slotb, p_src, p_len, p_snd, p_vb, s_ring, s_wmask);
        } else if (EDGPU_COPY_MODE(P) == 0 && P.src_addr) {   // same, two aligned loads per word (A/B)
            const int lane = tid & 63, wid = tid >> 6;
            for (uint32_t p = wid; p < n; p += THREADS / 64) {
                const uint32_t sb = p_slotb[p];
                if (sb == 0) continue;
                const uint32_t s = p_snd[p];
                const uint8_t* sp = reinterpret_cast<const uint8_t*>(p_src[p]);
                u32x4* ring = reinterpret_cast<u32x4*>(s_ring[s]);
                const uint64_t w0 = p_vb[p] >> 4;
                const uint32_t wm = s_wmask[s];
                const uint8_t* lim = sp + 4 + p_len[p];
                // all of a lane's (<= 3) words are loaded before its first store, as below
                const uint32_t nw = sb / 16;
                const u32x4 z = u32x4{0u, 0u, 0u, 0u};
                u32x4 v0 = lane < nw ? load16_unaligned(sp + 16 * lane, lim) : z;
                const u32x4 v1 = lane + 64 < nw ? load16_unaligned(sp + 16 * (lane + 64), lim) : z;
                const u32x4 v2 = lane + 128 < nw ? load16_unaligned(sp + 16 * (lane + 128), lim) : z;
                if (lane == 0) v0.x = slot_header(p_len[p]);
                if (lane < nw) ring[(w0 + lane) & wm] = v0;
                if (lane + 64 < nw) ring[(w0 + lane + 64) & wm] = v1;
                if (lane + 128 < nw) ring[(w0 + lane + 128) & wm] = v2;
            }
        } else if (EDGPU_COPY_MODE(P) == 0) {
            // kDepth packets per wave per round, and a slot is at most 129 words (2060 + 4 B),
            // so every lane issues all of its loads (<= 3 x 16 B per packet) before its first
            // store: a wave keeps kDepth whole slots in flight instead of waiting out one load
            // latency per 64 words of one slot.
            constexpr uint32_t kDepth = DEPTH, kW = THREADS / 64;
            const uint32_t lane = tid & 63, wid = tid >> 6;
            for (uint32_t p = wid; p < n; p += kDepth * kW) {
                uint32_t nw[kDepth];
                u32x4 v[kDepth][3];
#pragma unroll
                for (uint32_t d = 0; d < kDepth; d++) {
                    const uint32_t pd = p + d * kW;
                    nw[d] = pd < n ? p_slotb[pd] / 16 : 0u;
                    const u32x4* sp = reinterpret_cast<const u32x4*>(pd < n ? p_src[pd] : 0ull);
#pragma unroll
                    for (uint32_t k = 0; k < 3; k++) {
                        v[d][k] = u32x4{0u, 0u, 0u, 0u};
                        if (lane + 64 * k < nw[d]) v[d][k] = ing_ld(sp + lane + 64 * k);
                    }
                }
#pragma unroll
                for (uint32_t d = 0; d < kDepth; d++) {
                    if (nw[d] == 0) continue;
                    const uint32_t pd = p + d * kW;
                    u32x4* ring = reinterpret_cast<u32x4*>(s_ring[p_snd[pd]]);
                    const uint64_t w0 = p_vb[pd] >> 4;
                    const uint32_t wm = s_wmask[p_snd[pd]];
                    if (lane == 0) v[d][0].x = slot_header(p_len[pd]);
#pragma unroll
                    for (uint32_t k = 0; k < 3; k++)
                        if (lane + 64 * k < nw[d]) ing_st(ring + ((w0 + lane + 64 * k) & wm), v[d][k]);
                }
            }
        } else if (valid) {
            CopyJob j;
            j.ring = acc ? s_ring[ls] : 0ull;
            j.vword = vb >> 4;
            j.wmask = acc ? s_wmask[ls] : 0u;
            j.src_slot = slot;
            j.len = slotb ? len : 0u;
            j.sender = S.first_sender + ls;
            P.jobs[i] = j;
        }
        // ---- advance per-sender / per-stream state ----
        if (tid < (int)nsnd) {
            const uint64_t t = c_tot[tid];
            const uint32_t cnt = t & 1023;
            if (c_last[tid] >= 0) s_lastnz[tid] = (int64_t)(s_head[tid] + (c_last[tid] & 1023));
            s_head[tid] += cnt;
            s_vcount[tid] += (uint32_t)((t >> 10) & 1023);
            s_vbyte[tid] += t >> 20;
        }
        if (tid < (int)S.ntracks) s_count[tid] += (c_tot[2 * tid] & 1023) + (c_tot[2 * tid + 1] & 1023);
        if (tid < (int)nsnd) c_lastacc[tid] = -1;
        __syncthreads();
        EDGPU_ING_T(5);
    }

    if (tid < (int)nsnd) {
        SenderDev& D = P.senders[S.first_sender + tid];
        if (P.host_epoch) { D.batch_lo = D.head; D.batch_epoch = P.host_epoch; }   // (the head before the batch)
        D.head = s_head[tid]; D.vbyte_end = s_vbyte[tid]; D.vcount_end = s_vcount[tid];
        D.vclob = s_vclob[tid];
        D.key = s_klast[tid] ? (int64_t)(s_klast[tid] & kQiMask) : s_key[tid];
        D.valid_ssrc = s_valid[tid]; D.last_valid_s = s_lastv[tid]; D.last_nonzero = s_lastnz[tid];
        if (P.recv_time) {
            D.rt_has = s_rth[tid]; D.rt_ssrc = s_rts[tid]; D.rt_first_arrival = s_rta[tid]; D.rt_first_receive = s_rtr[tid];
            if (s_rtn) D.rt_nonmono = 1u;
        }
        // a copy pass the last tick still owes (edgpu_fanout_next): this batch must not lap what
        // that tick's remaining passes read
        if (pass_owed && (max(s_vbyte[tid], s_vclob[tid]) > D.fan_vlo + ((uint64_t)s_wmask[tid] + 1) * 16 ||
                      s_head[tid] > D.fan_lo + (uint64_t)s_pkmask[tid] + 1))
            atomicCAS(&P.totals->ingest_status, 0, EDGPU_RING_OVERFLOW);
    }
    if (tid < (int)S.ntracks) P.streams[S.first_stream + tid].packet_count = s_count[tid];
    if (tid == 0) P.sessions[P.seg_sess[seg]].video_key_flag = kflag ? 1u : 0u;
    // block totals: packets (< 2^21) and bytes (< 2^32) of the segment packed in one word, one
    // DPP scan per wave and one barrier
    const uint64_t wt = wave_inclusive_scan_u64((uint64_t)in_bytes << 21 | in_pk);
    if ((tid & 63) == 63) scan64[tid >> 6] = wt;
    __syncthreads();
    uint64_t t1 = 0, t2 = 0;
    if (tid == 0) {
        for (int w = 0; w < NW; w++) { t1 += scan64[w] & ((1ull << 21) - 1); t2 += scan64[w] >> 21; }
    }
    if (tid == 0 && !(EDGPU_ABL(P) & 16u)) {
        atomicAdd(&P.totals->cum_ingested_packets, (unsigned long long)t1);
        atomicAdd(&P.totals->cum_ingested_bytes, (unsigned long long)t2);
        atomicAdd(&P.totals->ing_pk[P.ing_slot], (unsigned long long)t1);
        atomicAdd(&P.totals->ing_b[P.ing_slot], (unsigned long long)t2);
    }
    if (seg == 0 && tid == 0) { P.totals->ing_pk[P.ing_slot ^ 1u] = 0; P.totals->ing_b[P.ing_slot ^ 1u] = 0; }
#ifdef EDGPU_AB_VARIANTS
    EDGPU_ING_T(6);
    if (tid == 0 && e > b) {
        for (int k = 1; k < 7; k++) atomicAdd(&P.totals->ing_ph[k], ph_t[k]);
        atomicAdd(&P.totals->ing_ph[0], 1ull);
    }
    if (tid == 0) {
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        atomicMin(&P.totals->ing_done_min, t);
        atomicMax(&P.totals->ing_done_max, t);
    }
#endif
}

// =========================================================================================
// Slot copy, blob -> byte rings.  Each group of kCopyLanes lanes copies one packet's slot as
// 16-B words, rewriting word 0's 4-byte prefix to the '$' 0 BE16(len) frame header.  A flat
// grid over packets keeps every CU busy regardless of how packets spread over sessions.
// =========================================================================================
#ifdef EDGPU_AB_VARIANTS
constexpr int kCopyThreads = 256, kCopyLanes = 16;

__global__ __launch_bounds__(kCopyThreads) void k_ingest_copy(IngestParams P) {
    const uint32_t g = blockIdx.x * (kCopyThreads / kCopyLanes) + threadIdx.x / kCopyLanes;
    const uint32_t lane = threadIdx.x % kCopyLanes;
    if (g >= P.npk) return;
    const CopyJob j = P.jobs[g];
    if (j.len == 0) return;
    const uint32_t nw = (j.len + 4 + 15) >> 4;
    // words a later packet of the same batch laps are left to it (k_ingest has already
    // advanced vbyte_end), so a batch larger than the ring stays deterministic
    const uint64_t vend = P.senders[j.sender].vbyte_end >> 4, cap = (uint64_t)j.wmask + 1;
    const uint64_t live = vend > cap ? vend - cap : 0ull;
    const u32x4* src = reinterpret_cast<const u32x4*>(P.blob + (uint64_t)j.src_slot * 16);
    u32x4* ring = reinterpret_cast<u32x4*>(j.ring);
    for (uint32_t k = lane; k < nw; k += kCopyLanes) {
        u32x4 v = src[k];
        if (k == 0) v.x = slot_header(j.len);
        if (j.vword + k >= live) ring[(j.vword + k) & j.wmask] = v;
    }
}
#endif  // EDGPU_AB_VARIANTS

// =========================================================================================
// Keyframe index + audio anchor: one wave per session segment.
// =========================================================================================

// =========================================================================================
// Fan-out planning
// =========================================================================================

// First index in [lo, hi) whose meta satisfies pred (monotone false..true), hi if none.
template <typename Pred>
__device__ uint64_t lower_bound_meta(const PktMeta* meta, uint32_t mask, uint64_t lo, uint64_t hi, Pred pred) {
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (pred(meta[mid & mask])) hi = mid; else lo = mid + 1;
    }
    return lo;
}

// lower_bound_meta for a whole wave: each round the 64 lanes probe 64 evenly spaced records
// and a ballot narrows the range 64-fold, so a 16k-record ring takes 3 dependent loads, not 14.
// Every lane of the wave must call it with the same arguments; all lanes get the result.
template <typename Pred>
__device__ uint64_t wave_lower_bound_meta(const PktMeta* meta, uint32_t mask, uint64_t lo, uint64_t hi, Pred pred) {
    const uint64_t lane = threadIdx.x & 63;
    while (lo < hi) {
        const uint64_t step = (hi - lo + 63) / 64;
        const uint64_t probe = min(lo + (lane + 1) * step - 1, hi - 1);
        const unsigned long long t = __ballot(pred(meta[probe & mask]) ? 1 : 0);
        if (t == 0) return hi;                               // pred(hi - 1) is false
        const uint64_t j = (uint64_t)(__ffsll(t) - 1);       // first probe that holds
        // the answer is in (probe j-1, probe j]: search below probe j, which is the fallback
        const uint64_t pj = min(lo + (j + 1) * step - 1, hi - 1);
        lo = j == 0 ? lo : min(lo + j * step - 1, hi - 1) + 1;
        hi = pj;
    }
    return hi;
}

// The first packet in [lo, hi) whose arrival is at least `cut`: GetClientBufferStartPacketOffset's
// walk from the oldest packet (ReflectorStream.cpp:1209-1227) and RemoveOldPackets' first young
// packet (:1245-1285).  Push times are monotone along a ring, so a binary search finds it -- until
// receive-time trailers rewrote arrivals on the sender (rt_nonmono, :1960-1994): then the walk
// itself, in arrival order as the reference walks its queue.  The wave form: every lane of the
// wave calls it with the same arguments and gets the result.
__device__ uint64_t first_arrival_at(const SenderDev& D, const PktMeta* meta, uint64_t lo, uint64_t hi, int64_t cut) {
    if (!D.rt_nonmono) return lower_bound_meta(meta, D.pk_mask, lo, hi, [&](const PktMeta& m) { return m.arrival >= cut; });
    for (; lo < hi; lo++)
        if (meta[lo & D.pk_mask].arrival >= cut) break;
    return lo;
}
__device__ uint64_t wave_first_arrival_at(const SenderDev& D, const PktMeta* meta, uint64_t lo, uint64_t hi, int64_t cut) {
    if (!D.rt_nonmono)
        return wave_lower_bound_meta(meta, D.pk_mask, lo, hi, [&](const PktMeta& m) { return m.arrival >= cut; });
    const uint64_t lane = threadIdx.x & 63;
    for (uint64_t b = lo; b < hi; b += 64) {
        const uint64_t i = b + lane;
        const unsigned long long t = __ballot(i < hi && meta[i & D.pk_mask].arrival >= cut ? 1 : 0);
        if (t) return b + (uint64_t)(__ffsll(t) - 1);
    }
    return hi;
}

// K1: per sender, one wave each -- ring tail, fFirstPacketInQueueForNewOutput
// (ReflectorStream.cpp:1058-1069).
__device__ __forceinline__ void reset_tick_totals(TickTotals* t) {
    t->relayed_packets = 0; t->relayed_bytes = 0; t->arena_bytes = 0;   // the ingest counters stay
    t->status = 0; t->nwork = 0; t->fan_next = 0; t->stream_errors = 0;
    t->fan_t0_min = ~0ull; t->fan_done_min = ~0ull; t->fan_done_max = 0;
#ifdef EDGPU_AB_VARIANTS
    // measurement builds: the last ingest's span and first workgroup exit, then a reset
    t->ing_last_span = t->ing_done_max - t->ing_t0_min; t->ing_last_first = t->ing_done_min - t->ing_t0_min;
    t->ing_t0_min = ~0ull; t->ing_done_min = ~0ull; t->ing_done_max = 0;
    for (int k = 0; k < 8; k++) { t->ing_last_ph[k] = t->ing_ph[k]; t->ing_ph[k] = 0; }
#endif
    // a pass the previous tick still owed is lost now (its host never called edgpu_fanout_next)
    if (t->pass_next[t->pass_slot & 1u] != kNoPass) t->cum_lost_passes++;
    t->pass_slot = 0;
    for (int k = 0; k < 2; k++) { t->pass_bytes[k] = 0; t->pass_desc[k] = 0; t->pass_next[k] = kNoPass; }
    t->grow_count = 0;
}

// Per-tick counter updates as one tiny launch (a hipMemsetAsync of a few bytes costs two fill
// kernels): which = 0 fan-out totals reset (when k_plan_senders, which does it itself, does not
// run), 1 the ingest counters of an empty batch (when k_ingest, which does it itself, does not run).
__global__ void k_totals_reset(TickTotals* t, int which) {
    if (threadIdx.x != 0) return;
    if (which == 0) reset_tick_totals(t);
    else for (int k = 0; k < 2; k++) { t->ing_pk[k] = 0; t->ing_b[k] = 0; }
}

// A sender ring lost a packet an output of its session needed (per-stream isolation: the
// session is marked, the tick goes on).
__device__ __forceinline__ void mark_stream_error(const PlanParams& P, uint32_t session) {
    if (atomicOr(&P.sessions[session].errors, kStreamRingOverflow) == 0u) atomicAdd(&P.totals->stream_errors, 1u);
}

__global__ __launch_bounds__(256) void k_plan_senders(PlanParams P) {
    if (blockIdx.x == 0 && threadIdx.x == 0) reset_tick_totals(P.totals);   // no later kernel has run
    const uint32_t s = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    if (s >= P.T.nsenders) return;                             // uniform per wave
    SenderDev& D = P.senders[s];
    const PktMeta* meta = reinterpret_cast<const PktMeta*>(D.meta);
    const uint64_t head = D.head;
    const uint64_t pk_cap = (uint64_t)D.pk_mask + 1;
    const uint64_t byte_cap = ((uint64_t)D.word_mask + 1) * 16;
    uint64_t lo = head > pk_cap ? head - pk_cap : 0;
    lo = max(lo, D.floor);                                    // a replica holds nothing older
    const uint64_t vend = D.vbyte_end, vhigh = max(vend, D.vclob);
    // oldest packet whose slot is still intact in the byte ring (no write since reached it: the
    // ingest's speculative copy may have written past vbyte_end, up to vclob)
    const uint64_t tail = wave_lower_bound_meta(meta, D.pk_mask, lo, head,
                                                [&](const PktMeta& m) { return vhigh - m.vbyte <= byte_cap; });
    int64_t ns = -1;
    if (D.key >= 0) {
        ns = D.key;
        if ((uint64_t)ns < tail) ns = -2;                      // key packet overwritten
    } else if (head > tail) {
        const int64_t cutoff = P.T.now - P.T.over_buffer_ms;  // now - arrival <= over buffer
        const uint64_t f = wave_first_arrival_at(D, meta, tail, head, cutoff);
        if (f < head) ns = (f == tail && tail > D.floor) ? -2 : (int64_t)f;   // -2: window exceeds ring
    }
    // Ring growth: the span the reference would still hold in its unbounded queue -- every packet
    // younger than sMaxPacketAgeMSec = 10 x the buffer (ReflectorStream.cpp:112-114), the key
    // packet and everything after it, and what last tick's outputs still read from (a blocked
    // output's bookmark keeps its packet, fNeededByOutput, RemoveOldPackets :1233-1289).  Measured
    // only once the ring holds more than half of either capacity; a span over half of one asks
    // the host to double that ring before the next ingest (GrowReq).
    if (P.T.grow_on && head > tail) {
        const uint64_t held_b = vend - meta[tail & D.pk_mask].vbyte;
        if (2 * (head - tail) > pk_cap || 2 * held_b > byte_cap) {
            const int64_t age_cut = P.T.now - 10 * P.T.over_buffer_ms;
            uint64_t r = wave_first_arrival_at(D, meta, tail, head, age_cut);
            if (D.key >= 0 && (uint64_t)D.key >= tail) r = min(r, (uint64_t)D.key);
            if (D.umin >= tail) r = min(r, D.umin);              // last tick's reads (before the reset below)
            const uint64_t need_pk = head - r;
            const uint64_t need_b = r < head ? vend - meta[r & D.pk_mask].vbyte : 0;
            uint64_t want_pk = pk_cap, want_b = byte_cap;
            while (2 * need_pk > want_pk && want_pk < P.T.grow_max_pk) want_pk *= 2;
            while (2 * need_b > want_b && want_b < P.T.grow_max_bytes) want_b *= 2;
            if ((threadIdx.x & 63) == 0 && (want_pk > pk_cap || want_b > byte_cap)) {
                const uint32_t k = atomicAdd(&P.totals->grow_count, 1u);
                if (k < kMaxGrow)
                    P.grow[k] = GrowReq{s, (uint32_t)(63 - __clzll((long long)want_pk)),
                                        (uint32_t)(63 - __clzll((long long)want_b)), 0u, tail, head};
                if (k == 0 && P.T.grow_flag) *(volatile uint32_t*)P.T.grow_flag = 1u;   // (a vector store)
            }
        }
    }
    if ((threadIdx.x & 63) == 0) {
        D.tail = tail;
        D.new_start = ns;
        D.umin = head;
    }
}

// Ring growth: a sender's ring entries [lo, lo + n) (monotonic indices) from a ring of mask
// `smask` to one of mask `dmask` (both powers of two minus one), entry v at v & mask in each.
template <typename T>
__global__ __launch_bounds__(256) void k_ring_move(const T* __restrict__ src, uint64_t smask, T* __restrict__ dst,
                                                   uint64_t dmask, uint64_t lo, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint64_t v = lo + i;
        dst[v & dmask] = src[v & smask];
    }
}

// K2: per sub-stream -- this tick's range and the bookmark / last-id commit
// (ReflectorStream.cpp:1092-1116; RTPSessionOutput.cpp:283-315, 624-639).
__global__ __launch_bounds__(256) void k_plan_subs(PlanParams P) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t bytes = 0;
    uint32_t count = 0;
    if (q < P.T.nsubs) {
        SubDev& Q = P.subs[q];
        Q.nonempty = 0; Q.count = 0; Q.bytes = 0;
        Q.was_new = Q.active && Q.bookmark < 0;
        if (Q.active) {
            SenderDev& D = P.senders[Q.sender];
            const PktMeta* meta = reinterpret_cast<const PktMeta*>(D.meta);
            const uint64_t head = D.head;
            bool have = false;
            uint64_t a = 0;
            Q.prev_last_id = Q.last_id;                 // for edgpu_fanout_blocked
            Q.prev_has_last = Q.has_last;
            Q.prev_sent_any = Q.sent_any;
            if (Q.bookmark >= 0) {                     // GetBookMarkedPacket: resume after it
                // (AT it when a blocked write left it unsent, or after a Q9 relocation)
                a = (uint64_t)Q.bookmark + (Q.resume_at ? 0u : 1u);
                // SendPacketsToOutput restarts AT the bookmarked packet (ReflectorStream.cpp:
                // 1138-1198); it went out or was empty at its first visit, so it is skipped --
                // unless the RTP-Info first-seq filter held it back and has just been lifted
                // by the client stream's first write (no RTP id recorded yet): then it goes now
                if (Q.rtp_info && Q.kind == 0 && !Q.has_last && (Q.sent_any || P.subs[q + 1].sent_any))
                    a = (uint64_t)Q.bookmark;
                have = true;
                if (a < D.tail && a < head) { mark_stream_error(P, D.session); a = D.tail; }
            } else if (D.new_start >= 0) {             // new output: key pointer / buffer start
                a = (uint64_t)D.new_start;
                have = true;
                if (Q.has_last)                        // PacketAlreadySent for a re-joined output
                    a = lower_bound_meta(meta, D.pk_mask, a, head,
                                         [&](const PktMeta& m) { return m.id > Q.last_id; });
            } else if (D.new_start == -2) {               // retried next tick (still a new output)
                mark_stream_error(P, D.session);
            }
            if (have) {
                // FilterPacket (RTPSessionOutput.cpp:249-280, Q10): until the client stream's
                // first write -- RTP or RTCP, its packet count (:643-653) -- RTP packets with
                // seq < FirstSeqNumber are skipped, a plain u16 compare with no wrap handling.
                // Zero-length packets never reach the filter (:571-572).  The RTP sender is
                // reflected before the RTCP sender in a tick, so the RTCP sibling's writes of
                // this tick do not count yet.
                if (Q.rtp_info && Q.kind == 0 && !Q.sent_any && !P.subs[q + 1].sent_any) {
                    while (a < head) {
                        const PktMeta m = meta[a & D.pk_mask];
                        if (m.len != 0 && m.seq >= Q.first_seq) break;
                        a++;
                    }
                }
                if (a < head) {
                    const PktMeta m = meta[a & D.pk_mask];
                    Q.a = a;
                    Q.vstart = m.vbyte;
                    Q.vcstart = m.vcount;
                    bytes = D.vbyte_end - m.vbyte;
                    count = D.vcount_end - m.vcount;
                    Q.bytes = bytes;
                    Q.count = count;
                    Q.nonempty = 1;
                    atomicMin((unsigned long long*)&D.umin, (unsigned long long)a);
                }
                // SendPacketsToOutput returns the newest visited packet; with sinks that never
                // block NeedRelocateBookMark (Q9) cannot fire: the bookmark is the newest packet.
                if (head > 0) { Q.bookmark = (int64_t)(head - 1); Q.resume_at = 0; }
                if (count > 0) {
                    Q.last_id = meta[(uint64_t)D.last_nonzero & D.pk_mask].id;
                    Q.has_last = 1;
                }
            }
        }
    }
    // block partials for the output-offset scan, and the block's largest sub-stream (the copy
    // passes of an over-capacity tick are cut so that any sub-stream fits one, k_plan_final)
    __shared__ uint64_t sb[4];
    __shared__ uint32_t sc[4];
    uint64_t tb; uint32_t tc;
    (void)block_exclusive_scan<uint64_t>(bytes, sb, tb);
    (void)block_exclusive_scan<uint32_t>(count, sc, tc);
    const uint64_t mb = block_reduce<uint64_t, OpMax>(bytes, sb);
    const uint32_t mc = block_reduce<uint32_t, OpMax>(count, sc);
    if (threadIdx.x == 0) {
        P.blk_bytes[blockIdx.x] = tb; P.blk_count[blockIdx.x] = tc;
        P.blk_maxb[blockIdx.x] = mb; P.blk_maxc[blockIdx.x] = mc;
    }
}

// Inclusive scan over a workgroup of up to 1024 threads: shuffles inside each wave, then the
// wave totals (wsum, one per wave) through LDS.  Every thread of the block must call it.
template <typename T>
__device__ __forceinline__ T wave_block_inclusive_scan(T v, T* wsum) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const T y = __shfl_up(v, o, 64);
        if (lane >= o) v += y;
    }
    if (lane == 63) wsum[w] = v;
    __syncthreads();
    T base = 0;
    for (int i = 0; i < w; i++) base += wsum[i];
    __syncthreads();                                  // wsum may be reused by the next call
    return v + base;
}

// K3: per sub-stream -- final arena / descriptor offsets and the public sub-stream table;
// per sender -- work items.  Each block adds up the K2 partials of the blocks before it (a few
// hundred at most), so the offsets need no separate scan launch; block 0 adds up all of them
// for the tick totals.  A sender's work items take their place with one atomicAdd on the
// tick's item count: items are independent, so their order only shapes the copy kernel's
// schedule (each sender's chunks stay consecutive).
__global__ __launch_bounds__(256) void k_plan_final(PlanParams P) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    __shared__ uint64_t sb[4];
    __shared__ uint32_t sc[4];
    // loads that do not wait for the K2 partials, issued first so that their latency overlaps the
    // partials' reduction: this row's size, and the work-item counts of the senders this lane
    // reserves for (below)
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
    const uint32_t gw = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    auto chunks_of = [&](const SenderDev& D) {
        return (uint32_t)(((D.head > D.umin ? D.head - D.umin : 0) + P.T.chunk - 1) / P.T.chunk);
    };
    uint64_t bytes = 0; uint32_t count = 0;
    if (q < P.T.nsubs) { bytes = P.subs[q].bytes; count = P.subs[q].count; }
    uint32_t res_nch = 0, res_base = 0;
    if (gw + lane * nwaves < P.T.nsenders) res_nch = chunks_of(P.senders[gw + lane * nwaves]);
    // Every block adds up all the K2 partials (a few hundred at most): the tick's totals, the
    // part before this block, and the largest sub-stream.
    uint64_t base_b, tb_all, mb;
    uint32_t base_c, tc_all, mc;
    {
        const uint32_t nb = P.T.nsub_blocks;
        uint64_t xb = 0, xba = 0, xmb = 0;
        uint32_t xc = 0, xca = 0, xmc = 0;
        for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) {
            const uint64_t b = P.blk_bytes[i];
            const uint32_t c = P.blk_count[i];
            xba += b; xca += c;
            if (i < blockIdx.x) { xb += b; xc += c; }
            xmb = max(xmb, P.blk_maxb[i]); xmc = max(xmc, P.blk_maxc[i]);
        }
        base_b = block_reduce<uint64_t, OpSum>(xb, sb); tb_all = block_reduce<uint64_t, OpSum>(xba, sb);
        mb = block_reduce<uint64_t, OpMax>(xmb, sb);
        base_c = block_reduce<uint32_t, OpSum>(xc, sc); tc_all = block_reduce<uint32_t, OpSum>(xca, sc);
        mc = block_reduce<uint32_t, OpMax>(xmc, sc);
    }
    // An over-capacity tick is delivered in copy passes over consecutive sub-stream rows
    // (edgpu_fanout_next), every pass within the arena and the descriptor array, so no output is
    // lost: the reference walks every output of every sender in each ReflectPackets
    // (ReflectorStream.cpp:1088-1120).  Row q belongs to pass  floor(B_q / W) + floor(C_q / Wc),
    // B_q / C_q its tick-global byte / descriptor offsets, W = arena - largest sub-stream (+ 16)
    // and Wc = descriptors - largest count + 1: both floors never fall from row to row, so a pass
    // id names one (byte window, descriptor window) pair (ids may skip), and a pass's rows --
    // which start inside its windows -- end within one arena / descriptor array of the windows'
    // starts, their offsets in the pass.  A tick that fits is pass 0 with global offsets.
    const bool fits = tb_all <= P.T.arena_bytes && tc_all <= P.T.max_desc;
    const bool impossible = mb > P.T.arena_bytes || mc > P.T.max_desc;   // one sub-stream is too large
    const uint64_t W = (fits || impossible) ? 16ull : ((P.T.arena_bytes - mb) & ~15ull) + 16;
    const uint32_t Wc = (fits || impossible) ? 1u : P.T.max_desc - mc + 1;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        P.totals->arena_bytes = tb_all;
        P.totals->relayed_packets = tc_all;
        P.totals->cum_relayed_packets += tc_all;
        if (!fits && impossible) atomicExch(&P.totals->status, EDGPU_OUT_OVERFLOW);
        if (fits) { P.totals->pass_bytes[0] = tb_all; P.totals->pass_desc[0] = tc_all; }
    }
    uint64_t tb; uint32_t tc;
    const uint64_t pb = block_exclusive_scan<uint64_t>(bytes, sb, tb);
    const uint32_t pc = block_exclusive_scan<uint32_t>(count, sc, tc);
    uint64_t end_b = 0; uint32_t end_c = 0, next = kNoPass;   // pass 0's extent, the next pass
    if (q < P.T.nsubs) {
        SubDev& Q = P.subs[q];
        uint64_t ob = base_b + pb;
        uint32_t od = base_c + pc, pass = 0;
        if (!fits) {
            const uint64_t kb = ob / W;
            const uint32_t kc = od / Wc;
            pass = (uint32_t)kb + kc;
            ob -= kb * W;
            od -= kc * Wc;
        }
        Q.out_base = ob;
        Q.desc_base = od;
        Q.pass = pass;
        edgpu_substream_out o;
        o.subscriber = Q.handle;
        o.track = Q.track;
        o.kind = Q.kind;
        o.transport = Q.transport;
        o.desc_base = Q.desc_base;
        o.desc_count = pass == 0 ? Q.count : 0u;
        o.out_base = Q.out_base;
        o.out_bytes = pass == 0 ? Q.bytes : 0ull;
        o.sender = Q.sender;
        o.flags = ((!Q.transport && !Q.rw) ? EDGPU_SUB_IDENTITY : 0u) | (Q.was_new ? EDGPU_SUB_NEW : 0u);
        P.sub_out[q] = o;
        if (Q.count > 0) Q.sent_any = 1;
        if (pass == 0) { end_b = ob + Q.bytes; end_c = od + Q.count; }
        else if (Q.count > 0) next = pass;
        const uint32_t pos = P.sub_pos[q];
        if (pos != 0xFFFFFFFFu) {
            FanSub f;
            f.dw = (int64_t)(Q.out_base >> 4) - (int64_t)(Q.vstart >> 4);
            f.off = (int64_t)(Q.out_base - Q.vstart) + (Q.transport ? 0 : 4);
            f.a = (Q.nonempty && pass == 0) ? Q.a : ~0ull;
            f.ch = Q.transport ? ((uint32_t)Q.channel << 8 | 1u) : 0u;
            f.db = Q.desc_base - Q.vcstart;
            f.rw = Q.rw;
            f.rw_ts = Q.rw_ts;
            f.rw_ssrc_be = __builtin_bswap32(Q.rw_ssrc);
            f._pad = 0;
            P.fansub[pos] = f;
        }
    }
    if (!fits) {                                       // uniform over the grid
        end_b = block_reduce<uint64_t, OpMax>(end_b, sb);
        end_c = block_reduce<uint32_t, OpMax>(end_c, sc);
        next = block_reduce<uint32_t, OpMin>(next, sc);
        if (threadIdx.x == 0) {
            if (end_b) atomicMax(&P.totals->pass_bytes[0], (unsigned long long)end_b);
            if (end_c) atomicMax(&P.totals->pass_desc[0], end_c);
            if (next != kNoPass) atomicMin(&P.totals->pass_next[0], next);
        }
    }
    // work items: one wave per sender (waves stride over senders), one lane per chunk.  Chunk
    // k covers packets [umin + k * chunk, min(umin + (k + 1) * chunk, head)), so every lane
    // loads its two boundary records at once instead of walking the chunks one by one.
    // the wave's senders are gw, gw + nwaves, ...: lane j reserves the items of the j-th.  The
    // block's reservations are one atomicAdd on the tick's item count, its lanes' bases a block
    // scan: one same-address atomic per block instead of one per sender (4096 serialised at one
    // L2 channel, each lane waiting for its return, were most of this kernel's fixed ~14 us)
    {
        __shared__ uint32_t s_wbase;
        uint32_t tot;
        const uint32_t pre = block_exclusive_scan<uint32_t>(res_nch, sc, tot);
        if (threadIdx.x == 0) s_wbase = tot ? atomicAdd(&P.totals->nwork, tot) : 0u;
        __syncthreads();
        res_base = s_wbase + pre;
    }
    uint32_t j = 0;
    for (uint32_t s = gw; s < P.T.nsenders; s += nwaves, j++) {
        const SenderDev& D = P.senders[s];
        const PktMeta* meta = reinterpret_cast<const PktMeta*>(D.meta);
        const uint64_t head = D.head, umin = D.umin, vend = D.vbyte_end;
        const uint32_t pkmask = D.pk_mask;
        uint32_t nch, chunk_base = 0;
        if (j < 64) {
            nch = (uint32_t)__shfl((int)res_nch, (int)j, 64);
            chunk_base = (uint32_t)__shfl((int)res_base, (int)j, 64);
        } else {
            nch = chunks_of(D);
            if (lane == 0 && nch) chunk_base = atomicAdd(&P.totals->nwork, nch);
            chunk_base = (uint32_t)__shfl((int)chunk_base, 0, 64);
        }
        if (lane == 0) {
            SenderDev& Dw = P.senders[s];
            Dw.fan_lo = nch ? umin : head;
            Dw.fan_vlo = nch ? meta[umin & pkmask].vbyte : vend;
        }
        FanWork it;
        it.ring = D.ring; it.meta = D.meta; it.wmask = D.word_mask; it.pkmask = pkmask;
        it.sender = s; it.qb = P.sub_range[2 * s]; it.qe = P.sub_range[2 * s + 1];
        for (uint32_t k = lane; k < nch; k += 64) {
            const uint64_t lo = umin + (uint64_t)k * P.T.chunk;
            const uint64_t hi = min(lo + P.T.chunk, head);
            const PktMeta& m = meta[lo & pkmask];
            const uint64_t vb0 = m.vbyte;
            const uint32_t vc0 = m.vcount;
            const uint64_t vb1 = hi < head ? meta[hi & pkmask].vbyte : vend;
            it.np = (uint32_t)(hi - lo);
            it.nw = (uint32_t)((vb1 - vb0) >> 4);
            it.vc0 = vc0;
            it.lo = lo;
            it.vb0 = vb0;
            P.work[chunk_base + k] = it;
        }
    }
}

// A later copy pass of an over-capacity tick (edgpu_fanout_next): the rows of pass T.pass_id
// become the tick's visible sub-streams and the copy kernel's targets (FanSub.a; every other
// row's record is skipped), with the pass's extent and the next pass id in slot pass_ord & 1.
// The work items and the FanSub offsets planned for the tick are reused as they are.
__global__ __launch_bounds__(256) void k_plan_pass(PlanParams P) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t slot = P.T.pass_ord & 1u;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        P.totals->fan_next = 0;                       // the copy kernel claims items from 0 again
        P.totals->pass_slot = slot;
        P.totals->pass_bytes[slot ^ 1u] = 0; P.totals->pass_desc[slot ^ 1u] = 0;
        P.totals->pass_next[slot ^ 1u] = kNoPass;     // for the pass after this one
    }
    __shared__ uint64_t sb[4];
    __shared__ uint32_t sc[4];
    uint64_t end_b = 0; uint32_t end_c = 0, next = kNoPass;
    if (q < P.T.nsubs) {
        const SubDev& Q = P.subs[q];
        const bool in = Q.pass == P.T.pass_id;
        edgpu_substream_out& o = P.sub_out[q];
        o.desc_base = Q.desc_base;
        o.out_base = Q.out_base;
        o.desc_count = in ? Q.count : 0u;
        o.out_bytes = in ? Q.bytes : 0ull;
        if (in) { end_b = Q.out_base + Q.bytes; end_c = Q.desc_base + Q.count; }
        else if (Q.count > 0 && Q.pass > P.T.pass_id) next = Q.pass;
        const uint32_t pos = P.sub_pos[q];
        if (pos != 0xFFFFFFFFu) P.fansub[pos].a = (in && Q.nonempty) ? Q.a : ~0ull;
    }
    end_b = block_reduce<uint64_t, OpMax>(end_b, sb);
    end_c = block_reduce<uint32_t, OpMax>(end_c, sc);
    next = block_reduce<uint32_t, OpMin>(next, sc);
    if (threadIdx.x == 0) {
        if (end_b) atomicMax(&P.totals->pass_bytes[slot], (unsigned long long)end_b);
        if (end_c) atomicMax(&P.totals->pass_desc[slot], end_c);
        if (next != kNoPass) atomicMin(&P.totals->pass_next[slot], next);
    }
}

// Egress backpressure (edgpu_fanout_blocked): one lane per report.  The sub-stream's tick
// wrote the non-empty packets of [a, head) in order; the socket took the first `sent`.
// SendPacketsToOutput stopped at the next one (ReflectorStream.cpp:1138-1198): it becomes the
// bookmark, relocated to the key frame when too old (NeedRelocateBookMark, :1293-1322, Q9);
// the stream's last-sent id is the last packet written (RTPSessionOutput.cpp:620-639).
__global__ void k_blocked(BlockedParams P) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    const edgpu_blocked b = P.reports[i];
    SubDev& Q = P.subs[b.substream];
    if (!Q.nonempty || b.sent >= Q.count) return;
    const SenderDev& D = P.senders[Q.sender];
    const PktMeta* meta = reinterpret_cast<const PktMeta*>(D.meta);
    const uint64_t head = D.head;
    // vcount = non-empty packets before a packet: the k-th written packet is the first whose
    // inclusive count exceeds vcstart + k
    auto kth = [&](uint32_t k) {
        return lower_bound_meta(meta, D.pk_mask, Q.a, head, [&](const PktMeta& m) {
            return m.vcount + (m.len != 0 ? 1u : 0u) > Q.vcstart + k; });
    };
    const uint64_t x = kth(b.sent);
    if (b.sent > 0) {
        Q.last_id = meta[kth(b.sent - 1) & D.pk_mask].id;
        Q.has_last = 1;
    } else {
        Q.last_id = Q.prev_last_id;
        Q.has_last = Q.prev_has_last;
        Q.sent_any = Q.prev_sent_any;
    }
    uint64_t unsent_bytes = 0;
    for (uint64_t k = x; k < head; k++) {
        const uint32_t len = meta[k & D.pk_mask].len;
        if (len) unsent_bytes += len + (Q.transport ? 4u : 0u);
    }
    const unsigned long long np = Q.count - b.sent;
    atomicAdd(&P.totals->relayed_packets, 0ull - np);
    atomicAdd(&P.totals->cum_relayed_packets, 0ull - np);
    atomicAdd(&P.totals->relayed_bytes, 0ull - unsent_bytes);
    atomicAdd(&P.totals->cum_relayed_bytes, 0ull - unsent_bytes);
    int64_t bm = (int64_t)x;
    const PktMeta mx = meta[x & D.pk_mask];
    if (P.now - mx.arrival > P.relocate_ms && D.key >= 0 && meta[(uint64_t)D.key & D.pk_mask].arrival > mx.arrival) {
        bm = D.key;
        atomicExch(&P.sessions[D.session].video_key_flag, 1u);
        atomicExch(&P.sessions[D.session].relocated, 1u);
    }
    Q.bookmark = bm;
    Q.resume_at = 1;
}

// =========================================================================================
// Fan-out
// =========================================================================================

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}

// -----------------------------------------------------------------------------------------
// k_fanout3: LDS-staged, line-aligned write-many.  The chunk is loaded from HBM into LDS once;
// for every sub-stream each lane then reads the word that lands on its lane of a 128-B-
// aligned destination window (the realignment is a per-sub-stream shift of the LDS read
// index), so every 1 KiB wave store covers whole cache lines.  A 16-B misaligned
// destination costs ~30 % of write bandwidth on MI355X (tools/store_peak2.hip), and the
// sub-streams' pieces start at arbitrary 16-B offsets.  TCP channel bytes are patched in
// registers before the single store.
// -----------------------------------------------------------------------------------------
template <int THREADS, int CHUNK>
constexpr int fanout3_lds() {
    return CHUNK * 129 * 16 + (CHUNK + 2) * 8 + CHUNK * 16 + ((((CHUNK * 129 + 31) / 32) + 3) & ~3) * 4 +
           (THREADS < 256 ? THREADS : 256) * 36 + (THREADS / 64) * 8;
}

template <int THREADS, int CHUNK>
__global__ __attribute__((amdgpu_flat_work_group_size(1, THREADS)))
void k_fanout3(FanoutParams P) {
    constexpr int CWORDS = CHUNK * 129;
    constexpr int NW = (CWORDS + 7 + THREADS - 1) / THREADS;
    constexpr int NWAVES = THREADS / 64;
    constexpr int QB = THREADS < 256 ? THREADS : 256;                  // sub-streams per LDS batch
    const uint32_t nwork = P.totals->nwork;
    if (P.totals->status == EDGPU_OUT_OVERFLOW) return;
    const int tid = threadIdx.x;
    // All LDS is one dynamic region carved at 16-B-aligned offsets (Guideline 17: no static
    // __shared__ in front of it), so the ds_read_b128 of the chunk words stay aligned.
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int SM = ((CWORDS + 31) / 32 + 3) & ~3;                  // startmap words, x4
    u32x4* cbuf = reinterpret_cast<u32x4*>(lds);                       // CWORDS words
    uint64_t* m_vb = reinterpret_cast<uint64_t*>(cbuf + CWORDS);       // CHUNK + 2
    uint32_t* m_id = reinterpret_cast<uint32_t*>(m_vb + CHUNK + 2);    // CHUNK (multiple of 4)
    uint32_t* m_len = m_id + CHUNK;
    uint32_t* m_vc = m_len + CHUNK;
    uint32_t* m_nzp = m_vc + CHUNK;                                    // CHUNK: ordinal -> packet
    uint32_t* startmap = m_nzp + CHUNK;                                // SM
    int64_t* q_dw0 = reinterpret_cast<int64_t*>(startmap + SM);        // QB
    int64_t* q_off = q_dw0 + QB;
    uint32_t* q_fw = reinterpret_cast<uint32_t*>(q_off + QB);
    uint32_t* q_ch = q_fw + QB;
    uint32_t* q_db = q_ch + QB;
    uint32_t* q_p0 = q_db + QB;
    uint32_t* q_hl = q_p0 + QB;
    unsigned long long* s_red = reinterpret_cast<unsigned long long*>(q_hl + QB);   // NWAVES
    unsigned long long wire = 0, inb = 0;
    u32x4* out = reinterpret_cast<u32x4*>(P.arena);

    for (uint32_t w = blockIdx.x; w < nwork; w += gridDim.x) {
        const FanWork it = P.work[w];
        const SenderDev& D = P.senders[it.sender];
        const uint64_t lo = it.lo;
        const uint64_t head = D.head;
        const uint32_t np = (uint32_t)min((uint64_t)CHUNK, head - lo);
        const PktMeta* meta = reinterpret_cast<const PktMeta*>(D.meta);
        if (tid < (int)np) {
            const PktMeta m = meta[(lo + tid) & D.pk_mask];
            m_vb[tid] = m.vbyte; m_id[tid] = (uint32_t)m.id; m_len[tid] = m.len; m_vc[tid] = m.vcount;
            inb += m.len;
        }
        if (tid == (int)np) m_vb[np] = (lo + np == head) ? D.vbyte_end : meta[(lo + np) & D.pk_mask].vbyte;
        for (int k = tid; k < (int)((CWORDS + 31) / 32); k += THREADS) startmap[k] = 0;
        __syncthreads();
        const uint64_t vb0 = m_vb[0];
        const uint32_t nw = uni((uint32_t)((m_vb[np] - vb0) >> 4));
        if (tid < (int)np && m_len[tid] != 0) {
            const uint32_t sw = (uint32_t)((m_vb[tid] - vb0) >> 4);
            atomicOr(&startmap[sw >> 5], 1u << (sw & 31));
            m_nzp[m_vc[tid] - m_vc[0]] = tid;              // non-empty ordinal -> packet
        }
        // chunk HBM -> LDS (buffer loads, one 32-bit offset per lane; wrap handled per word)
        {
            const uint32_t wmask = uni(D.word_mask);
            const uint32_t rstart = uni((uint32_t)((vb0 >> 4) & wmask));
            const bool wraps = rstart + nw > wmask + 1;
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                reinterpret_cast<u32x4*>(D.ring) + (wraps ? 0u : rstart), 0,
                wraps ? (wmask + 1) * 16 : nw * 16, 0x00020000);
#pragma unroll
            for (int j = 0; j < (CWORDS + THREADS - 1) / THREADS; j++) {
                const uint32_t wi = tid + j * THREADS;
                if (wi < nw)
                    cbuf[wi] = __builtin_amdgcn_raw_buffer_load_b128(
                        rs, (wraps ? ((rstart + wi) & wmask) : wi) * 16u, 0, 0);
            }
        }
        const uint32_t qb = P.sub_range[2 * it.sender], qe = P.sub_range[2 * it.sender + 1];
        for (uint32_t q0 = qb; q0 < qe; q0 += QB) {
            const uint32_t nq = min((uint32_t)QB, qe - q0);
            if (tid < (int)nq) {
                const SubDev& Q = P.subs[P.sub_index[q0 + tid]];
                uint32_t fw = 0xFFFFFFFFu, p0 = 0xFFFFFFFFu;
                if (Q.nonempty && Q.a < lo + np) {
                    const uint64_t first = Q.a > lo ? Q.a : lo;
                    p0 = (uint32_t)(first - lo);
                    fw = (uint32_t)((m_vb[p0] - vb0) >> 4);
                }
                q_fw[tid] = fw;
                q_p0[tid] = p0;
                q_dw0[tid] = (int64_t)(Q.out_base >> 4) + ((int64_t)(vb0 - Q.vstart) >> 4);
                q_off[tid] = (int64_t)(Q.out_base - Q.vstart) + (Q.transport ? 0 : 4);
                q_ch[tid] = Q.transport ? ((uint32_t)Q.channel << 8) : 0u;
                q_db[tid] = Q.desc_base - Q.vcstart;
                q_hl[tid] = Q.transport ? 4u : 0u;
            }
            __syncthreads();
            for (uint32_t q = 0; q < nq && !(EDGPU_ABL(P) & 2u); q++) {
                const uint32_t fw = uni(q_fw[q]);
                if (fw >= nw) continue;
                const int64_t A = (int64_t)uni64((uint64_t)q_dw0[q]) + fw;     // first dest word
                const uint32_t s = (uint32_t)(A & 7);                          // words past a 128-B line
                // descriptor from the exact first word; lanes below it get a wrapped (huge)
                // offset and are dropped by the range check, as are lanes past the chunk
                const __amdgpu_buffer_rsrc_t os = __builtin_amdgcn_make_buffer_rsrc(
                    out + A, 0, (nw - fw) * 16, 0x00020000);
                const uint32_t chbits = uni(q_ch[q]);
#pragma unroll
                for (int j = 0; j < NW; j++) {
                    const uint32_t lane_w = tid + j * THREADS;               // word in the aligned window
                    const uint32_t src = fw + lane_w - s;                    // chunk word it carries
                    const uint32_t srcc = src < (uint32_t)CWORDS ? src : 0u;
                    u32x4 v = cbuf[srcc];
                    if (chbits && ((startmap[srcc >> 5] >> (srcc & 31)) & 1u)) v.x |= chbits;
                    __builtin_amdgcn_raw_buffer_store_b128(v, os, (lane_w - s) * 16u, 0, 0);
                }
            }
            // descriptors: one wave per sub-stream, lanes mapped onto a 128-B-aligned window of
            // the sub-stream's descriptor array (8 descriptors per line)
            {
                const int lane = tid & 63, wv = tid >> 6;
                // non-empty packets of this chunk: ordinals [0, nzc)
                const uint32_t nzc = (uint32_t)__builtin_amdgcn_readfirstlane(
                    (int)(np ? m_vc[np - 1] - m_vc[0] + (m_len[np - 1] != 0) : 0));
                for (uint32_t q = wv; q < (EDGPU_ABL(P) & 1u ? 0u : nq); q += NWAVES) {
                    const uint32_t p0 = q_p0[q];
                    if (p0 >= np) continue;
                    const uint32_t o0 = m_vc[p0] - m_vc[0];                   // first ordinal
                    if (o0 >= nzc) continue;
                    const uint32_t d0 = q_db[q] + m_vc[p0];                   // its descriptor
                    const uint32_t sh = d0 & 7;
                    const uint32_t o = o0 + lane - sh;                        // ordinal of this lane
                    if (lane >= (int)sh && o < nzc) {
                        const uint32_t p = m_nzp[o];
                        const uint32_t len = m_len[p];
                        const uint64_t off = (uint64_t)(q_off[q] + (int64_t)m_vb[p]);
                        const uint32_t wlen = len + q_hl[q];
                        u32x4 dv;
                        dv.x = (uint32_t)off; dv.y = (uint32_t)(off >> 32); dv.z = wlen; dv.w = m_id[p];
                        if (d0 - sh + lane < P.max_desc) reinterpret_cast<u32x4*>(P.desc)[d0 - sh + lane] = dv;
                        wire += wlen;
                    }
                }
            }
            __syncthreads();
        }
    }
    unsigned long long a = wire, b = inb;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { a += __shfl_down(a, o, 64); b += __shfl_down(b, o, 64); }
    if ((tid & 63) == 0) s_red[tid >> 6] = a;
    __syncthreads();
    if (tid == 0) {
        unsigned long long tot = 0;
        for (int i = 0; i < NWAVES; i++) tot += s_red[i];
        if (tot) { atomicAdd(&P.totals->relayed_bytes, tot); atomicAdd(&P.totals->cum_relayed_bytes, tot); }
    }
    __syncthreads();
    if ((tid & 63) == 0) s_red[tid >> 6] = b;
    __syncthreads();
    if (tid == 0) {
        unsigned long long tot = 0;
        for (int i = 0; i < NWAVES; i++) tot += s_red[i];
        if (tot) atomicAdd(&P.totals->cum_fanout_in_bytes, tot);
    }
}

// -----------------------------------------------------------------------------------------
// k_fanout4: k_fanout3's line-aligned LDS write-many, restructured so that loading a chunk never
// stalls the store stream.
//   * Everything a work item needs before its loads comes from one 64-B FanWork record
//     (k_plan_final), read through the constant address space, so it lands in SGPRs: the
//     ring's buffer resource is scalar and the chunk's 16-B loads issue back to back.
//     (k_fanout3 built that resource from a per-lane load, which the compiler lowers to a
//     waterfall loop that waits for every load in turn.)
//   * Sub-stream parameters are one 48-B FanSub per sub-stream in sender order, also scalar
//     loads: no sub_index -> SubDev chain and no per-sender LDS batch.
//   * The NEXT item's chunk words and packet metadata are loaded into registers as soon as
//     this item's LDS image is complete, so their HBM latency runs under this item's stores;
//     the LDS image is refilled from those registers after the end-of-item barrier.
//   * The slot-start bitmap (TCP channel patch) is double-buffered by item parity, so
//     clearing it needs no extra barrier.
// Stores: per sub-stream, lanes walk the destination in whole 128-B lines (k_fanout3), with a
// uniform trip count, so no store instruction is issued for words past the chunk.
// -----------------------------------------------------------------------------------------
// Loads a record written by an earlier kernel through the constant address space: uniform
// addresses become scalar (s_load) loads, whose results live in SGPRs.
template <typename T>
__device__ __forceinline__ T const_load(const T* p) {
    typedef __attribute__((address_space(4))) const uint32_t cu32;
    static_assert(sizeof(T) % 4 == 0, "");
    T v;
    uint32_t* d = reinterpret_cast<uint32_t*>(&v);
    cu32* src = (cu32*)p;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); i++) d[i] = src[i];
    return v;
}

// The per-output patch of one 16-B arena word (word `w` of the chunk's LDS image `cb`, slot
// starts marked in bitmap `sm`): the RTSP-interleaved channel byte (RTSPSessionInterface.cpp:
// 329-336) and the rewrite stage (kRw*).  A slot's first word holds the 4-B '$' 0 BE16(len)
// header and packet bytes 0..11: RTP seq (bytes 2-3), timestamp (4-7) and SSRC (8-11), or an
// RTCP packet's sender SSRC (4-7); an SR's RTP timestamp (packet bytes 16-19) is in the second
// word.  Fields past the packet's length are left alone; CSRC lists and extensions are never
// touched.
// The patched form of a slot's first word (computed for every lane, selected by `start`).
__device__ __forceinline__ u32x4 fan_patch_start(u32x4 v, const FanSub& f, bool start) {
    u32x4 p = v;
    if (f.ch & 1u) p.x |= f.ch & 0xFF00u;
    if (f.rw) {
        const uint32_t len = ((v.x >> 8) & 0xFF00u) | (v.x >> 24);
        if (!(f.rw & kRwRtcp)) {
            const bool ok = len >= 12;
            const uint32_t seq = (((v.y >> 8) & 0xFF00u) | (v.y >> 24)) + (f.rw >> 16);
            const uint32_t ny = (v.y & 0xFFFFu) | ((seq >> 8) & 0xFFu) << 16 | (seq & 0xFFu) << 24;
            const uint32_t nz = __builtin_bswap32(__builtin_bswap32(v.z) + f.rw_ts);
            p.y = ok ? ny : v.y;
            p.z = ok ? nz : v.z;
            if (f.rw & kRwSsrc) p.w = ok ? f.rw_ssrc_be : v.w;
        } else if (f.rw & kRwSsrc) {
            p.z = len >= 8 ? f.rw_ssrc_be : v.z;
        }
    }
    return start ? p : v;
}

// The per-output patch of one 16-B arena word (word `w` of the chunk's LDS image `cb`, slot
// starts marked in bitmap `sm`): the RTSP-interleaved channel byte (RTSPSessionInterface.cpp:
// 329-336) and the rewrite stage (kRw*).  A slot's first word holds the 4-B '$' 0 BE16(len)
// header and packet bytes 0..11: RTP seq (bytes 2-3), timestamp (4-7) and SSRC (8-11), or an
// RTCP packet's sender SSRC (4-7); an SR's RTP timestamp (packet bytes 16-19) is in the second
// word.  Fields past the packet's length are left alone; CSRC lists and extensions are never
// touched.  Branch-free on the per-word test; the flags (f.ch, f.rw) are uniform.
__device__ __forceinline__ u32x4 fan_patch(u32x4 v, const FanSub& f, uint32_t w, const uint32_t* sm, const u32x4* cb) {
    const bool start = (sm[w >> 5] >> (w & 31)) & 1u;
    if ((f.rw & kRwRtcp) && !start && w > 0 && ((sm[(w - 1) >> 5] >> ((w - 1) & 31)) & 1u)) {   // RTCP only: rare
        const u32x4 h = cb[w - 1];
        const uint32_t hl = ((h.x >> 8) & 0xFF00u) | (h.x >> 24);
        if (hl >= 20 && ((h.y >> 8) & 0xFFu) == 200u) v.y = __builtin_bswap32(__builtin_bswap32(v.y) + f.rw_ts);
    }
    return fan_patch_start(v, f, start);
}

// fan_patch with the slot-start test as a divergent branch: the patch arithmetic runs only on
// lanes that hold a slot's first word (and only in waves that have one), in place, with no
// per-dword selects.  Same result as fan_patch.
__device__ __forceinline__ u32x4 fan_patch_branchy(u32x4 v, const FanSub& f, uint32_t w, const uint32_t* sm,
                                                   const u32x4* cb) {
    const bool start = (sm[w >> 5] >> (w & 31)) & 1u;
    if ((f.rw & kRwRtcp) && !start && w > 0 && ((sm[(w - 1) >> 5] >> ((w - 1) & 31)) & 1u)) {   // RTCP only: rare
        const u32x4 h = cb[w - 1];
        const uint32_t hl = ((h.x >> 8) & 0xFF00u) | (h.x >> 24);
        if (hl >= 20 && ((h.y >> 8) & 0xFFu) == 200u) v.y = __builtin_bswap32(__builtin_bswap32(v.y) + f.rw_ts);
    }
    if (start) {
        if (f.ch & 1u) v.x |= f.ch & 0xFF00u;
        if (f.rw) {
            const uint32_t len = ((v.x >> 8) & 0xFF00u) | (v.x >> 24);
            if (!(f.rw & kRwRtcp)) {
                if (len >= 12) {
                    const uint32_t seq = (((v.y >> 8) & 0xFF00u) | (v.y >> 24)) + (f.rw >> 16);
                    v.y = (v.y & 0xFFFFu) | ((seq >> 8) & 0xFFu) << 16 | (seq & 0xFFu) << 24;
                    v.z = __builtin_bswap32(__builtin_bswap32(v.z) + f.rw_ts);
                    if (f.rw & kRwSsrc) v.w = f.rw_ssrc_be;
                }
            } else if ((f.rw & kRwSsrc) && len >= 8) {
                v.z = f.rw_ssrc_be;
            }
        }
    }
    return v;
}

// Bits [c0, c0 + 64) of a slot-start bitmap of `nw32` words as one wave-uniform mask (bit l =
// word c0 + l; words before 0 or past the bitmap read as 0).  Every lane reads the same three
// LDS words (a broadcast), so the per-word test becomes a shift of an SGPR pair.
__device__ __forceinline__ uint64_t row_mask(const uint32_t* sm, int c0, int nw32) {
    const int b = c0 >> 5, sh = c0 & 31;
    auto word = [&](int i) -> uint64_t { return (i >= 0 && i < nw32) ? (uint64_t)sm[i] : 0ull; };
    const uint64_t lo = word(b) | word(b + 1) << 32, hi = word(b + 2);
    return (lo >> sh) | (sh ? hi << (64 - sh) : 0ull);
}

// LFS: FanSub records staged in LDS per work item (up to kLfs), so the store loop's per-window
// record read is an LDS broadcast instead of a scalar load that can miss the scalar cache
constexpr int kLfs = 64;
template <int THREADS, int CHUNK, int LFS = 0>
constexpr int fanout4_lds() {
    return CHUNK * kSlotWordsMax * 16 + (CHUNK + 2) * 8 + 4 * CHUNK * 4 +
           2 * ((((CHUNK * kSlotWordsMax + 31) / 32) + 3) & ~3) * 4 + (THREADS / 64) * 8 +
           (LFS ? kLfs * (int)sizeof(FanSub) : 0);
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));

// Issues one work item's loads into registers: the chunk's slot words (NL per lane) and, for
// lanes < np, the packet's metadata as raw words (ma = vbyte, id low; mb = len, vcount), decoded
// only when the LDS image is written, so the registers stay exactly as loaded while the loads
// are in flight.  All are buffer loads (vector-memory counter only; a flat load would also hold
// the LDS counter that the store loop waits on).
template <int THREADS, int NL, int LAUX = 0>
__device__ __forceinline__ void fan4_issue(const FanWork& it, int tid, u32x4 (&r)[NL], u32x3& ma, u32x2& mb,
                                           bool skip_words = false) {
    const uint32_t wmask = it.wmask, nw = it.nw;
    const uint32_t rstart = (uint32_t)(it.vb0 >> 4) & wmask;
    const bool wraps = rstart + nw > wmask + 1;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<u32x4*>(it.ring) + (wraps ? 0u : rstart), 0, wraps ? (wmask + 1) * 16 : nw * 16, 0x00020000);
#pragma unroll
    for (int j = 0; j < NL; j++) {
        const uint32_t wi = tid + j * THREADS;
        if ((uint32_t)(j * THREADS) < nw && !skip_words)   // uniform: no load past the chunk's lines
            r[j] = __builtin_amdgcn_raw_buffer_load_b128(
                rs, wraps ? (wi < nw ? ((rstart + wi) & wmask) * 16u : 0xFFFFFFFFu) : wi * 16u, 0, LAUX);
    }
    const __amdgpu_buffer_rsrc_t ms = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(it.meta), 0, (it.pkmask + 1) * (uint32_t)sizeof(PktMeta), 0x00020000);
    const uint32_t mo = (uint32_t)tid < it.np ? (uint32_t)((it.lo + tid) & it.pkmask) * (uint32_t)sizeof(PktMeta) : 0xFFFFFFE0u;
    ma = __builtin_amdgcn_raw_buffer_load_b96(ms, mo, 0, 0);
    mb = __builtin_amdgcn_raw_buffer_load_b64(ms, mo + 24u, 0, 0);
}

// AUX: cache policy of the arena stores (0 plain; A/B variants: 2 nt, 16 sc1, 17 sc0 sc1);
// DNT: non-temporal descriptor stores; LAUX: cache policy of the chunk loads.
// SU: store-loop unroll (SU LDS reads in flight before the SU stores of a sub-stream window;
// needs the VGPRs of 1 workgroup per CU at 1024 threads)
// WPE: minimum waves per SIMD the register allocation must allow (8 = two 1024-thread
// workgroups per CU, i.e. <= 64 VGPRs); 0 leaves it to the compiler.
// PM: how the store loop finds slot starts for the per-output patch: 0 one bitmap bit per lane
// (LDS read per word), 1 one wave-uniform 64-bit mask per wave row (row_mask).
// DYN: work items claimed from a tick-global counter (one atomic per item, two items ahead of
// use) instead of a static stride over blockIdx, so unequal items cannot leave a long tail.
// PACE (A/B of store issue rate): 1 every window takes the patch path (an identity window then
// pays the rewrite's bitmap read per word); 2 s_sleep after every store row.
// HW: the two halves of the workgroup write two sub-streams' windows at once (each half walks
// its window with THREADS/2 lanes), so one window's record / offset chain overlaps the other's
// stores.
template <int THREADS, int CHUNK, int AUX = 0, int DNT = 0, int LAUX = 0, int SU = 1, int WPE = 0, int PM = 0,
          int LFS = 0, int DYN = 0, int PACE = 0, int HW = 0>
__global__ __attribute__((amdgpu_flat_work_group_size(1, THREADS), amdgpu_waves_per_eu(WPE ? WPE : 1)))
void k_fanout4(FanoutParams P) {
    constexpr int CWORDS = CHUNK * kSlotWordsMax;
    constexpr int NL = (CWORDS + THREADS - 1) / THREADS;              // chunk words per lane
    constexpr int NWAVES = THREADS / 64;
    constexpr int SM = ((CWORDS + 31) / 32 + 3) & ~3;                  // bitmap words, x4
    static_assert(CHUNK <= 56, "descriptor windows assume one wave covers a chunk's packets");
    const uint32_t nwork = uni(P.totals->nwork);
    if (uni((uint32_t)P.totals->status) == (uint32_t)EDGPU_OUT_OVERFLOW) return;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const uint32_t wv = uni((uint32_t)tid >> 6);
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    u32x4* cbuf = reinterpret_cast<u32x4*>(lds);                       // CWORDS words
    uint64_t* m_vb = reinterpret_cast<uint64_t*>(cbuf + CWORDS);       // CHUNK + 2
    uint32_t* m_id = reinterpret_cast<uint32_t*>(m_vb + CHUNK + 2);
    uint32_t* m_len = m_id + CHUNK;
    uint32_t* m_vc = m_len + CHUNK;
    uint32_t* m_nzp = m_vc + CHUNK;                                    // non-empty ordinal -> packet
    uint32_t* smap = m_nzp + CHUNK;                                    // 2 x SM, by item parity
    unsigned long long* s_red = reinterpret_cast<unsigned long long*>(smap + 2 * SM);
    uint32_t* s_fs = reinterpret_cast<uint32_t*>(s_red + NWAVES);       // LFS: kLfs FanSub records
    constexpr uint32_t kFsw = sizeof(FanSub) / 4;                      // dwords per record
    static_assert(!LFS || kLfs * kFsw <= (uint32_t)THREADS, "one staged dword per lane");
    // the item's FanSub q as SGPRs: from the LDS copy (LFS) or a scalar load
    auto fansub = [&](const FanWork& w, uint32_t q) -> FanSub {
        if constexpr (LFS) {
            if (q - w.qb < (uint32_t)kLfs) {
                FanSub f;
                uint32_t* d = reinterpret_cast<uint32_t*>(&f);
                const uint32_t* src = s_fs + (q - w.qb) * kFsw;
#pragma unroll
                for (uint32_t i = 0; i < kFsw; i++) d[i] = (uint32_t)__builtin_amdgcn_readfirstlane((int)src[i]);
                return f;
            }
        }
        return const_load(P.fansub + q);
    };
    uint32_t fsw = 0;                                                  // LFS: this lane's staged dword
    u32x4* out = reinterpret_cast<u32x4*>(P.arena);
    unsigned long long wire = 0, inb = 0;

    for (int k = tid; k < 2 * SM; k += THREADS) smap[k] = 0;
    u32x4 r[NL];
    u32x3 ma;
    u32x2 mb;
    // DYN: s_claim[par] holds the item claimed for use two items later (written by thread 0
    // after an image barrier, read by everyone after the next one)
    __shared__ uint32_t s_claim[2];
    uint32_t w = blockIdx.x;
    if constexpr (DYN) {
        if (tid == 0) {
            s_claim[0] = atomicAdd(&P.totals->fan_next, 1u);
            s_claim[1] = atomicAdd(&P.totals->fan_next, 1u);
        }
        __syncthreads();
        w = s_claim[0];
    }
    FanWork nx;
    if (w < nwork) {
        nx = const_load(P.work + w);
        fan4_issue<THREADS, NL, LAUX>(nx, tid, r, ma, mb, (EDGPU_ABL(P) & 4u) != 0);
        if constexpr (LFS) {
            const uint32_t nq = min(nx.qe - nx.qb, (uint32_t)kLfs);
            if ((uint32_t)tid < nq * kFsw) fsw = reinterpret_cast<const uint32_t*>(P.fansub + nx.qb)[tid];
        }
    }
    uint32_t wnext = DYN ? s_claim[1] : 0u;      // DYN: the item to prefetch during this one
    uint32_t wpref = 0;                          // the item whose loads are in flight
    for (uint32_t par = 0; w < nwork; w = wpref, par ^= 1u) {
        const FanWork it = nx;
        const uint64_t lo = it.lo, vb0 = it.vb0;
        const uint32_t np = it.np, nw = it.nw, vc0 = it.vc0;
        uint32_t* sm = smap + par * SM;
        // ---- this item's LDS image, from the registers loaded one item earlier ----------
#pragma unroll
        for (int j = 0; j < NL; j++) {
            const uint32_t wi = tid + j * THREADS;
            if ((uint32_t)(j * THREADS) < nw && wi < nw) cbuf[wi] = r[j];
        }
        if ((uint32_t)tid < np) {
            const uint64_t vbyte = (uint64_t)ma.y << 32 | ma.x;
            const uint32_t len = mb.x & 0xFFFFu, vcount = mb.y;          // len:16 | seq:16
            m_vb[tid] = vbyte; m_id[tid] = ma.z; m_len[tid] = len; m_vc[tid] = vcount;
            inb += len;
            if (len != 0) {
                const uint32_t sw = (uint32_t)((vbyte - vb0) >> 4);
                atomicOr(&sm[sw >> 5], 1u << (sw & 31));
                m_nzp[vcount - vc0] = tid;
            }
        }
        if (tid == 0) m_vb[np] = vb0 + (uint64_t)nw * 16;
        if constexpr (LFS) {
            if ((uint32_t)tid < min(it.qe - it.qb, (uint32_t)kLfs) * kFsw) s_fs[tid] = fsw;
        }
        __syncthreads();
        // ---- the other parity's bitmap is free now: clear it for the next item ----------
        for (int k = tid; k < SM; k += THREADS) smap[(par ^ 1u) * SM + k] = 0;
        // ---- next item's loads, in flight under this item's stores ------------------------
        uint32_t wn = w + gridDim.x;
        if constexpr (DYN) {
            wn = wnext;                                            // claimed one item ago
            if (tid == 0) s_claim[par] = atomicAdd(&P.totals->fan_next, 1u);   // for the item after it
        }
        wpref = wn;
        if (wn < nwork) {
            nx = const_load(P.work + wn);
            fan4_issue<THREADS, NL, LAUX>(nx, tid, r, ma, mb, (EDGPU_ABL(P) & 4u) != 0);
            if constexpr (LFS) {
                const uint32_t nq = min(nx.qe - nx.qb, (uint32_t)kLfs);
                if ((uint32_t)tid < nq * kFsw) fsw = reinterpret_cast<const uint32_t*>(P.fansub + nx.qb)[tid];
            }
        }
        // ---- write the chunk to every sub-stream of the sender ----------------------------
        constexpr uint32_t WT = HW ? THREADS / 2 : THREADS;                    // lanes per window
        const uint32_t wtid = HW ? (uint32_t)tid % WT : (uint32_t)tid;
        const uint32_t q0 = HW ? uni((uint32_t)tid / WT) : 0u;
        for (uint32_t q = it.qb + q0; q < it.qe && !(EDGPU_ABL(P) & 2u); q += HW ? 2u : 1u) {
            const FanSub f = fansub(it, q);
            if (f.a >= lo + np) continue;
            const uint32_t p0 = f.a > lo ? (uint32_t)(f.a - lo) : 0u;
            const uint32_t fw = uni((uint32_t)((m_vb[p0] - vb0) >> 4));
            const int64_t A = f.dw + (int64_t)(vb0 >> 4) + fw;                 // first dest word
            if (A < 0 || (uint64_t)A + (nw - fw) > P.arena_words) { set_status(&P.totals->status, EDGPU_OUT_OVERFLOW); continue; }
            const uint32_t s = (uint32_t)(A & 7);                              // words past a line
            const __amdgpu_buffer_rsrc_t os = __builtin_amdgcn_make_buffer_rsrc(out + A, 0, (nw - fw) * 16, 0x00020000);
            const bool patch = PACE == 1 || (f.ch & 1u) || f.rw;               // uniform
            const uint32_t nj = (nw - fw + s + WT - 1) / WT;
            for (uint32_t j = 0; j < nj; j += SU) {
                u32x4 v[SU];
                uint32_t srcc[SU];
#pragma unroll
                for (int k = 0; k < SU; k++) {
                    const uint32_t src = fw + wtid + (j + k) * WT - s;         // chunk word of the lane's
                    srcc[k] = src < (uint32_t)CWORDS ? src : 0u;               // word of the aligned window
                    if (k == 0 || j + k < nj) v[k] = cbuf[srcc[k]];            // uniform guard
                }
#pragma unroll
                for (int k = 0; k < SU; k++) {
                    if (k > 0 && j + k >= nj) break;
                    if (patch) {
                        if (PM == 0 || (f.rw & kRwRtcp)) {
                            v[k] = fan_patch(v[k], f, srcc[k], sm, cbuf);
                        } else {
                            const int c0 = (int)(fw + (j + k) * WT + (wtid & ~63u)) - (int)s;
                            const uint64_t m = uni64(row_mask(sm, c0, SM));
                            if (m) v[k] = fan_patch_start(v[k], f, (m >> lane) & 1u);
                        }
                    }
                    __builtin_amdgcn_raw_buffer_store_b128(v[k], os, (wtid + (j + k) * WT - s) * 16u, 0, AUX);
                }
                if constexpr (PACE == 2) __builtin_amdgcn_s_sleep(1);
            }
        }
        // ---- descriptors: one wave per sub-stream, a 128-B-aligned window of its array ----
        {
            const uint32_t nzc = np ? m_vc[np - 1] - vc0 + (m_len[np - 1] != 0) : 0u;
            for (uint32_t q = it.qb + wv; q < it.qe && !(EDGPU_ABL(P) & 1u); q += NWAVES) {
                const FanSub f = fansub(it, q);
                if (f.a >= lo + np) continue;
                const uint32_t p0 = f.a > lo ? (uint32_t)(f.a - lo) : 0u;
                const uint32_t o0 = m_vc[p0] - vc0;                            // first ordinal
                if (o0 >= nzc) continue;
                const uint32_t d0 = f.db + m_vc[p0];
                const uint32_t sh = d0 & 7;
                const uint32_t o = o0 + lane - sh;
                if ((uint32_t)lane >= sh && o < nzc) {
                    const uint32_t p = m_nzp[o];
                    const uint32_t len = m_len[p];
                    const uint64_t off = (uint64_t)(f.off + (int64_t)m_vb[p]);
                    const uint32_t wlen = len + ((f.ch & 1u) ? 4u : 0u);
                    u32x4 dv;
                    dv.x = (uint32_t)off; dv.y = (uint32_t)(off >> 32); dv.z = wlen; dv.w = m_id[p];
                    if (d0 - sh + lane < P.max_desc) {
                        if constexpr (DNT) __builtin_nontemporal_store(dv, reinterpret_cast<u32x4*>(P.desc) + d0 - sh + lane);
                        else reinterpret_cast<u32x4*>(P.desc)[d0 - sh + lane] = dv;
                    }
                    wire += wlen;
                }
            }
        }
        __syncthreads();
        if constexpr (DYN) wnext = s_claim[par];                  // visible after the barrier
    }
    unsigned long long a = wire, b = inb;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { a += __shfl_down(a, o, 64); b += __shfl_down(b, o, 64); }
    if (lane == 0) s_red[tid >> 6] = a;
    __syncthreads();
    if (tid == 0) {
        unsigned long long tot = 0;
        for (int i = 0; i < NWAVES; i++) tot += s_red[i];
        if (tot) { atomicAdd(&P.totals->relayed_bytes, tot); atomicAdd(&P.totals->cum_relayed_bytes, tot); }
    }
    __syncthreads();
    if (lane == 0) s_red[tid >> 6] = b;
    __syncthreads();
    if (tid == 0) {
        unsigned long long tot = 0;
        for (int i = 0; i < NWAVES; i++) tot += s_red[i];
        if (tot) atomicAdd(&P.totals->cum_fanout_in_bytes, tot);
    }
}

// -----------------------------------------------------------------------------------------
// k_fanout6: k_fanout4<..., nt, dyn> with TWO LDS images and one barrier per work item.
// k_fanout4 fills its single image from the prefetch registers, waits at a barrier, writes the
// item out, and waits again before the image may be refilled: every wave idles twice per item
// while the slowest one catches up.  Here a wave that has written out item i from image i&1
// fills image (i+1)&1 from the registers right away -- the other waves may still be reading
// image i&1 -- and the one barrier then means both "image i+1 complete" and "image i free".
// The slot-start bitmaps rotate through three buffers so that each is cleared one barrier
// before it is filled.  LDS: two 66-KB images (one 1024-thread workgroup per CU, as k_fanout4's
// default already runs).
// -----------------------------------------------------------------------------------------
template <int THREADS, int CHUNK>
struct Fan6 {
    static constexpr int CWORDS = CHUNK * kSlotWordsMax;
    static constexpr int NL = (CWORDS + THREADS - 1) / THREADS;
    static constexpr int NWAVES = THREADS / 64;
    static constexpr int SM = ((CWORDS + 31) / 32 + 3) & ~3;
    // per image: chunk words, then m_vb (CHUNK + 2 x u64), m_id / m_len / m_vc / m_nzp (CHUNK x u32)
    static constexpr int IMG = CWORDS * 16 + (CHUNK + 2) * 8 + 4 * CHUNK * 4;
    static constexpr int lds() { return 2 * IMG + 3 * SM * 4 + NWAVES * 8; }
};
template <int THREADS, int CHUNK>
constexpr int fanout6_lds() { return Fan6<THREADS, CHUNK>::lds(); }

// PP: the per-output patch as per-packet fix-ups.  The rows store every word that is not a
// packet's first word (nor, for an RTCP rewrite, its second); then one wave writes those words,
// patched, one lane per packet of the window.  The words are disjoint, so no ordering is
// needed, and the patch arithmetic runs once per packet instead of on every stored word.
// PF: each sub-stream window's FanSub record is loaded one window ahead (while the previous
// window's rows are stored), instead of in up to three dependent scalar-load round trips at the
// window's start.
// BP: the patch as a divergent branch on the slot-start test (fan_patch_branchy).
template <int THREADS, int CHUNK, int AUX = 2, int PP = 0, int PF = 0, int BP = 0>
__global__ __attribute__((amdgpu_flat_work_group_size(1, THREADS))) void k_fanout6(FanoutParams P) {
    using F = Fan6<THREADS, CHUNK>;
    constexpr int CWORDS = F::CWORDS, NL = F::NL, NWAVES = F::NWAVES, SM = F::SM;
    static_assert(CHUNK <= 56, "descriptor windows assume one wave covers a chunk's packets");
    const uint32_t nwork = uni(P.totals->nwork);
    if (uni((uint32_t)P.totals->status) == (uint32_t)EDGPU_OUT_OVERFLOW) return;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const uint32_t wv = uni((uint32_t)tid >> 6);
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    struct Img { u32x4* cb; uint64_t* vb; uint32_t *id, *len, *vc, *nzp; };
    auto img = [&](uint32_t b) {
        unsigned char* base = lds + b * F::IMG;
        Img m;
        m.cb = reinterpret_cast<u32x4*>(base);
        m.vb = reinterpret_cast<uint64_t*>(base + CWORDS * 16);
        m.id = reinterpret_cast<uint32_t*>(m.vb + CHUNK + 2);
        m.len = m.id + CHUNK; m.vc = m.len + CHUNK; m.nzp = m.vc + CHUNK;
        return m;
    };
    uint32_t* smb = reinterpret_cast<uint32_t*>(lds + 2 * F::IMG);       // 3 x SM bitmap words
    unsigned long long* s_red = reinterpret_cast<unsigned long long*>(smb + 3 * SM);
    u32x4* out = reinterpret_cast<u32x4*>(P.arena);
    unsigned long long wire = 0, inb = 0;
    u32x4 r[NL];
    u32x3 ma;
    u32x2 mb;
    __shared__ uint32_t s_claim[2];

    // one item's LDS image and slot-start bitmap (bitmap `sm` cleared beforehand), from the
    // registers its loads landed in
    auto fill = [&](const FanWork& it, const Img& m, uint32_t* sm) {
        const uint32_t nw = it.nw, np = it.np;
#pragma unroll
        for (int j = 0; j < NL; j++) {
            const uint32_t wi = tid + j * THREADS;
            if ((uint32_t)(j * THREADS) < nw && wi < nw) m.cb[wi] = r[j];
        }
        if ((uint32_t)tid < np) {
            const uint64_t vbyte = (uint64_t)ma.y << 32 | ma.x;
            const uint32_t len = mb.x & 0xFFFFu, vcount = mb.y;          // len:16 | seq:16
            m.vb[tid] = vbyte; m.id[tid] = ma.z; m.len[tid] = len; m.vc[tid] = vcount;
            inb += len;
            if (len != 0) {
                const uint32_t sw = (uint32_t)((vbyte - it.vb0) >> 4);
                atomicOr(&sm[sw >> 5], 1u << (sw & 31));
                m.nzp[vcount - it.vc0] = tid;
            }
        }
        if (tid == 0) m.vb[np] = it.vb0 + (uint64_t)nw * 16;
    };

    for (int k = tid; k < 3 * SM; k += THREADS) smb[k] = 0;
    if (tid == 0) { s_claim[0] = atomicAdd(&P.totals->fan_next, 1u); s_claim[1] = atomicAdd(&P.totals->fan_next, 1u); }
#ifdef EDGPU_AB_VARIANTS
    if (tid == 0) atomicMin(&P.totals->fan_t0_min, (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
    __syncthreads();
    uint32_t w = s_claim[0], wnext = s_claim[1];
    FanWork cur, nx;
    if (w < nwork) {
        cur = const_load(P.work + w);
        fan4_issue<THREADS, NL>(cur, tid, r, ma, mb);
        fill(cur, img(0), smb);
    }
    if (wnext < nwork) {
        nx = const_load(P.work + wnext);
        fan4_issue<THREADS, NL>(nx, tid, r, ma, mb);
    }
    __syncthreads();                                   // image 0 complete; s_claim read by all
    if (tid == 0) s_claim[0] = atomicAdd(&P.totals->fan_next, 1u);      // the item after next
    for (uint32_t i = 0; w < nwork; i++) {
        const FanWork it = cur;
        const Img m = img(i & 1u);
        uint32_t* sm = smb + (i % 3u) * SM;
        const uint64_t lo = it.lo, vb0 = it.vb0;
        const uint32_t np = it.np, nw = it.nw, vc0 = it.vc0;
        // ---- write the chunk to every sub-stream of the sender ----------------------------
        FanSub fnext;
        bool have_next = false;                                            // PF: fnext is record q
        for (uint32_t q = it.qb; q < it.qe && !(EDGPU_ABL(P) & 2u); q++) {
            const FanSub f = (PF && have_next) ? fnext : const_load(P.fansub + q);
            have_next = false;
            if (f.a >= lo + np) continue;
            const uint32_t p0 = f.a > lo ? (uint32_t)(f.a - lo) : 0u;
            const uint32_t fw = uni((uint32_t)((m.vb[p0] - vb0) >> 4));
            const int64_t A = f.dw + (int64_t)(vb0 >> 4) + fw;                 // first dest word
            if (A < 0 || (uint64_t)A + (nw - fw) > P.arena_words) { set_status(&P.totals->status, EDGPU_OUT_OVERFLOW); continue; }
            const uint32_t s = (uint32_t)(A & 7);                              // words past a line
            const __amdgpu_buffer_rsrc_t os = __builtin_amdgcn_make_buffer_rsrc(out + A, 0, (nw - fw) * 16, 0x00020000);
            const bool patch = (f.ch & 1u) || f.rw;                            // uniform
            const uint32_t nj = (nw - fw + s + THREADS - 1) / THREADS;
            if (PF && q + 1 < it.qe) { fnext = const_load(P.fansub + q + 1); have_next = true; }
            if (PP && patch) {
                const bool second = (f.rw & kRwRtcp) != 0;                     // the SR timestamp word too
                for (uint32_t j = 0; j < nj; j++) {
                    const uint32_t src = fw + tid + j * THREADS - s;
                    const uint32_t srcc = src < (uint32_t)CWORDS ? src : 0u;
                    const u32x4 v = m.cb[srcc];
                    bool skip = (sm[srcc >> 5] >> (srcc & 31)) & 1u;
                    if (second && srcc > 0) skip |= (sm[(srcc - 1) >> 5] >> ((srcc - 1) & 31)) & 1u;
                    if (!skip) __builtin_amdgcn_raw_buffer_store_b128(v, os, (tid + j * THREADS - s) * 16u, 0, AUX);
                }
                if (wv == (q - it.qb) % NWAVES) {                              // one wave: the packets
                    const uint32_t p = p0 + lane;
                    const uint32_t len = p < np ? m.len[p] : 0u;
                    if (len != 0) {
                        const uint32_t st = (uint32_t)((m.vb[p] - vb0) >> 4);  // the slot's first word
                        const u32x4 h = m.cb[st];
                        __builtin_amdgcn_raw_buffer_store_b128(fan_patch_start(h, f, true), os, (st - fw) * 16u, 0, AUX);
                        if (second && len >= 13) {                             // a second word in the slot
                            u32x4 v1 = m.cb[st + 1];
                            if (len >= 20 && ((h.y >> 8) & 0xFFu) == 200u)     // an SR: its RTP timestamp
                                v1.y = __builtin_bswap32(__builtin_bswap32(v1.y) + f.rw_ts);
                            __builtin_amdgcn_raw_buffer_store_b128(v1, os, (st + 1 - fw) * 16u, 0, AUX);
                        }
                    }
                }
                continue;
            }
            for (uint32_t j = 0; j < nj; j++) {
                const uint32_t src = fw + tid + j * THREADS - s;               // chunk word of the lane's
                const uint32_t srcc = src < (uint32_t)CWORDS ? src : 0u;       // word of the aligned window
                u32x4 v = m.cb[srcc];
                if (patch) v = BP ? fan_patch_branchy(v, f, srcc, sm, m.cb) : fan_patch(v, f, srcc, sm, m.cb);
                __builtin_amdgcn_raw_buffer_store_b128(v, os, (tid + j * THREADS - s) * 16u, 0, AUX);
            }
        }
        // ---- descriptors: one wave per sub-stream, a 128-B-aligned window of its array ----
        {
            const uint32_t nzc = np ? m.vc[np - 1] - vc0 + (m.len[np - 1] != 0) : 0u;
            for (uint32_t q = it.qb + wv; q < it.qe && !(EDGPU_ABL(P) & 1u); q += NWAVES) {
                const FanSub f = const_load(P.fansub + q);
                if (f.a >= lo + np) continue;
                const uint32_t p0 = f.a > lo ? (uint32_t)(f.a - lo) : 0u;
                const uint32_t o0 = m.vc[p0] - vc0;                            // first ordinal
                if (o0 >= nzc) continue;
                const uint32_t d0 = f.db + m.vc[p0];
                const uint32_t sh = d0 & 7;
                const uint32_t o = o0 + lane - sh;
                if ((uint32_t)lane >= sh && o < nzc) {
                    const uint32_t p = m.nzp[o];
                    const uint32_t len = m.len[p];
                    const uint64_t off = (uint64_t)(f.off + (int64_t)m.vb[p]);
                    const uint32_t wlen = len + ((f.ch & 1u) ? 4u : 0u);
                    u32x4 dv;
                    dv.x = (uint32_t)off; dv.y = (uint32_t)(off >> 32); dv.z = wlen; dv.w = m.id[p];
                    if (d0 - sh + lane < P.max_desc) reinterpret_cast<u32x4*>(P.desc)[d0 - sh + lane] = dv;
                    wire += wlen;
                }
            }
        }
        // ---- the next item's image, while other waves may still read this one ------------
        // Bitmap buffers rotate by three: item i+2's (last read by item i-1, before the previous
        // barrier) is cleared now, one barrier before it is filled; item i+1's was cleared one
        // item ago.
        {
            uint32_t* sc = smb + ((i + 2) % 3u) * SM;
            for (int k = tid; k < SM; k += THREADS) sc[k] = 0;
        }
        if (wnext < nwork) fill(nx, img((i + 1) & 1u), smb + ((i + 1) % 3u) * SM);
        __syncthreads();                     // image i+1 complete, image i free, s_claim visible
        cur = nx;
        w = wnext;
        wnext = s_claim[i & 1u];
        if (wnext < nwork) {
            nx = const_load(P.work + wnext);
            fan4_issue<THREADS, NL>(nx, tid, r, ma, mb);
        }
        if (tid == 0) s_claim[(i + 1) & 1u] = atomicAdd(&P.totals->fan_next, 1u);
    }
    unsigned long long a = wire, b = inb;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { a += __shfl_down(a, o, 64); b += __shfl_down(b, o, 64); }
    if (lane == 0) s_red[tid >> 6] = a;
    __syncthreads();
    if (tid == 0) {
        unsigned long long tot = 0;
        for (int k = 0; k < NWAVES; k++) tot += s_red[k];
        if (tot) { atomicAdd(&P.totals->relayed_bytes, tot); atomicAdd(&P.totals->cum_relayed_bytes, tot); }
    }
    __syncthreads();
    if (lane == 0) s_red[tid >> 6] = b;
    __syncthreads();
    if (tid == 0) {
        unsigned long long tot = 0;
        for (int k = 0; k < NWAVES; k++) tot += s_red[k];
        if (tot) atomicAdd(&P.totals->cum_fanout_in_bytes, tot);
    }
#ifdef EDGPU_AB_VARIANTS
    if (tid == 0) {
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        atomicMin(&P.totals->fan_done_min, t);
        atomicMax(&P.totals->fan_done_max, t);
    }
#endif
}

// -----------------------------------------------------------------------------------------
// k_fanout5: the write-many at low wave count with asynchronous chunk staging.  Measured on
// the box (tools/store_peak3.hip): the same line-aligned window stores reach ~5.8 TB/s with 4
// waves per CU and no load phases, against ~5.3 TB/s at 32 waves per CU with load phases
// between chunks.  So each CU runs few waves, and the next chunk (slot words and packet
// metadata) is staged by LDS-DMA (global_load_lds_dwordx4, no VGPRs) into the other half of a
// double-buffered LDS image while the current chunk is written out.  Barriers are raw
// s_barrier with explicit counter waits, so the DMA stays in flight across them; the one
// vmcnt(0) per item (which also retires that item's stores) is where the next image lands.
// -----------------------------------------------------------------------------------------
template <int THREADS, int CHUNK>
struct Fan5 {
    static constexpr int CWORDS = CHUNK * kSlotWordsMax;
    static constexpr int NLD = (CWORDS + THREADS - 1) / THREADS;       // DMA words per lane
    static constexpr int CBUF = NLD * THREADS;                         // words per image
    static constexpr int SM = ((CWORDS + 31) / 32 + 3) & ~3;
    static constexpr int NWAVES = THREADS / 64;
    // per buffer: chunk words, 2 metadata words per packet; then bitmaps, ordinals, reduction
    static constexpr int lds() {
        return 2 * CBUF * 16 + 2 * 2 * CHUNK * 16 + 2 * SM * 4 + 2 * CHUNK * 4 + NWAVES * 8;
    }
};

template <int THREADS, int CHUNK>
constexpr int fanout5_lds() { return Fan5<THREADS, CHUNK>::lds(); }

typedef __attribute__((address_space(3))) void* lptr_t;

// One global_load_lds_dwordx4: 16 B per lane from `g` into LDS at M0 + 16 * lane.  Issued from
// inline asm so the compiler's counter pass does not see an LDS write in flight (it would
// otherwise wait for the DMA before every later LDS access, serialising the pipeline); the
// kernel waits for it explicitly (vmcnt(0) at the top of the next item).
__device__ __forceinline__ void glds16(const void* g, uint32_t lds_base) {
    uint32_t keep;                                     // M0 is reserved: save and restore it
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds_base) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(void* p) { return uni((uint32_t)(size_t)(lptr_t)p); }

// LDS-DMA of one work item into image `img` / metadata `mimg` (both wave-linear: lane l of a
// wave-instruction lands at base + 16 l).  Lanes past the chunk re-read a valid word.
template <int THREADS, int CHUNK>
__device__ __forceinline__ void fan5_stage(const FanWork& it, int tid, u32x4* img, u32x4* mimg) {
    using F = Fan5<THREADS, CHUNK>;
    const uint32_t wmask = it.wmask, nw = it.nw;
    const uint32_t r0 = (uint32_t)(it.vb0 >> 4);
    const u32x4* ring = reinterpret_cast<const u32x4*>(it.ring);
    const uint32_t wbase = uni((uint32_t)tid & ~63u);
    const uint32_t ibase = lds_addr(img) + wbase * 16u;
#pragma unroll
    for (int j = 0; j < F::NLD; j++) {
        if ((uint32_t)(j * THREADS) < nw) {                    // uniform
            const uint32_t wi = j * THREADS + tid;
            const uint32_t src = (r0 + min(wi, nw - 1)) & wmask;
            glds16(ring + src, ibase + (uint32_t)(j * THREADS) * 16u);
        }
    }
    if (tid < 2 * CHUNK && it.np) {      // metadata: 2 words per packet; exec-masked lanes write nothing
        const uint32_t p = min((uint32_t)tid >> 1, it.np - 1);
        const u32x4* meta = reinterpret_cast<const u32x4*>(it.meta);
        const uint64_t e = (it.lo + p) & it.pkmask;
        glds16(meta + 2 * e + (tid & 1), lds_addr(mimg) + wbase * 16u);
    }
}

template <int THREADS, int CHUNK, int AUX = 0>
__global__ __attribute__((amdgpu_flat_work_group_size(1, THREADS)))
void k_fanout5(FanoutParams P) {
    using F = Fan5<THREADS, CHUNK>;
    constexpr int CWORDS = F::CWORDS, SM = F::SM, NWAVES = F::NWAVES;
    static_assert(CHUNK <= 56 && 2 * CHUNK <= THREADS, "");
    const uint32_t nwork = uni(P.totals->nwork);
    if (uni((uint32_t)P.totals->status) == (uint32_t)EDGPU_OUT_OVERFLOW) return;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const uint32_t wv = uni((uint32_t)tid >> 6);
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    u32x4* cimg = reinterpret_cast<u32x4*>(lds);                       // 2 x CBUF words
    u32x4* mimg = cimg + 2 * F::CBUF;                                  // 2 x 2*CHUNK words
    uint32_t* smap = reinterpret_cast<uint32_t*>(mimg + 4 * CHUNK);    // 2 x SM
    uint32_t* nzp = smap + 2 * SM;                                     // 2 x CHUNK
    unsigned long long* s_red = reinterpret_cast<unsigned long long*>(nzp + 2 * CHUNK);
    u32x4* out = reinterpret_cast<u32x4*>(P.arena);
    unsigned long long wire = 0, inb = 0;

    for (int k = tid; k < 2 * SM; k += THREADS) smap[k] = 0;
    uint32_t w = blockIdx.x;
    FanWork cur, nxt;
    if (w < nwork) {
        cur = const_load(P.work + w);
        fan5_stage<THREADS, CHUNK>(cur, tid, cimg, mimg);
    }
    if (w + gridDim.x < nwork) nxt = const_load(P.work + w + gridDim.x);
    for (uint32_t b = 0; w < nwork; w += gridDim.x, b ^= 1u) {
        const uint64_t lo = cur.lo, vb0 = cur.vb0;
        const uint32_t np = cur.np, nw = cur.nw, vc0 = cur.vc0;
        u32x4* cb = cimg + b * F::CBUF;
        const u32x4* mb = mimg + b * 2 * CHUNK;
        uint32_t* sm = smap + b * SM;
        uint32_t* nz = nzp + b * CHUNK;
        // this item's image has landed (this also retires the previous item's stores), and
        // every wave is past the previous item: the other buffer is free
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const uint32_t wn = w + gridDim.x;
        if (wn < nwork) fan5_stage<THREADS, CHUNK>(nxt, tid, cimg + (b ^ 1u) * F::CBUF, mimg + (b ^ 1u) * 2 * CHUNK);
        // slot-start bitmap and non-empty ordinals of this item; clear the other bitmap
        for (int k = tid; k < SM; k += THREADS) smap[(b ^ 1u) * SM + k] = 0;
        if ((uint32_t)tid < np) {
            const u32x4 m0 = mb[2 * tid], m1 = mb[2 * tid + 1];
            const uint64_t vbyte = (uint64_t)m0.y << 32 | m0.x;
            inb += m1.z & 0xFFFFu;                                     // len:16 | seq:16
            if ((m1.z & 0xFFFFu) != 0) {
                const uint32_t sw = (uint32_t)((vbyte - vb0) >> 4);
                atomicOr(&sm[sw >> 5], 1u << (sw & 31));
                nz[m1.w - vc0] = tid;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const FanWork it = cur;
        cur = nxt;
        if (wn + gridDim.x < nwork) nxt = const_load(P.work + wn + gridDim.x);
        // ---- write the chunk to every sub-stream of the sender (k_fanout3's line-aligned
        // windows, uniform trip count) ----
        for (uint32_t q = it.qb; q < it.qe && !(EDGPU_ABL(P) & 2u); q++) {
            const FanSub f = const_load(P.fansub + q);
            if (f.a >= lo + np) continue;
            const uint32_t p0 = f.a > lo ? (uint32_t)(f.a - lo) : 0u;
            const u32x4 mp = mb[2 * p0];
            const uint32_t fw = uni((uint32_t)((((uint64_t)mp.y << 32 | mp.x) - vb0) >> 4));
            const int64_t A = f.dw + (int64_t)(vb0 >> 4) + fw;
            if (A < 0 || (uint64_t)A + (nw - fw) > P.arena_words) { set_status(&P.totals->status, EDGPU_OUT_OVERFLOW); continue; }
            const uint32_t s = (uint32_t)(A & 7);
            const __amdgpu_buffer_rsrc_t os = __builtin_amdgcn_make_buffer_rsrc(out + A, 0, (nw - fw) * 16, 0x00020000);
            const bool patch = (f.ch & 1u) || f.rw;                            // uniform
            const uint32_t nj = (nw - fw + s + THREADS - 1) / THREADS;
            for (uint32_t j = 0; j < nj; j++) {
                const uint32_t lw = tid + j * THREADS;
                const uint32_t src = fw + lw - s;
                const uint32_t srcc = src < (uint32_t)CWORDS ? src : 0u;
                u32x4 v = cb[srcc];
                if (patch) v = fan_patch(v, f, srcc, sm, cb);
                __builtin_amdgcn_raw_buffer_store_b128(v, os, (lw - s) * 16u, 0, AUX);
            }
        }
        // ---- descriptors: one wave per sub-stream, 128-B-aligned windows ----
        {
            const u32x4 ml = mb[2 * (np - 1) + 1];
            const uint32_t nzc = np ? ml.w - vc0 + ((ml.z & 0xFFFFu) != 0) : 0u;
            for (uint32_t q = it.qb + wv; q < it.qe && !(EDGPU_ABL(P) & 1u); q += NWAVES) {
                const FanSub f = const_load(P.fansub + q);
                if (f.a >= lo + np) continue;
                const uint32_t p0 = f.a > lo ? (uint32_t)(f.a - lo) : 0u;
                const uint32_t vcp0 = mb[2 * p0 + 1].w;
                const uint32_t o0 = vcp0 - vc0;
                if (o0 >= nzc) continue;
                const uint32_t d0 = f.db + vcp0;
                const uint32_t sh = d0 & 7;
                const uint32_t o = o0 + lane - sh;
                if ((uint32_t)lane >= sh && o < nzc) {
                    const uint32_t p = nz[o];
                    const u32x4 m0 = mb[2 * p], m1 = mb[2 * p + 1];
                    const uint64_t off = (uint64_t)(f.off + (int64_t)((uint64_t)m0.y << 32 | m0.x));
                    const uint32_t wlen = (m1.z & 0xFFFFu) + ((f.ch & 1u) ? 4u : 0u);
                    u32x4 dv;
                    dv.x = (uint32_t)off; dv.y = (uint32_t)(off >> 32); dv.z = wlen; dv.w = m0.z;
                    if (d0 - sh + lane < P.max_desc) reinterpret_cast<u32x4*>(P.desc)[d0 - sh + lane] = dv;
                    wire += wlen;
                }
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned long long a = wire, bb = inb;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { a += __shfl_down(a, o, 64); bb += __shfl_down(bb, o, 64); }
    if (lane == 0) s_red[tid >> 6] = a;
    __syncthreads();
    if (tid == 0) {
        unsigned long long tot = 0;
        for (int i = 0; i < NWAVES; i++) tot += s_red[i];
        if (tot) { atomicAdd(&P.totals->relayed_bytes, tot); atomicAdd(&P.totals->cum_relayed_bytes, tot); }
    }
    __syncthreads();
    if (lane == 0) s_red[tid >> 6] = bb;
    __syncthreads();
    if (tid == 0) {
        unsigned long long tot = 0;
        for (int i = 0; i < NWAVES; i++) tot += s_red[i];
        if (tot) atomicAdd(&P.totals->cum_fanout_in_bytes, tot);
    }
}

// =========================================================================================
// Session images: export the serveable part of a session's rings into a
// contiguous buffer that another GPU imports into a replica session; a subscriber joining
// the replica receives exactly what it would receive joining the owner.
// =========================================================================================

__device__ uint64_t sender_tail(const SenderDev& D) {
    const PktMeta* meta = reinterpret_cast<const PktMeta*>(D.meta);
    const uint64_t head = D.head, pk_cap = (uint64_t)D.pk_mask + 1;
    const uint64_t byte_cap = ((uint64_t)D.word_mask + 1) * 16, vend = max(D.vbyte_end, D.vclob);
    uint64_t lo = head > pk_cap ? head - pk_cap : 0;
    lo = max(lo, D.floor);
    return lower_bound_meta(meta, D.pk_mask, lo, head,
                            [&](const PktMeta& m) { return vend - m.vbyte <= byte_cap; });
}

// RTP-Info PLAY (HaveStreamBuffers, QTSSReflectorModule.cpp:1804-1865): per track,
// HasFirstRTP and ReflectorSender::GetFirstPacketInfo (ReflectorStream.cpp:728-753) -- the
// oldest RTP-sender packet whose age is within the window (GetClientBufferStartPacketOffset,
// :1201-1231), its sequence number and RTP timestamp (ReflectorStream.h:160-189).
__global__ void k_first_packet_info(const FirstInfoQuery* Q, FirstInfoResult* R, const SenderDev* senders, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const FirstInfoQuery q = Q[i];
    const SenderDev& D = senders[q.rtp_sender];
    FirstInfoResult r{0u, 0u, 0u, 0u};
    const bool has_rtp = D.head > 0 || (q.rtcp_sender != 0xFFFFFFFFu && senders[q.rtcp_sender].head > 0);
    if (has_rtp) {
        const PktMeta* meta = reinterpret_cast<const PktMeta*>(D.meta);
        const uint64_t f = first_arrival_at(D, meta, sender_tail(D), D.head, q.cutoff);
        r.found = 2;
        if (f < D.head) {
            const PktMeta m = meta[f & D.pk_mask];
            r.found = 1;
            r.seq = m.seq;
            if (m.len >= 8) {     // packet bytes 4..7 sit in the slot's first 16-B word
                const uint8_t* ring = reinterpret_cast<const uint8_t*>(D.ring);
                const uint64_t mask = ((uint64_t)D.word_mask + 1) * 16 - 1;
                r.rtptime = __builtin_bswap32(*reinterpret_cast<const uint32_t*>(ring + ((m.vbyte + 8) & mask)));
            }
        }
    }
    R[i] = r;
}

// Export plan, one thread per sender: which packets the image carries.  A full image starts
// at the key pointer, or (no key) at the oldest packet inside the new-output window -- the
// same start k_plan_senders would pick for a new output at `now` or later (Q7).
__global__ void k_image_plan(ImageParams P) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= P.nplan) return;
    ImgPlan& E = P.plan[j];
    const SenderDev& D = P.senders[E.sender];
    const PktMeta* meta = reinterpret_cast<const PktMeta*>(D.meta);
    const uint64_t head = D.head, tail = sender_tail(D);
    uint64_t floor = head;
    if (E.from != kImageFull) {
        floor = E.from;
        if (floor > head) { set_status(P.status, EDGPU_BAD_ARGUMENT); floor = head; }
        else if (floor < tail) { set_status(P.status, EDGPU_RING_OVERFLOW); floor = tail; }
    } else if (D.key >= 0) {
        floor = (uint64_t)D.key;
        if (floor < tail) { set_status(P.status, EDGPU_RING_OVERFLOW); floor = tail; }
    } else if (head > tail) {
        const int64_t cutoff = P.now - P.over_buffer_ms;
        floor = first_arrival_at(D, meta, tail, head, cutoff);
        if (floor < head && floor == tail && tail > D.floor) set_status(P.status, EDGPU_RING_OVERFLOW);
    }
    if (E.from == kImageFull && head > tail && floor > tail) {
        // an RTP-Info PLAY on the replica reads the first packet of the over-buffer window
        // (GetFirstPacketInfo, ReflectorStream.cpp:728-753), which may precede the key pointer
        const int64_t cutoff = P.now - P.over_buffer_ms;
        const uint64_t w = first_arrival_at(D, meta, tail, head, cutoff);
        if (w < floor) floor = w;
    }
    E.floor = floor;
    E.vbyte_floor = floor < head ? meta[floor & D.pk_mask].vbyte : D.vbyte_end;
    E.nmeta = head - floor;
    E.nbytes = D.vbyte_end - E.vbyte_floor;
}

// Export pack, one workgroup per sender: metadata and slot bytes out of the rings (unwrapped).
__global__ __launch_bounds__(256) void k_image_pack(ImageParams P) {
    const ImgPlan E = P.plan[blockIdx.x];
    const SenderDev& D = P.senders[E.sender];
    uint8_t* img = P.buf + E.image_base;
    const PktMeta* meta = reinterpret_cast<const PktMeta*>(D.meta);
    PktMeta* om = reinterpret_cast<PktMeta*>(img + E.meta_off);
    for (uint64_t i = threadIdx.x; i < E.nmeta; i += blockDim.x) om[i] = meta[(E.floor + i) & D.pk_mask];
    const u32x4* ring = reinterpret_cast<const u32x4*>(D.ring);
    u32x4* ob = reinterpret_cast<u32x4*>(img + E.bytes_off);
    const uint64_t w0 = E.vbyte_floor >> 4, nw = E.nbytes >> 4;
    for (uint64_t w = threadIdx.x; w < nw; w += blockDim.x) ob[w] = ring[(w0 + w) & D.word_mask];
    if (threadIdx.x == 0) {
        const SessionDev& S = P.sessions[E.session];
        ImgSender r;
        r.floor = E.floor; r.head = D.head; r.vbyte_floor = E.vbyte_floor; r.vbyte_end = D.vbyte_end;
        r.vcount_end = D.vcount_end; r.valid_ssrc = D.valid_ssrc; r.last_valid_s = D.last_valid_s;
        r.key = D.key; r.last_nonzero = D.last_nonzero;
        r.meta_off = E.meta_off; r.bytes_off = E.bytes_off;
        r.delta = E.from != kImageFull; r.flags = D.flags; r.nonmono = D.rt_nonmono; r._pad = 0;
        reinterpret_cast<ImgSender*>(img + sizeof(ImgHeader) + S.ntracks * sizeof(ImgStream))[E.ls] = r;
        if (E.first) {
            ImgHeader h;
            h.magic = kImageMagic; h.version = kImageVersion; h.ntracks = S.ntracks; h.nsenders = 2 * S.ntracks;
            h.bytes = E.image_bytes; h.now = P.now; h.video_key_flag = S.video_key_flag; h.delta = r.delta;
            h._pad[0] = h._pad[1] = h._pad[2] = 0;
            *reinterpret_cast<ImgHeader*>(img) = h;
            ImgStream* st = reinterpret_cast<ImgStream*>(img + sizeof(ImgHeader));
            for (uint32_t t = 0; t < S.ntracks; t++) st[t] = ImgStream{P.streams[S.first_stream + t].packet_count, 0};
        }
    }
}

// Import, one workgroup per (image, sender): validate, copy into the replica's rings at the
// same virtual positions, then take over the owner's sender state.
__global__ __launch_bounds__(256) void k_image_apply(ImageParams P) {
    const ImgPlan E = P.plan[blockIdx.x];
    SenderDev& D = P.senders[E.sender];
    const SessionDev& S = P.sessions[E.session];
    const uint8_t* img = P.buf + E.image_base;
    const ImgHeader h = *reinterpret_cast<const ImgHeader*>(img);
    if (h.magic != kImageMagic || h.version != kImageVersion || h.ntracks != S.ntracks || h.nsenders != 2 * S.ntracks) {
        if (threadIdx.x == 0) set_status(P.status, EDGPU_BAD_ARGUMENT);
        return;
    }
    const ImgSender r = reinterpret_cast<const ImgSender*>(img + sizeof(ImgHeader) + h.ntracks * sizeof(ImgStream))[E.ls];
    const uint64_t nmeta = r.head - r.floor, nbytes = r.vbyte_end - r.vbyte_floor;
    if ((r.delta && r.floor != D.head) || (r.flags & ~kSndRtcpPort) != (D.flags & ~kSndRtcpPort)) {
        if (threadIdx.x == 0) set_status(P.status, EDGPU_BAD_ARGUMENT);
        return;
    }
    if (nmeta > (uint64_t)D.pk_mask + 1 || nbytes > ((uint64_t)D.word_mask + 1) * 16) {
        if (threadIdx.x == 0) set_status(P.status, EDGPU_RING_OVERFLOW);
        return;
    }
    const PktMeta* im = reinterpret_cast<const PktMeta*>(img + r.meta_off);
    PktMeta* meta = reinterpret_cast<PktMeta*>(D.meta);
    for (uint64_t i = threadIdx.x; i < nmeta; i += blockDim.x) meta[(r.floor + i) & D.pk_mask] = im[i];
    const u32x4* ib = reinterpret_cast<const u32x4*>(img + r.bytes_off);
    u32x4* ring = reinterpret_cast<u32x4*>(D.ring);
    const uint64_t w0 = r.vbyte_floor >> 4, nw = nbytes >> 4;
    for (uint64_t w = threadIdx.x; w < nw; w += blockDim.x) ring[(w0 + w) & D.word_mask] = ib[w];
    if (threadIdx.x == 0) {
        if (!r.delta) D.floor = r.floor;
        D.head = r.head; D.vbyte_end = r.vbyte_end; D.vcount_end = r.vcount_end;
        D.valid_ssrc = r.valid_ssrc; D.last_valid_s = r.last_valid_s;
        D.key = r.key; D.last_nonzero = r.last_nonzero;
        D.rt_nonmono |= r.nonmono;               // arrivals the owner rewrote travel with its packets
        if (E.first) {
            const ImgStream* st = reinterpret_cast<const ImgStream*>(img + sizeof(ImgHeader));
            for (uint32_t t = 0; t < S.ntracks; t++) P.streams[S.first_stream + t].packet_count = st[t].packet_count;
            P.sessions[E.session].video_key_flag = h.video_key_flag;
        }
    }
}

// Import fit (ring growth), one thread per (image, sender): a replica's rings must hold what its
// owner's image carries, so the image part's packets / bytes go back (nmeta / nbytes, with the
// sender's oldest kept index in floor) when they exceed the rings, else 0.  An image that does not
// match its replica (header, size) is left to k_image_apply to reject.  E.image_bytes: the image's
// size in the buffer.
__global__ void k_image_fit(ImageParams P) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= P.nplan) return;
    ImgPlan& E = P.plan[j];
    E.nmeta = 0;
    E.nbytes = 0;
    const SenderDev& D = P.senders[E.sender];
    const uint32_t nt = P.sessions[E.session].ntracks;
    const uint8_t* img = P.buf + E.image_base;
    if (E.image_bytes < sizeof(ImgHeader) + nt * sizeof(ImgStream) + 2 * nt * sizeof(ImgSender)) return;
    const ImgHeader h = *reinterpret_cast<const ImgHeader*>(img);
    if (h.magic != kImageMagic || h.version != kImageVersion || h.ntracks != nt || h.nsenders != 2 * nt) return;
    const ImgSender r = reinterpret_cast<const ImgSender*>(img + sizeof(ImgHeader) + nt * sizeof(ImgStream))[E.ls];
    if (r.head < r.floor || r.vbyte_end < r.vbyte_floor) return;
    const uint64_t nmeta = r.head - r.floor, nbytes = r.vbyte_end - r.vbyte_floor;
    if (nmeta <= (uint64_t)D.pk_mask + 1 && nbytes <= ((uint64_t)D.word_mask + 1) * 16) return;
    E.nmeta = nmeta;
    E.nbytes = nbytes;
    E.floor = D.tail > D.floor ? D.tail : D.floor;
}

}  // namespace edgpu

// ---------------------------------------------------------------------------------------
// Launch wrappers (internal C++ API used by edgpu_engine.cpp)
namespace edgpu {
thread_local uint64_t tl_launches = 0;

// edgpu_arena_gather: one workgroup per region, 16-B words (offsets / lengths are slot-aligned)
__global__ __launch_bounds__(256) void k_arena_gather(const u32x4* arena, const edgpu_region* reg, const uint64_t* dst_off,
                                                      u32x4* dst) {
    const edgpu_region r = reg[blockIdx.x];
    const u32x4* s = arena + r.offset / 16;
    u32x4* d = dst + dst_off[blockIdx.x] / 16;
    for (uint64_t w = threadIdx.x; w < r.bytes / 16; w += blockDim.x) __builtin_nontemporal_store(s[w], d + w);
}
hipError_t launch_arena_gather(const uint8_t* arena, const edgpu_region* reg, const uint64_t* dst_off, uint32_t n,
                               uint8_t* dst, hipStream_t st) {
    if (n) EDGPU_LAUNCH(k_arena_gather, dim3(n), dim3(256), 0, st, reinterpret_cast<const u32x4*>(arena), reg,
                              dst_off, reinterpret_cast<u32x4*>(dst));
    return hipGetLastError();
}

// Device -> pinned host copy by stores over PCIe: a grid-stride sweep of 16-B words (53 GB/s on
// the MI355X box for a 52 MB read against 29 GB/s for hipMemcpyAsync, tools/pcie_d2h.hip); the
// last `bytes % 16` bytes by one lane.  src / dst 16-B aligned (checked by the caller).
__global__ __launch_bounds__(256) void k_copy_to_pinned(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                        uint64_t bytes) {
    const uint64_t words = bytes / 16;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < words; i += (uint64_t)gridDim.x * 256ull)
        __builtin_nontemporal_store(src[i], dst + i);
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (uint64_t b = words * 16; b < bytes; b++)
            reinterpret_cast<uint8_t*>(dst)[b] = reinterpret_cast<const uint8_t*>(src)[b];
}
hipError_t launch_copy_to_pinned(void* dst, const void* src, uint64_t bytes, hipStream_t st) {
    if (bytes) EDGPU_LAUNCH(k_copy_to_pinned, dim3(1024), dim3(256), 0, st, reinterpret_cast<const u32x4*>(src),
                                  reinterpret_cast<u32x4*>(dst), bytes);
    return hipGetLastError();
}

// edgpu_debug_stall: one wave that waits `ticks` of the device's constant-rate clock (s_memrealtime,
// sleeping between reads) and exits -- a stand-in for a stuck kernel, to exercise the watchdog.
// Every lane reaches the exit: the condition is the clock alone.
__global__ __launch_bounds__(64) void k_stall(uint64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}
hipError_t launch_stall(uint64_t ticks, hipStream_t st) {
    EDGPU_LAUNCH(k_stall, dim3(1), dim3(64), 0, st, ticks);
    return hipGetLastError();
}

// edgpu_fanout_arrivals: the arrival time of every descriptor of the last tick.  One wave per
// sub-stream walks its range [a, head) of the sender's metadata ring; descriptor i is the i-th
// non-empty packet from `a` (vcount - vcstart), exactly as k_fanout4 numbered them.
__global__ __launch_bounds__(256) void k_desc_arrival(const SubDev* subs, const SenderDev* senders, uint32_t nsubs,
                                                      uint32_t pass, int64_t* out) {
    const uint32_t q = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (q >= nsubs) return;
    const SubDev& Q = subs[q];
    if (!Q.active || !Q.nonempty || Q.count == 0 || Q.pass != pass) return;   // the current copy pass's rows
    const SenderDev& D = senders[Q.sender];
    const PktMeta* meta = reinterpret_cast<const PktMeta*>(D.meta);
    for (uint64_t p = Q.a + lane; p < D.head; p += 64) {
        const PktMeta m = meta[p & D.pk_mask];
        const uint32_t i = m.vcount - Q.vcstart;
        if (m.len != 0 && i < Q.count) out[Q.desc_base + i] = m.arrival;
    }
}
hipError_t launch_desc_arrival(const SubDev* subs, const SenderDev* senders, uint32_t nsubs, uint32_t pass,
                               int64_t* out, hipStream_t st) {
    if (nsubs) EDGPU_LAUNCH(k_desc_arrival, dim3((nsubs + 3) / 4), dim3(256), 0, st, subs, senders, nsubs, pass, out);
    return hipGetLastError();
}

// edgpu_fanout_sources: per descriptor of the current pass, the blob slot of its packet when the
// packet came with the last host batch (ingest epoch `epoch`), else kNoSource.  Numbered as
// k_desc_arrival numbers them; out[] was filled with kNoSource first.
__global__ __launch_bounds__(256) void k_desc_source(const SubDev* subs, const SenderDev* senders, uint32_t nsubs,
                                                     uint32_t pass, uint32_t epoch, uint32_t* out) {
    const uint32_t q = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (q >= nsubs) return;
    const SubDev& Q = subs[q];
    if (!Q.active || !Q.nonempty || Q.count == 0 || Q.pass != pass) return;
    const SenderDev& D = senders[Q.sender];
    if (D.batch_epoch != epoch) return;
    const PktMeta* meta = reinterpret_cast<const PktMeta*>(D.meta);
    const uint32_t* src = reinterpret_cast<const uint32_t*>(D.meta + ((uint64_t)D.pk_mask + 1) * sizeof(PktMeta));
    for (uint64_t p = max(Q.a, D.batch_lo) + lane; p < D.head; p += 64) {
        const PktMeta m = meta[p & D.pk_mask];
        const uint32_t i = m.vcount - Q.vcstart;
        if (m.len != 0 && i < Q.count) out[Q.desc_base + i] = src[p & D.pk_mask];
    }
}
hipError_t launch_desc_source(const SubDev* subs, const SenderDev* senders, uint32_t nsubs, uint32_t pass,
                              uint32_t epoch, uint32_t* out, hipStream_t st) {
    if (nsubs) EDGPU_LAUNCH(k_desc_source, dim3((nsubs + 3) / 4), dim3(256), 0, st, subs, senders, nsubs, pass,
                                  epoch, out);
    return hipGetLastError();
}

// edgpu_fanout_rows: one wave per selected sub-stream (sel[2k] its row, sel[2k + 1] its first
// output row); each of its descriptors with the packet's arrival and batch slot, numbered as
// k_desc_arrival numbers them.  Rows past `nrows` are not written.
__global__ __launch_bounds__(256) void k_sub_rows(const SubDev* subs, const SenderDev* senders, const edgpu_out_desc* desc,
                                                  const uint32_t* sel, uint32_t nsel, uint32_t nsubs, uint32_t pass,
                                                  uint32_t epoch, edgpu_packet_row* rows, uint64_t nrows) {
    const uint32_t k = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (k >= nsel) return;
    const uint32_t q = sel[2 * k];
    const uint64_t base = sel[2 * k + 1];
    if (q >= nsubs) return;
    const SubDev& Q = subs[q];
    if (!Q.active || !Q.nonempty || Q.count == 0 || Q.pass != pass) return;
    const SenderDev& D = senders[Q.sender];
    const PktMeta* meta = reinterpret_cast<const PktMeta*>(D.meta);
    const uint32_t* src = reinterpret_cast<const uint32_t*>(D.meta + ((uint64_t)D.pk_mask + 1) * sizeof(PktMeta));
    const uint64_t from_batch = (epoch && D.batch_epoch == epoch) ? D.batch_lo : ~0ull;
    for (uint64_t p = Q.a + lane; p < D.head; p += 64) {
        const PktMeta m = meta[p & D.pk_mask];
        const uint32_t i = m.vcount - Q.vcstart;
        if (m.len == 0 || i >= Q.count || base + i >= nrows) continue;
        const edgpu_out_desc o = desc[Q.desc_base + i];
        edgpu_packet_row r;
        r.offset = o.offset;
        r.len = o.len;
        r.packet_id = o.packet_id;
        r.arrival = m.arrival;
        r.source = p >= from_batch ? src[p & D.pk_mask] : EDGPU_NO_SOURCE;
        r._pad = 0;
        rows[base + i] = r;
    }
}
// edgpu_fanout_active: the sub-stream rows of the current pass that carry descriptors or are new,
// in table order.  k_sub_active_count: per workgroup of 256 rows its count; k_sub_active_write: its base
// (the counts of the workgroups before it, reduced in LDS), each active row's rank (wave ballots
// + the waves' counts), the row and its index stored at base + rank (straight into pinned host
// memory when the caller gave it); the last workgroup stores the total.
__global__ __launch_bounds__(256) void k_sub_active_count(const edgpu_substream_out* sub, uint32_t n, uint32_t* blk) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const int act = i < n && (sub[i].desc_count != 0 || (sub[i].flags & EDGPU_SUB_NEW));
    const int c = __syncthreads_count(act);
    if (threadIdx.x == 0) blk[blockIdx.x] = (uint32_t)c;
}

__global__ __launch_bounds__(256) void k_sub_active_write(const edgpu_substream_out* sub, uint32_t n, const uint32_t* blk,
                                                          edgpu_substream_out* rows, uint32_t* q, uint32_t cap,
                                                          uint32_t* total) {
    __shared__ uint32_t s_part[256];
    __shared__ uint32_t s_wave[4];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    uint32_t part = 0;
    for (uint32_t b = tid; b < blockIdx.x; b += 256) part += blk[b];
    s_part[tid] = part;
    const uint32_t i = blockIdx.x * 256 + tid;
    const bool act = i < n && (sub[i].desc_count != 0 || (sub[i].flags & EDGPU_SUB_NEW));
    const uint64_t m = __ballot(act);
    if (lane == 0) s_wave[wid] = (uint32_t)__popcll(m);
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (tid < s) s_part[tid] += s_part[tid + s];
        __syncthreads();
    }
    uint32_t pos = s_part[0];
    for (int w = 0; w < wid; w++) pos += s_wave[w];
    pos += (uint32_t)__popcll(m & ((1ull << lane) - 1));
    if (act && pos < cap) {
        rows[pos] = sub[i];
        q[pos] = i;
    }
    if (blockIdx.x == gridDim.x - 1 && tid == 0)
        *total = s_part[0] + s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
}

hipError_t launch_sub_active(const edgpu_substream_out* sub, uint32_t n, uint32_t* blk, edgpu_substream_out* rows,
                             uint32_t* q, uint32_t cap, uint32_t* total, hipStream_t st) {
    const uint32_t nb = (n + 255) / 256;
    if (!nb) return hipSuccess;
    EDGPU_LAUNCH(k_sub_active_count, dim3(nb), dim3(256), 0, st, sub, n, blk);
    EDGPU_LAUNCH(k_sub_active_write, dim3(nb), dim3(256), 0, st, sub, n, blk, rows, q, cap, total);
    return hipGetLastError();
}

hipError_t launch_sub_rows(const SubDev* subs, const SenderDev* senders, const edgpu_out_desc* desc, const uint32_t* sel,
                           uint32_t nsel, uint32_t nsubs, uint32_t pass, uint32_t epoch, edgpu_packet_row* rows,
                           uint64_t nrows, hipStream_t st) {
    if (nsel) EDGPU_LAUNCH(k_sub_rows, dim3((nsel + 3) / 4), dim3(256), 0, st, subs, senders, desc, sel, nsel,
                                 nsubs, pass, epoch, rows, nrows);
    return hipGetLastError();
}


hipError_t launch_ingest(const IngestParams& p, uint32_t nseg, hipStream_t st) {
    if (nseg == 0) {                         // still the (empty) ingest's counters
        EDGPU_LAUNCH(k_totals_reset, dim3(1), dim3(64), 0, st, p.totals, 1);
        return hipGetLastError();
    }
    // descriptor batches in the blob take the speculative copy (k_ingest SPEC); frames inside a
    // TCP byte stream find their lengths in their own first bytes and keep the header-first order
    const bool spec = !p.tcp_groups && !p.src_addr && EDGPU_COPY_MODE(p) == 0 && p.spec_min && p.npk >= (uint64_t)p.spec_min * nseg;
#ifdef EDGPU_AB_VARIANTS   // measurement builds: the ingest shapes of Appendix A.2
    static const int depth = [] { const char* v = getenv("EDGPU_INGEST_DEPTH"); return v ? atoi(v) : 4; }();
    static const int threads = [] { const char* v = getenv("EDGPU_INGEST_THREADS"); return v && atoi(v) == 512 ? 512 : 256; }();
    if (threads == 512) EDGPU_LAUNCH((k_ingest<4, 512>), dim3(nseg), dim3(512), 0, st, p);
    else if (depth == 2) EDGPU_LAUNCH(k_ingest<2>, dim3(nseg), dim3(kIngestThreads), 0, st, p);
    else if (spec && !getenv("EDGPU_INGEST_NOSPEC")) EDGPU_LAUNCH((k_ingest<4, kIngestThreads, true>), dim3(nseg), dim3(kIngestThreads), 0, st, p);
    else EDGPU_LAUNCH(k_ingest<4>, dim3(nseg), dim3(kIngestThreads), 0, st, p);
    if (p.npk && EDGPU_COPY_MODE(p) == 1) {
        const uint32_t per = kCopyThreads / kCopyLanes;
        EDGPU_LAUNCH(k_ingest_copy, dim3((p.npk + per - 1) / per), dim3(kCopyThreads), 0, st, p);
    }
#else
    if (spec) EDGPU_LAUNCH((k_ingest<4, kIngestThreads, true>), dim3(nseg), dim3(kIngestThreads), 0, st, p);
    else EDGPU_LAUNCH(k_ingest<4>, dim3(nseg), dim3(kIngestThreads), 0, st, p);
#endif
    return hipGetLastError();
}
hipError_t launch_image(const ImageParams& p, int phase, hipStream_t st) {
    if (p.nplan == 0) return hipSuccess;
    if (phase == 0) EDGPU_LAUNCH(k_image_plan, dim3((p.nplan + 255) / 256), dim3(256), 0, st, p);
    else if (phase == 1) EDGPU_LAUNCH(k_image_pack, dim3(p.nplan), dim3(256), 0, st, p);
    else if (phase == 2) EDGPU_LAUNCH(k_image_apply, dim3(p.nplan), dim3(256), 0, st, p);
    else EDGPU_LAUNCH(k_image_fit, dim3((p.nplan + 255) / 256), dim3(256), 0, st, p);
    return hipGetLastError();
}
hipError_t launch_first_packet_info(const FirstInfoQuery* q, FirstInfoResult* r, const SenderDev* senders,
                                    uint32_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    EDGPU_LAUNCH(k_first_packet_info, dim3((n + 63) / 64), dim3(64), 0, st, q, r, senders, n);
    return hipGetLastError();
}
hipError_t launch_blocked(const BlockedParams& p, hipStream_t st) {
    if (p.n) EDGPU_LAUNCH(k_blocked, dim3((p.n + 63) / 64), dim3(64), 0, st, p);
    return hipGetLastError();
}

hipError_t launch_plan(const PlanParams& p, hipStream_t st) {
    const uint32_t nsb = p.T.nsenders ? (p.T.nsenders + 255) / 256 : 0;
    if (nsb) EDGPU_LAUNCH(k_plan_senders, dim3((p.T.nsenders + 3) / 4), dim3(256), 0, st, p);
    else EDGPU_LAUNCH(k_totals_reset, dim3(1), dim3(64), 0, st, p.totals, 0);
    if (p.T.nsub_blocks) EDGPU_LAUNCH(k_plan_subs, dim3(p.T.nsub_blocks), dim3(256), 0, st, p);
    const uint32_t nfb = max(p.T.nsub_blocks, nsb);
    if (nfb) EDGPU_LAUNCH(k_plan_final, dim3(nfb), dim3(256), 0, st, p);
    return hipGetLastError();
}
// A sender ring moved into a larger one (ring growth): kind 0 the PktMeta ring, 1 its blob-slot
// array (uint32 per entry), 2 the byte ring (16-B words); entries [lo, lo + n).
hipError_t launch_ring_move(int kind, const void* src, uint64_t smask, void* dst, uint64_t dmask, uint64_t lo, uint64_t n,
                            hipStream_t st) {
    if (!n) return hipSuccess;
    const uint64_t nb = (n + 255) / 256;
    const uint32_t blocks = (uint32_t)(nb < 4096 ? nb : 4096);
    if (kind == 0)
        EDGPU_LAUNCH(k_ring_move<PktMeta>, dim3(blocks), dim3(256), 0, st, (const PktMeta*)src, smask, (PktMeta*)dst, dmask, lo, n);
    else if (kind == 1)
        EDGPU_LAUNCH(k_ring_move<uint32_t>, dim3(blocks), dim3(256), 0, st, (const uint32_t*)src, smask, (uint32_t*)dst, dmask, lo, n);
    else
        EDGPU_LAUNCH(k_ring_move<u32x4>, dim3(blocks), dim3(256), 0, st, (const u32x4*)src, smask, (u32x4*)dst, dmask, lo, n);
    return hipGetLastError();
}
hipError_t launch_plan_pass(const PlanParams& p, hipStream_t st) {
    EDGPU_LAUNCH(k_plan_pass, dim3(max(p.T.nsub_blocks, 1u)), dim3(256), 0, st, p);
    return hipGetLastError();
}
// Fan-out variants (EDGPU_FANOUT env var, for A/B measurement).  Each entry: kernel,
// threads per workgroup, packets per work item.
static int occupancy_of(const void* fn, int threads, int lds) {
    int blocks = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, threads, lds) != hipSuccess) return 1;
    return blocks > 0 ? blocks : 1;
}
struct FanoutVariant { const void* fn; int threads; int chunk; int lds; int max_wg_per_cu = 0; };
#ifdef EDGPU_AB_VARIANTS
static const FanoutVariant kVariants[] = {
    {(const void*)k_fanout3<1024, 32>, 1024, 32, fanout3_lds<1024, 32>()},          // 0 r01 LDS, aligned
    {(const void*)k_fanout3<512, 16>, 512, 16, fanout3_lds<512, 16>()},             // 1
    {(const void*)k_fanout4<1024, 32>, 1024, 32, fanout4_lds<1024, 32>()},          // 2 scalar headers, prefetch
    {(const void*)k_fanout4<512, 32>, 512, 32, fanout4_lds<512, 32>()},             // 3
    {(const void*)k_fanout4<1024, 16>, 1024, 16, fanout4_lds<1024, 16>()},          // 4
    {(const void*)k_fanout4<512, 16>, 512, 16, fanout4_lds<512, 16>()},             // 5
    {(const void*)k_fanout5<256, 32>, 256, 32, fanout5_lds<256, 32>()},             // 6 LDS-DMA, 4 waves/CU
    {(const void*)k_fanout5<512, 32>, 512, 32, fanout5_lds<512, 32>()},             // 7
    {(const void*)k_fanout5<128, 16>, 128, 16, fanout5_lds<128, 16>()},             // 8
    {(const void*)k_fanout5<256, 16>, 256, 16, fanout5_lds<256, 16>()},             // 9
    {(const void*)k_fanout4<1024, 32, 2>, 1024, 32, fanout4_lds<1024, 32>()},       // 10 nt arena stores
    {(const void*)k_fanout4<1024, 32, 16>, 1024, 32, fanout4_lds<1024, 32>()},      // 11 sc1
    {(const void*)k_fanout4<1024, 32, 17>, 1024, 32, fanout4_lds<1024, 32>()},      // 12 sc0 sc1
    {(const void*)k_fanout4<1024, 32, 2, 1>, 1024, 32, fanout4_lds<1024, 32>()},    // 13 nt arena + descriptors
    {(const void*)k_fanout4<1024, 32, 2, 1, 2>, 1024, 32, fanout4_lds<1024, 32>()}, // 14 ... + nt chunk loads
    {(const void*)k_fanout4<1024, 32, 2, 0, 2>, 1024, 32, fanout4_lds<1024, 32>()}, // 15 nt arena + nt loads
    {(const void*)k_fanout5<256, 32, 2>, 256, 32, fanout5_lds<256, 32>()},          // 16 LDS-DMA + nt arena
    {(const void*)k_fanout5<512, 32, 2>, 512, 32, fanout5_lds<512, 32>()},          // 17
    {(const void*)k_fanout4<512, 32, 2>, 512, 32, fanout4_lds<512, 32>()},          // 18 nt, 512 threads
    {(const void*)k_fanout4<1024, 16, 2>, 1024, 16, fanout4_lds<1024, 16>()},       // 19 nt, 16-packet chunks
    {(const void*)k_fanout4<1024, 36, 2>, 1024, 36, fanout4_lds<1024, 36>()},       // 20 nt, 36 (2 WG/CU)
    {(const void*)k_fanout4<1024, 48, 2>, 1024, 48, fanout4_lds<1024, 48>()},       // 21 nt, 48 (1 WG/CU)
    {(const void*)k_fanout4<1024, 56, 2>, 1024, 56, fanout4_lds<1024, 56>()},       // 22 nt, 56 (1 WG/CU)
    {(const void*)k_fanout4<1024, 56, 2, 0, 0, 4>, 1024, 56, fanout4_lds<1024, 56>()}, // 23 + 4-deep store loop
    {(const void*)k_fanout4<1024, 56, 2, 0, 0, 2>, 1024, 56, fanout4_lds<1024, 56>()}, // 24 + 2-deep
    {(const void*)k_fanout4<1024, 32, 2, 0, 0, 2>, 1024, 32, fanout4_lds<1024, 32>()}, // 25 32, 2-deep
    {(const void*)k_fanout4<1024, 32, 2, 0, 0, 1, 8>, 1024, 32, fanout4_lds<1024, 32>()}, // 26 32, <= 64 VGPRs
    {(const void*)k_fanout4<1024, 32, 2, 0, 0, 1, 0, 1>, 1024, 32, fanout4_lds<1024, 32>()}, // 27 row-mask patch
    {(const void*)k_fanout4<1024, 56, 2, 0, 0, 1, 0, 1>, 1024, 56, fanout4_lds<1024, 56>()}, // 28 56, row-mask
    {(const void*)k_fanout4<1024, 32, 2, 0, 0, 1, 0, 0, 1>, 1024, 32, fanout4_lds<1024, 32, 1>()}, // 29 LDS FanSub
    {(const void*)k_fanout4<1024, 56, 2, 0, 0, 1, 0, 0, 1>, 1024, 56, fanout4_lds<1024, 56, 1>()}, // 30 56, LDS FanSub
    {(const void*)k_fanout4<1024, 32, 2, 0, 0, 1, 0, 0, 0, 1>, 1024, 32, fanout4_lds<1024, 32>()}, // 31 dynamic items
    {(const void*)k_fanout4<1024, 56, 2, 0, 0, 1, 0, 0, 0, 1>, 1024, 56, fanout4_lds<1024, 56>()}, // 32 56, dynamic
    {(const void*)k_fanout4<1024, 32, 2, 0, 0, 1, 8, 0, 0, 1>, 1024, 32, fanout4_lds<1024, 32>()}, // 33 32, <= 64 VGPRs, dynamic
    {(const void*)k_fanout4<1024, 48, 2, 0, 0, 1, 0, 0, 0, 1>, 1024, 48, fanout4_lds<1024, 48>()}, // 34 48, dynamic
    {(const void*)k_fanout4<1024, 32, 2, 0, 0, 1, 0, 0, 0, 1, 1>, 1024, 32, fanout4_lds<1024, 32>()}, // 35 dyn, patch path always
    {(const void*)k_fanout4<1024, 32, 2, 0, 0, 1, 0, 0, 0, 1, 2>, 1024, 32, fanout4_lds<1024, 32>()}, // 36 dyn, s_sleep per row
    {(const void*)k_fanout4<1024, 32, 2, 0, 0, 1, 0, 0, 0, 1, 0, 1>, 1024, 32, fanout4_lds<1024, 32>()}, // 37 dyn, two windows at once
    {(const void*)k_fanout4<1024, 56, 2, 0, 0, 1, 0, 0, 0, 1, 0, 1>, 1024, 56, fanout4_lds<1024, 56>()}, // 38 56, dyn, two windows
    {(const void*)k_fanout6<1024, 32>, 1024, 32, fanout6_lds<1024, 32>()},          // 39 two images, one barrier per item
    {(const void*)k_fanout6<1024, 16>, 1024, 16, fanout6_lds<1024, 16>()},          // 40 same, 16-packet chunks (2 WG/CU)
    {(const void*)k_fanout6<1024, 18>, 1024, 18, fanout6_lds<1024, 18>()},          // 41 18 packets (2 WG/CU)
    {(const void*)k_fanout6<1024, 12>, 1024, 12, fanout6_lds<1024, 12>()},          // 42 12 packets (2 WG/CU)
    {(const void*)k_fanout6<512, 16>, 512, 16, fanout6_lds<512, 16>()},             // 43 16 packets, 512 threads
    {(const void*)k_fanout6<1024, 16>, 1024, 16, fanout6_lds<1024, 16>(), 1},       // 44 = 40 at one workgroup per CU
    {(const void*)k_fanout6<1024, 18>, 1024, 18, fanout6_lds<1024, 18>(), 1},       // 45 = 41 at one workgroup per CU
    {(const void*)k_fanout4<1024, 16, 2, 0, 0, 1, 0, 0, 0, 1>, 1024, 16, fanout4_lds<1024, 16>()}, // 46 16, dynamic (k_fanout4)
    {(const void*)k_fanout4<1024, 16, 2, 0, 0, 1, 0, 1, 0, 1>, 1024, 16, fanout4_lds<1024, 16>()}, // 47 16, dynamic, row-mask patch
    {(const void*)k_fanout4<1024, 24, 2, 0, 0, 1, 0, 0, 0, 1>, 1024, 24, fanout4_lds<1024, 24>()}, // 48 24, dynamic
    {(const void*)k_fanout4<1024, 24, 2, 0, 0, 1, 0, 1, 0, 1>, 1024, 24, fanout4_lds<1024, 24>()}, // 49 24, dynamic, row-mask patch
    {(const void*)k_fanout6<1024, 16, 2, 1>, 1024, 16, fanout6_lds<1024, 16>()},    // 50 16, per-packet patch
    {(const void*)k_fanout6<1024, 32, 2, 1>, 1024, 32, fanout6_lds<1024, 32>()},    // 51 32, per-packet patch
    {(const void*)k_fanout6<1024, 14>, 1024, 14, fanout6_lds<1024, 14>()},          // 52 14 packets
    {(const void*)k_fanout6<1024, 20>, 1024, 20, fanout6_lds<1024, 20>()},          // 53 20
    {(const void*)k_fanout6<1024, 22>, 1024, 22, fanout6_lds<1024, 22>()},          // 54 22 (a C2 window: 2 rows)
    {(const void*)k_fanout6<1024, 23>, 1024, 23, fanout6_lds<1024, 23>()},          // 55 23
    {(const void*)k_fanout6<768, 16>, 768, 16, fanout6_lds<768, 16>()},             // 56 768 threads: a C2 window in 2 rows
    {(const void*)k_fanout6<768, 18>, 768, 18, fanout6_lds<768, 18>()},             // 57
    {(const void*)k_fanout6<896, 16>, 896, 16, fanout6_lds<896, 16>()},             // 58
    {(const void*)k_fanout6<768, 12>, 768, 12, fanout6_lds<768, 12>()},             // 59
    {(const void*)k_fanout6<1024, 16, 2, 0, 1>, 1024, 16, fanout6_lds<1024, 16>()}, // 60 16, FanSub one window ahead
    {(const void*)k_fanout6<1024, 32, 2, 0, 1>, 1024, 32, fanout6_lds<1024, 32>()}, // 61 32, same
    {(const void*)k_fanout6<1024, 16, 2, 0, 0, 1>, 1024, 16, fanout6_lds<1024, 16>()}, // 62 16, branchy patch
    {(const void*)k_fanout6<1024, 32, 2, 0, 0, 1>, 1024, 32, fanout6_lds<1024, 32>()}, // 63 32, branchy patch
};
static const char* const kVariantNames[] = {"k_fanout3<1024,32>", "k_fanout3<512,16>", "k_fanout4<1024,32>",
                                            "k_fanout4<512,32>", "k_fanout4<1024,16>", "k_fanout4<512,16>",
                                            "k_fanout5<256,32>", "k_fanout5<512,32>", "k_fanout5<128,16>", "k_fanout5<256,16>",
                                            "k_fanout4<1024,32,nt>", "k_fanout4<1024,32,sc1>", "k_fanout4<1024,32,sc0sc1>",
                                            "k_fanout4<1024,32,nt,ntdesc>", "k_fanout4<1024,32,nt,ntdesc,ntload>",
                                            "k_fanout4<1024,32,nt,ntload>", "k_fanout5<256,32,nt>", "k_fanout5<512,32,nt>",
                                            "k_fanout4<512,32,nt>", "k_fanout4<1024,16,nt>",
                                            "k_fanout4<1024,36,nt>", "k_fanout4<1024,48,nt>", "k_fanout4<1024,56,nt>",
                                            "k_fanout4<1024,56,nt,su4>", "k_fanout4<1024,56,nt,su2>",
                                            "k_fanout4<1024,32,nt,su2>", "k_fanout4<1024,32,nt,wpe8>",
                                            "k_fanout4<1024,32,nt,rowmask>", "k_fanout4<1024,56,nt,rowmask>",
                                            "k_fanout4<1024,32,nt,ldsfansub>", "k_fanout4<1024,56,nt,ldsfansub>",
                                            "k_fanout4<1024,32,nt,dyn>", "k_fanout4<1024,56,nt,dyn>",
                                            "k_fanout4<1024,32,nt,wpe8,dyn>", "k_fanout4<1024,48,nt,dyn>",
                                            "k_fanout4<1024,32,nt,dyn,patchall>", "k_fanout4<1024,32,nt,dyn,sleep>",
                                            "k_fanout4<1024,32,nt,dyn,2win>", "k_fanout4<1024,56,nt,dyn,2win>",
                                            "k_fanout6<1024,32,nt,dyn>", "k_fanout6<1024,16,nt,dyn>",
                                            "k_fanout6<1024,18,nt,dyn>", "k_fanout6<1024,12,nt,dyn>", "k_fanout6<512,16,nt,dyn>",
                                            "k_fanout6<1024,16,nt,dyn,1wg>", "k_fanout6<1024,18,nt,dyn,1wg>",
                                            "k_fanout4<1024,16,nt,dyn>", "k_fanout4<1024,16,nt,rowmask,dyn>",
                                            "k_fanout4<1024,24,nt,dyn>", "k_fanout4<1024,24,nt,rowmask,dyn>",
                                            "k_fanout6<1024,16,nt,dyn,pp>", "k_fanout6<1024,32,nt,dyn,pp>",
                                            "k_fanout6<1024,14,nt,dyn>", "k_fanout6<1024,20,nt,dyn>",
                                            "k_fanout6<1024,22,nt,dyn>", "k_fanout6<1024,23,nt,dyn>",
                                            "k_fanout6<768,16,nt,dyn>", "k_fanout6<768,18,nt,dyn>",
                                            "k_fanout6<896,16,nt,dyn>", "k_fanout6<768,12,nt,dyn>",
                                            "k_fanout6<1024,16,nt,dyn,pf>", "k_fanout6<1024,32,nt,dyn,pf>",
                                            "k_fanout6<1024,16,nt,dyn,bp>", "k_fanout6<1024,32,nt,dyn,bp>"};
#else
// The shipped library: the two defaults.  The measurement build above keeps
// their numbers (31 and 40) and every variant they were chosen over.
static const FanoutVariant kVariants[] = {
    {(const void*)k_fanout4<1024, 32, 2, 0, 0, 1, 0, 0, 0, 1>, 1024, 32, fanout4_lds<1024, 32>()}, // 0 = AB 31
    {(const void*)k_fanout6<1024, 16>, 1024, 16, fanout6_lds<1024, 16>()},                           // 1 = AB 40
};
static const char* const kVariantNames[] = {"k_fanout4<1024,32,nt,dyn>", "k_fanout6<1024,16,nt,dyn>"};
#endif
static const int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);
static_assert(sizeof(kVariantNames) / sizeof(kVariantNames[0]) == sizeof(kVariants) / sizeof(kVariants[0]),
              "one name per fan-out variant");
// Defaults (items claimed dynamically, non-temporal arena stores): k_fanout6<1024,16> when no
// sub-stream of the tick needs a per-output patch (all UDP, identity: the reference's parity
// mode), k_fanout4<1024,32> when some do (RTSP-interleaved channel byte or a rewrite).  The
// 16-packet chunks are ~4 % faster on identity windows but ~25 % slower through the patch path
// (profiles/r02z9_*).
#ifdef EDGPU_AB_VARIANTS
static const int kDefaultVariant = 31;   // k_fanout4<1024,32,nt,dyn>: the patching default
static const int kDefaultPlain = 40;     // k_fanout6<1024,16,nt,dyn>: every sub-stream identity UDP
static const int kFirstRewriting = 2;    // k_fanout3 (0, 1) reads SubDev directly and has no rewrite stage
#else
static const int kDefaultVariant = 0;
static const int kDefaultPlain = 1;
static const int kFirstRewriting = 0;
#endif
int fanout_default(bool patching) { return patching ? kDefaultVariant : kDefaultPlain; }
// edgpu_subscriber_rewrite refuses a variant without a rewrite stage
bool fanout_rewrites(int variant) {
    if (variant < 0 || variant >= kNumVariants) variant = kDefaultVariant;
    return variant >= kFirstRewriting;
}
int fanout_chunk(int variant) {
    if (variant < 0 || variant >= kNumVariants) variant = kDefaultVariant;
    return kVariants[variant].chunk;
}
const char* fanout_name(int variant) {
    if (variant < 0 || variant >= kNumVariants) variant = kDefaultVariant;
    return kVariantNames[variant];
}
hipError_t launch_fanout(const FanoutParams& p, int variant, int num_cus, hipStream_t st) {
    if (variant < 0 || variant >= kNumVariants) variant = kDefaultVariant;
    static int occ[64] = {0};
    const FanoutVariant& v = kVariants[variant];
    if (!occ[variant]) {
        if (v.lds > 48 * 1024) (void)hipFuncSetAttribute(v.fn, hipFuncAttributeMaxDynamicSharedMemorySize, v.lds);
        occ[variant] = occupancy_of(v.fn, v.threads, v.lds);
        if (v.max_wg_per_cu && occ[variant] > v.max_wg_per_cu) occ[variant] = v.max_wg_per_cu;
    }
    void* args[] = {(void*)&p};
    ++tl_launches;
    return hipLaunchKernel(v.fn, dim3(num_cus * occ[variant]), dim3(v.threads), args, v.lds, st);
}
}  // namespace edgpu
