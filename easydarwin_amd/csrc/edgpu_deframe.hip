// edgpu_deframe.hip -- RTSP-interleaved push ingest on gfx950: '$'-deframing of pusher TCP reads.
//
// Reference behaviour (RTSPRequestStream::ReadRequest, Server.tproj/RTSPRequestStream.cpp:65-171,
// called per readable event by RTSPSession::Run, RTSPSession.cpp:240-262): a connection's bytes
// collect in a 2 KiB request buffer; a '$' at a frame boundary starts a frame of 4 + BE16(len)
// bytes that is handed to ProcessRTPData once complete; anything else is an RTSP request; a
// frame that cannot fit the 2047 usable buffer bytes ends the connection.  The CPU walks that
// chain one header at a time.
//
// Here a session's stream (carried partial frame ++ this call's reads) is cut into 32 KiB
// chunks.  A frame starts at most kTcpMaxFrame - 1 bytes before a chunk boundary, so the true
// walk enters each chunk at a '$' within its first kTcpMaxFrame bytes.
//   k_tcp_walk     two chunks per wave: finds their candidates (aligned 16-B loads, all
//                  lanes), walks every candidate to the chunk end at once (a lane each, half a
//                  wave per chunk; header bytes only), records its first kTcpFrames frame starts
//                  and links its exit to the next chunk's candidate.
//   k_tcp_resolve  one workgroup per session: follows the links in LDS (one hop per chunk),
//                  scans the chunks' frame counts.
//   k_tcp_scan     sessions -> ingest segments, capacity check (one workgroup).
//   k_tcp_finish   one wave per session: descriptors for the chunks the walk did not record
//                  (re-walked), the staging of a frame that starts in the carried bytes, the new
//                  carry and the per-read report.
// k_ingest then finds every recorded frame itself -- its chunk from the per-chunk frame ends,
// its start from the walk's records, its length and channel from its '$' header -- and copies
// it out of the TCP bytes into the sender rings (IngestParams.tcp_groups): no per-frame
// descriptor pass.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "edgpu.h"
#include "edgpu_device.h"
#include "edgpu_params.h"
#include "edgpu_bytes.h"

namespace edgpu {

namespace {

// A session's stream in this call: carry[0, clen) ++ raw[0, len - clen).
struct TcpView {
    const uint8_t* carry;
    const uint8_t* raw;     // P.raw + raw_off
    uint32_t clen;
    uint64_t len;
};

__device__ __forceinline__ TcpView tcp_view(const TcpParams& P, const TcpGroup& G) {
    TcpView v;
    v.carry = P.carry + (uint64_t)G.session * kTcpCarry;
    v.raw = P.raw + G.raw_off;
    v.clen = G.carry_len;
    v.len = G.len;
    return v;
}

__device__ __forceinline__ uint32_t tbyte(const TcpView& v, uint64_t p) {
    return p < v.clen ? v.carry[p] : v.raw[p - v.clen];
}

// One step of ReadRequest's '$' branch at frame boundary `pos`: kWalkRun with the frame length,
// or why the walk stops there.
__device__ __forceinline__ uint32_t tcp_step(const TcpView& v, uint64_t pos, uint32_t& flen) {
    if (pos >= v.len) return kWalkPartial;                         // nothing left (carry 0)
    uint32_t b0, b2, b3;
    if (pos >= v.clen && pos + 4 <= v.len) {                       // the common case: 3 loads at once
        const uint8_t* q = v.raw + (pos - v.clen);
        b0 = q[0]; b2 = q[2]; b3 = q[3];
    } else {
        b0 = tbyte(v, pos);
        b2 = pos + 2 < v.len ? tbyte(v, pos + 2) : 0u;
        b3 = pos + 3 < v.len ? tbyte(v, pos + 3) : 0u;
    }
    if (b0 != 0x24u) return kWalkMessage;
    if (pos + 4 > v.len) return kWalkPartial;
    flen = 4 + (b2 << 8 | b3);
    if (flen > kTcpMaxFrame) return v.len - pos >= kTcpMaxFrame ? kWalkDropped : kWalkPartial;
    if (pos + flen > v.len) return kWalkPartial;
    return kWalkRun;
}

// Walks from `pos` until reaching `end` or a stop; counts frames, recording the first
// kTcpFrames starts (chunk offsets from `start`) in `rec` when given.
//
// Each step's header load waits on the previous frame's length, so a chunk's ~23 frames are ~23
// HBM latencies in a row.  With kTcpSpec > 0 the walk also guesses: after a frame of length L it
// loads the headers at pos + j·L (j < kTcpSpec) at once, as if the next frames had length L too
// (FU-A fragments of one video frame all do), then checks them in order.  A guessed header is
// used only once every frame before it had length exactly L, i.e. once it is known to be the
// true next frame start, and each is judged by tcp_step's own rules, so the walk's frames, stop
// code and exit are the sequential walk's; a wrong guess costs nothing but its loads.
__device__ __forceinline__ uint32_t tcp_walk(const TcpView& v, uint64_t& pos, uint64_t start, uint64_t end,
                                             uint32_t& nf, uint16_t* rec) {
    nf = 0;
    while (pos < end) {
        uint32_t flen = 0;
        const uint32_t code = tcp_step(v, pos, flen);
        if (code != kWalkRun) return code;
        if (rec && nf < kTcpFrames) rec[nf] = (uint16_t)(pos - start);
        nf++;
        pos += flen;
        if constexpr (kTcpSpec > 0) {
            const uint32_t L = flen;
            bool more = pos >= v.clen;                        // guesses only in the raw reads
            while (more) {                                    // one burst of kTcpSpec guesses
                more = false;
                uint32_t h[kTcpSpec ? kTcpSpec : 1];          // b0 | b2 << 8 | b3 << 16, or ~0u
#pragma unroll
                for (uint32_t j = 0; j < kTcpSpec; j++) {
                    const uint64_t q = pos + (uint64_t)j * L;
                    h[j] = ~0u;
                    if (q < end && q + 4 <= v.len) {          // tcp_step's fast branch at q
                        const uint8_t* b = v.raw + (q - v.clen);
                        h[j] = (uint32_t)b[0] | (uint32_t)b[2] << 8 | (uint32_t)b[3] << 16;
                    }
                }
#pragma unroll
                for (uint32_t j = 0; j < kTcpSpec; j++) {
                    if (h[j] == ~0u) break;                   // past the chunk / near the stream end
                    if ((h[j] & 0xFFu) != 0x24u) return kWalkMessage;
                    const uint32_t fl = 4 + ((h[j] >> 8 & 0xFFu) << 8 | (h[j] >> 16));
                    if (fl > kTcpMaxFrame) return v.len - pos >= kTcpMaxFrame ? kWalkDropped : kWalkPartial;
                    if (pos + fl > v.len) return kWalkPartial;
                    if (rec && nf < kTcpFrames) rec[nf] = (uint16_t)(pos - start);
                    nf++;
                    pos += fl;
                    if (fl != L) break;                       // later guesses are off the chain
                    if (j == kTcpSpec - 1) more = true;       // every guess held: guess on
                }
            }
        }
    }
    return kWalkRun;
}

// '$' bytes among the first kTcpMaxFrame bytes of the chunk at `start` (offsets, in order; the
// first kTcpCands kept in `list`); the stream's first chunk has the single candidate 0.  One
// wave: aligned 16-B blocks, one per lane per round (the window spans at most 129 blocks),
// a per-byte '$' mask, and a wave prefix sum for the order; returns the full count
// (> kTcpCands: overflow).  Chunks after the first start past the carried bytes (a chunk is
// longer than the carry), so the window lies in the raw reads.
__device__ __forceinline__ uint32_t dollar_mask(u32x4 w) {
    uint32_t m = 0;
    const uint32_t d[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int i = 0; i < 16; i++)
        m |= (((d[i >> 2] >> (8 * (i & 3))) & 0xFFu) == 0x24u ? 1u : 0u) << i;
    return m;
}

[[maybe_unused]] __device__ uint32_t tcp_candidates(const TcpView& v, uint64_t start, uint16_t* list, int lane) {
    if (start == 0) {
        if (lane == 0) list[0] = 0;
        return 1;
    }
    const uint64_t wend = min(start + (uint64_t)kTcpMaxFrame, v.len);
    const uintptr_t lo = (uintptr_t)(v.raw + (start - v.clen));
    const uintptr_t hi = (uintptr_t)(v.raw + (wend - v.clen));
    const uintptr_t al = lo & ~(uintptr_t)15;
    uint32_t n = 0;
    for (uint32_t round = 0; al + 16 * 64 * (uintptr_t)round < hi; round++) {
        const uintptr_t b = al + 16 * (uintptr_t)(lane + 64 * round);
        uint32_t mask = 0;
        if (b < hi) {
            mask = dollar_mask(*reinterpret_cast<const u32x4*>(b));
            if (b < lo) mask &= ~((1u << (uint32_t)(lo - b)) - 1u);
            if (b + 16 > hi) mask &= (1u << (uint32_t)(hi - b)) - 1u;
        }
        const uint32_t cnt = (uint32_t)__popc(mask);
        uint32_t incl = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        uint32_t idx = n + incl - cnt;
        while (mask) {
            const int i = __ffs(mask) - 1;
            mask &= mask - 1;
            if (idx < kTcpCands) list[idx] = (uint16_t)(b + i - lo);
            idx++;
        }
        n += __shfl(incl, 63, 64);
    }
    return n;
}

// The same over two windows (a chunk's own and the next chunk's) with every block of both
// loaded before the first is scanned: one load latency instead of up to six in a row.  A window
// spans at most 129 blocks, so three rounds of 64 lanes hold it.
struct CandWin {
    uintptr_t lo = 0, hi = 0, al = 0;
    bool first = false, none = true;
};

[[maybe_unused]] __device__ __forceinline__ CandWin cand_window(const TcpView& v, uint64_t start, bool want) {
    CandWin w;
    if (!want) return w;
    w.none = false;
    if (start == 0) { w.first = true; return w; }
    const uint64_t wend = min(start + (uint64_t)kTcpMaxFrame, v.len);
    w.lo = (uintptr_t)(v.raw + (start - v.clen));
    w.hi = (uintptr_t)(v.raw + (wend - v.clen));
    w.al = w.lo & ~(uintptr_t)15;
    return w;
}

[[maybe_unused]] __device__ __forceinline__ uint32_t cand_scan(const CandWin& w, const u32x4 (&blk)[3], uint16_t* list, int lane) {
    if (w.none) return 0;
    if (w.first) {
        if (lane == 0) list[0] = 0;
        return 1;
    }
    uint32_t n = 0;
#pragma unroll
    for (uint32_t round = 0; round < 3; round++) {
        if (w.al + 16 * 64 * (uintptr_t)round >= w.hi) break;          // uniform
        const uintptr_t b = w.al + 16 * (uintptr_t)(lane + 64 * round);
        uint32_t mask = 0;
        if (b < w.hi) {
            mask = dollar_mask(blk[round]);
            if (b < w.lo) mask &= ~((1u << (uint32_t)(w.lo - b)) - 1u);
            if (b + 16 > w.hi) mask &= (1u << (uint32_t)(w.hi - b)) - 1u;
        }
        const uint32_t cnt = (uint32_t)__popc(mask);
        uint32_t incl = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        uint32_t idx = n + incl - cnt;
        while (mask) {
            const int i = __ffs(mask) - 1;
            mask &= mask - 1;
            if (idx < kTcpCands) list[idx] = (uint16_t)(b + i - w.lo);
            idx++;
        }
        n += __shfl(incl, 63, 64);
    }
    return n;
}

[[maybe_unused]] __device__ __forceinline__ void cand_load(const CandWin& w, u32x4 (&blk)[3], int lane) {
#pragma unroll
    for (uint32_t round = 0; round < 3; round++) {
        const uintptr_t b = w.al + 16 * (uintptr_t)(lane + 64 * round);
        blk[round] = u32x4{0u, 0u, 0u, 0u};
        if (!w.none && !w.first && b < w.hi) blk[round] = *reinterpret_cast<const u32x4*>(b);
    }
}

template <typename T>
__device__ __forceinline__ T block_exclusive_scan256(T v, T* scratch, T& total) {
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
    for (int w = 0; w < 4; w++) {
        T t = scratch[w];
        if (w < wid) base += t;
        tot += t;
    }
    __syncthreads();
    total = tot;
    return base + x - v;
}

}  // namespace

// ---- k_tcp_walk: CPW chunks per wave (kTcpWalkCpw), 4 waves per workgroup ----
// The walk is bound by how many waves are resident (~16k chunks at 32 KiB, ~2 waves per wave
// slot; profiles/r02z31_tcp_walk_sq/), and a chunk's true walk keeps one lane busy while its few
// false candidates end within a step or two.  With CPW = 2 a wave finds both chunks' candidates
// (all 64 lanes, one chunk after the other) and then walks them side by side, lanes 0-31 and
// 32-63 (candidates past 32 in a second pass): half the waves for the same chains.
constexpr int kWalkWaves = 4;

namespace {

struct WalkChunk {
    TcpView v;
    uint64_t start, end;
    uint32_t c, n, nn;
    bool valid;
};

__device__ __forceinline__ WalkChunk walk_chunk_setup(const TcpParams& P, uint32_t c, uint16_t* own, uint16_t* next,
                                                      int lane) {
    WalkChunk w{};
    w.c = c;
    w.valid = c < P.nchunks;
    if (!w.valid) return w;
    const TcpGroup G = P.groups[P.chunk_group[c]];
    w.v = tcp_view(P, G);
    w.start = (uint64_t)(c - G.first_chunk) * kTcpChunk;
    w.end = min(w.start + kTcpChunk, w.v.len);
    if constexpr (EDGPU_TCP_CAND_FUSED) {              // both windows' blocks loaded at once (A/B)
        const CandWin wo = cand_window(w.v, w.start, true), wn = cand_window(w.v, w.end, w.end < w.v.len);
        u32x4 bo[3], bn[3];
        cand_load(wo, bo, lane);
        cand_load(wn, bn, lane);
        w.n = cand_scan(wo, bo, own, lane);
        w.nn = cand_scan(wn, bn, next, lane);
    } else {
        w.n = tcp_candidates(w.v, w.start, own, lane);
        w.nn = w.end < w.v.len ? tcp_candidates(w.v, w.end, next, lane) : 0u;
    }
    return w;
}

// Candidate k of chunk w: walk to the chunk end, record the frame starts, link the exit to the
// next chunk's candidate.
__device__ __forceinline__ void walk_candidate(const TcpParams& P, const WalkChunk& w, uint32_t k,
                                               const uint16_t* own, const uint16_t* next) {
    const size_t ci = (size_t)w.c * kTcpCands + k;
    uint64_t pos = w.start + own[k];
    uint32_t nf;
    const uint32_t code = tcp_walk(w.v, pos, w.start, w.end, nf, P.offs + ci * kTcpFrames);
    uint8_t link = 0xFE;
    if (code == kWalkRun && pos < w.v.len) {                // continues in the next chunk
        link = 0xFF;
        if (w.nn <= kTcpCands) {
            const uint32_t q = (uint32_t)(pos - w.end);
            for (uint32_t i = 0; i < w.nn; i++)
                if (next[i] == q) { link = (uint8_t)i; break; }
        }
    }
    TcpCand r;
    r.q = own[k];
    r.exit = (uint32_t)(pos - w.start);
    r.nframes = nf;
    r.code = code;
    P.cands[ci] = r;
    P.links[ci] = link;
}

}  // namespace

template <int CPW>
__global__ __launch_bounds__(64 * kWalkWaves) __attribute__((amdgpu_waves_per_eu(EDGPU_TCP_WALK_WPE)))
void k_tcp_walk(TcpParams P) {
    static_assert(CPW == 1 || CPW == 2 || CPW == 4, "one, two or four chunks per wave");
    constexpr uint32_t LPC = 64 / CPW;                      // walking lanes per chunk
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __shared__ uint16_t s_own[kWalkWaves][CPW][kTcpCands], s_next[kWalkWaves][CPW][kTcpCands];
    __shared__ WalkChunk s_w[kWalkWaves][CPW];              // each chunk's setup, for its lanes
    const uint32_t c0 = (blockIdx.x * kWalkWaves + wid) * CPW;
    WalkChunk a = walk_chunk_setup(P, c0, s_own[wid][0], s_next[wid][0], lane);
    if (lane == 0) s_w[wid][0] = a;
#pragma unroll
    for (int h = 1; h < CPW; h++) {
        WalkChunk b{};
        if (a.valid && a.end < a.v.len && c0 + h < P.nchunks && P.chunk_group[c0 + h] == P.chunk_group[c0 + h - 1]) {
            // chunk h follows chunk h - 1 in the same stream: its own candidate window is the
            // previous chunk's next window, already scanned -- copy the list, scan only its next
            b.c = c0 + h;
            b.valid = true;
            b.v = a.v;
            b.start = a.end;
            b.end = min(b.start + kTcpChunk, b.v.len);
            b.n = a.nn;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if ((uint32_t)lane < kTcpCands) s_own[wid][h][lane] = s_next[wid][h - 1][lane];
            b.nn = b.end < b.v.len ? tcp_candidates(b.v, b.end, s_next[wid][h], lane) : 0u;
        } else {
            b = walk_chunk_setup(P, c0 + h, s_own[wid][h], s_next[wid][h], lane);
        }
        if (lane == 0) s_w[wid][h] = b;
        a = b;
    }
    __syncthreads();
    const int h = lane / (int)LPC;                          // this lane's chunk
    const WalkChunk m = CPW == 1 ? a : s_w[wid][h];
    const uint32_t sub = (uint32_t)lane % LPC;
    if (!m.valid) return;
    if (sub == 0) P.ncand[m.c] = m.n;
    if (m.n > kTcpCands) return;
    for (uint32_t k = sub; k < m.n; k += LPC) walk_candidate(P, m, k, s_own[wid][h], s_next[wid][h]);
}

// ---- k_tcp_resolve: one workgroup per session; thread 0 follows the links ----
constexpr uint32_t kPiece = 256;        // chunks per LDS pass

__global__ __launch_bounds__(256) void k_tcp_resolve(TcpParams P) {
    const uint32_t g = blockIdx.x;
    const int tid = threadIdx.x;
    const TcpGroup G = P.groups[g];
    const TcpView v = tcp_view(P, G);
    __shared__ uint8_t s_link[kPiece * kTcpCands];
    __shared__ uint8_t s_idx[kPiece];                 // candidate index, 0xFD sequential, 0xFF idle
    __shared__ uint32_t s_nf[kPiece], s_exit[kPiece], s_code[kPiece], s_entry[kPiece];
    __shared__ uint32_t scan32[4];
    __shared__ uint32_t s_stop_code;
    __shared__ uint64_t s_stop;
    if (tid == 0) { s_stop_code = kWalkRun; s_stop = v.len; }
    // chain state (thread 0)
    int j = 0;                  // candidate of the current chunk, -1: search for `entry`
    uint64_t entry = 0;
    bool stopped = false;
    uint32_t fb = 0;
    for (uint32_t k0 = 0; k0 < G.nchunks; k0 += kPiece) {
        const uint32_t np = min(kPiece, G.nchunks - k0);
        const uint32_t c0 = G.first_chunk + k0;
        {
            const uint32_t* src = reinterpret_cast<const uint32_t*>(P.links + (size_t)c0 * kTcpCands);
            uint32_t* dst = reinterpret_cast<uint32_t*>(s_link);
            for (uint32_t w = tid; w < np * kTcpCands / 4; w += 256) dst[w] = src[w];
        }
        __syncthreads();
        if (tid == 0) {
            for (uint32_t kk = 0; kk < np; kk++) {
                const uint32_t c = c0 + kk;
                const uint64_t start = (uint64_t)(k0 + kk) * kTcpChunk;
                const uint64_t end = min(start + kTcpChunk, v.len);
                if (stopped) { s_idx[kk] = 0xFF; continue; }
                const uint32_t n = P.ncand[c];
                if (j < 0) {
                    if (n <= kTcpCands) {                      // entry among the candidates?
                        const uint32_t q = (uint32_t)(entry - start);
                        const TcpCand* cc = P.cands + (size_t)c * kTcpCands;
                        int lo = 0, hi = (int)n - 1;
                        while (lo <= hi) {
                            const int mid = (lo + hi) >> 1;
                            const uint32_t qm = cc[mid].q;
                            if (qm == q) { j = mid; break; }
                            if (qm < q) lo = mid + 1; else hi = mid - 1;
                        }
                    }
                    if (j < 0) {
                        uint64_t pos = entry;
                        uint32_t nf = 0, code;
                        if (n <= kTcpCands) code = kWalkMessage;                        // not a '$'
                        else code = tcp_walk(v, pos, start, end, nf, nullptr);          // too many candidates
                        s_idx[kk] = 0xFD;
                        s_entry[kk] = (uint32_t)(entry - start);
                        s_nf[kk] = nf; s_code[kk] = code; s_exit[kk] = (uint32_t)(pos - start);
                        if (code != kWalkRun || pos >= v.len) stopped = true;
                        else entry = pos;
                        continue;
                    }
                }
                s_idx[kk] = (uint8_t)j;
                const uint8_t l = s_link[kk * kTcpCands + j];
                if (l == 0xFE) {
                    stopped = true;
                } else if (l == 0xFF) {
                    entry = start + P.cands[(size_t)c * kTcpCands + j].exit;
                    j = -1;
                } else {
                    j = l;
                }
            }
        }
        __syncthreads();
        // per chunk of the piece: its true walk's frame count, then the scan
        uint32_t nf = 0, ent = kTcpNone, cand = kTcpNone;
        if ((uint32_t)tid < np) {
            const uint32_t c = c0 + tid;
            const uint64_t start = (uint64_t)(k0 + tid) * kTcpChunk;
            const uint8_t idx = s_idx[tid];
            uint32_t code = kWalkRun, ex = 0;
            bool terminal = false;
            if (idx < kTcpCands) {
                const TcpCand r = P.cands[(size_t)c * kTcpCands + idx];
                nf = r.nframes; ent = r.q; code = r.code; ex = r.exit; cand = idx;
                terminal = s_link[tid * kTcpCands + idx] == 0xFE;
            } else if (idx == 0xFD) {
                nf = s_nf[tid]; ent = s_entry[tid]; code = s_code[tid]; ex = s_exit[tid];
                terminal = code != kWalkRun || start + ex >= v.len;
            }
            if (terminal) { s_stop_code = code; s_stop = start + ex; }
        }
        uint32_t tnf;
        const uint32_t pnf = block_exclusive_scan256<uint32_t>(nf, scan32, tnf);
        if ((uint32_t)tid < np) {
            TcpChunkRes R;
            R.entry = nf ? ent : kTcpNone;
            R.fbase = fb + pnf;
            R.nframes = nf;
            R.cand = cand;
            P.chunkres[c0 + tid] = R;
        }
        fb += tnf;
        __syncthreads();
    }
    if (tid == 0) {
        TcpGroup& W = P.groups[g];
        W.nframes = fb;
        // a walk that ran off the end of the stream stops there: everything framed
        const uint32_t code = s_stop_code;
        W.code = (code == kWalkPartial && s_stop >= v.len) ? kWalkRun : code;
        W.stop = s_stop;
    }
}

// ---- k_tcp_walk_seg: the walk in segments of P.seg chunks, one wave per segment ----
// A candidate walk covers its whole segment: chunk after chunk it records the frames in that
// chunk's row of the same candidate index and links the row to itself in the next chunk, and at
// the segment's end it links to the next segment's candidate as k_tcp_walk does at a chunk's.  So
// k_tcp_resolve follows the links unchanged, and only a segment's first chunk has a candidate
// window: P.seg x fewer windows (2 KiB per 32-KiB chunk, 0.03 GB at C2) and false candidates
// than k_tcp_walk, for walks P.seg x longer -- still beside the fan-out.  The
// other chunks of a segment report more candidates than kept, so a search that lands there (only
// after a sequential fallback) walks sequentially.
__global__ __launch_bounds__(64 * kWalkWaves) __attribute__((amdgpu_waves_per_eu(EDGPU_TCP_WALK_WPE)))
void k_tcp_walk_seg(TcpParams P) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __shared__ uint16_t s_own[kWalkWaves][kTcpCands], s_next[kWalkWaves][kTcpCands];
    const uint32_t c = blockIdx.x * kWalkWaves + wid;
    if (c >= P.nchunks) return;                                   // (per wave: no block barrier below)
    const TcpGroup G = P.groups[P.chunk_group[c]];
    const uint32_t k = c - G.first_chunk;
    if (k % P.seg) {
        if (lane == 0) P.ncand[c] = kTcpCands + 1;
        return;
    }
    const TcpView v = tcp_view(P, G);
    const uint32_t kend = min(k + P.seg, G.nchunks);              // the segment: chunks [k, kend)
    const uint64_t start = (uint64_t)k * kTcpChunk, send = min((uint64_t)kend * kTcpChunk, v.len);
    const uint32_t n = tcp_candidates(v, start, s_own[wid], lane);
    const uint32_t nn = send < v.len ? tcp_candidates(v, send, s_next[wid], lane) : 0u;
    if (lane == 0) P.ncand[c] = n;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");        // the lists, written lane by lane
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (n > kTcpCands) return;                                     // (uniform)
    for (uint32_t j = (uint32_t)lane; j < n; j += 64) {
        uint64_t pos = start + s_own[wid][j];
        for (uint32_t kk = k; kk < kend; kk++) {
            const uint64_t cs = (uint64_t)kk * kTcpChunk, ce = min(cs + kTcpChunk, v.len);
            const size_t ci = (size_t)(G.first_chunk + kk) * kTcpCands + j;
            const uint64_t entry = pos;
            uint32_t nf;
            const uint32_t code = tcp_walk(v, pos, cs, ce, nf, P.offs + ci * kTcpFrames);
            uint8_t link = 0xFE;
            bool more = false;
            if (code == kWalkRun && pos < v.len) {
                if (kk + 1 < kend) {                              // the same walk, the next chunk
                    link = (uint8_t)j;
                    more = true;
                } else {                                          // the next segment's candidate
                    link = 0xFF;
                    if (nn <= kTcpCands) {
                        const uint32_t q = (uint32_t)(pos - send);
                        for (uint32_t i = 0; i < nn; i++)
                            if (s_next[wid][i] == q) { link = (uint8_t)i; break; }
                    }
                }
            }
            TcpCand r;
            r.q = (uint32_t)(entry - cs);
            r.exit = (uint32_t)(pos - cs);
            r.nframes = nf;
            r.code = code;
            P.cands[ci] = r;
            P.links[ci] = link;
            if (!more) break;
        }
    }
}

// ---- k_tcp_chain: k_tcp_walk + k_tcp_resolve in one, each stream walked in order ----
// One lane per session: its walk enters each chunk where the previous chunk's ended, so it reads
// only the true chain's headers -- no candidate windows, no false candidates (the parallel walk's
// ~0.05 GB of the two, r06 C2: DESIGN §5.4).  The hops are one dependent load each; the lanes of a
// wave hop side by side, so 1024 sessions are 16 waves, which keep ~1024 header loads in flight
// beside the previous tick's fan-out.  It writes what k_tcp_resolve writes (chunk results with the
// walk's records as candidate row 0, the group's frames / stop code / stop position), so
// k_tcp_scan, k_tcp_finish and k_ingest run unchanged.
__global__ __launch_bounds__(64) void k_tcp_chain(TcpParams P) {
    const uint32_t g = blockIdx.x * 64 + threadIdx.x;
    if (g >= P.ngroups) return;
    const TcpGroup G = P.groups[g];
    const TcpView v = tcp_view(P, G);
    uint64_t pos = 0, stop = v.len;
    uint32_t fb = 0, stop_code = kWalkRun;
    bool stopped = false;
    for (uint32_t k = 0; k < G.nchunks; k++) {
        const uint32_t c = G.first_chunk + k;
        TcpChunkRes R;
        R.fbase = fb;
        if (stopped) {
            R.entry = kTcpNone; R.nframes = 0; R.cand = kTcpNone;
            P.chunkres[c] = R;
            continue;
        }
        const uint64_t start = (uint64_t)k * kTcpChunk, end = min(start + kTcpChunk, v.len);
        const uint64_t entry = pos;
        uint32_t nf = 0;
        const uint32_t code = tcp_walk(v, pos, start, end, nf, P.offs + (size_t)c * kTcpCands * kTcpFrames);
        TcpCand r;
        r.q = (uint32_t)(entry - start);
        r.exit = (uint32_t)(pos - start);
        r.nframes = nf;
        r.code = code;
        P.cands[(size_t)c * kTcpCands] = r;
        R.entry = nf ? r.q : kTcpNone;
        R.nframes = nf;
        R.cand = 0;
        P.chunkres[c] = R;
        fb += nf;
        if (code != kWalkRun || pos >= v.len) { stopped = true; stop_code = code; stop = pos; }
    }
    TcpGroup& W = P.groups[g];
    W.nframes = fb;
    // a walk that ran off the end of the stream stops there: everything framed
    W.code = (stop_code == kWalkPartial && stop >= v.len) ? kWalkRun : stop_code;
    W.stop = stop;
}

// ---- k_tcp_scan: one 1024-thread workgroup; sessions -> ingest segments ----
// Each thread takes a run of consecutive sessions (one for up to 1024 sessions): all frame
// counts are loaded at once, one block scan places them.
constexpr int kScanThreads = 1024;
__global__ __launch_bounds__(kScanThreads) void k_tcp_scan(TcpParams P) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    constexpr int NW = kScanThreads / 64;
    __shared__ uint32_t s_w[NW];
    const uint32_t per = (P.ngroups + kScanThreads - 1) / kScanThreads;
    const uint32_t g0 = tid * per, g1 = min(g0 + per, P.ngroups);
    uint32_t mine = 0;
    for (uint32_t g = g0; g < g1; g++) mine += P.groups[g].nframes;
    uint32_t x = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[wid] = x;
    __syncthreads();
    uint32_t base = 0, fb = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
        const uint32_t t = s_w[w];
        if (w < wid) base += t;
        fb += t;
    }
    const bool over = fb > P.max_desc;
    uint32_t at = base + x - mine;
    for (uint32_t g = g0; g < g1; g++) {
        const uint32_t nf = P.groups[g].nframes;
        P.groups[g].frame_base = at;
        P.seg_off[g] = over ? 0u : at;
        P.seg_sess[g] = P.groups[g].session;
        at += nf;
    }
    if (tid == 0) {
        P.seg_off[P.ngroups] = over ? 0u : fb;
        P.tot->frames = fb;
        P.tot->status = over ? EDGPU_OUT_OVERFLOW : 0;
    }
}

// ---- k_tcp_finish: one wave per session ----
// k_ingest finds the frames of every chunk whose true walk was recorded itself (IngestParams.
// tcp_groups).  This wave does the rest of the session: a descriptor and a source address per
// frame of the chunks the walk did not record (re-walked here: a chunk entered by the sequential
// fallback, or with more than kTcpFrames frames); the staging of a frame that starts in the
// carried bytes (only the stream's first frame can), then the new carry -- only this wave reads
// the carried bytes after the walk -- and the whole per-read report, frame counts included: a
// recorded chunk's frame ends are its next recorded start (its walk's exit for the last), so the
// report needs no header and is complete when the deframe is, before k_ingest has run.
// A session with no stream bytes has no chunk; its report is the zeros the host cleared.
__global__ __launch_bounds__(64) void k_tcp_finish(TcpParams P) {
    const uint32_t g = blockIdx.x;
    const int lane = threadIdx.x;
    const bool over = P.tot->status != 0;
    const TcpGroup G = P.groups[g];
    const TcpView v = tcp_view(P, G);
    const TcpRead* rd = P.reads + G.first_read;
    __shared__ uint64_t s_pos[64];
    __shared__ uint32_t s_m;
    __shared__ uint64_t s_next;
    // the session's read starts and arrivals (up to 64 reads) in LDS: a frame's read is found by
    // a binary search there instead of a chain of dependent global loads
    __shared__ uint64_t s_rstart[64];
    __shared__ int64_t s_rarr[64];
    __shared__ uint8_t s_carry[kTcpCarry];
    __shared__ uint32_t s_frames[64];                 // per read (up to 64 reads), else global atomics
    const bool lds_reads = G.nreads <= 64;
    if (lds_reads && (uint32_t)lane < G.nreads) { s_rstart[lane] = rd[lane].start; s_rarr[lane] = rd[lane].arrival; }
    s_frames[lane] = 0;
    __syncthreads();
    auto count_frame = [&](uint32_t r) {
        if (lds_reads) atomicAdd(&s_frames[r], 1u);
        else atomicAdd(&P.results[G.first_read + r].frames, 1u);
    };
    for (uint32_t k0 = 0; !over && k0 < G.nchunks; k0 += 64) {
        // the chunks the walk did not record, 64 at a time
        const uint32_t k = k0 + (uint32_t)lane;
        bool rewalk = false;
        if (k < G.nchunks) {
            const TcpChunkRes R = P.chunkres[G.first_chunk + k];
            rewalk = R.entry != kTcpNone && (R.cand == kTcpNone || R.nframes > kTcpFrames);
        }
        uint64_t todo = __ballot(rewalk);
        while (todo) {
            const uint32_t kk = k0 + (uint32_t)(__ffsll((unsigned long long)todo) - 1);
            todo &= todo - 1;
            const TcpChunkRes R = P.chunkres[G.first_chunk + kk];
            const uint64_t start = (uint64_t)kk * kTcpChunk;
            const uint64_t end = min(start + kTcpChunk, v.len);
            uint32_t done = 0;
            uint64_t pos = start + R.entry;
            while (done < R.nframes) {
                if (lane == 0) {                              // the next up to 64 frames
                    uint32_t mm = 0;
                    uint64_t p = pos;
                    while (mm < 64 && p < end) {
                        uint32_t flen = 0;
                        if (tcp_step(v, p, flen) != kWalkRun) break;
                        s_pos[mm++] = p;
                        p += flen;
                    }
                    s_m = mm;
                    s_next = p;
                }
                __syncthreads();
                const uint32_t m = s_m;
                pos = s_next;
                if ((uint32_t)lane < m) {
                    const uint64_t p = s_pos[lane];
                    uint32_t flen = 0;
                    tcp_step(v, p, flen);
                    const uint64_t last = p + flen - 1;
                    int lo = 0, hi = (int)G.nreads - 1;          // last read starting at or before `last`
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if ((lds_reads ? s_rstart[mid] : rd[mid].start) <= last) lo = mid; else hi = mid - 1;
                    }
                    const uint32_t fi = G.frame_base + R.fbase + done + lane;
                    edgpu_pkt_desc d;
                    d.slot = 0;
                    d.len = (uint16_t)(flen - 4);
                    d.channel = (uint8_t)tbyte(v, p + 1);
                    d.flags = 0;
                    d.arrival_ms = lds_reads ? s_rarr[lo] : rd[lo].arrival;
                    P.desc[fi] = d;
                    const uint8_t* a = p >= v.clen ? v.raw + (p - v.clen) : P.stage + (uint64_t)g * kTcpCarry;
                    P.src_addr[fi] = (uint64_t)(uintptr_t)a;
                    count_frame((uint32_t)lo);
                }
                done += m;
                __syncthreads();
                if (m == 0) break;
            }
        }
    }
    // the recorded chunks' frames, counted per read: frame f of a chunk ends where frame f + 1
    // starts (the walk's exit for the last) and belongs to the read holding its last byte.  A lane
    // per recorded frame (kTcpFrames = 32: two chunks per wave, eight per pass, their loads issued
    // together); the chunk table comes through LDS 64 chunks at a time.
    static_assert(kTcpFrames == 32, "two chunks per wave");
    __shared__ uint32_t s_cnf[64], s_cci[64];         // recorded frames (0: none) / candidate row
    for (uint32_t c0 = 0; !over && c0 < G.nchunks; c0 += 64) {
        const uint32_t nc = min(64u, G.nchunks - c0);
        if ((uint32_t)lane < nc) {
            const TcpChunkRes R = P.chunkres[G.first_chunk + c0 + lane];
            const bool rec = R.entry != kTcpNone && R.cand != kTcpNone && R.nframes <= kTcpFrames;
            s_cnf[lane] = rec ? R.nframes : 0u;
            s_cci[lane] = rec ? R.cand : 0u;
        }
        __syncthreads();
        for (uint32_t k0 = 0; k0 < nc; k0 += 8) {
            uint32_t nxt[4];
            bool on[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t k = k0 + 2 * u + (uint32_t)(lane >> 5), f = (uint32_t)lane & 31u;
                const uint32_t nf = k < nc ? s_cnf[k] : 0u;
                on[u] = f < nf;
                nxt[u] = 0;
                if (on[u]) {
                    const size_t ci = (size_t)(G.first_chunk + c0 + k) * kTcpCands + s_cci[k];
                    nxt[u] = f + 1 < nf ? (uint32_t)P.offs[ci * kTcpFrames + f + 1] : P.cands[ci].exit;
                }
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if (!on[u]) continue;
                const uint32_t k = k0 + 2 * u + (uint32_t)(lane >> 5);
                const uint64_t last = (uint64_t)(c0 + k) * kTcpChunk + nxt[u] - 1;
                int lo = 0, hi = (int)G.nreads - 1;       // last read starting at or before `last`
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if ((lds_reads ? s_rstart[mid] : rd[mid].start) <= last) lo = mid; else hi = mid - 1;
                }
                count_frame((uint32_t)lo);
            }
        }
        __syncthreads();
    }
    __syncthreads();
    // a frame that starts in the carried bytes -- the stream's first, at position 0 -- is staged
    // contiguously for k_ingest before the carry is overwritten
    if (!over && G.nchunks && v.clen) {
        const TcpChunkRes R0 = P.chunkres[G.first_chunk];
        if (R0.entry == 0) {                                  // uniform
            uint32_t flen = 0;
            tcp_step(v, 0, flen);
            uint8_t* dst = P.stage + (uint64_t)g * kTcpCarry;
            for (uint32_t b = lane; b < ((flen + 15) & ~15u); b += 64)
                dst[b] = b < flen ? (uint8_t)tbyte(v, b) : 0u;
        }
    }
    // ---- the carry + per-read results ----
    const uint32_t code = G.code;
    const uint64_t stop = G.stop;
    uint32_t ncarry = 0;
    if (!over && code == kWalkPartial) ncarry = (uint32_t)(v.len - stop);
    if (over) ncarry = G.carry_len;
    if (!over) {
        __syncthreads();                                      // the staging above has read the carry
        for (uint32_t b = lane; b < ncarry; b += 64) s_carry[b] = (uint8_t)tbyte(v, stop + b);
        __syncthreads();
        uint8_t* dst = P.carry + (uint64_t)G.session * kTcpCarry;
        for (uint32_t b = lane; b < ncarry; b += 64) dst[b] = s_carry[b];
    }
    for (uint32_t i = lane; i < G.nreads; i += 64) {
        const TcpRead r = P.reads[G.first_read + i];
        edgpu_tcp_result& o = P.results[G.first_read + i];
        uint32_t consumed = r.len;
        int32_t status = 0;
        if (over) {
            consumed = 0;
            o.frames = 0;
        } else {
            if (lds_reads) o.frames = s_frames[i];
            if (code == kWalkMessage || code == kWalkDropped) {
                consumed = stop <= r.start ? 0u : (uint32_t)min<uint64_t>(stop - r.start, r.len);
                const uint64_t at = code == kWalkMessage ? stop : stop + kTcpMaxFrame - 1;
                if (r.start + r.len > at) status = code == kWalkMessage ? EDGPU_TCP_MESSAGE : EDGPU_TCP_DROPPED;
            }
        }
        o.consumed = consumed;
        o.status = status;
        o.carry = ncarry;
    }
}

hipError_t launch_deframe(const TcpParams& p, hipStream_t st) {
    if (p.walk == 1) {
        if (p.ngroups) EDGPU_LAUNCH(k_tcp_chain, dim3((p.ngroups + 63) / 64), dim3(64), 0, st, p);
    } else {
        if (p.nchunks && p.walk == 2)
            EDGPU_LAUNCH(k_tcp_walk_seg, dim3((p.nchunks + kWalkWaves - 1) / kWalkWaves), dim3(64 * kWalkWaves), 0, st, p);
        else if (p.nchunks)
            EDGPU_LAUNCH(k_tcp_walk<kTcpWalkCpw>, dim3((p.nchunks + kWalkWaves * kTcpWalkCpw - 1) / (kWalkWaves * kTcpWalkCpw)),
                         dim3(64 * kWalkWaves), 0, st, p);
        EDGPU_LAUNCH(k_tcp_resolve, dim3(p.ngroups), dim3(256), 0, st, p);
    }
    EDGPU_LAUNCH(k_tcp_scan, dim3(1), dim3(kScanThreads), 0, st, p);
    EDGPU_LAUNCH(k_tcp_finish, dim3(p.ngroups), dim3(64), 0, st, p);
    return hipGetLastError();
}

}  // namespace edgpu
