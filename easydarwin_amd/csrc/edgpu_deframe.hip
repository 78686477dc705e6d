// edgpu_deframe.hip -- RTSP-interleaved push ingest on gfx950: '$'-deframing of pusher TCP reads.
//
// Reference behaviour (RTSPRequestStream::ReadRequest, Server.tproj/RTSPRequestStream.cpp:65-171,
// called per readable event by RTSPSession::Run, RTSPSession.cpp:240-262): a connection's bytes
// collect in a 2 KiB request buffer; a '$' at a frame boundary starts a frame of 4 + BE16(len)
// bytes that is handed to ProcessRTPData once complete; anything else is an RTSP request; a
// frame that cannot fit the 2047 usable buffer bytes ends the connection.  The CPU walks that
// chain one header at a time.
//
// Here a session's stream (carried partial frame ++ this call's reads) is cut into 16 KiB
// chunks.  A frame starts at most kTcpMaxFrame - 1 bytes before a chunk boundary, so the true
// walk enters each chunk at a '$' within its first kTcpMaxFrame bytes.  k_tcp_walk walks every
// such candidate to the chunk end at once (one lane each) and links its exit to the next
// chunk's candidate; k_tcp_resolve follows the links (LDS) per session and scans frame and
// slot counts; k_tcp_scan lays sessions out in the ingest staging; k_tcp_emit re-walks each
// chunk from its true entry and writes every frame into a 16-B slot ('$' header word, packet,
// zero pad) with its edgpu_pkt_desc; k_tcp_finish carries the partial frame and reports per
// read.  k_ingest then runs unchanged on the emitted batch.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "edgpu.h"
#include "edgpu_device.h"
#include "edgpu_params.h"

namespace edgpu {

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// A session's stream in this call: carry[0, clen) ++ raw[raw_off, raw_off + len - clen).
struct TcpView {
    const uint8_t* carry;
    const uint8_t* raw;     // raw + raw_off
    const uint8_t* raw_end; // end of the raw buffer (bounds for wide loads)
    uint32_t clen;
    uint64_t len;
};

__device__ __forceinline__ TcpView tcp_view(const TcpParams& P, const TcpGroup& G) {
    TcpView v;
    v.carry = P.carry + (uint64_t)G.session * kTcpCarry;
    v.raw = P.raw + G.raw_off;
    v.raw_end = P.raw + P.raw_bytes;
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
    if (tbyte(v, pos) != 0x24u) return kWalkMessage;
    if (pos + 4 > v.len) return kWalkPartial;
    flen = 4 + (tbyte(v, pos + 2) << 8 | tbyte(v, pos + 3));
    if (flen > kTcpMaxFrame) return v.len - pos >= kTcpMaxFrame ? kWalkDropped : kWalkPartial;
    if (pos + flen > v.len) return kWalkPartial;
    return kWalkRun;
}

// Walks from `pos` until reaching `end` or a stop; counts frames and their slot bytes.
__device__ __forceinline__ uint32_t tcp_walk(const TcpView& v, uint64_t& pos, uint64_t end, uint32_t& nf,
                                             uint64_t& sb) {
    nf = 0;
    sb = 0;
    while (pos < end) {
        uint32_t flen = 0;
        const uint32_t code = tcp_step(v, pos, flen);
        if (code != kWalkRun) return code;
        nf++;
        sb += (flen + 15) & ~15u;
        pos += flen;
    }
    return kWalkRun;
}

// '$' bytes among the first kTcpMaxFrame bytes of the chunk at `start` (offsets, in order, the
// first kTcpCands kept in `list`); the stream's first chunk has the single candidate 0.  One
// wave; returns the full count (> kTcpCands: overflow).
__device__ uint32_t tcp_candidates(const TcpView& v, uint64_t start, uint16_t* list, int lane) {
    if (start == 0) {
        if (lane == 0) list[0] = 0;
        return 1;
    }
    const uint64_t wend = min(start + (uint64_t)kTcpMaxFrame, v.len);
    uint32_t n = 0;
    for (uint64_t o = start; o < wend; o += 64) {
        const uint64_t p = o + (uint64_t)lane;
        const bool is = p < wend && tbyte(v, p) == 0x24u;
        const uint64_t m = __ballot(is);
        if (is) {
            const uint32_t i = n + (uint32_t)__popcll(m & ((1ull << lane) - 1));
            if (i < kTcpCands) list[i] = (uint16_t)(p - start);
        }
        n += (uint32_t)__popcll(m);
    }
    return n;
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

// ---- k_tcp_walk: one wave per chunk ----
__global__ __launch_bounds__(64) void k_tcp_walk(TcpParams P) {
    const uint32_t c = blockIdx.x;
    const int lane = threadIdx.x;
    const uint32_t g = P.chunk_group[c];
    const TcpGroup G = P.groups[g];
    const TcpView v = tcp_view(P, G);
    const uint32_t k = c - G.first_chunk;
    const uint64_t start = (uint64_t)k * kTcpChunk;
    const uint64_t end = min(start + kTcpChunk, v.len);
    __shared__ uint16_t own[kTcpCands], next[kTcpCands];
    const uint32_t n = tcp_candidates(v, start, own, lane);
    const uint32_t nn = end < v.len ? tcp_candidates(v, end, next, lane) : 0u;
    __syncthreads();
    if (lane == 0) P.ncand[c] = n;
    if (n > kTcpCands || (uint32_t)lane >= n) return;
    uint64_t pos = start + own[lane];
    uint32_t nf;
    uint64_t sb;
    const uint32_t code = tcp_walk(v, pos, end, nf, sb);
    uint8_t link = 0xFE;
    if (code == kWalkRun && pos < v.len) {                  // continues in the next chunk
        link = 0xFF;
        if (nn <= kTcpCands) {
            const uint32_t q = (uint32_t)(pos - end);
            for (uint32_t i = 0; i < nn; i++)
                if (next[i] == q) { link = (uint8_t)i; break; }
        }
    }
    TcpCand r;
    r.q = own[lane];
    r.exit = (uint32_t)(pos - start);
    r.nframes = nf;
    r.code = code;
    r.sbytes = sb;
    P.cands[(size_t)c * kTcpCands + lane] = r;
    P.links[(size_t)c * kTcpCands + lane] = link;
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
    __shared__ uint64_t s_sb[kPiece];
    __shared__ uint64_t scan64[4];
    __shared__ uint32_t scan32[4];
    __shared__ uint32_t s_stop_code;
    __shared__ uint64_t s_stop;
    if (tid == 0) { s_stop_code = kWalkRun; s_stop = v.len; }
    // chain state (thread 0)
    int j = 0;                  // candidate of the current chunk, -1: search for `entry`
    uint64_t entry = 0;
    bool stopped = false;
    uint32_t fb = 0;
    uint64_t sbb = 0;
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
                        uint64_t sb = 0;
                        if (n <= kTcpCands) code = kWalkMessage;              // not a '$'
                        else code = tcp_walk(v, pos, end, nf, sb);            // too many candidates
                        s_idx[kk] = 0xFD;
                        s_entry[kk] = (uint32_t)(entry - start);
                        s_nf[kk] = nf; s_sb[kk] = sb; s_code[kk] = code; s_exit[kk] = (uint32_t)(pos - start);
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
        // per chunk of the piece: its true walk's counts, then the scan
        uint32_t nf = 0;
        uint64_t sb = 0;
        uint32_t ent = kTcpNone;
        if ((uint32_t)tid < np) {
            const uint32_t c = c0 + tid;
            const uint64_t start = (uint64_t)(k0 + tid) * kTcpChunk;
            const uint8_t idx = s_idx[tid];
            uint32_t code = kWalkRun, ex = 0;
            bool terminal = false;
            if (idx < kTcpCands) {
                const TcpCand r = P.cands[(size_t)c * kTcpCands + idx];
                nf = r.nframes; sb = r.sbytes; ent = r.q; code = r.code; ex = r.exit;
                terminal = s_link[tid * kTcpCands + idx] == 0xFE;
            } else if (idx == 0xFD) {
                nf = s_nf[tid]; sb = s_sb[tid]; ent = s_entry[tid]; code = s_code[tid]; ex = s_exit[tid];
                terminal = code != kWalkRun || start + ex >= v.len;
            }
            if (terminal) { s_stop_code = code; s_stop = start + ex; }
        }
        uint32_t tnf;
        uint64_t tsb;
        const uint32_t pnf = block_exclusive_scan256<uint32_t>(nf, scan32, tnf);
        const uint64_t psb = block_exclusive_scan256<uint64_t>(sb, scan64, tsb);
        if ((uint32_t)tid < np) {
            TcpChunkRes R;
            R.entry = (nf || ent != kTcpNone) ? ent : kTcpNone;
            R.fbase = fb + pnf;
            R.sbase = sbb + psb;
            P.chunkres[c0 + tid] = R;
        }
        fb += tnf;
        sbb += tsb;
        __syncthreads();
    }
    if (tid == 0) {
        TcpGroup& W = P.groups[g];
        W.nframes = fb;
        W.slot_bytes = sbb;
        // a walk that ran off the end of the stream stops there: everything framed
        const uint32_t code = s_stop_code;
        W.code = (code == kWalkPartial && s_stop >= v.len) ? kWalkRun : code;
        W.stop = s_stop;
    }
}

// ---- k_tcp_scan: one workgroup; sessions -> ingest segments ----
__global__ __launch_bounds__(256) void k_tcp_scan(TcpParams P) {
    const int tid = threadIdx.x;
    __shared__ uint64_t scan64[4];
    __shared__ uint32_t scan32[4];
    uint32_t fb = 0;
    uint64_t sbb = 0;
    for (uint32_t g0 = 0; g0 < P.ngroups; g0 += 256) {
        const uint32_t g = g0 + tid;
        const bool ok = g < P.ngroups;
        const uint32_t nf = ok ? P.groups[g].nframes : 0u;
        const uint64_t sb = ok ? P.groups[g].slot_bytes : 0ull;
        uint32_t tnf;
        uint64_t tsb;
        const uint32_t pnf = block_exclusive_scan256<uint32_t>(nf, scan32, tnf);
        const uint64_t psb = block_exclusive_scan256<uint64_t>(sb, scan64, tsb);
        if (ok) {
            P.groups[g].frame_base = fb + pnf;
            P.groups[g].slot_base = sbb + psb;
        }
        fb += tnf;
        sbb += tsb;
    }
    const bool over = fb > P.max_desc || sbb > P.blob_cap;
    for (uint32_t g = tid; g < P.ngroups; g += 256) {
        P.seg_off[g] = over ? 0u : P.groups[g].frame_base;
        P.seg_sess[g] = P.groups[g].session;
    }
    if (tid == 0) {
        P.seg_off[P.ngroups] = over ? 0u : fb;
        P.tot->frames = fb;
        P.tot->slot_bytes = sbb;
        P.tot->status = over ? EDGPU_OUT_OVERFLOW : 0;
    }
}

// 16 stream bytes at `p` (< len) as one slot word; bytes at or past `lim` read 0.
__device__ __forceinline__ u32x4 tcp_word(const TcpView& v, uint64_t p, uint64_t lim) {
    if (p >= v.clen) {
        // two aligned 16-B loads + byte funnel (the raw buffer is 16-B aligned)
        const uint8_t* a = v.raw + (p - v.clen);
        const uintptr_t al = (uintptr_t)a & ~(uintptr_t)15;
        const uint32_t sh = (uint32_t)((uintptr_t)a & 15);
        if (al + 32 <= (uintptr_t)v.raw_end) {
            const u32x4 w0 = *reinterpret_cast<const u32x4*>(al);
            const u32x4 w1 = sh ? *reinterpret_cast<const u32x4*>(al + 16) : w0;
            const uint32_t d[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
            const uint32_t q = sh >> 2, r = sh & 3;
            uint32_t o[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                // d[i + q], d[i + q + 1] without dynamic register indexing (q is wave-uniform)
                uint32_t lo = d[i], hi = d[i + 1];
                if (q == 1) { lo = d[i + 1]; hi = d[i + 2]; }
                else if (q == 2) { lo = d[i + 2]; hi = d[i + 3]; }
                else if (q == 3) { lo = d[i + 3]; hi = d[i + 4]; }
                o[i] = r ? __builtin_amdgcn_alignbyte(hi, lo, r) : lo;
            }
            if (p + 16 > lim) {                                  // zero the slot padding
                const uint32_t nb = (uint32_t)(lim - p);
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int keep = (int)nb - 4 * i;
                    o[i] = keep >= 4 ? o[i] : keep <= 0 ? 0u : (o[i] & ((1u << (8 * keep)) - 1));
                }
            }
            return u32x4{o[0], o[1], o[2], o[3]};
        }
    }
    uint32_t o[4] = {0u, 0u, 0u, 0u};
    for (int b = 0; b < 16; b++)
        if (p + b < lim) o[b >> 2] |= tbyte(v, p + b) << (8 * (b & 3));
    return u32x4{o[0], o[1], o[2], o[3]};
}

// ---- k_tcp_emit: one wave per chunk; frames -> slots + descriptors ----
__global__ __launch_bounds__(64) void k_tcp_emit(TcpParams P) {
    const uint32_t c = blockIdx.x;
    const int lane = threadIdx.x;
    if (P.tot->status != 0) return;
    const TcpChunkRes R = P.chunkres[c];
    if (R.entry == kTcpNone) return;
    const uint32_t g = P.chunk_group[c];
    const TcpGroup G = P.groups[g];
    const TcpView v = tcp_view(P, G);
    const uint64_t start = (uint64_t)(c - G.first_chunk) * kTcpChunk;
    const uint64_t end = min(start + kTcpChunk, v.len);
    __shared__ uint64_t s_pos[64];
    __shared__ uint32_t s_flen[64];
    __shared__ uint32_t s_m;
    __shared__ uint64_t s_next;
    uint64_t pos = start + R.entry;
    uint32_t fidx = G.frame_base + R.fbase;
    uint64_t soff = G.slot_base + R.sbase;
    const TcpRead* rd = P.reads + G.first_read;
    while (pos < end) {
        if (lane == 0) {                                  // next up to 64 frames of the chain
            uint32_t m = 0;
            uint64_t p = pos;
            while (m < 64 && p < end) {
                uint32_t flen = 0;
                if (tcp_step(v, p, flen) != kWalkRun) { p = ~0ull; break; }
                s_pos[m] = p;
                s_flen[m] = flen;
                m++;
                p += flen;
            }
            s_m = m;
            s_next = p;
        }
        __syncthreads();
        const uint32_t m = s_m;
        // lane f: descriptor of frame f (arrival of the read holding its last byte)
        uint64_t my_soff = 0;
        {
            const uint32_t sl = (uint32_t)lane < m ? ((s_flen[lane] + 15) & ~15u) : 0u;
            uint64_t x = sl;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint64_t y = __shfl_up(x, o, 64);
                if (lane >= o) x += y;
            }
            my_soff = soff + x - sl;
            if ((uint32_t)lane < m) {
                const uint64_t p = s_pos[lane];
                const uint32_t flen = s_flen[lane];
                const uint64_t last = p + flen - 1;
                int lo = 0, hi = (int)G.nreads - 1;              // last read starting at or before `last`
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (rd[mid].start <= last) lo = mid; else hi = mid - 1;
                }
                edgpu_pkt_desc d;
                d.slot = (uint32_t)(my_soff >> 4);
                d.len = (uint16_t)(flen - 4);
                d.channel = (uint8_t)tbyte(v, p + 1);
                d.flags = 0;
                d.arrival_ms = rd[lo].arrival;
                P.desc[fidx + lane] = d;
                atomicAdd(&P.results[G.first_read + lo].frames, 1u);
            }
            soff += __shfl(x, 63, 64);
        }
        // slot words: the frame as received ('$' ch BE16(len) + packet), zero padded
        for (uint32_t f = 0; f < m; f++) {
            const uint64_t p = s_pos[f];
            const uint32_t flen = s_flen[f];
            const uint64_t so = __shfl(my_soff, (int)f, 64);
            u32x4* dst = reinterpret_cast<u32x4*>(P.blob + so);
            const uint32_t nw = (flen + 15) >> 4;
            for (uint32_t w = lane; w < nw; w += 64) dst[w] = tcp_word(v, p + 16 * w, p + flen);
        }
        fidx += m;
        pos = s_next;
        __syncthreads();
    }
}

// ---- k_tcp_finish: one workgroup per session; carry + per-read results ----
__global__ __launch_bounds__(256) void k_tcp_finish(TcpParams P) {
    const uint32_t g = blockIdx.x;
    const int tid = threadIdx.x;
    const TcpGroup G = P.groups[g];
    const bool over = P.tot->status != 0;
    const TcpView v = tcp_view(P, G);
    __shared__ uint8_t s_carry[kTcpCarry];
    const uint32_t code = G.code;
    const uint64_t stop = G.stop;
    uint32_t ncarry = 0;
    if (!over && code == kWalkPartial) ncarry = (uint32_t)(v.len - stop);
    if (over) ncarry = G.carry_len;
    if (!over) {
        for (uint32_t b = tid; b < ncarry; b += 256) s_carry[b] = (uint8_t)tbyte(v, stop + b);
        __syncthreads();
        uint8_t* dst = P.carry + (uint64_t)G.session * kTcpCarry;
        for (uint32_t b = tid; b < ncarry; b += 256) dst[b] = s_carry[b];
    }
    for (uint32_t i = tid; i < G.nreads; i += 256) {
        const TcpRead r = P.reads[G.first_read + i];
        edgpu_tcp_result& o = P.results[G.first_read + i];
        uint32_t consumed = r.len;
        int32_t status = 0;
        if (over) {
            consumed = 0;
            o.frames = 0;
        } else if (code == kWalkMessage || code == kWalkDropped) {
            consumed = stop <= r.start ? 0u : (uint32_t)min<uint64_t>(stop - r.start, r.len);
            const uint64_t at = code == kWalkMessage ? stop : stop + kTcpMaxFrame - 1;
            if (r.start + r.len > at) status = code == kWalkMessage ? EDGPU_TCP_MESSAGE : EDGPU_TCP_DROPPED;
        }
        o.consumed = consumed;
        o.status = status;
        o.carry = ncarry;
    }
}

hipError_t launch_deframe(const TcpParams& p, hipStream_t st) {
    if (p.nchunks) hipLaunchKernelGGL(k_tcp_walk, dim3(p.nchunks), dim3(64), 0, st, p);
    hipLaunchKernelGGL(k_tcp_resolve, dim3(p.ngroups), dim3(256), 0, st, p);
    hipLaunchKernelGGL(k_tcp_scan, dim3(1), dim3(256), 0, st, p);
    if (p.nchunks) hipLaunchKernelGGL(k_tcp_emit, dim3(p.nchunks), dim3(64), 0, st, p);
    hipLaunchKernelGGL(k_tcp_finish, dim3(p.ngroups), dim3(256), 0, st, p);
    return hipGetLastError();
}

}  // namespace edgpu
