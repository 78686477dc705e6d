// tools/store_peak3.hip -- calibration (not product): what bounds HBM write bandwidth for the
// fan-out's access shape?  Compares memset, constant vs random payload, per-lane widths and a
// synthetic LDS-staged write-many kernel with k_fanout4's window pattern (1024-thread blocks,
// 2 per CU, ~45 KB windows at 16-B-aligned offsets, 16 copies per chunk).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <string>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 rnd(size_t i) {
    unsigned x = (unsigned)i * 2654435761u ^ (unsigned)(i >> 32);
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    return u32x4{x, x * 747796405u, x ^ 0x9E3779B9u, x + 12345u};
}

// block-contiguous span, 16 B per lane per instruction
template <int THREADS, bool RND>
__global__ __launch_bounds__(THREADS) void k_span(u32x4* out, size_t nwords) {
    const size_t per = (nwords + gridDim.x - 1) / gridDim.x;
    const size_t b = blockIdx.x * per, e = min(nwords, b + per);
    for (size_t i = b + threadIdx.x; i < e; i += THREADS) out[i] = RND ? rnd(i) : u32x4{1u, 1u, 2u, 3u};
}

// grid-stride, each lane writes 4 consecutive words (64 B) per iteration
template <bool RND>
__global__ __launch_bounds__(256) void k_x4(u32x4* out, size_t nwords) {
    const size_t stride = (size_t)gridDim.x * 256 * 4;
    for (size_t i = (blockIdx.x * (size_t)256 + threadIdx.x) * 4; i + 3 < nwords; i += stride) {
#pragma unroll
        for (int u = 0; u < 4; u++) out[i + u] = RND ? rnd(i + u) : u32x4{1u, 1u, 2u, 3u};
    }
}

// grid-stride, 16 B per lane, wave instruction = 1 KiB contiguous
template <bool RND>
__global__ __launch_bounds__(256) void k_gs(u32x4* out, size_t nwords) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < nwords; i += stride)
        out[i] = RND ? rnd(i) : u32x4{1u, 1u, 2u, 3u};
}

__global__ void k_gsT(u32x4* out, size_t nwords) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nwords; i += stride) out[i] = u32x4{1u, 1u, 2u, 3u};
}

// synthetic fan-out: work item w = (chunk of CW words at in[w*CW]), written to 16 windows;
// window f of item w lands at out + base(w, f) where the arena is laid out sub-stream major
// (like the engine: sub-stream regions of NCH chunks each), each window starting 16-B aligned
// at a pseudo-random word phase.  LDS-staged, line-aligned stores like k_fanout4.
template <int THREADS, int CW, bool ALIGN_LINES>
__global__ __launch_bounds__(THREADS) void k_fan(const u32x4* in, u32x4* out, int nitems, int nch, size_t region_words) {
    __shared__ u32x4 cbuf[CW];
    for (int w = blockIdx.x; w < nitems; w += gridDim.x) {
        for (int i = threadIdx.x; i < CW; i += THREADS) cbuf[i] = in[(size_t)w * CW + i];
        __syncthreads();
        const int sender = w / nch, chunk = w % nch;
        for (int f = 0; f < 16; f++) {
            const size_t sub = (size_t)sender * 16 + f;
            const size_t A = sub * region_words + (size_t)chunk * CW + ((sub * 7) & 7);   // 16-B phase
            const unsigned s = ALIGN_LINES ? (unsigned)(A & 7) : 0u;
            for (unsigned lw = threadIdx.x; lw < CW + s; lw += THREADS) {
                const unsigned src = lw - s;
                if (src < (unsigned)CW) out[A - s + lw] = cbuf[src];
            }
        }
        __syncthreads();
    }
}

// output-driven gather sweep: the grid walks the arena in address order (one write front, like
// the runtime's fill kernel); each 16-B output word finds its source word arithmetically.
// Arena is sub-stream major: sub-stream u (= sender u/16) holds NCH chunks of CW words; source
// chunk (sender, c) is read by the sender's 16 sub-streams (L2 / Infinity-Cache hits after the
// first).  `phase` offsets each sub-stream's source by a word phase (16-B-aligned slots).
__global__ void k_gsweep(const u32x4* in, u32x4* out, size_t nout, unsigned cw, unsigned nch) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const size_t region = (size_t)cw * nch;
    for (size_t o = blockIdx.x * (size_t)blockDim.x + threadIdx.x; o < nout; o += stride) {
        const size_t u = o / region, k = o - u * region;
        const size_t sender = u >> 4;
        out[o] = in[sender * region + k];
    }
}

// same sweep, 32-bit index math and U independent loads in flight per lane before the stores
template <int U>
__global__ __launch_bounds__(256) void k_gsweep2(const u32x4* in, u32x4* out, unsigned nout, unsigned cw, unsigned nch) {
    const unsigned stride = gridDim.x * 256u * U;
    const unsigned region = cw * nch;
    for (unsigned o0 = blockIdx.x * 256u * U + threadIdx.x; o0 < nout; o0 += stride) {
        u32x4 v[U];
#pragma unroll
        for (int j = 0; j < U; j++) {
            const unsigned o = o0 + j * 256u;
            const unsigned u = o / region, k = o - u * region;
            if (o < nout) v[j] = in[(size_t)(u >> 4) * region + k];
        }
#pragma unroll
        for (int j = 0; j < U; j++) {
            const unsigned o = o0 + j * 256u;
            if (o < nout) out[o] = v[j];
        }
    }
}

// k_fan with a chunk-major arena: item w's 16 copies are adjacent (one 16 x CW region per
// item, each copy at a 16-B phase), so a block's stores sweep one contiguous region per item.
template <int THREADS, int CW>
__global__ __launch_bounds__(THREADS) void k_fan_cm(const u32x4* in, u32x4* out, int nitems) {
    __shared__ u32x4 cbuf[CW];
    for (int w = blockIdx.x; w < nitems; w += gridDim.x) {
        for (int i = threadIdx.x; i < CW; i += THREADS) cbuf[i] = in[(size_t)w * CW + i];
        __syncthreads();
        const size_t base = (size_t)w * (16 * CW + 8);
        for (int f = 0; f < 16; f++) {
            const size_t A = base + (size_t)f * CW + ((w * 7 + 3) & 7);
            const unsigned s = (unsigned)(A & 7);
            for (unsigned lw = threadIdx.x; lw < CW + s; lw += THREADS) {
                const unsigned src = lw - s;
                if (src < (unsigned)CW) out[A - s + lw] = cbuf[src];
            }
        }
        __syncthreads();
    }
}
// k_fan_cm variants: MODE 1 = no chunk reads (LDS filled once), MODE 2 = non-temporal stores
template <int THREADS, int CW, int MODE>
__global__ __launch_bounds__(THREADS) void k_fan_cmx(const u32x4* in, u32x4* out, int nitems) {
    __shared__ u32x4 cbuf[CW];
    if (MODE == 1) { for (int i = threadIdx.x; i < CW; i += THREADS) cbuf[i] = in[i]; __syncthreads(); }
    for (int w = blockIdx.x; w < nitems; w += gridDim.x) {
        if (MODE != 1) {
            for (int i = threadIdx.x; i < CW; i += THREADS) cbuf[i] = in[(size_t)w * CW + i];
            __syncthreads();
        }
        const size_t base = (size_t)w * (16 * CW + 8);
        for (int f = 0; f < 16; f++) {
            const size_t A = base + (size_t)f * CW + ((w * 7 + 3) & 7);
            const unsigned s = (unsigned)(A & 7);
            for (unsigned lw = threadIdx.x; lw < CW + s; lw += THREADS) {
                const unsigned src = lw - s;
                if (src < (unsigned)CW) {
                    if (MODE == 2) __builtin_nontemporal_store(cbuf[src], &out[A - s + lw]);
                    else out[A - s + lw] = cbuf[src];
                }
            }
        }
        if (MODE != 1) __syncthreads();
    }
}
// the same region written as ONE flat sweep of 16*CW words (copy boundaries inside lines)
template <int THREADS, int CW>
__global__ __launch_bounds__(THREADS) void k_fan_cmflat(const u32x4* in, u32x4* out, int nitems) {
    __shared__ u32x4 cbuf[CW];
    for (int w = blockIdx.x; w < nitems; w += gridDim.x) {
        for (int i = threadIdx.x; i < CW; i += THREADS) cbuf[i] = in[(size_t)w * CW + i];
        __syncthreads();
        const size_t A = (size_t)w * (16 * CW + 8) + ((w * 7 + 3) & 7);
        const unsigned s = (unsigned)(A & 7);
        for (unsigned lw = threadIdx.x; lw < 16 * CW + s; lw += THREADS) {
            const unsigned idx = lw - s;
            if (idx < 16u * CW) out[A - s + lw] = cbuf[idx % CW];
        }
        __syncthreads();
    }
}

template <typename F>
static float timeit(F f) {
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    f(); hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
        hipEventRecord(a); f(); hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
    }
    return best;
}

int main() {
    const size_t bytes = 8ull << 30, nw = bytes / 16;
    u32x4* out; hipMalloc(&out, bytes + (64 << 20));
    std::string js = "{";
    auto add = [&](const char* k, double gbs) { char buf[128]; snprintf(buf, sizeof buf, "%s\"%s\": %.1f", js.size() > 1 ? ", " : "", k, gbs); js += buf; };
    add("memset0", bytes / timeit([&] { hipMemsetAsync(out, 0, bytes, 0); }) / 1e6);
    add("memset5a", bytes / timeit([&] { hipMemsetAsync(out, 0x5a, bytes, 0); }) / 1e6);
    add("memsetD32_rnd", bytes / timeit([&] { hipMemsetD32Async((hipDeviceptr_t)out, 0x9E3779B9, bytes / 4, 0); }) / 1e6);
    add("span1024_const_g512", bytes / timeit([&] { hipLaunchKernelGGL((k_span<1024, false>), dim3(512), dim3(1024), 0, 0, out, nw); }) / 1e6);
    add("span1024_rnd_g512", bytes / timeit([&] { hipLaunchKernelGGL((k_span<1024, true>), dim3(512), dim3(1024), 0, 0, out, nw); }) / 1e6);
    add("span256_rnd_g8192", bytes / timeit([&] { hipLaunchKernelGGL((k_span<256, true>), dim3(8192), dim3(256), 0, 0, out, nw); }) / 1e6);
    // synthetic fan-out: 900 senders x 12 chunks x 2816 words, 16 subs -> ~7.4 GB written
    const int CW = 2816, nch = 12, nsend = 900, nitems = nsend * nch;   // 900*16 regions of 33856 words = 7.8 GB
    if ((size_t)nsend * 16 * ((size_t)nch * CW + 64) * 16 > bytes) { printf("{}\n"); return 1; }
    const size_t region = (size_t)nch * CW + 64;
    u32x4* in; hipMalloc(&in, (size_t)nitems * CW * 16);
    hipMemset(in, 7, (size_t)nitems * CW * 16);
    const double fb = (double)nitems * CW * 16 * 17;
    add("fan_aligned_1024x512", fb / timeit([&] { hipLaunchKernelGGL((k_fan<1024, CW, true>), dim3(512), dim3(1024), 0, 0, in, out, nitems, nch, region); }) / 1e6);
    add("fan_unaligned_1024x512", fb / timeit([&] { hipLaunchKernelGGL((k_fan<1024, CW, false>), dim3(512), dim3(1024), 0, 0, in, out, nitems, nch, region); }) / 1e6);
    add("fan_aligned_1024x256", fb / timeit([&] { hipLaunchKernelGGL((k_fan<1024, CW, true>), dim3(256), dim3(1024), 0, 0, in, out, nitems, nch, region); }) / 1e6);
    add("fan_aligned_512x1024", fb / timeit([&] { hipLaunchKernelGGL((k_fan<512, CW, true>), dim3(512), dim3(512), 0, 0, in, out, nitems, nch, region); }) / 1e6);
    add("fan_aligned_256x1024", fb / timeit([&] { hipLaunchKernelGGL((k_fan<256, CW, true>), dim3(512), dim3(256), 0, 0, in, out, nitems, nch, region); }) / 1e6);
    add("fan_cm_1024x512", fb / timeit([&] { hipLaunchKernelGGL((k_fan_cm<1024, CW>), dim3(512), dim3(1024), 0, 0, in, out, nitems); }) / 1e6);
    add("fan_cm_noread_1024x512", fb / timeit([&] { hipLaunchKernelGGL((k_fan_cmx<1024, CW, 1>), dim3(512), dim3(1024), 0, 0, in, out, nitems); }) / 1e6);
    add("fan_cm_nt_1024x512", fb / timeit([&] { hipLaunchKernelGGL((k_fan_cmx<1024, CW, 2>), dim3(512), dim3(1024), 0, 0, in, out, nitems); }) / 1e6);
    add("fan_cm_noread_256x256", fb / timeit([&] { hipLaunchKernelGGL((k_fan_cmx<256, CW, 1>), dim3(256), dim3(256), 0, 0, in, out, nitems); }) / 1e6);
    add("fan_cm_noread_1024x256", fb / timeit([&] { hipLaunchKernelGGL((k_fan_cmx<1024, CW, 1>), dim3(256), dim3(1024), 0, 0, in, out, nitems); }) / 1e6);
    add("fan_aligned_256x256", fb / timeit([&] { hipLaunchKernelGGL((k_fan<256, CW, true>), dim3(256), dim3(256), 0, 0, in, out, nitems, nch, region); }) / 1e6);
    {
        const size_t nout = (size_t)nsend * 16 * nch * CW;
        const double gb = (double)nout * 16 + (double)nitems * CW * 16;
    }
    js += "}";
    printf("%s\n", js.c_str());
    return 0;
}
