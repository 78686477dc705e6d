// tools/store_peak6.hip -- calibration (not product): does splitting a tick into session groups
// (ingest g, then fan-out g) let the fan-out's chunk reads hit the Infinity Cache (MALL)?
// store_peak5 showed the write-many at 5.66 TB/s when its sources were just written by another
// kernel and fit in the MALL (cm_nt_fresh_128MB), against ~5.0 TB/s when a tick's whole 486 MB
// comes from HBM.  Here the source is written piece by piece, as the ingest would write one
// group's slots, and each piece is fanned out right after it was written.  Timed: the whole
// sequence (writes + fan-outs), and the fan-out launches alone, for G = 1 .. 16 groups.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <string>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// chunk-major write-many (store_peak5's k_fan_cm, nt stores): items [i0, i0 + n), each its own
// chunk of the source, 16 line-aligned copies at 16-B phases
template <int THREADS, int CW>
__global__ __launch_bounds__(THREADS) void k_fan_cm(const u32x4* in, u32x4* out, int i0, int n) {
    __shared__ u32x4 cbuf[CW];
    for (int k = blockIdx.x; k < n; k += gridDim.x) {
        const int w = i0 + k;
        const size_t sw = (size_t)w * CW;
        for (int i = threadIdx.x; i < CW; i += THREADS) cbuf[i] = in[sw + i];
        __syncthreads();
        const size_t base = (size_t)w * (16 * CW + 8);
        for (int f = 0; f < 16; f++) {
            const size_t A = base + (size_t)f * CW + ((w * 7 + 3) & 7);
            const unsigned s = (unsigned)(A & 7);
            for (unsigned lw = threadIdx.x; lw < CW + s; lw += THREADS) {
                const unsigned src = lw - s;
                if (src < (unsigned)CW) __builtin_nontemporal_store(cbuf[src], &out[A - s + lw]);
            }
        }
        __syncthreads();
    }
}

// the "ingest": a streaming copy from a staging buffer into the source piece (plain stores, as
// k_ingest's slot stores)
__global__ __launch_bounds__(256) void k_copy(const u32x4* src, u32x4* dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

int main() {
    const int CW = 2816, nitems = 900 * 12;                          // 486 MB of sources, 7.8 GB out
    const size_t item_w = CW;
    u32x4 *in, *stage, *out;
    if (hipMalloc(&in, (size_t)nitems * item_w * 16) != hipSuccess ||
        hipMalloc(&stage, (size_t)nitems * item_w * 16) != hipSuccess ||
        hipMalloc(&out, (size_t)nitems * (16 * CW + 8) * 16 + (1 << 20)) != hipSuccess) return 1;
    hipMemset(stage, 7, (size_t)nitems * item_w * 16);
    hipMemset(in, 3, (size_t)nitems * item_w * 16);
    hipEvent_t ev[2 * 16 + 2];
    for (auto& e : ev) hipEventCreate(&e);
    const double fan_b = (double)nitems * item_w * 16 * 17, copy_b = (double)nitems * item_w * 16 * 2;
    std::string js = "{";
    auto add = [&](const std::string& k, double v) {
        char buf[160]; snprintf(buf, sizeof buf, "%s\"%s\": %.4f", js.size() > 1 ? ", " : "", k.c_str(), v); js += buf;
    };
    const int groups[] = {1, 2, 4, 6, 8, 12, 16};
    for (int G : groups) {
        float best_tot = 1e30f, best_fan = 1e30f;
        for (int rep = 0; rep < 6; rep++) {
            hipEventRecord(ev[0]);
            for (int g = 0; g < G; g++) {
                const int i0 = (int)((long)nitems * g / G), i1 = (int)((long)nitems * (g + 1) / G);
                hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, 0, stage + (size_t)i0 * item_w,
                                   in + (size_t)i0 * item_w, (size_t)(i1 - i0) * item_w);
                hipEventRecord(ev[1 + 2 * g]);
                hipLaunchKernelGGL((k_fan_cm<1024, CW>), dim3(512), dim3(1024), 0, 0, in, out, i0, i1 - i0);
                hipEventRecord(ev[2 + 2 * g]);
            }
            hipEventSynchronize(ev[2 * G]);
            float tot, fan = 0, ms;
            hipEventElapsedTime(&tot, ev[0], ev[2 * G]);
            for (int g = 0; g < G; g++) { hipEventElapsedTime(&ms, ev[1 + 2 * g], ev[2 + 2 * g]); fan += ms; }
            if (rep > 0) { if (tot < best_tot) best_tot = tot; if (fan < best_fan) best_fan = fan; }
        }
        add("G" + std::to_string(G) + "_total_ms", best_tot);
        add("G" + std::to_string(G) + "_fan_ms", best_fan);
        add("G" + std::to_string(G) + "_fan_GBps", fan_b / best_fan / 1e6);
        add("G" + std::to_string(G) + "_copy_GBps", copy_b / (best_tot - best_fan) / 1e6);
    }
    js += "}";
    printf("%s\n", js.c_str());
    return 0;
}
