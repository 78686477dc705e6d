// tools/store_peak5.hip -- calibration (not product): does the write-many lose its ~13 %
// read/write-mix penalty when the chunk reads hit the memory-side Infinity Cache (MALL)?
// store_peak3's chunk-major synthetic (fan_cm: 16 adjacent copies per item, line-aligned
// windows at 16-B phases, 1024 threads, 2 blocks per CU), but the chunk sources cycle over a
// footprint of F MiB instead of streaming 484 MB once.  F well below the 256 MB MALL (and above
// the 8 x 4 MB of L2) shows what a cache-resident source would buy; F = all is the engine case.
// Variants: plain or non-temporal arena stores (does an nt write stream evict the source?),
// and "fresh": the source is rewritten by a copy kernel right before each timed launch.
// Prints GB/s counted like store_peak3's fan modes: source once + 16 copies per item.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <string>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int THREADS, int CW, bool NT>
__global__ __launch_bounds__(THREADS) void k_fan_cm(const u32x4* in, u32x4* out, int nitems, int nsrc) {
    __shared__ u32x4 cbuf[CW];
    for (int w = blockIdx.x; w < nitems; w += gridDim.x) {
        const size_t sw = (size_t)(w % nsrc) * CW;
        for (int i = threadIdx.x; i < CW; i += THREADS) cbuf[i] = in[sw + i];
        __syncthreads();
        const size_t base = (size_t)w * (16 * CW + 8);
        for (int f = 0; f < 16; f++) {
            const size_t A = base + (size_t)f * CW + ((w * 7 + 3) & 7);
            const unsigned s = (unsigned)(A & 7);
            for (unsigned lw = threadIdx.x; lw < CW + s; lw += THREADS) {
                const unsigned src = lw - s;
                if (src < (unsigned)CW) {
                    if (NT) __builtin_nontemporal_store(cbuf[src], &out[A - s + lw]);
                    else out[A - s + lw] = cbuf[src];
                }
            }
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_touch(u32x4* p, size_t n, unsigned salt) {
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        p[i] = u32x4{(unsigned)i ^ salt, salt, 1u, 2u};
}

template <typename F, typename P>
static float timeit2(F f, P pre) {
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    pre(); f(); hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
        pre();
        hipEventRecord(a); f(); hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
    }
    return best;
}

int main() {
    const int CW = 2816, nch = 12, nsend = 900, nitems = nsend * nch;   // 7.8 GB written
    const size_t item_b = (size_t)CW * 16;                              // 45 KB per chunk
    u32x4 *in, *out;
    if (hipMalloc(&in, (size_t)nitems * item_b) != hipSuccess ||
        hipMalloc(&out, (size_t)nitems * (16 * CW + 8) * 16 + (1 << 20)) != hipSuccess) return 1;
    hipMemset(in, 7, (size_t)nitems * item_b);
    const double fb = (double)nitems * item_b * 17;
    std::string js = "{";
    auto add = [&](const std::string& k, double gbs) {
        char buf[160]; snprintf(buf, sizeof buf, "%s\"%s\": %.1f", js.size() > 1 ? ", " : "", k.c_str(), gbs); js += buf;
    };
    const int foot_mb[] = {16, 64, 128, 192, 0};       // 0 = every item its own chunk (486 MB)
    for (int fm : foot_mb) {
        const int nsrc = fm ? (int)(((size_t)fm << 20) / item_b) : nitems;
        const std::string tag = fm ? std::to_string(fm) + "MB" : std::string("all");
        auto none = [] {};
        auto fresh = [&] { hipLaunchKernelGGL(k_touch, dim3(2048), dim3(256), 0, 0, in, (size_t)nsrc * CW, 5u); };
        add("cm_plain_" + tag, fb / timeit2([&] { hipLaunchKernelGGL((k_fan_cm<1024, CW, false>), dim3(512), dim3(1024), 0, 0, in, out, nitems, nsrc); }, none) / 1e6);
        add("cm_nt_" + tag, fb / timeit2([&] { hipLaunchKernelGGL((k_fan_cm<1024, CW, true>), dim3(512), dim3(1024), 0, 0, in, out, nitems, nsrc); }, none) / 1e6);
        if (fm == 128 || fm == 0)
            add("cm_nt_fresh_" + tag, fb / timeit2([&] { hipLaunchKernelGGL((k_fan_cm<1024, CW, true>), dim3(512), dim3(1024), 0, 0, in, out, nitems, nsrc); }, fresh) / 1e6);
    }
    js += "}";
    printf("%s\n", js.c_str());
    return 0;
}
