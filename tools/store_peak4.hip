// tools/store_peak4.hip -- calibration (not product): would a DESTINATION-major fan-out beat
// k_fanout4's chunk-major write-many?  Same synthetic arena as store_peak3's k_fan (900 senders
// x 12 chunks x 2816 words, 16 sub-streams each, 16-B-phased regions), but each workgroup owns
// ONE sub-stream region and copies its sender's source range straight from global memory into
// it (line-aligned stores, U loads in flight per lane).  With the XCD swizzle the 16 workgroups
// of a sender are dispatched consecutively on one XCD, so 15 of 16 source reads can hit its L2.
// Prints GB/s counted like store_peak3's fan modes: source once + 16 copies.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <string>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int THREADS, int U, bool SWZ, bool NT>
__global__ __launch_bounds__(THREADS) void k_dst(const u32x4* in, u32x4* out, int ntask, unsigned n, size_t region) {
    const int b = blockIdx.x;
    const int t = SWZ ? (b % 8) * (ntask / 8) + b / 8 : b;             // XCD-contiguous task ranges
    const int sender = t >> 4;
    const u32x4* src = in + (size_t)sender * n;
    const size_t A = (size_t)t * region + ((t * 7) & 7);               // 16-B phase per region
    const unsigned s = (unsigned)(A & 7);
    u32x4* dst = out + (A - s);
    for (unsigned i0 = threadIdx.x; i0 < n + s; i0 += THREADS * U) {
        u32x4 v[U];
#pragma unroll
        for (int j = 0; j < U; j++) {
            const unsigned lw = i0 + j * THREADS, w = lw - s;
            if (lw < n + s && w < n) v[j] = src[w];
        }
#pragma unroll
        for (int j = 0; j < U; j++) {
            const unsigned lw = i0 + j * THREADS, w = lw - s;
            if (lw < n + s && w < n) {
                if (NT) __builtin_nontemporal_store(v[j], dst + lw);
                else dst[lw] = v[j];
            }
        }
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
    const int CW = 2816, nch = 12, nsend = 896;                       // ntask % 8 == 0
    const unsigned n = (unsigned)nch * CW;
    const int ntask = nsend * 16;
    const size_t region = (size_t)n + 64;
    u32x4 *in, *out;
    if (hipMalloc(&in, (size_t)nsend * n * 16) != hipSuccess || hipMalloc(&out, (size_t)ntask * region * 16) != hipSuccess) return 1;
    hipMemset(in, 7, (size_t)nsend * n * 16);
    const double fb = (double)nsend * n * 16 * 17;
    std::string js = "{";
    auto add = [&](const char* k, double gbs) { char buf[128]; snprintf(buf, sizeof buf, "%s\"%s\": %.1f", js.size() > 1 ? ", " : "", k, gbs); js += buf; };
    add("dst1024_u2_swz", fb / timeit([&] { hipLaunchKernelGGL((k_dst<1024, 2, true, false>), dim3(ntask), dim3(1024), 0, 0, in, out, ntask, n, region); }) / 1e6);
    add("dst1024_u4_swz", fb / timeit([&] { hipLaunchKernelGGL((k_dst<1024, 4, true, false>), dim3(ntask), dim3(1024), 0, 0, in, out, ntask, n, region); }) / 1e6);
    add("dst1024_u4_swz_nt", fb / timeit([&] { hipLaunchKernelGGL((k_dst<1024, 4, true, true>), dim3(ntask), dim3(1024), 0, 0, in, out, ntask, n, region); }) / 1e6);
    add("dst1024_u4_noswz_nt", fb / timeit([&] { hipLaunchKernelGGL((k_dst<1024, 4, false, true>), dim3(ntask), dim3(1024), 0, 0, in, out, ntask, n, region); }) / 1e6);
    add("dst512_u4_swz_nt", fb / timeit([&] { hipLaunchKernelGGL((k_dst<512, 4, true, true>), dim3(ntask), dim3(512), 0, 0, in, out, ntask, n, region); }) / 1e6);
    add("dst256_u8_swz_nt", fb / timeit([&] { hipLaunchKernelGGL((k_dst<256, 8, true, true>), dim3(ntask), dim3(256), 0, 0, in, out, ntask, n, region); }) / 1e6);
    printf("%s}\n", js.c_str());
    return 0;
}
