// tools/store_peak.hip -- calibration microbenchmark (not part of the product): the HBM
// write / copy ceilings for the fan-out's access shape on this MI355X.
//   write: every lane stores 16-B words to a contiguous region (8 GiB), plain vs nt
//   fanout-shaped: 1 KiB read once from a source, written to 16 destinations 64 MiB apart
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void k_write(u32x4* out, size_t nwords) {
    size_t i = blockIdx.x * (size_t)256 + threadIdx.x;
    u32x4 v = {(unsigned)i, 1u, 2u, 3u};
    for (; i < nwords; i += (size_t)gridDim.x * 256) {
        if (NT) __builtin_nontemporal_store(v, &out[i]); else out[i] = v;
    }
}

template <bool NT, int FAN>
__global__ __launch_bounds__(256) void k_fan(const u32x4* in, u32x4* out, size_t nin, size_t stride) {
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < nin; i += (size_t)gridDim.x * 256) {
        u32x4 v = in[i];
#pragma unroll
        for (int f = 0; f < FAN; f++) {
            if (NT) __builtin_nontemporal_store(v, &out[f * stride + i]); else out[f * stride + i] = v;
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
    const size_t bytes = 8ull << 30, nw = bytes / 16;
    u32x4* out; hipMalloc(&out, bytes);
    u32x4* in; hipMalloc(&in, bytes / 16);
    hipMemset(in, 1, bytes / 16);
    int grid = 256 * 8;
    float t0 = timeit([&] { hipLaunchKernelGGL((k_write<false>), dim3(grid), dim3(256), 0, 0, out, nw); });
    float t1 = timeit([&] { hipLaunchKernelGGL((k_write<true>), dim3(grid), dim3(256), 0, 0, out, nw); });
    const size_t nin = nw / 16, stride = nin;
    float t2 = timeit([&] { hipLaunchKernelGGL((k_fan<false, 16>), dim3(grid), dim3(256), 0, 0, in, out, nin, stride); });
    float t3 = timeit([&] { hipLaunchKernelGGL((k_fan<true, 16>), dim3(grid), dim3(256), 0, 0, in, out, nin, stride); });
    printf("{\"write_plain_GBps\": %.1f, \"write_nt_GBps\": %.1f, \"fan16_plain_GBps\": %.1f, \"fan16_nt_GBps\": %.1f}\n",
           bytes / t0 / 1e6, bytes / t1 / 1e6, (bytes + bytes / 16) / t2 / 1e6, (bytes + bytes / 16) / t3 / 1e6);
    return 0;
}
