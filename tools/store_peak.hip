// tools/store_peak.hip -- calibration microbenchmark (not part of the product): HBM write
// and copy ceilings on this MI355X for the access shapes the fan-out uses.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <string>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// grid-stride, one 16-B word per lane per iteration (1 KiB per wave instruction)
template <bool NT, int UNROLL>
__global__ __launch_bounds__(256) void k_write(u32x4* out, size_t nwords) {
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = blockIdx.x * (size_t)256 + threadIdx.x;
    u32x4 v = {(unsigned)i, 1u, 2u, 3u};
    for (; i + (UNROLL - 1) * stride < nwords; i += UNROLL * stride) {
#pragma unroll
        for (int u = 0; u < UNROLL; u++) {
            if (NT) __builtin_nontemporal_store(v, &out[i + u * stride]); else out[i + u * stride] = v;
        }
    }
    for (; i < nwords; i += stride) out[i] = v;
}

// block-contiguous: each block owns a contiguous span and sweeps it 1 KiB per wave-instruction
template <int THREADS>
__global__ __launch_bounds__(THREADS) void k_write_span(u32x4* out, size_t nwords) {
    const size_t per = (nwords + gridDim.x - 1) / gridDim.x;
    const size_t b = blockIdx.x * per, e = min(nwords, b + per);
    u32x4 v = {1u, 1u, 2u, 3u};
    for (size_t i = b + threadIdx.x; i < e; i += THREADS) out[i] = v;
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

__global__ __launch_bounds__(256) void k_copy(const u32x4* in, u32x4* out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) out[i] = in[i];
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
    u32x4* in; hipMalloc(&in, bytes / 2);
    hipMemset(in, 1, bytes / 2);
    std::string js = "{";
    auto add = [&](const char* k, double gbs) { char buf[128]; snprintf(buf, sizeof buf, "%s\"%s\": %.1f", js.size() > 1 ? ", " : "", k, gbs); js += buf; };
    for (int g : {4, 8, 16, 64}) {
        int grid = 256 * g;
        char name[64];
        snprintf(name, sizeof name, "write_plain_g%d", g);
        add(name, bytes / timeit([&] { hipLaunchKernelGGL((k_write<false, 1>), dim3(grid), dim3(256), 0, 0, out, nw); }) / 1e6);
        snprintf(name, sizeof name, "write_plain_u4_g%d", g);
        add(name, bytes / timeit([&] { hipLaunchKernelGGL((k_write<false, 4>), dim3(grid), dim3(256), 0, 0, out, nw); }) / 1e6);
    }
    add("write_nt_g8", bytes / timeit([&] { hipLaunchKernelGGL((k_write<true, 1>), dim3(2048), dim3(256), 0, 0, out, nw); }) / 1e6);
    add("write_span256_g2048", bytes / timeit([&] { hipLaunchKernelGGL((k_write_span<256>), dim3(2048), dim3(256), 0, 0, out, nw); }) / 1e6);
    add("write_span1024_g1024", bytes / timeit([&] { hipLaunchKernelGGL((k_write_span<1024>), dim3(1024), dim3(1024), 0, 0, out, nw); }) / 1e6);
    add("memset_async", bytes / timeit([&] { hipMemsetAsync(out, 0, bytes, 0); }) / 1e6);
    add("copy_4GiB_rw", 2.0 * (bytes / 2) / timeit([&] { hipLaunchKernelGGL(k_copy, dim3(2048), dim3(256), 0, 0, in, out, nw / 2); }) / 1e6);
    const size_t nin = nw / 16, stride = nin;
    add("fan16_plain", (bytes + bytes / 16) / timeit([&] { hipLaunchKernelGGL((k_fan<false, 16>), dim3(2048), dim3(256), 0, 0, in, out, nin, stride); }) / 1e6);
    add("write_1GiB_plain_g8", (bytes / 8) / timeit([&] { hipLaunchKernelGGL((k_write<false, 1>), dim3(2048), dim3(256), 0, 0, out, nw / 8); }) / 1e6);
    js += "}";
    printf("%s\n", js.c_str());
    return 0;
}
