// Device -> host readback calibration for the drop-in's per-tick readback (a tick's distinct
// bytes, ~52 MB at C2 with 100-ms ticks): hipMemcpyAsync into pinned memory (one call, or split
// over several streams), against a kernel that stores straight into the pinned host buffer over
// PCIe.  Prints one JSON line.  Build: hipcc --offload-arch=gfx950 -O3 tools/pcie_d2h.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_store_host(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull)
        __builtin_nontemporal_store(src[i], &dst[i]);
}

int main(int argc, char** argv) {
    const uint64_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 0) : 52ull << 20) & ~15ull;
    const int reps = 10;
    void* d = nullptr;
    void* h = nullptr;
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(d, 0x5A, bytes));
    CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
    hipStream_t st[4];
    for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    auto time = [&](auto fn) {
        fn(); CK(hipDeviceSynchronize());
        double best = 1e30, sum = 0;
        for (int r = 0; r < reps; r++) {
            auto a = std::chrono::steady_clock::now();
            fn();
            CK(hipDeviceSynchronize());
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
            best = std::min(best, ms); sum += ms;
        }
        return std::make_pair(best, sum / reps);
    };
    auto copy_split = [&](int k) {
        return [&, k]() {
            const uint64_t part = ((bytes / k) + 15) & ~15ull;
            for (int i = 0; i < k; i++) {
                const uint64_t o = part * i;
                if (o >= bytes) break;
                CK(hipMemcpyAsync((char*)h + o, (const char*)d + o, std::min(part, bytes - o), hipMemcpyDeviceToHost, st[i]));
            }
        };
    };
    auto kern = [&](int blocks) {
        return [&, blocks]() {
            hipLaunchKernelGGL(k_store_host, dim3(blocks), dim3(256), 0, st[0], (const u32x4*)d, (u32x4*)h, bytes / 16);
        };
    };
    printf("{\"bytes\": %llu", (unsigned long long)bytes);
    for (int k : {1, 2, 4}) {
        auto r = time(copy_split(k));
        printf(", \"memcpy_streams%d\": {\"best_ms\": %.3f, \"mean_ms\": %.3f, \"GBps\": %.1f}", k, r.first, r.second, bytes / r.first / 1e6);
    }
    for (int b : {256, 1024, 4096}) {
        auto r = time(kern(b));
        printf(", \"kernel_store_%d\": {\"best_ms\": %.3f, \"mean_ms\": %.3f, \"GBps\": %.1f}", b, r.first, r.second, bytes / r.first / 1e6);
    }
    // check the kernel path's bytes
    const unsigned char* p = (const unsigned char*)h;
    bool ok = true;
    for (uint64_t i = 0; i < bytes; i += 4093) ok &= p[i] == 0x5A;
    printf(", \"kernel_bytes_ok\": %s}\n", ok ? "true" : "false");
    return 0;
}
