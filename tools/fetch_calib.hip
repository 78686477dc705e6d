// fetch_calib.hip -- what a narrow load costs in HBM traffic on gfx950, and how FETCH_SIZE
// tallies it (MI355X_MICROARCH.md: "Other access widths are uncalibrated: calibrate on a known
// byte count in your own access pattern").  The ingest's header phase and the deframe walk read
// 4-48 B per frame at scattered offsets; their traffic figures double FETCH_SIZE
// as for a wide stream.  Each pattern below touches a known set of 128-B lines of a buffer far
// larger than the 256-MiB Infinity Cache; its duration against the full stream's says how many
// bytes per line the memory really moved, and a rocprofv3 --pmc pass gives the counters.
//
//   stream        16 B per lane, coalesced, every byte                    (lines: all)
//   l128_o0_16    16 B at the start of every 128-B line                  (lines: all)
//   l128_o48_16   16 B at byte 48 of every line
//   l128_o40_48   48 B (three 16-B loads) from byte 40 of every line
//   l64_o0_16     16 B at the start of every 64-B half line              (lines: all)
//   l256_o0_16    16 B at the start of every other line                  (lines: half)
//   l128_o0_4     4 B at the start of every line                         (lines: all)
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
// Run:   tools/fetch_calib [GiB] [reps]  -> one JSON line per pattern
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// every lane folds what it loaded; a store that never happens keeps the loads alive
__device__ __forceinline__ void sink(uint32_t acc, uint32_t* out) {
    if (acc == 0x9E3779B9u) out[threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_stream(const u32x4* __restrict__ p, uint64_t n16, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        const u32x4 v = p[i];
        acc ^= v.x + v.y + v.z + v.w;
    }
    sink(acc, out);
}

// one unit of `stride` bytes per lane: NL 16-B loads from byte OFF of it
template <uint32_t NL>
__global__ __launch_bounds__(256) void k_strided(const uint8_t* __restrict__ p, uint64_t nunits, uint32_t stride,
                                                 uint32_t off, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nunits; i += (uint64_t)gridDim.x * 256) {
        const u32x4* q = reinterpret_cast<const u32x4*>(p + i * stride + off);
#pragma unroll
        for (uint32_t k = 0; k < NL; k++) {
            const u32x4 v = q[k];
            acc ^= v.x + v.y + v.z + v.w;
        }
    }
    sink(acc, out);
}

__global__ __launch_bounds__(256) void k_dword(const uint8_t* __restrict__ p, uint64_t nunits, uint32_t stride,
                                               uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nunits; i += (uint64_t)gridDim.x * 256)
        acc ^= *reinterpret_cast<const uint32_t*>(p + i * stride);
    sink(acc, out);
}

__global__ void k_fill(uint32_t* p, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        p[i] = (uint32_t)(i * 2654435761u);
}

int main(int argc, char** argv) {
    const uint64_t gib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 4;
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    const uint64_t bytes = gib << 30;
    uint8_t* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 4096));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint32_t*)buf, bytes / 4);
    CK(hipDeviceSynchronize());
    const dim3 grid(256 * 8 * 4), blk(256);   // 32 waves per CU: enough loads in flight
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct Pat {
        const char* name;
        int kind;           // 0 stream, 1 strided 16-B loads, 2 dword
        uint32_t stride, off, nl;
    } pats[] = {
        {"stream", 0, 16, 0, 1},         {"l128_o0_16", 1, 128, 0, 1}, {"l128_o48_16", 1, 128, 48, 1},
        {"l128_o40_48", 1, 128, 40, 3},  {"l64_o0_16", 1, 64, 0, 1},   {"l256_o0_16", 1, 256, 0, 1},
        {"l128_o0_4", 2, 128, 0, 1},
    };
    for (const Pat& pt : pats) {
        const uint64_t nunits = bytes / pt.stride;
        auto launch = [&]() {
            if (pt.kind == 0)
                hipLaunchKernelGGL(k_stream, grid, blk, 0, 0, (const u32x4*)buf, bytes / 16, out);
            else if (pt.kind == 2)
                hipLaunchKernelGGL(k_dword, grid, blk, 0, 0, buf, nunits, pt.stride, out);
            else if (pt.nl == 3)
                hipLaunchKernelGGL(k_strided<3>, grid, blk, 0, 0, buf, nunits, pt.stride, pt.off, out);
            else
                hipLaunchKernelGGL(k_strided<1>, grid, blk, 0, 0, buf, nunits, pt.stride, pt.off, out);
        };
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; r++) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double per = ms / reps;
        const uint64_t lines = pt.stride >= 128 ? bytes / pt.stride : bytes / 128;
        const uint64_t loaded = pt.kind == 0 ? bytes : nunits * (pt.kind == 2 ? 4ull : 16ull * pt.nl);
        printf("{\"pattern\": \"%s\", \"ms\": %.4f, \"lines_touched\": %llu, \"bytes_loaded\": %llu, "
               "\"lines_per_ns\": %.3f}\n",
               pt.name, per, (unsigned long long)lines, (unsigned long long)loaded, lines / per / 1e6);
        fflush(stdout);
    }
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
