// tools/store_peak2.hip -- calibration (not product): what limits a read-once/write-16x
// fan-out on MI355X?  All variants move 512 MiB in -> 8 GiB out.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <string>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// A: grid-stride lane-per-word, 16 destinations `stride` words apart (naive)
__global__ __launch_bounds__(256) void k_a(const u32x4* in, u32x4* out, size_t nin, size_t stride) {
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < nin; i += (size_t)gridDim.x * 256) {
        u32x4 v = in[i];
#pragma unroll
        for (int f = 0; f < 16; f++) out[f * stride + i] = v;
    }
}
// B: block-chunked like k_fanout2: block owns chunk of CW words (register staged), writes the
// chunk to 16 destinations one after the other (each a contiguous span)
template <int T, int NW, bool READ>
__global__ __launch_bounds__(T) void k_b(const u32x4* in, u32x4* out, size_t nin, size_t stride, size_t mis = 0) {
    const size_t cw = (size_t)T * NW;
    for (size_t c = blockIdx.x; c * cw < nin; c += gridDim.x) {
        u32x4 r[NW];
#pragma unroll
        for (int j = 0; j < NW; j++) {
            size_t i = c * cw + j * T + threadIdx.x;
            if (READ) r[j] = i < nin ? in[i] : u32x4{0, 0, 0, 0};
            else r[j] = u32x4{(unsigned)i, 1u, 2u, 3u};
        }
        for (int f = 0; f < 16; f++) {
#pragma unroll
            for (int j = 0; j < NW; j++) {
                size_t i = c * cw + j * T + threadIdx.x;
                if (i < nin) out[f * stride + i + mis * (f + 1)] = r[j];
            }
        }
    }
}
// C: chunk-major layout: chunk c's 16 copies are adjacent (block writes 16*CW contiguous)
template <int T, int NW>
__global__ __launch_bounds__(T) void k_c(const u32x4* in, u32x4* out, size_t nin) {
    const size_t cw = (size_t)T * NW;
    for (size_t c = blockIdx.x; c * cw < nin; c += gridDim.x) {
        u32x4 r[NW];
#pragma unroll
        for (int j = 0; j < NW; j++) {
            size_t i = c * cw + j * T + threadIdx.x;
            r[j] = i < nin ? in[i] : u32x4{0, 0, 0, 0};
        }
        u32x4* o = out + c * cw * 16;
        for (int f = 0; f < 16; f++) {
#pragma unroll
            for (int j = 0; j < NW; j++) {
                size_t i = c * cw + j * T + threadIdx.x;
                if (i < nin) o[f * cw + j * T + threadIdx.x] = r[j];
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
    const size_t out_bytes = 8ull << 30, nin = (out_bytes / 16) / 16;
    u32x4* out; hipMalloc(&out, out_bytes + (64 << 20));
    u32x4* in; hipMalloc(&in, nin * 16);
    hipMemset(in, 1, nin * 16);
    const double B = out_bytes + nin * 16.0;
    std::string js = "{";
    auto add = [&](const char* k, float ms) { char buf[160]; snprintf(buf, sizeof buf, "%s\"%s\": %.1f", js.size() > 1 ? ", " : "", k, B / ms / 1e6); js += buf; };
    const size_t s_pow2 = nin, s_odd = nin + 4096 * 7 + 48;
    add("A_pow2", timeit([&] { hipLaunchKernelGGL(k_a, dim3(2048), dim3(256), 0, 0, in, out, nin, s_pow2); }));
    add("A_odd", timeit([&] { hipLaunchKernelGGL(k_a, dim3(2048), dim3(256), 0, 0, in, out, nin, s_odd); }));
    add("B512x6_read_odd", timeit([&] { hipLaunchKernelGGL((k_b<512, 6, true>), dim3(512), dim3(512), 0, 0, in, out, nin, s_odd); }));
    add("B512x6_noread_odd", timeit([&] { hipLaunchKernelGGL((k_b<512, 6, false>), dim3(512), dim3(512), 0, 0, in, out, nin, s_odd); }));
    add("B512x6_read_odd_g2048", timeit([&] { hipLaunchKernelGGL((k_b<512, 6, true>), dim3(2048), dim3(512), 0, 0, in, out, nin, s_odd); }));
    add("B256x6_read_odd_g2048", timeit([&] { hipLaunchKernelGGL((k_b<256, 6, true>), dim3(2048), dim3(256), 0, 0, in, out, nin, s_odd); }));
    add("B256x2_read_odd_g4096", timeit([&] { hipLaunchKernelGGL((k_b<256, 2, true>), dim3(4096), dim3(256), 0, 0, in, out, nin, s_odd); }));
    add("B256x2_noread_odd_g4096", timeit([&] { hipLaunchKernelGGL((k_b<256, 2, false>), dim3(4096), dim3(256), 0, 0, in, out, nin, s_odd); }));
    add("B1024x4_read_odd_g256", timeit([&] { hipLaunchKernelGGL((k_b<1024, 4, true>), dim3(256), dim3(1024), 0, 0, in, out, nin, s_odd); }));
    add("B512x6_read_s528k", timeit([&] { hipLaunchKernelGGL((k_b<512, 6, true>), dim3(512), dim3(512), 0, 0, in, out, nin, (size_t)33000); }));
    add("C512x6_read", timeit([&] { hipLaunchKernelGGL((k_c<512, 6>), dim3(512), dim3(512), 0, 0, in, out, nin); }));
    add("C512x6_read_g2048", timeit([&] { hipLaunchKernelGGL((k_c<512, 6>), dim3(2048), dim3(512), 0, 0, in, out, nin); }));
    add("C1024x4_read_g256", timeit([&] { hipLaunchKernelGGL((k_c<1024, 4>), dim3(256), dim3(1024), 0, 0, in, out, nin); }));
    add("C256x8_read_g2048", timeit([&] { hipLaunchKernelGGL((k_c<256, 8>), dim3(2048), dim3(256), 0, 0, in, out, nin); }));
    add("B1024x4_read_odd_mis1", timeit([&] { hipLaunchKernelGGL((k_b<1024, 4, true>), dim3(256), dim3(1024), 0, 0, in, out, nin, s_odd, (size_t)1); }));
    add("B1024x4_read_odd_mis3", timeit([&] { hipLaunchKernelGGL((k_b<1024, 4, true>), dim3(256), dim3(1024), 0, 0, in, out, nin, s_odd, (size_t)3); }));
    add("B1024x4_read_odd_al", timeit([&] { hipLaunchKernelGGL((k_b<1024, 4, true>), dim3(256), dim3(1024), 0, 0, in, out, nin, s_odd, (size_t)0); }));
    add("B1024x4_read_odd_al_g512", timeit([&] { hipLaunchKernelGGL((k_b<1024, 4, true>), dim3(512), dim3(1024), 0, 0, in, out, nin, s_odd, (size_t)0); }));
    add("B1024x4_read_odd_mis1_g512", timeit([&] { hipLaunchKernelGGL((k_b<1024, 4, true>), dim3(512), dim3(1024), 0, 0, in, out, nin, s_odd, (size_t)1); }));
    js += "}";
    printf("%s\n", js.c_str());
    return 0;
}
