// tools/repro_fpi.hip -- isolates the mechanism behind the r01 stale RTP-Info result (DESIGN
// §4.9).  The r01 engine ran each RTP-Info PLAY query as:
//     hipMallocAsync(Q), hipMallocAsync(R)                   (stream-ordered pool)
//     hipMemcpyAsync(Q <- pageable std::vector, H2D)
//     k_first_packet_info<<<...>>>(Q, R)                     (writes every R[i])
//     hipMemcpyAsync(pageable std::vector <- R, D2H)
//     hipFreeAsync(Q), hipFreeAsync(R); hipStreamSynchronize
// and rarely returned the PREVIOUS query's result.  Both buffers come back from the pool with
// the previous call's contents, so two orderings explain that: (a) the kernel read a stale Q
// (the H2D copy of the new query landed after the kernel read it) or (b) the D2H copy read a
// stale R (before the kernel's write).  Here every query carries a nonce and the kernel stamps
// each result with (the nonce it read, a device-side launch counter), so a mismatch says which:
//     result nonce = previous, stamp = this launch    -> (a) stale query read by the kernel
//     result nonce = previous, stamp = previous launch -> (b) stale result read by the copy
// Modes: 0 the r01 pattern above; 1 persistent device buffers + pinned host staging (the r01
// fix, as the engine runs it now); 2 the r01 pattern behind a ~20-us kernel on the stream (the
// PLAY query ran behind ingest work).  Prints one JSON line.  Usage: repro_fpi [iters] [mode]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

struct Q { unsigned nonce, pad[3]; };
struct R { unsigned nonce, launch, pad[2]; };

__global__ void k_stamp(const Q* q, R* r, unsigned n, unsigned* counter) {
    __shared__ unsigned launch;
    if (threadIdx.x == 0) launch = atomicAdd(counter, 1u) + 1u;
    __syncthreads();
    const unsigned i = threadIdx.x;
    if (i < n) { R o; o.nonce = q[i].nonce; o.launch = launch; o.pad[0] = o.pad[1] = 0; r[i] = o; }
}

__global__ void k_busy(long long cycles) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {}
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    const int mode = argc > 2 ? atoi(argv[2]) : 0;
    const unsigned n = 2;                       // tracks per query
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    unsigned* counter;
    CK(hipMalloc(&counter, 4));
    CK(hipMemset(counter, 0, 4));
    Q* dq = nullptr; R* dr = nullptr; Q* hq = nullptr; R* hr = nullptr;
    if (mode == 1) {
        CK(hipMalloc(&dq, 16 * sizeof(Q))); CK(hipMalloc(&dr, 16 * sizeof(R)));
        CK(hipHostMalloc((void**)&hq, 16 * sizeof(Q), hipHostMallocDefault));
        CK(hipHostMalloc((void**)&hr, 16 * sizeof(R), hipHostMallocDefault));
    }
    long stale_query = 0, stale_result = 0, other = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int it = 1; it <= iters; it++) {
        std::vector<Q> q(n);
        std::vector<R> r(n);
        for (unsigned i = 0; i < n; i++) q[i].nonce = (unsigned)it * 16u + i;
        if (mode == 0 || mode == 2) {
            if (mode == 2) hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, st, 40000LL);
            CK(hipMallocAsync((void**)&dq, n * sizeof(Q), st));
            CK(hipMallocAsync((void**)&dr, n * sizeof(R), st));
            CK(hipMemcpyAsync(dq, q.data(), n * sizeof(Q), hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, st, dq, dr, n, counter);
            CK(hipGetLastError());
            CK(hipMemcpyAsync(r.data(), dr, n * sizeof(R), hipMemcpyDeviceToHost, st));
            CK(hipFreeAsync(dq, st));
            CK(hipFreeAsync(dr, st));
            CK(hipStreamSynchronize(st));
        } else {
            for (unsigned i = 0; i < n; i++) hq[i] = q[i];
            CK(hipMemcpyAsync(dq, hq, n * sizeof(Q), hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, st, dq, dr, n, counter);
            CK(hipGetLastError());
            CK(hipMemcpyAsync(hr, dr, n * sizeof(R), hipMemcpyDeviceToHost, st));
            CK(hipStreamSynchronize(st));
            for (unsigned i = 0; i < n; i++) r[i] = hr[i];
        }
        for (unsigned i = 0; i < n; i++) {
            if (r[i].nonce == q[i].nonce && r[i].launch == (unsigned)it) continue;
            if (r[i].launch == (unsigned)it) stale_query++;
            else if (r[i].launch + 1 == (unsigned)it) stale_result++;
            else other++;
        }
    }
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("{\"mode\": %d, \"iters\": %d, \"results\": %d, \"stale_query_read_by_kernel\": %ld, "
           "\"stale_result_read_by_copy\": %ld, \"other\": %ld, \"seconds\": %.3f}\n",
           mode, iters, iters * (int)n, stale_query, stale_result, other, s);
    return 0;
}
