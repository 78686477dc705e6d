// edgpu_bytes.h -- byte-stream loads shared by the ingest and deframe kernels (device code).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace edgpu {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// The 16 bytes at `p` (any alignment) as four little-endian words; bytes at or past `lim`
// read as 0.  Only aligned 16-B blocks holding a byte of [p, lim) are loaded (p < lim), so
// the loads never leave the pages of the bytes asked for.
__device__ __forceinline__ u32x4 load16_unaligned(const uint8_t* p, const uint8_t* lim) {
    const uintptr_t a = (uintptr_t)p;
    const uintptr_t al = a & ~(uintptr_t)15;
    const uint32_t sh = (uint32_t)(a & 15);
    const u32x4 w0 = *reinterpret_cast<const u32x4*>(al);
    u32x4 w1 = w0;
    if (sh && al + 16 < (uintptr_t)lim) w1 = *reinterpret_cast<const u32x4*>(al + 16);
    const uint32_t d[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
    const uint32_t q = sh >> 2, r = sh & 3;
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        // d[i + q], d[i + q + 1] without dynamic register indexing
        uint32_t lo = d[i], hi = d[i + 1];
        if (q == 1) { lo = d[i + 1]; hi = d[i + 2]; }
        else if (q == 2) { lo = d[i + 2]; hi = d[i + 3]; }
        else if (q == 3) { lo = d[i + 3]; hi = d[i + 4]; }
        o[i] = r ? __builtin_amdgcn_alignbyte(hi, lo, r) : lo;
    }
    if (p + 16 > lim) {
        const int nb = (int)(lim - p);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int keep = nb - 4 * i;
            o[i] = keep >= 4 ? o[i] : keep <= 0 ? 0u : (o[i] & ((1u << (8 * keep)) - 1));
        }
    }
    return u32x4{o[0], o[1], o[2], o[3]};
}

// The 16 bytes at offset `sh` (0..15) of the 32-byte pair (lo, hi) of aligned blocks.
__device__ __forceinline__ u32x4 funnel16(u32x4 w0, u32x4 w1, uint32_t sh) {
    const uint32_t d[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
    const uint32_t q = sh >> 2, r = sh & 3;
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint32_t lo = d[i], hi = d[i + 1];
        if (q == 1) { lo = d[i + 1]; hi = d[i + 2]; }
        else if (q == 2) { lo = d[i + 2]; hi = d[i + 3]; }
        else if (q == 3) { lo = d[i + 3]; hi = d[i + 4]; }
        o[i] = r ? __builtin_amdgcn_alignbyte(hi, lo, r) : lo;
    }
    return u32x4{o[0], o[1], o[2], o[3]};
}

// Bytes at or past `nb` (0..16) of a 16-B word cleared.
__device__ __forceinline__ u32x4 keep16(u32x4 v, int nb) {
    uint32_t o[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int keep = nb - 4 * i;
        o[i] = keep >= 4 ? o[i] : keep <= 0 ? 0u : (o[i] & ((1u << (8 * keep)) - 1));
    }
    return u32x4{o[0], o[1], o[2], o[3]};
}

// Lane l gets lane l + 1's value of `v`; lane 63 gets `last` (DPP wave_shl:1, one VALU op per
// dword -- no LDS traffic, unlike a __shfl).
__device__ __forceinline__ u32x4 wave_next(u32x4 v, u32x4 last) {
    return u32x4{(uint32_t)__builtin_amdgcn_update_dpp((int)last.x, (int)v.x, 0x130, 0xF, 0xF, false),
                 (uint32_t)__builtin_amdgcn_update_dpp((int)last.y, (int)v.y, 0x130, 0xF, 0xF, false),
                 (uint32_t)__builtin_amdgcn_update_dpp((int)last.z, (int)v.z, 0x130, 0xF, 0xF, false),
                 (uint32_t)__builtin_amdgcn_update_dpp((int)last.w, (int)v.w, 0x130, 0xF, 0xF, false)};
}

}  // namespace edgpu
