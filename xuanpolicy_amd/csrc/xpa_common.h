// Shared device helpers for the gfx950 kernels of xuanpolicy_amd (wave64, CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/xuanpolicy_amd.h"

#define XPA_API extern "C" __attribute__((visibility("default")))

static inline int xpa_launch_status() { return (int)hipGetLastError(); }

constexpr int kWave = 64;

// ---- counter hash RNG (bit-identical to oracle/synth_env.py: mix32 / hash4 / u01) ----------------
__device__ __forceinline__ uint32_t xpa_mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ uint32_t xpa_hash4(uint32_t seed, uint32_t k0, uint32_t k1, uint32_t k2) {
    uint32_t h = xpa_mix32(seed);
    h = xpa_mix32(h ^ k0);
    h = xpa_mix32(h ^ k1);
    return xpa_mix32(h ^ k2);
}

__device__ __forceinline__ float xpa_u01(uint32_t h) { return (float)(h >> 8) * (1.0f / 16777216.0f); }

// ---- wave reductions (fixed butterfly order -> deterministic) ------------------------------------
template <typename T>
__device__ __forceinline__ T xpa_wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <typename T>
__device__ __forceinline__ T xpa_wave_max(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Block sum over `nwaves` waves through LDS scratch (nwaves entries); result valid in all threads.
template <typename T>
__device__ __forceinline__ T xpa_block_sum(T v, T *scratch, int nwaves) {
    v = xpa_wave_sum(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) scratch[w] = v;
    __syncthreads();
    T s = T(0);
    for (int i = 0; i < nwaves; ++i) s += scratch[i];
    return s;
}
