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

// ---- hidden activation + dot product of the rollout value / policy heads -------------------------
// (shared so K14's value head and the value-fused GAE scan form V(s) with the same arithmetic, bit for bit)
// ACT: 0 identity, 1 LeakyReLU(slope), 2 tanh.
template <int ACT>
__device__ __forceinline__ float4 xpa_act4(float4 z, float slope) {
    if (ACT == 1) {
        z.x = z.x > 0.f ? z.x : z.x * slope; z.y = z.y > 0.f ? z.y : z.y * slope;
        z.z = z.z > 0.f ? z.z : z.z * slope; z.w = z.w > 0.f ? z.w : z.w * slope;
    } else if (ACT == 2) {
        z.x = tanhf(z.x); z.y = tanhf(z.y); z.z = tanhf(z.z); z.w = tanhf(z.w);
    }
    return z;
}

// explicit fma chain: left to fp-contract, hipcc picked fma(x, x', y y') in one kernel and fma(y, y', x x') in
// another, so the "same" dot product differed by an ulp between K14 and the value-fused scan
__device__ __forceinline__ float xpa_dot4(float4 a, float4 b) {
    return fmaf(a.w, b.w, fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)));
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

// ---- inter-workgroup hand-off inside one launch (ticketed "last block merges") -------------------
// Producer: xpa_store_agent for every handed-off value (write-through, sc1), then xpa_drain() and the
// block barrier, then one lane takes the ticket (xpa_ticket).  Consumer (the last block): xpa_load_agent
// (sc1 loads).  No __threadfence(): on gfx950 an agent-scope release is a full L2 write-back
// (buffer_wbl2 sc1) per block — 76 us for a ~150-block finalize behind the update's GEMMs (r01).
template <typename T>
__device__ __forceinline__ void xpa_store_agent(T *p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T xpa_load_agent(const T *p) {
    return __hip_atomic_load(const_cast<T *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void xpa_drain() { __builtin_amdgcn_s_waitcnt(0); }
__device__ __forceinline__ unsigned xpa_ticket(unsigned *t) {
    return __hip_atomic_fetch_add(t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
