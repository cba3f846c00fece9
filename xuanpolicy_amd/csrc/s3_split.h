// The three-way bf16 split of f32 operands for the bf16 matrix cores (K40 sgemm3.hip, K16S head.hip).
//
// x = hi + mid + lo EXACTLY: hi = bf16_rn(x), mid = bf16_rn(x - hi), lo = bf16_rn(x - hi - mid); both residuals are
// exact in f32 and 3 x 8 significant bits cover the f32 significand: exact for 2^-100 <= |x| < 3.39e38 (bf16's largest
// finite value; below 2^-100 lo drops bits under 2^-24 of x, tests/test_split_model_cpu.py).  A product
// a b keeps the six terms above 2^-24 relative, summed smallest first into one f32 accumulator:
//     am bm + ah bl + al bh + ah bm + am bh + ah bh
// (dropped: am bl, al bm, al bl <= 2^-25 relative).  Each bf16 x bf16 product is exact in f32.  An infinite or NaN
// operand gives NaN (inf - inf in the residual) where the f32 GEMM might give inf: the callers' operands are finite.
#pragma once
#include <hip/hip_runtime.h>

typedef __bf16 xpa_bf16x8 __attribute__((ext_vector_type(8)));
typedef float xpa_f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void xpa_split3(float x, __bf16 &hi, __bf16 &mid, __bf16 &lo) {
    hi = (__bf16)x;
    const float r1 = x - (float)hi;
    mid = (__bf16)r1;
    const float r2 = r1 - (float)mid;
    lo = (__bf16)r2;
}

// the 8 f32 of an MFMA fragment (two quads) -> its three bf16 fragments
__device__ __forceinline__ void xpa_split8(const float4 &q0, const float4 &q1, xpa_bf16x8 &h, xpa_bf16x8 &m,
                                           xpa_bf16x8 &l) {
    const float v[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        __bf16 a, b, c;
        xpa_split3(v[j], a, b, c);
        h[j] = a;
        m[j] = b;
        l[j] = c;
    }
}

// acc += A . B over one 16-k step from the split fragments (the six products, smallest first)
__device__ __forceinline__ xpa_f32x16 xpa_mfma_s3(const xpa_bf16x8 &ah, const xpa_bf16x8 &am, const xpa_bf16x8 &al,
                                                  const xpa_bf16x8 &bh, const xpa_bf16x8 &bm, const xpa_bf16x8 &bl,
                                                  xpa_f32x16 acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
    return acc;
}
