// C3 / C5 convolutional trunk (AC_CNN_Atari / Basic_CNN), the elementwise passes around the MIOpen
// convolutions and hipBLASLt GEMMs, gfx950.  Every tensor is NHWC ([rows = B*H*W, C] row-major), the layout the
// uint8 frames arrive in, so no pass needs a permute.
//
//   K20 xpa_frames_to_f32    uint8 frames -> float32 / 255, as the reference's `observations / 255.0` (NumPy
//                            float64 division) + torch.as_tensor(..., float32) (xuance/torch/representations/
//                            cnn.py:89-92): a 256-entry table of float32(i / 255.0) in LDS, so every value is the
//                            reference's double-rounded one bit for bit.  1 B read + 4 B written per pixel.
//   K21 xpa_bias_act         y = act(y + b) in place over [rows, C]: the conv's bias (run bias-free by MIOpen)
//                            and the ReLU of cnn_block / mlp_block (xuance/torch/utils/layers.py:8-57) in one
//                            pass instead of MIOpen's bias op + torch's activation (8 B per element).
//   K22 xpa_act_bwd_bias     dz = dh * act'(h) in place + per-block column sums of dz (the bias gradient), one
//                            pass over [rows, C] (12 B per element): the ReLU backward and the bias-gradient
//                            reduction of the conv / fc layers; a fixed grid (<= 2048 blocks) so the f64 finalize
//                            (xpa_colsum_finalize) reads few partials.  K10's form for conv-sized row counts.
#include "xpa_common.h"

namespace {

typedef float f4v __attribute__((ext_vector_type(4)));

// Lane = one dword (4 pixels) per step of 64 dwords: every load instruction reads 256 contiguous bytes of the
// wave and every store writes 1 KiB contiguous (a lane that converted 16 B and wrote 4 float4 made each store
// instruction hit 64 B strides, 4.5x slower: r02 C3 trace); 4 dwords in flight per lane.
__global__ __launch_bounds__(256) void frames_to_f32_kernel(const unsigned *__restrict__ src, int64_t n4,
                                                            f4v *__restrict__ dst) {
    __shared__ float lut[256];
    lut[threadIdx.x] = (float)((double)threadIdx.x / 255.0);  // NumPy: uint8 / 255.0 in f64, then float32
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t base = wave * 256; base < n4; base += nw * 256) {  // a wave's 4 x 64 dwords per step
        unsigned w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t i = base + k * 64 + lane;
            w[k] = i < n4 ? __builtin_nontemporal_load(src + i) : 0u;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t i = base + k * 64 + lane;
            const unsigned x = w[k];
            const f4v o = {lut[x & 0xffu], lut[(x >> 8) & 0xffu], lut[(x >> 16) & 0xffu], lut[x >> 24]};
            if (i < n4) __builtin_nontemporal_store(o, dst + i);
        }
    }
}

// the scalar remainder (n % 16, or every element of a misaligned buffer)
__global__ __launch_bounds__(256) void frames_to_f32_tail(const uint8_t *__restrict__ src, int64_t n0, int64_t n,
                                                          float *__restrict__ dst) {
    for (int64_t i = n0 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        dst[i] = (float)((double)src[i] / 255.0);
}

template <int ACT>
__device__ __forceinline__ float act_fwd(float z, float slope) {
    if (ACT == 1) return z > 0.f ? z : z * slope;
    if (ACT == 2) return tanhf(z);
    return z;
}

// C % 4 == 0, C / 4 divides 256: a thread's column quad is fixed across the grid-stride loop (the stride,
// gridDim * 256 quads, is a multiple of C / 4), so its bias quad is loaded once.
template <int ACT, bool BIAS>
__global__ __launch_bounds__(256) void bias_act_kernel(f4v *__restrict__ y, int64_t n4, int cq,
                                                       const f4v *__restrict__ b, float slope) {
    const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
    f4v bq = {0.f, 0.f, 0.f, 0.f};
    if (BIAS) bq = b[i0 % cq];
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = i0; i < n4; i += stride) {
        f4v v = y[i];
        if (BIAS) v += bq;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = act_fwd<ACT>(v[e], slope);
        y[i] = v;
    }
}

template <int ACT>
__device__ __forceinline__ float act_grad(float dh, float h, float slope) {
    if (ACT == 1) return h > 0.f ? dh : dh * slope;  // mask from the OUTPUT: h > 0 <=> z > 0 for slope >= 0
    if (ACT == 2) return dh * (1.0f - h * h);
    return dh;
}

constexpr int kBiasGradBlocks = 2048;
constexpr int kUnroll = 4;

// Thread = (row group g, column quad c4); the block's row groups stride the rows by gridDim * groups; kUnroll
// rows' loads are issued before any of their (in-place) stores.  LDS combine of the row groups in a fixed order.
template <int ACT>
__global__ __launch_bounds__(256) void act_bwd_bias_kernel(const float *dh, const float *__restrict__ h,
                                                           int64_t rows, int C, float slope, float *dz,
                                                           float *__restrict__ partials) {
    extern __shared__ __attribute__((aligned(16))) f4v s_acc[];
    const int cq = C / 4, groups = 256 / cq;
    const int c4 = threadIdx.x % cq, g = threadIdx.x / cq;
    f4v acc = {0.f, 0.f, 0.f, 0.f};
    const int64_t stride = (int64_t)gridDim.x * groups;
    for (int64_t r0 = (int64_t)blockIdx.x * groups + g; r0 < rows; r0 += kUnroll * stride) {
        f4v d[kUnroll], hv[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t r = r0 + u * stride;
            const int64_t off = (r < rows ? r : r0) * C + 4 * c4;
            d[u] = *reinterpret_cast<const f4v *>(dh + off);
            if (ACT != 0) hv[u] = *reinterpret_cast<const f4v *>(h + off);
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t r = r0 + u * stride;
            if (r < rows) {
                f4v v = d[u];
                if (ACT != 0) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = act_grad<ACT>(v[e], hv[u][e], slope);
                    if (dz) *reinterpret_cast<f4v *>(dz + r * C + 4 * c4) = v;
                }
                acc += v;
            }
        }
    }
    s_acc[g * cq + c4] = acc;
    __syncthreads();
    if ((int)threadIdx.x < cq) {
        f4v t = {0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < groups; ++k) t += s_acc[k * cq + threadIdx.x];
        *reinterpret_cast<f4v *>(partials + (int64_t)blockIdx.x * C + 4 * threadIdx.x) = t;
    }
}

// K23: global max over the HW positions of NHWC [B, HW, C] (Basic_CNN's AdaptiveMaxPool2d((1, 1))), thread = (b, c),
// consecutive threads = consecutive channels (each hw step of a wave reads 256 contiguous bytes), 4 positions' loads
// in flight.  torch's rule (AdaptiveMaxPooling2d.cu): max starts at -inf with index 0, and a position replaces it
// when `val > max || isnan(val)` — the first maximum wins, the last NaN wins.
__global__ __launch_bounds__(256) void global_maxpool_kernel(const float *__restrict__ x, int64_t B, int HW, int C,
                                                             float *__restrict__ out, int32_t *__restrict__ argmax) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= B * C) return;
    const int64_t b = i / C;
    const int c = (int)(i - b * C);
    const float *p = x + b * (int64_t)HW * C + c;
    float m = -__builtin_inff();
    int am = 0;
    int hw = 0;
    for (; hw + 4 <= HW; hw += 4) {
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = p[(int64_t)(hw + u) * C];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (v[u] > m || __builtin_isnan(v[u])) {
                m = v[u];
                am = hw + u;
            }
    }
    for (; hw < HW; ++hw) {
        const float v = p[(int64_t)hw * C];
        if (v > m || __builtin_isnan(v)) {
            m = v;
            am = hw;
        }
    }
    out[i] = m;
    argmax[i] = am;
}

// K24: the backward of K23 fused into K22 — the pooled gradient routed to each (b, c)'s argmax position (0
// elsewhere), times act'(h), written as the conv output's dz, with the bias-gradient partials (K22's grid / layout).
template <int ACT>
__global__ __launch_bounds__(256) void maxpool_act_bwd_bias_kernel(const float *__restrict__ dout,
                                                                   const int32_t *__restrict__ argmax,
                                                                   const float *__restrict__ h, int64_t rows, int HW,
                                                                   int C, float slope, float *__restrict__ dz,
                                                                   float *__restrict__ partials) {
    extern __shared__ __attribute__((aligned(16))) f4v s_acc[];
    const int cq = C / 4, groups = 256 / cq;
    const int c4 = threadIdx.x % cq, g = threadIdx.x / cq;
    f4v acc = {0.f, 0.f, 0.f, 0.f};
    const int64_t stride = (int64_t)gridDim.x * groups;
    for (int64_t r = (int64_t)blockIdx.x * groups + g; r < rows; r += stride) {
        const int64_t b = r / HW;
        const int hw = (int)(r - b * HW);
        const f4v hv = *reinterpret_cast<const f4v *>(h + r * C + 4 * c4);
        f4v v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t bc = b * C + 4 * c4 + e;
            v[e] = argmax[bc] == hw ? dout[bc] : 0.f;
            v[e] = act_grad<ACT>(v[e], hv[e], slope);
        }
        *reinterpret_cast<f4v *>(dz + r * C + 4 * c4) = v;
        acc += v;
    }
    s_acc[g * cq + c4] = acc;
    __syncthreads();
    if ((int)threadIdx.x < cq) {
        f4v t = {0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < groups; ++k) t += s_acc[k * cq + threadIdx.x];
        *reinterpret_cast<f4v *>(partials + (int64_t)blockIdx.x * C + 4 * threadIdx.x) = t;
    }
}

int grid_for(int64_t work, int64_t per_block, int64_t cap) {
    int64_t g = (work + per_block - 1) / per_block;
    if (g > cap) g = cap;
    return (int)(g < 1 ? 1 : g);
}


// ---- K25: the first conv straight from the uint8 frames, on the fp32 matrix cores -------------------------------
// y[b, oy, ox, n] = act(sum_{ky, kx, c} (x[b, oy S - P + ky, ox S - P + kx, c] / 255) W[n, c, ky, kx] + bias[n]) for
// C = 4 input channels (one pixel = one dword), an 8 x 8 kernel (K = 256) and 32 output channels (N = 32): the
// implicit GEMM [rows = B OH OW, 256] x [256, 32] with v_mfma_f32_32x32x2_f32 (exact f32 fma chains).  Lane (h, i)
// of a wave owns output row i of a 32-row tile and pixel 2 t + h of each pixel pair t: it loads that pixel's dword
// (0 outside the frame: the zero padding) and feeds its 4 bytes, as exact f32 integers (v_cvt_f32_ubyte, one VALU
// op per MFMA), as the MFMA's k = h for channels c = 0..3, with the matching weights W[n, c, ky, kx] / 255 read from
// an LDS image [pixel][n][c] (one ds_read_b128 per pixel): sum x (w / 255) instead of the reference's
// sum float(x / 255) w — one f32 rounding per term either way (the scale rounds on the weight instead of the
// frame), the same order of difference as any fp32 summation order.  Replaces K20 + MIOpen's conv + K21 for the forward (the uint8 frames are read
// once, the f32 frame copy is never written).  Wave = 2 row tiles (2 accumulators), block = 4 waves = 256 rows,
// grid-stride over row blocks (<= 4 blocks per CU) so the weight image is staged once per block.
constexpr int kC1Rows = 256;

typedef float f32x16 __attribute__((ext_vector_type(16)));

// Loads: 4 chunks of 8 pixel pairs (two kernel rows); chunk c + 1's 16 dwords per lane are requested before chunk
// c's 64 MFMAs (a two-buffer register ring, fully unrolled), addresses as 32-bit offsets from each row tile's frame.
template <int ACT>
__device__ __forceinline__ void conv1_load_chunk(unsigned (&v)[2][8], const unsigned *const (&xr)[2], const int (&by)[2],
                                                 const int (&bx)[2], int H, int W, int chunk, int h) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int p = 16 * chunk + 2 * j + h, ky = p >> 3, kx = p & 7;
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            const int iy = by[rt] + ky, ix = bx[rt] + kx;
            const bool inb = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
            const unsigned d = xr[rt][inb ? iy * W + ix : 0];
            v[rt][j] = inb ? d : 0u;
        }
    }
}

__device__ __forceinline__ void conv1_mfma_chunk(f32x16 (&acc)[2], const unsigned (&v)[2][8], const float *sB, int chunk,
                                                 int h, int i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int p = 16 * chunk + 2 * j + h;
        const f4v b4 = *reinterpret_cast<const f4v *>(sB + (p * 32 + i) * 4);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) {
                const float a = (float)((v[rt][j] >> (8 * c)) & 0xffu);  // v_cvt_f32_ubyte<c>
                acc[rt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b4[c], acc[rt], 0, 0, 0);
            }
        }
    }
}

template <int ACT>
__global__ __launch_bounds__(256, 4) void conv1_u8_fwd_kernel(const unsigned *__restrict__ x, int64_t rows, int H,
                                                              int W, int OH, int OW, int S, int P,
                                                              const float *__restrict__ w, const float *__restrict__ bias,
                                                              float slope, float *__restrict__ y) {
    __shared__ __attribute__((aligned(16))) float sB[64 * 32 * 4];  // [pixel p = ky 8 + kx][n][c]
    const int t = threadIdx.x;
    for (int e = t; e < 64 * 32 * 4; e += 256) {
        const int c = e & 3, n = (e >> 2) & 31, p = e >> 7;
        sB[e] = w[((n * 4 + c) * 8 + (p >> 3)) * 8 + (p & 7)] / 255.0f;  // the 1 / 255 scale on the weight side
    }
    __syncthreads();
    const int lane = t & 63, h = lane >> 5, i = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const float bc = bias[i];
    const int64_t ohw = (int64_t)OH * OW;
    for (int64_t blk = blockIdx.x; blk * kC1Rows < rows; blk += gridDim.x) {
        const int64_t r0 = blk * kC1Rows + wave * 64;
        int by[2], bx[2];
        const unsigned *xr[2];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            const int64_t m = r0 + rt * 32 + i;
            const int64_t mc = m < rows ? m : rows - 1;
            const int64_t b = mc / ohw;
            const int rem = (int)(mc - b * ohw);
            const int oy = rem / OW, ox = rem - (rem / OW) * OW;
            by[rt] = oy * S - P;
            bx[rt] = ox * S - P;
            xr[rt] = x + b * H * W;
        }
        f32x16 acc[2];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[rt][r] = 0.f;
        unsigned va[2][8], vb[2][8];
        // sched_barrier: keep the ring order (hipcc otherwise hoists all 64 loads and their 64-bit addresses: 248
        // VGPRs, 2 waves per SIMD)
        conv1_load_chunk<ACT>(va, xr, by, bx, H, W, 0, h);
        conv1_load_chunk<ACT>(vb, xr, by, bx, H, W, 1, h);
        __builtin_amdgcn_sched_barrier(0);
        conv1_mfma_chunk(acc, va, sB, 0, h, i);
        __builtin_amdgcn_sched_barrier(0);
        conv1_load_chunk<ACT>(va, xr, by, bx, H, W, 2, h);
        __builtin_amdgcn_sched_barrier(0);
        conv1_mfma_chunk(acc, vb, sB, 1, h, i);
        __builtin_amdgcn_sched_barrier(0);
        conv1_load_chunk<ACT>(vb, xr, by, bx, H, W, 3, h);
        __builtin_amdgcn_sched_barrier(0);
        conv1_mfma_chunk(acc, va, sB, 2, h, i);
        __builtin_amdgcn_sched_barrier(0);
        conv1_mfma_chunk(acc, vb, sB, 3, h, i);
        // C/D map: row = (r & 3) + 8 (r >> 2) + 4 h, column n = i
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t m = r0 + rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m < rows) y[m * 32 + i] = act_fwd<ACT>(acc[rt][r] + bc, slope);
            }
    }
}
}  // namespace

XPA_API int xpa_frames_to_f32(const uint8_t *src, int64_t n, float *dst, xpa_stream_t stream) {
    if (n < 0 || (n > 0 && (!src || !dst))) return (int)hipErrorInvalidValue;
    if (n == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const bool vec = ((uintptr_t)src % 4 == 0) && ((uintptr_t)dst % 16 == 0);
    const int64_t n4 = vec ? n / 4 : 0;
    if (n4 > 0) {  // 1024 dwords per block per step, <= 8 blocks per CU, grid-stride beyond that
        const int g = grid_for(n4, 1024, 256 * 8);
        hipLaunchKernelGGL(frames_to_f32_kernel, dim3((unsigned)g), dim3(256), 0, s, (const unsigned *)src, n4,
                           (f4v *)dst);
    }
    const int64_t n0 = n4 * 4;
    if (n0 < n)
        hipLaunchKernelGGL(frames_to_f32_tail, dim3((unsigned)grid_for(n - n0, 256, 4096)), dim3(256), 0, s, src, n0,
                           n, dst);
    return xpa_launch_status();
}

XPA_API int xpa_bias_act(int act, float *y, int64_t rows, int64_t cols, const float *bias, float slope,
                         xpa_stream_t stream) {
    if (rows <= 0 || cols <= 0 || cols % 4 || 256 % (cols / 4) || !y || act < 0 || act > 2)
        return (int)hipErrorInvalidValue;
    if (((uintptr_t)y | (uintptr_t)(bias ? bias : y)) % 16) return (int)hipErrorInvalidValue;
    const int cq = (int)(cols / 4);
    const int64_t n4 = rows * cq;
    const int g = grid_for(n4, 256, 256 * 8 * 4);
    hipStream_t s = (hipStream_t)stream;
#define XPA_BA(A_, B_)                                                                                          \
    hipLaunchKernelGGL((bias_act_kernel<A_, B_>), dim3((unsigned)g), dim3(256), 0, s, (f4v *)y, n4, cq,          \
                       (const f4v *)bias, slope)
    if (bias) {
        if (act == 0) XPA_BA(0, true);
        else if (act == 1) XPA_BA(1, true);
        else XPA_BA(2, true);
    } else {
        if (act == 0) return 0;
        if (act == 1) XPA_BA(1, false);
        else XPA_BA(2, false);
    }
#undef XPA_BA
    return xpa_launch_status();
}

XPA_API int64_t xpa_act_bwd_bias_num_partials(int64_t rows, int64_t cols) {
    if (rows <= 0 || cols <= 0 || cols % 4 || 256 % (cols / 4)) return 0;
    const int64_t groups = 256 / (cols / 4);
    return grid_for(rows, groups * kUnroll, kBiasGradBlocks);
}

XPA_API int xpa_act_bwd_bias(int act, const float *dh, const float *h, int64_t rows, int64_t cols, float slope,
                             float *dz, float *partials, xpa_stream_t stream) {
    const int64_t G = xpa_act_bwd_bias_num_partials(rows, cols);
    if (G <= 0 || !dh || !partials || act < 0 || act > 2 || (act != 0 && !h)) return (int)hipErrorInvalidValue;
    if (((uintptr_t)dh | (uintptr_t)(h ? h : dh) | (uintptr_t)(dz ? dz : dh) | (uintptr_t)partials) % 16)
        return (int)hipErrorInvalidValue;
    const int C = (int)cols;
    const size_t lds = 256 * sizeof(f4v);
    hipStream_t s = (hipStream_t)stream;
#define XPA_ABB(A_)                                                                                               \
    hipLaunchKernelGGL((act_bwd_bias_kernel<A_>), dim3((unsigned)G), dim3(256), lds, s, dh, h, rows, C, slope, dz, \
                       partials)
    if (act == 0) XPA_ABB(0);
    else if (act == 1) XPA_ABB(1);
    else XPA_ABB(2);
#undef XPA_ABB
    return xpa_launch_status();
}

XPA_API int xpa_global_maxpool(const float *x, int64_t batch, int64_t hw, int64_t channels, float *out,
                               int32_t *argmax, xpa_stream_t stream) {
    if (batch <= 0 || hw <= 0 || channels <= 0 || hw > (1 << 30) || channels > (1 << 20) || !x || !out || !argmax)
        return (int)hipErrorInvalidValue;
    const int64_t n = batch * channels;
    hipLaunchKernelGGL(global_maxpool_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x,
                       batch, (int)hw, (int)channels, out, argmax);
    return xpa_launch_status();
}

XPA_API int xpa_maxpool_act_bwd_bias(int act, const float *dout, const int32_t *argmax, const float *h, int64_t batch,
                                     int64_t hw, int64_t channels, float slope, float *dz, float *partials,
                                     xpa_stream_t stream) {
    const int64_t rows = batch * hw;
    const int64_t G = xpa_act_bwd_bias_num_partials(rows, channels);
    if (G <= 0 || hw > (1 << 30) || !dout || !argmax || !h || !dz || !partials || act < 0 || act > 2)
        return (int)hipErrorInvalidValue;
    if (((uintptr_t)h | (uintptr_t)dz | (uintptr_t)partials) % 16) return (int)hipErrorInvalidValue;
    const size_t lds = 256 * sizeof(f4v);
    hipStream_t s = (hipStream_t)stream;
#define XPA_MPB(A_)                                                                                              \
    hipLaunchKernelGGL((maxpool_act_bwd_bias_kernel<A_>), dim3((unsigned)G), dim3(256), lds, s, dout, argmax, h, \
                       rows, (int)hw, (int)channels, slope, dz, partials)
    if (act == 0) XPA_MPB(0);
    else if (act == 1) XPA_MPB(1);
    else XPA_MPB(2);
#undef XPA_MPB
    return xpa_launch_status();
}

XPA_API int xpa_conv1_u8_fwd(int act, const uint8_t *x, int64_t batch, int64_t height, int64_t width, int64_t channels,
                             int64_t kernel, int64_t stride, int64_t pad, const float *w, const float *bias,
                             int64_t out_channels, float slope, float *y, xpa_stream_t stream) {
    if (batch <= 0 || channels != 4 || kernel != 8 || out_channels != 32 || stride < 1 || pad < 0 || act < 0 ||
        act > 2 || !x || !w || !bias || !y || ((uintptr_t)x % 4) || height + 2 * pad < kernel ||
        width + 2 * pad < kernel || height * width > (1 << 30))
        return (int)hipErrorInvalidValue;
    const int64_t OH = (height + 2 * pad - kernel) / stride + 1, OW = (width + 2 * pad - kernel) / stride + 1;
    const int64_t rows = batch * OH * OW;
    const int64_t blocks = (rows + kC1Rows - 1) / kC1Rows;
    const dim3 grid((unsigned)(blocks < 1024 ? blocks : 1024)), block(256);
    hipStream_t s = (hipStream_t)stream;
#define XPA_C1(A_)                                                                                                   \
    hipLaunchKernelGGL((conv1_u8_fwd_kernel<A_>), grid, block, 0, s, (const unsigned *)x, rows, (int)height,           \
                       (int)width, (int)OH, (int)OW, (int)stride, (int)pad, w, bias, slope, y)
    if (act == 0) XPA_C1(0);
    else if (act == 1) XPA_C1(1);
    else XPA_C1(2);
#undef XPA_C1
    return xpa_launch_status();
}
