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
#include "s3_split.h"

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
#pragma clang fp contract(off)  // no product here fuses into its consumer (K26B's split): one value per input everywhere
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
                                                                   float *__restrict__ partials, int *__restrict__ err) {
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
            const int am = argmax[bc];
            if (err && hw == 0 && (am < 0 || am >= HW)) atomicAdd(err, 1);  // K23 writes only in-range indices
            v[e] = am == hw ? dout[bc] : 0.f;
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
// Pixel of slot j (0..7) of a chunk for lane half h: the dword form pairs pixels 2j + h; X2 (even W, S and P, 8-B
// aligned frames) loads pixels 4q + 2h and 4q + 2h + 1 (same kernel row, even column: both in or both out of the frame)
// as one 8-B load into slots 2q, 2q + 1 — half the load instructions (the address units bound the dword form).
template <bool X2>
__device__ __forceinline__ int conv1_pix(int chunk, int j, int h) {
    return X2 ? 16 * chunk + 4 * (j >> 1) + 2 * h + (j & 1) : 16 * chunk + 2 * j + h;
}

template <bool X2>
__device__ __forceinline__ void conv1_load_chunk(unsigned (&v)[2][8], const unsigned *const (&xr)[2], const int (&by)[2],
                                                 const int (&bx)[2], int H, int W, int chunk, int h) {
    if (X2) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int p = conv1_pix<true>(chunk, 2 * q, h), ky = p >> 3, kx = p & 7;
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) {
                const int iy = by[rt] + ky, ix = bx[rt] + kx;
                const bool inb = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
                const uint2 d = *reinterpret_cast<const uint2 *>(xr[rt] + (inb ? iy * W + ix : 0));
                v[rt][2 * q] = inb ? d.x : 0u;
                v[rt][2 * q + 1] = inb ? d.y : 0u;
            }
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int p = conv1_pix<false>(chunk, j, h), ky = p >> 3, kx = p & 7;
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            const int iy = by[rt] + ky, ix = bx[rt] + kx;
            const bool inb = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
            const unsigned d = xr[rt][inb ? iy * W + ix : 0];
            v[rt][j] = inb ? d : 0u;
        }
    }
}

template <bool X2>
__device__ __forceinline__ void conv1_mfma_chunk(f32x16 (&acc)[2], const unsigned (&v)[2][8], const float *sB, int chunk,
                                                 int h, int i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int p = conv1_pix<X2>(chunk, j, h);
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

template <int ACT, bool X2>
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
    // The geometry of a row block for this lane's two rows (clamped past the end: loads stay in bounds).
    auto geometry = [&](int64_t blk, int (&by)[2], int (&bx)[2], const unsigned *(&xr)[2]) {
        const int64_t r0 = blk * kC1Rows + wave * 64;
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
    };
    int64_t blk = blockIdx.x;
    if (blk * kC1Rows >= rows) return;
    int by[2], bx[2];
    const unsigned *xr[2];
    geometry(blk, by, bx, xr);
    unsigned va[2][8], vb[2][8];
    // sched_barrier: keep the ring order (hipcc otherwise hoists all 64 loads and their 64-bit addresses: 248
    // VGPRs, 2 waves per SIMD).  The ring runs on across row blocks: the next block's chunks 0 and 1 are requested
    // during this block's chunks 2 and 3, so no block starts with an exposed load round trip.
    conv1_load_chunk<X2>(va, xr, by, bx, H, W, 0, h);
    conv1_load_chunk<X2>(vb, xr, by, bx, H, W, 1, h);
    for (;;) {
        f32x16 acc[2];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[rt][r] = 0.f;
        __builtin_amdgcn_sched_barrier(0);
        conv1_mfma_chunk<X2>(acc, va, sB, 0, h, i);
        __builtin_amdgcn_sched_barrier(0);
        conv1_load_chunk<X2>(va, xr, by, bx, H, W, 2, h);
        __builtin_amdgcn_sched_barrier(0);
        conv1_mfma_chunk<X2>(acc, vb, sB, 1, h, i);
        __builtin_amdgcn_sched_barrier(0);
        conv1_load_chunk<X2>(vb, xr, by, bx, H, W, 3, h);
        __builtin_amdgcn_sched_barrier(0);
        conv1_mfma_chunk<X2>(acc, va, sB, 2, h, i);
        __builtin_amdgcn_sched_barrier(0);
        const int64_t r0 = blk * kC1Rows + wave * 64;
        const int64_t nblk = blk + gridDim.x;
        const bool more = nblk * kC1Rows < rows;  // block-uniform
        if (more) {
            geometry(nblk, by, bx, xr);
            conv1_load_chunk<X2>(va, xr, by, bx, H, W, 0, h);
        }
        __builtin_amdgcn_sched_barrier(0);
        conv1_mfma_chunk<X2>(acc, vb, sB, 3, h, i);
        __builtin_amdgcn_sched_barrier(0);
        if (more) conv1_load_chunk<X2>(vb, xr, by, bx, H, W, 1, h);
        // C/D map: row = (r & 3) + 8 (r >> 2) + 4 h, column n = i
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t m = r0 + rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m < rows) y[m * 32 + i] = act_fwd<ACT>(acc[rt][r] + bc, slope);
            }
        if (!more) break;
        blk = nblk;
    }
}

// ---- K25B: K25 on the bf16 matrix cores (r05) ---------------------------------------------------------------------
// A byte is exact in bf16 (8 significant bits), so the frames need no split: only the weight side w / 255 (f32) is cut
// into its exact three-way bf16 split (s3_split.h) and a 16-k step is 3 v_mfma_f32_32x32x16_bf16 (lo, mid, hi:
// smallest first) instead of 8 v_mfma_f32_32x32x2_f32 — 96 against 512 MFMA cycles per 16 k.  Each product
// x (w / 255)_plane is exact in f32 and x (mid + lo) has at most 24 significant bits, so a single tap's term reaches the
// accumulator as x (w / 255) rounded once, as in K25; the sum over taps rounds in another (fixed) order.
// k order: step s (16 k) = pixels 4 s .. 4 s + 3 (kernel row s / 2); lane half h feeds pixels 4 s + 2 h and 4 s + 2 h + 1
// (a horizontally adjacent pair: one 8-B load in the X2 form) x 4 channels = its 8 k, the byte order of the two
// dwords.  B image in LDS: [step 16][plane 3][lane 64] x 8 bf16 = 48 KiB, one ds_read_b128 per plane per step shared
// by the wave's two row tiles.  Block = 8 waves x 64 rows, 2 blocks per CU, grid-stride over row blocks with K25's
// register ring (chunk = 4 steps = 2 kernel rows).
constexpr int kC1BRows = 512;

typedef unsigned u32x4v __attribute__((ext_vector_type(4)));

// 8 bytes -> 8 bf16 (each byte's f32 is exact; its bf16 is the f32's top half): v_cvt_f32_ubyte<c> + v_perm_b32
__device__ __forceinline__ xpa_bf16x8 c1b_bytes(unsigned d0, unsigned d1) {
    u32x4v r;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const unsigned d = q < 2 ? d0 : d1, c = 16 * (q & 1);
        const unsigned f0 = __float_as_uint((float)((d >> c) & 0xffu));
        const unsigned f1 = __float_as_uint((float)((d >> (c + 8)) & 0xffu));
        r[q] = __builtin_amdgcn_perm(f1, f0, 0x07060302u);
    }
    return __builtin_bit_cast(xpa_bf16x8, r);
}

// Range-checked buffer loads (a tap outside the frame gets an offset past the record count: the hardware returns
// zeros), so no select consumes a load and the wait for chunk c + 1 lands after chunk c's MFMAs.
template <bool X2>
__device__ __forceinline__ void c1b_load_chunk(uint2 (&v)[2][4], __amdgpu_buffer_rsrc_t rx, const int (&xo)[2],
                                               const int (&by)[2], const int (&bx)[2], int H, int W, int chunk, int h) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int s = 4 * chunk + j, ky = s >> 1, kx = 4 * (s & 1) + 2 * h;
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            const int iy = by[rt] + ky, ix = bx[rt] + kx;
            const bool yin = (unsigned)iy < (unsigned)H;
            const int o = xo[rt] + (iy * W + ix) * 4;
            if (X2) {  // ix even, W even: both pixels in or both out
                const bool inb = yin && (unsigned)ix < (unsigned)W;
                v[rt][j] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rx, inb ? o : INT32_MIN, 0, 0));
            } else {
                const bool in0 = yin && (unsigned)ix < (unsigned)W, in1 = yin && (unsigned)(ix + 1) < (unsigned)W;
                v[rt][j].x = __builtin_amdgcn_raw_buffer_load_b32(rx, in0 ? o : INT32_MIN, 0, 0);
                v[rt][j].y = __builtin_amdgcn_raw_buffer_load_b32(rx, in1 ? o + 4 : INT32_MIN, 0, 0);
            }
        }
    }
}

__device__ __forceinline__ void c1b_mfma_chunk(f32x16 (&acc)[2], const uint2 (&v)[2][4], const xpa_bf16x8 *sB,
                                               int chunk, int lane) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const xpa_bf16x8 *b = sB + (4 * chunk + j) * 3 * 64 + lane;
        const xpa_bf16x8 bh = b[0], bm = b[64], bl = b[128];
        xpa_bf16x8 a[2];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) a[rt] = c1b_bytes(v[rt][j].x, v[rt][j].y);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) acc[rt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[rt], bl, acc[rt], 0, 0, 0);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) acc[rt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[rt], bm, acc[rt], 0, 0, 0);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) acc[rt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[rt], bh, acc[rt], 0, 0, 0);
    }
}

template <int ACT, bool X2>
__global__ __launch_bounds__(512, 2) void conv1_u8_fwd_bf16_kernel(const unsigned *__restrict__ x, int64_t rows, int H,
                                                                   int W, int OH, int OW, int S, int P,
                                                                   const float *__restrict__ w,
                                                                   const float *__restrict__ bias, float slope,
                                                                   float *__restrict__ y) {
    __shared__ xpa_bf16x8 sB[16 * 3 * 64];  // [step][plane hi, mid, lo][lane]
    const int t = threadIdx.x;
    for (int e = t; e < 16 * 64; e += 512) {
        const int s = e >> 6, l = e & 63, n = l & 31, hh = l >> 5;
        xpa_bf16x8 ph, pm, pl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int p = 4 * s + 2 * hh + (j >> 2), c = j & 3;
            __bf16 a, b, cc;
            xpa_split3(w[((n * 4 + c) * 8 + (p >> 3)) * 8 + (p & 7)] / 255.0f, a, b, cc);
            ph[j] = a;
            pm[j] = b;
            pl[j] = cc;
        }
        sB[(s * 3 + 0) * 64 + l] = ph;
        sB[(s * 3 + 1) * 64 + l] = pm;
        sB[(s * 3 + 2) * 64 + l] = pl;
    }
    __syncthreads();
    const int lane = t & 63, h = lane >> 5, i = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const float bc = bias[i];
    const int64_t ohw = (int64_t)OH * OW;
    // the frames as one buffer record (the entry guarantees < 2^31 bytes)
    const int nb = (int)(((rows - 1) / ohw + 1) * H * W * 4);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned *>(x), 0, nb, 0x00020000);
    auto geometry = [&](int64_t blk, int (&by)[2], int (&bx)[2], int (&xr)[2]) {
        const int64_t r0 = blk * kC1BRows + wave * 64;
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            const int64_t m = r0 + rt * 32 + i;
            const int64_t mc = m < rows ? m : rows - 1;
            const int64_t b = mc / ohw;
            const int rem = (int)(mc - b * ohw);
            const int oy = rem / OW, ox = rem - (rem / OW) * OW;
            by[rt] = oy * S - P;
            bx[rt] = ox * S - P;
            xr[rt] = (int)(b * H * W * 4);
        }
    };
    int64_t blk = blockIdx.x;
    if (blk * kC1BRows >= rows) return;
    int by[2], bx[2], xr[2];
    geometry(blk, by, bx, xr);
    uint2 va[2][4], vb[2][4];
    c1b_load_chunk<X2>(va, rx, xr, by, bx, H, W, 0, h);
    c1b_load_chunk<X2>(vb, rx, xr, by, bx, H, W, 1, h);
    for (;;) {
        f32x16 acc[2];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[rt][r] = 0.f;
        __builtin_amdgcn_sched_barrier(0);
        c1b_mfma_chunk(acc, va, sB, 0, lane);
        __builtin_amdgcn_sched_barrier(0);
        c1b_load_chunk<X2>(va, rx, xr, by, bx, H, W, 2, h);
        __builtin_amdgcn_sched_barrier(0);
        c1b_mfma_chunk(acc, vb, sB, 1, lane);
        __builtin_amdgcn_sched_barrier(0);
        c1b_load_chunk<X2>(vb, rx, xr, by, bx, H, W, 3, h);
        __builtin_amdgcn_sched_barrier(0);
        c1b_mfma_chunk(acc, va, sB, 2, lane);
        __builtin_amdgcn_sched_barrier(0);
        const int64_t r0 = blk * kC1BRows + wave * 64;
        const int64_t nblk = blk + gridDim.x;
        const bool more = nblk * kC1BRows < rows;  // block-uniform
        if (more) {
            geometry(nblk, by, bx, xr);
            c1b_load_chunk<X2>(va, rx, xr, by, bx, H, W, 0, h);
        }
        __builtin_amdgcn_sched_barrier(0);
        c1b_mfma_chunk(acc, vb, sB, 3, lane);
        __builtin_amdgcn_sched_barrier(0);
        if (more) c1b_load_chunk<X2>(vb, rx, xr, by, bx, H, W, 1, h);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t m = r0 + rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m < rows) y[m * 32 + i] = act_fwd<ACT>(acc[rt][r] + bc, slope);
            }
        if (!more) break;
        blk = nblk;
    }
}

// ---- K27: data gradient of a stride-s, 2s x 2s conv (the Nature CNN's second conv: 4 x 4 stride 2, 32 -> 64) ------
// dX[b, iy, ix, n] = sum_{ky, kx, co} dY[b, oy, ox, co] W[co, n, ky, kx] over iy = oy s - P + ky, ix likewise.  With a
// 2s kernel every input pixel takes exactly the taps (oy0 - dy, ky0 + dy s) x (ox0 - dx, kx0 + dx s), dy, dx in
// {0, 1}, where oy0 = (iy + P) / s and ky0 = (iy + P) % s: the s x s residue classes (ky0, kx0) each form a plain
// implicit GEMM [rows of the class, K = 4 taps x 64 co] x [K, 32] whose weight operand is uniform over the class.  A
// block owns 256 rows of one class (waves of 2 x 32 rows, v_mfma_f32_32x32x2_f32 as K25): lane (h, i) loads, for its
// row i and tap t, the dY quads 2 j + h (16 B: channels 4q .. 4q + 3; 0 where the tap's output pixel is outside the
// map) and feeds their 4 components as the MFMA's k = h against W[4 q + c, n, ky_t, kx_t] from the class's LDS image
// [tap][co quad][n][4].  Chunks of (tap, half of its 64 channels) in a two-buffer register ring.  Replaces MIOpen's
// stride-2 backward-data kernel (27 % of the fp32 MFMA peak at the C3 update, r02 trace).
constexpr int kDgRows = 256;

struct DgradGeom {
    int H, W, OH, OW, S, P;
    int ny[2], nx[2], iy0[2], ix0[2];  // per residue (s <= 2): rows / first index of the class
    int64_t tiles[4];                  // block-tile prefix ends of the (ry, rx) classes in order 00, 01, 10, 11
    int64_t B;
};

// A tile's per-lane geometry: for its two rows, the dY element offset of every tap (clamped to 0 when the tap's
// output pixel is outside the map, flagged in ok) and the dX row (-1 past the class's rows).
struct DgradRows {
    int off[2][4];
    bool ok[2][4];
    int64_t orow[2];
};

__device__ __forceinline__ int dgrad_class(const DgradGeom &g, int64_t tile) {
    return tile < g.tiles[0] ? 0 : tile < g.tiles[1] ? 1 : tile < g.tiles[2] ? 2 : 3;
}

__device__ __forceinline__ void dgrad_rows(const DgradGeom &g, int64_t gtile, int wave, int i, DgradRows &q) {
    const int cls = dgrad_class(g, gtile);
    const int64_t tile = gtile - (cls ? g.tiles[cls - 1] : 0);
    const int ry = cls >> 1, rx = cls & 1;
    const int ny = g.ny[ry], nx = g.nx[rx];
    const int64_t per_img = (int64_t)ny * nx, rows = g.B * per_img;
    const int64_t r0 = tile * kDgRows + wave * 64;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
        const int64_t m = r0 + rt * 32 + i;
        const bool mv = m < rows;
        const int64_t mc = mv ? m : 0;
        const int64_t b = mc / per_img;
        const int rem = (int)(mc - b * per_img);
        const int ay = rem / nx, ax = rem - (rem / nx) * nx;
        const int iy = g.iy0[ry] + g.S * ay, ix = g.ix0[rx] + g.S * ax;
        q.orow[rt] = mv ? (b * g.H + iy) * g.W + ix : -1;
        const int oy0 = (iy + g.P) / g.S, ox0 = (ix + g.P) / g.S;
#pragma unroll
        for (int tap = 0; tap < 4; ++tap) {
            const int oy = oy0 - (tap >> 1), ox = ox0 - (tap & 1);
            const bool v = mv && (unsigned)oy < (unsigned)g.OH && (unsigned)ox < (unsigned)g.OW;
            q.ok[rt][tap] = v;
            q.off[rt][tap] = v ? (int)(((b * g.OH + oy) * g.OW + ox) * 64) : 0;
        }
    }
}

__device__ __forceinline__ void dgrad_load_chunk(f4v (&v)[2][4], const float *__restrict__ dy, const DgradRows &q,
                                                 int tap, int half, int h) {  // every load from a clamped address
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c4 = 2 * (4 * half + j) + h;  // channel quad
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            const f4v d = *reinterpret_cast<const f4v *>(dy + q.off[rt][tap] + 4 * c4);
            const f4v z = {0.f, 0.f, 0.f, 0.f};
            v[rt][j] = q.ok[rt][tap] ? d : z;
        }
    }
}

__device__ __forceinline__ void dgrad_mfma_chunk(f32x16 (&acc)[2], const f4v (&v)[2][4], const float *sB, int tap,
                                                 int half, int h, int i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int q = 2 * (4 * half + j) + h;
        const f4v b4 = *reinterpret_cast<const f4v *>(sB + ((tap * 16 + q) * 32 + i) * 4);
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
                acc[rt] = __builtin_amdgcn_mfma_f32_32x32x2f32(v[rt][j][c], b4[c], acc[rt], 0, 0, 0);
    }
}

// Persistent blocks over contiguous ranges of the class-major tile list: a block re-stages the weight image only when
// its range crosses into the next residue class (at most 3 times), and the register ring runs on across tiles (the
// next tile's first chunk is requested during the current tile's last one).
constexpr int kDgGrid = 512;  // 2 blocks per CU resident (191 VGPRs)

__global__ __launch_bounds__(256, 2) void conv_dgrad_s2k_kernel(const float *__restrict__ dy, const float *__restrict__ w,
                                                                DgradGeom g, float *__restrict__ dx) {
    __shared__ __attribute__((aligned(16))) float sB[4 * 16 * 32 * 4];  // [tap][co quad][n][4]
    __shared__ int64_t s_orow[4][32];
    const int t = threadIdx.x;
    const int lane = t & 63, h = lane >> 5, i = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int64_t T = g.tiles[3];
    const int64_t t0 = T * blockIdx.x / gridDim.x, t1 = T * (blockIdx.x + 1) / gridDim.x;
    if (t0 >= t1) return;
    const int K = 2 * g.S;
    int staged = -1;
    DgradRows cur, nxt;
    dgrad_rows(g, t0, wave, i, cur);
    f4v va[2][4], vb[2][4];
    dgrad_load_chunk(va, dy, cur, 0, 0, h);
    for (int64_t tile = t0; tile < t1; ++tile) {
        const int cls = dgrad_class(g, tile);
        if (cls != staged) {  // block-uniform
            const int ry = cls >> 1, rx = cls & 1;
            __syncthreads();
            for (int e = t; e < 4 * 16 * 32 * 4; e += 256) {  // W [64 co][32 n][K][K]
                const int c = e & 3, n = (e >> 2) & 31, q = (e >> 7) & 15, tap = e >> 11;
                const int ky = ry + (tap >> 1) * g.S, kx = rx + (tap & 1) * g.S;
                sB[e] = w[(((4 * q + c) * 32 + n) * K + ky) * K + kx];
            }
            __syncthreads();
            staged = cls;
        }
        const bool more = tile + 1 < t1;
        f32x16 acc[2];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[rt][r] = 0.f;
        // 8 chunks (tap, half of the 64 channels): chunk k + 1 requested before chunk k's 32 MFMAs
#pragma unroll
        for (int tap = 0; tap < 4; ++tap) {
            dgrad_load_chunk(vb, dy, cur, tap, 1, h);
            __builtin_amdgcn_sched_barrier(0);
            dgrad_mfma_chunk(acc, va, sB, tap, 0, h, i);
            __builtin_amdgcn_sched_barrier(0);
            if (tap + 1 < 4) {
                dgrad_load_chunk(va, dy, cur, tap + 1, 0, h);
            } else if (more) {
                dgrad_rows(g, tile + 1, wave, i, nxt);
                dgrad_load_chunk(va, dy, nxt, 0, 0, h);
            }
            __builtin_amdgcn_sched_barrier(0);
            dgrad_mfma_chunk(acc, vb, sB, tap, 1, h, i);
            __builtin_amdgcn_sched_barrier(0);
        }
        // C/D map: row = (r & 3) + 8 (r >> 2) + 4 h of the tile, column n = i; the tile's rows are scattered pixels
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            // every lane learns the output offsets of its 16 rows from the row owners (lane i, h = 0)
            __builtin_amdgcn_wave_barrier();
            if (h == 0) s_orow[wave][i] = cur.orow[rt];
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
                const int64_t o = s_orow[wave][row];
                if (o >= 0) dx[o * 32 + i] = acc[rt][r];
            }
        }
        if (more) cur = nxt;
    }
}

// ---- K27B: K27 on the bf16 matrix cores (r05) -------------------------------------------------------------------
// The same residue-class implicit GEMMs with both operands f32: dY split three ways in registers, the class's weight
// operand split three ways into an LDS image [step 16][plane 3][lane 64] x 8 bf16 (48 KiB), six products per 16-k
// step (s3_split.h: f32-GEMM accuracy).  Step s = (tap s / 4, channels 16 (s % 4) .. + 15); lane half h feeds channels
// 16 (s % 4) + 8 h .. + 7 — two adjacent dY quads (32 B).  A chunk (tap, half of its 64 channels) is 2 steps; K27's
// ring, persistent tile ranges and output scatter are unchanged.  4 x 6 MFMAs of 32 cycles per (tap, half) and row tile
// against K27's 16 x 64.
// dY through a range-checked buffer record (a tap outside the map reads zeros: no select consumes a load)
__device__ __forceinline__ void dgrad_b_load_chunk(f4v (&v)[2][4], __amdgpu_buffer_rsrc_t rdy, const DgradRows &q,
                                                   int tap, int half, int h) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c4 = 4 * (2 * half + (j >> 1)) + 2 * h + (j & 1);  // channel quad
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            const int o = q.ok[rt][tap] ? 4 * (q.off[rt][tap] + 4 * c4) : INT32_MIN;
            v[rt][j] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rdy, o, 0, 0));
        }
    }
}

__device__ __forceinline__ void dgrad_b_mfma_chunk(f32x16 (&acc)[2], const f4v (&v)[2][4], const xpa_bf16x8 *sB,
                                                   int tap, int half, int lane) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const xpa_bf16x8 *b = sB + (4 * tap + 2 * half + k) * 3 * 64 + lane;
        const xpa_bf16x8 bh = b[0], bm = b[64], bl = b[128];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            xpa_bf16x8 ah, am, al;
            const f4v q0 = v[rt][2 * k], q1 = v[rt][2 * k + 1];
            xpa_split8(float4{q0[0], q0[1], q0[2], q0[3]}, float4{q1[0], q1[1], q1[2], q1[3]}, ah, am, al);
            acc[rt] = xpa_mfma_s3(ah, am, al, bh, bm, bl, acc[rt]);
        }
    }
}

template <int OCC>
__global__ __launch_bounds__(256, OCC) void conv_dgrad_s2k_bf16_kernel(const float *__restrict__ dy,
                                                                     const float *__restrict__ w, DgradGeom g,
                                                                     float *__restrict__ dx) {
    __shared__ xpa_bf16x8 sB[16 * 3 * 64];  // [step][plane hi, mid, lo][lane]
    __shared__ int64_t s_orow[4][32];
    const int t = threadIdx.x;
    const int lane = t & 63, h = lane >> 5, i = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int64_t T = g.tiles[3];
    const int64_t t0 = T * blockIdx.x / gridDim.x, t1 = T * (blockIdx.x + 1) / gridDim.x;
    if (t0 >= t1) return;
    const int K = 2 * g.S;
    int staged = -1;
    const __amdgpu_buffer_rsrc_t rdy = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(dy), 0, (int)(g.B * g.OH * g.OW * 256), 0x00020000);  // the entry: < 2^31 bytes
    DgradRows cur, nxt;
    dgrad_rows(g, t0, wave, i, cur);
    f4v va[2][4], vb[2][4];
    dgrad_b_load_chunk(va, rdy, cur, 0, 0, h);
    for (int64_t tile = t0; tile < t1; ++tile) {
        const int cls = dgrad_class(g, tile);
        if (cls != staged) {  // block-uniform
            const int ry = cls >> 1, rx = cls & 1;
            __syncthreads();
            for (int e = t; e < 16 * 64; e += 256) {  // W [64 co][32 n][K][K] -> B[k = (tap, co)][n]
                const int s = e >> 6, l = e & 63, n = l & 31, hh = l >> 5, tap = s >> 2;
                const int ky = ry + (tap >> 1) * g.S, kx = rx + (tap & 1) * g.S;
                xpa_bf16x8 ph, pm, pl;
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int co = 16 * (s & 3) + 8 * hh + u;
                    __bf16 a, b, c;
                    xpa_split3(w[((co * 32 + n) * K + ky) * K + kx], a, b, c);
                    ph[u] = a;
                    pm[u] = b;
                    pl[u] = c;
                }
                sB[(s * 3 + 0) * 64 + l] = ph;
                sB[(s * 3 + 1) * 64 + l] = pm;
                sB[(s * 3 + 2) * 64 + l] = pl;
            }
            __syncthreads();
            staged = cls;
        }
        const bool more = tile + 1 < t1;
        f32x16 acc[2];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[rt][r] = 0.f;
#pragma unroll
        for (int tap = 0; tap < 4; ++tap) {
            dgrad_b_load_chunk(vb, rdy, cur, tap, 1, h);
            __builtin_amdgcn_sched_barrier(0);
            dgrad_b_mfma_chunk(acc, va, sB, tap, 0, lane);
            __builtin_amdgcn_sched_barrier(0);
            if (tap + 1 < 4) {
                dgrad_b_load_chunk(va, rdy, cur, tap + 1, 0, h);
            } else if (more) {
                dgrad_rows(g, tile + 1, wave, i, nxt);
                dgrad_b_load_chunk(va, rdy, nxt, 0, 0, h);
            }
            __builtin_amdgcn_sched_barrier(0);
            dgrad_b_mfma_chunk(acc, vb, sB, tap, 1, lane);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            __builtin_amdgcn_wave_barrier();
            if (h == 0) s_orow[wave][i] = cur.orow[rt];
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
                const int64_t o = s_orow[wave][row];
                if (o >= 0) dx[o * 32 + i] = acc[rt][r];
            }
        }
        if (more) cur = nxt;
    }
}

// ---- K26: the first conv's weight gradient straight from the uint8 frames ----------------------------------------
// dW[n, c, ky, kx] = sum_rows dz[row, n] x[row's pixel (ky, kx), c] / 255 for K25's conv (4 channels, 8 x 8, 32
// outputs; dz NHWC [B, OH, OW, 32] after the activation backward).  Split over rows: wave w of a block streams its
// share of rows two at a time (the MFMA's k = the row pair), A = dz^T (lane (h, i): dz[row 2s + h][n = i], one f32
// load), B = the frames: lane (h, j) loads the dword of pixel 32 g + j (g = 0, 1) of its row and feeds byte c to output
// tile (g, c) — so one load of dz + two pixel dwords feed 8 MFMAs into 8 32 x 32 tiles (128 accumulator registers):
// [32 n] x [256 = (g, c, j)].  The block's 4 waves are added in order through LDS and the block writes one partial row
// (8192 floats, the weight layout [n][c][ky][kx], divided by 255 once); xpa_colsum_finalize sums the partials in f64.
constexpr int kWgBlocks = 512;

// X2 (even W, S, P and an 8-B aligned frame buffer: the Nature CNN's 84 / 4 / 2): lane j loads pixels 2j and 2j + 1 of
// its row (kernel row j / 4, columns 2 (j % 4), + 1) as one 8-B load and feeds tile (parity, c) with byte c of pixel
// 2j + parity — 2 load instructions per 8 MFMAs instead of 3 (r02: the dword form was address-unit bound).
// ACT >= 0: dz is the gradient at the block's OUTPUT (before the activation) and the block's activation backward +
// bias-gradient partials run here (K22 folded in: dz = dh act'(y) never goes to HBM); y = the forward's output.
template <bool X2, int ACT>
__global__ __launch_bounds__(256, 2) void conv1_u8_wgrad_kernel(const float *__restrict__ dz, const unsigned *__restrict__ x,
                                                                int64_t rows, int H, int W, int OH, int OW, int S,
                                                                int P, float *__restrict__ partial,
                                                                const float *__restrict__ y, float slope,
                                                                float *__restrict__ bias_partial) {
    __shared__ __attribute__((aligned(16))) float s_red[64 * 16 * 8];  // one wave's accumulators, lane-major
    float bsum = 0.f;
    const int t = threadIdx.x, lane = t & 63, h = lane >> 5, j = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    // this wave's row range (row pairs split evenly over every wave of the grid)
    const int64_t pairs = (rows + 1) / 2, nw = (int64_t)gridDim.x * 4, gw = (int64_t)blockIdx.x * 4 + wave;
    const int64_t p0 = pairs * gw / nw, p1 = pairs * (gw + 1) / nw;
    f32x16 acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[q][r] = 0.f;
    // this lane's row 2 p + h, tracked incrementally as (b, oy, ox); groups of 4 row pairs, the next group's loads
    // (4 dz values + 8 pixel dwords per lane) requested before the current group's 32 MFMAs
    int64_t m = 2 * p0 + h;
    const int64_t ohw = (int64_t)OH * OW;
    int64_t b = m / ohw;
    int rem = (int)(m - b * ohw);
    int oy = rem / OW, ox = rem - (rem / OW) * OW;
    // dword form: pixel 32 g + j (ky = 4 g + j / 8, kx = j % 8); X2: pixels 2j + g (ky = j / 4, kx = 2 (j % 4) + g)
    const int ky0 = X2 ? (j >> 2) : (j >> 3), kx = X2 ? 2 * (j & 3) : (j & 7);
    constexpr int U = 4;
    float an[U];
    unsigned dn[U][2];
    auto load_group = [&](int64_t pp) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool mv = pp + u < p1 && m < rows;
            an[u] = dz[(mv ? m : 0) * 32 + j];
            if (ACT >= 0) an[u] = act_grad<ACT>(an[u], y[(mv ? m : 0) * 32 + j], slope);
            if (X2) {  // both pixels in or both out: ix even, W even
                const int iy = oy * S - P + ky0, ix = ox * S - P + kx;
                const bool inb = mv && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
                const uint2 v = *reinterpret_cast<const uint2 *>(x + ((mv ? b : 0) * H + (inb ? iy : 0)) * W +
                                                                 (inb ? ix : 0));
                dn[u][0] = inb ? v.x : 0u;
                dn[u][1] = inb ? v.y : 0u;
            } else {
#pragma unroll
                for (int g = 0; g < 2; ++g) {
                    const int iy = oy * S - P + 4 * g + ky0, ix = ox * S - P + kx;
                    const bool inb = mv && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
                    const unsigned v = x[((mv ? b : 0) * H + (inb ? iy : 0)) * W + (inb ? ix : 0)];
                    dn[u][g] = inb ? v : 0u;
                }
            }
            if (!mv) an[u] = 0.f;
            m += 2;  // advance this lane's row by 2
            ox += 2;
            while (ox >= OW) {
                ox -= OW;
                if (++oy >= OH) {
                    oy = 0;
                    ++b;
                }
            }
        }
    };
    if (p0 < p1) load_group(p0);
    for (int64_t pp = p0; pp < p1; pp += U) {
        float a[U];
        unsigned d[U][2];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            a[u] = an[u];
            d[u][0] = dn[u][0];
            d[u][1] = dn[u][1];
        }
        if (pp + U < p1) load_group(pp + U);
        if (ACT >= 0) {
#pragma unroll
            for (int u = 0; u < U; ++u) bsum += a[u];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    acc[4 * g + c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], (float)((d[u][g] >> (8 * c)) & 0xffu),
                                                                          acc[4 * g + c], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
    if (ACT >= 0) {  // bias partial: lane (h, j)'s sums over its rows, both halves and the 4 waves in a fixed order
        __shared__ float s_b[4][64];
        s_b[wave][lane] = bsum;
        __syncthreads();
        if (t < 32) {
            float tb = 0.f;
            for (int w = 0; w < 4; ++w) tb += s_b[w][t] + s_b[w][t + 32];
            bias_partial[(int64_t)blockIdx.x * 32 + t] = tb;
        }
    }
    // waves 1..3 added into wave 0 in order
    for (int src = 1; src < 4; ++src) {
        __syncthreads();
        if (wave == src) {
#pragma unroll
            for (int q = 0; q < 8; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r) s_red[(q * 16 + r) * 64 + lane] = acc[q][r];
        }
        __syncthreads();
        if (wave == 0) {
#pragma unroll
            for (int q = 0; q < 8; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[q][r] += s_red[(q * 16 + r) * 64 + lane];
        }
    }
    if (wave != 0) return;
    // D of tile (g, c): row n = (r & 3) + 8 (r >> 2) + 4 h, column j = pixel 32 g + j (X2: 2 j + g) -> W[n][c][ky][kx]
    float *pr = partial + (int64_t)blockIdx.x * 8192;
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = (r & 3) + 8 * (r >> 2) + 4 * h;
                pr[(n * 4 + c) * 64 + (X2 ? 2 * j + g : 32 * g + j)] = acc[4 * g + c][r] / 255.0f;
            }
}

// ---- K26B: K26 on the bf16 matrix cores (r05) -------------------------------------------------------------------
// The same [32 n] x [256 taps] product over rows with the MFMA's k = 16 rows (v_mfma_f32_32x32x16_bf16): lane (h, j)
// owns rows 16 s + 8 h + u (u < 8) of step s — A = dz^T (dz[row][n = j], cut into its exact three-way bf16 split:
// 3 products), B = the frames (byte c of the pixel dwords of those 8 rows, exact in bf16) — so a step is 8 tiles x 3
// MFMAs against K26's 8 row pairs x 8 tiles of v_mfma_f32_32x32x2_f32 (768 against 4096 MFMA cycles per 16 rows).
// Each product is exact in f32; the sum over rows rounds in another fixed order than K26's.  The accumulator layout,
// the in-order wave reduction, the bias partials and the partial layout are K26's.
template <bool X2, int ACT>
__global__ __launch_bounds__(256, 2) void conv1_u8_wgrad_bf16_kernel(const float *__restrict__ dz,
                                                                     const unsigned *__restrict__ x, int64_t rows, int H,
                                                                     int W, int OH, int OW, int S, int P,
                                                                     float *__restrict__ partial,
                                                                     const float *__restrict__ y, float slope,
                                                                     float *__restrict__ bias_partial) {
    __shared__ __attribute__((aligned(16))) float s_red[64 * 16 * 8];
    float bsum = 0.f;
    const int t = threadIdx.x, lane = t & 63, h = lane >> 5, j = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int64_t steps = (rows + 15) / 16, nw = (int64_t)gridDim.x * 4, gw = (int64_t)blockIdx.x * 4 + wave;
    const int64_t s0 = steps * gw / nw, s1 = steps * (gw + 1) / nw;
    f32x16 acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[q][r] = 0.f;
    int64_t m = 16 * s0 + 8 * h;
    const int64_t ohw = (int64_t)OH * OW;
    const int64_t mc0 = m < rows ? m : 0;
    int64_t b = mc0 / ohw;
    int rem = (int)(mc0 - b * ohw);
    int oy = rem / OW, ox = rem - (rem / OW) * OW;
    const int ky0 = X2 ? (j >> 2) : (j >> 3), kx = X2 ? 2 * (j & 3) : (j & 7);
    auto advance = [&](int n) {
        m += n;
        ox += n;
        while (ox >= OW) {
            ox -= OW;
            if (++oy >= OH) {
                oy = 0;
                ++b;
            }
        }
    };
    // range-checked buffer loads (rows past the end and taps outside the frame read zeros; the entry guarantees
    // < 2^31 bytes per record), raw dz / y kept in the ring: no VALU op consumes a load before the next step's MFMAs
    const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(dz), 0,
                                                                        (int)(rows * 128), 0x00020000);
    const __amdgpu_buffer_rsrc_t ryy = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(ACT >= 0 ? y : dz), 0,
                                                                         (int)(rows * 128), 0x00020000);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned *>(x), 0, (int)(((rows - 1) / ohw + 1) * H * W * 4), 0x00020000);
    float an[8], yn[8];
    uint2 dn[8];
    auto load_step = [&]() {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const bool mv = m < rows;
            const int oz = mv ? (int)(m * 128) + 4 * j : INT32_MIN;
            an[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rz, oz, 0, 0));
            if (ACT >= 0) yn[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ryy, oz, 0, 0));
            const int xb = (int)(b * H * W * 4);
            if (X2) {
                const int iy = oy * S - P + ky0, ix = ox * S - P + kx;
                const bool inb = mv && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
                dn[u] = __builtin_bit_cast(
                    uint2, __builtin_amdgcn_raw_buffer_load_b64(rx, inb ? xb + (iy * W + ix) * 4 : INT32_MIN, 0, 0));
            } else {
#pragma unroll
                for (int g = 0; g < 2; ++g) {
                    const int iy = oy * S - P + 4 * g + ky0, ix = ox * S - P + kx;
                    const bool inb = mv && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
                    const unsigned v =
                        __builtin_amdgcn_raw_buffer_load_b32(rx, inb ? xb + (iy * W + ix) * 4 : INT32_MIN, 0, 0);
                    if (g) dn[u].y = v;
                    else dn[u].x = v;
                }
            }
            advance(1);
        }
        advance(8);  // the other half's 8 rows
    };
    if (s0 < s1) load_step();
    for (int64_t st = s0; st < s1; ++st) {
        float a[8];
        uint2 d[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            a[u] = ACT >= 0 ? act_grad<ACT>(an[u], yn[u], slope) : an[u];  // a row past the end: 0 act'(0) = 0
            d[u] = dn[u];
        }
        if (st + 1 < s1) load_step();
        if (ACT >= 0) {
#pragma unroll
            for (int u = 0; u < 8; ++u) bsum += a[u];
        }
        __builtin_amdgcn_sched_barrier(0);
        xpa_bf16x8 ah, am, al;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            __bf16 p, q, r;
            xpa_split3(a[u], p, q, r);
            ah[u] = p;
            am[u] = q;
            al[u] = r;
        }
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                u32x4v bb;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const unsigned d0 = g ? d[2 * q].y : d[2 * q].x, d1 = g ? d[2 * q + 1].y : d[2 * q + 1].x;
                    const unsigned f0 = __float_as_uint((float)((d0 >> (8 * c)) & 0xffu));
                    const unsigned f1 = __float_as_uint((float)((d1 >> (8 * c)) & 0xffu));
                    bb[q] = __builtin_amdgcn_perm(f1, f0, 0x07060302u);
                }
                const xpa_bf16x8 bv = __builtin_bit_cast(xpa_bf16x8, bb);
                f32x16 &ac = acc[4 * g + c];
                ac = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bv, ac, 0, 0, 0);
                ac = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bv, ac, 0, 0, 0);
                ac = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bv, ac, 0, 0, 0);
            }
        __builtin_amdgcn_sched_barrier(0);
    }
    if (ACT >= 0) {
        __shared__ float s_b[4][64];
        s_b[wave][lane] = bsum;
        __syncthreads();
        if (t < 32) {
            float tb = 0.f;
            for (int w = 0; w < 4; ++w) tb += s_b[w][t] + s_b[w][t + 32];
            bias_partial[(int64_t)blockIdx.x * 32 + t] = tb;
        }
    }
    for (int src = 1; src < 4; ++src) {
        __syncthreads();
        if (wave == src) {
#pragma unroll
            for (int q = 0; q < 8; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r) s_red[(q * 16 + r) * 64 + lane] = acc[q][r];
        }
        __syncthreads();
        if (wave == 0) {
#pragma unroll
            for (int q = 0; q < 8; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[q][r] += s_red[(q * 16 + r) * 64 + lane];
        }
    }
    if (wave != 0) return;
    float *pr = partial + (int64_t)blockIdx.x * 8192;
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = (r & 3) + 8 * (r >> 2) + 4 * h;
                pr[(n * 4 + c) * 64 + (X2 ? 2 * j + g : 32 * g + j)] = acc[4 * g + c][r] / 255.0f;
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
                                     int32_t *err, xpa_stream_t stream) {
    const int64_t rows = batch * hw;
    const int64_t G = xpa_act_bwd_bias_num_partials(rows, channels);
    if (G <= 0 || hw > (1 << 30) || !dout || !argmax || !h || !dz || !partials || act < 0 || act > 2)
        return (int)hipErrorInvalidValue;
    if (((uintptr_t)h | (uintptr_t)dz | (uintptr_t)partials) % 16) return (int)hipErrorInvalidValue;
    const size_t lds = 256 * sizeof(f4v);
    hipStream_t s = (hipStream_t)stream;
#define XPA_MPB(A_)                                                                                              \
    hipLaunchKernelGGL((maxpool_act_bwd_bias_kernel<A_>), dim3((unsigned)G), dim3(256), lds, s, dout, argmax, h, \
                       rows, (int)hw, (int)channels, slope, dz, partials, err)
    if (act == 0) XPA_MPB(0);
    else if (act == 1) XPA_MPB(1);
    else XPA_MPB(2);
#undef XPA_MPB
    return xpa_launch_status();
}

// r05: bit 0 = K25B (the conv1 forward on the bf16 matrix cores), bit 1 = K26B (its weight gradient likewise), bit 2 =
// K27B (the conv2 data gradient likewise); a cleared bit selects the fp32-MFMA form.  Returns the previous mask.
static int g_conv1_bf16 = 7;
XPA_API int xpa_conv1_form(int mask) {
    const int prev = g_conv1_bf16;
    if (mask >= 0) g_conv1_bf16 = mask;
    return prev;
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
    hipStream_t s = (hipStream_t)stream;
    const bool x2 = width % 2 == 0 && stride % 2 == 0 && pad % 2 == 0 && (uintptr_t)x % 8 == 0;
    if ((g_conv1_bf16 & 1) && batch * height * width * 4 < ((int64_t)1 << 31)) {  // K25B (one buffer record)
        const int64_t blocks = (rows + kC1BRows - 1) / kC1BRows;
        const dim3 grid((unsigned)(blocks < 512 ? blocks : 512)), block(512);
#define XPA_C1B(A_)                                                                                                  \
    if (x2)                                                                                                          \
        hipLaunchKernelGGL((conv1_u8_fwd_bf16_kernel<A_, true>), grid, block, 0, s, (const unsigned *)x, rows,        \
                           (int)height, (int)width, (int)OH, (int)OW, (int)stride, (int)pad, w, bias, slope, y);     \
    else                                                                                                             \
        hipLaunchKernelGGL((conv1_u8_fwd_bf16_kernel<A_, false>), grid, block, 0, s, (const unsigned *)x, rows,       \
                           (int)height, (int)width, (int)OH, (int)OW, (int)stride, (int)pad, w, bias, slope, y)
        if (act == 0) XPA_C1B(0);
        else if (act == 1) XPA_C1B(1);
        else XPA_C1B(2);
#undef XPA_C1B
        return xpa_launch_status();
    }
    const int64_t blocks = (rows + kC1Rows - 1) / kC1Rows;
    const dim3 grid((unsigned)(blocks < 1024 ? blocks : 1024)), block(256);
#define XPA_C1(A_)                                                                                                   \
    if (x2)                                                                                                          \
        hipLaunchKernelGGL((conv1_u8_fwd_kernel<A_, true>), grid, block, 0, s, (const unsigned *)x, rows,             \
                           (int)height, (int)width, (int)OH, (int)OW, (int)stride, (int)pad, w, bias, slope, y);     \
    else                                                                                                             \
        hipLaunchKernelGGL((conv1_u8_fwd_kernel<A_, false>), grid, block, 0, s, (const unsigned *)x, rows,            \
                           (int)height, (int)width, (int)OH, (int)OW, (int)stride, (int)pad, w, bias, slope, y)
    if (act == 0) XPA_C1(0);
    else if (act == 1) XPA_C1(1);
    else XPA_C1(2);
#undef XPA_C1
    return xpa_launch_status();
}

XPA_API int xpa_conv_dgrad_s2k(const float *dy, int64_t batch, int64_t out_h, int64_t out_w, int64_t out_channels,
                               const float *w, int64_t in_channels, int64_t kernel, int64_t stride, int64_t pad,
                               int64_t in_h, int64_t in_w, float *dx, xpa_stream_t stream) {
    if (batch <= 0 || out_channels != 64 || in_channels != 32 || stride < 1 || stride > 2 || kernel != 2 * stride ||
        pad < 0 || pad >= stride * 2 || in_h < 1 || in_w < 1 || !dy || !w || !dx || ((uintptr_t)dy % 16) ||
        out_h != (in_h + 2 * pad - kernel) / stride + 1 || out_w != (in_w + 2 * pad - kernel) / stride + 1 ||
        out_h < 1 || out_w < 1)
        return (int)hipErrorInvalidValue;
    DgradGeom g{};
    g.H = (int)in_h; g.W = (int)in_w; g.OH = (int)out_h; g.OW = (int)out_w; g.S = (int)stride; g.P = (int)pad;
    g.B = batch;
    for (int r = 0; r < 2; ++r) {
        const int s_ = (int)stride;
        const int y0 = (((r - (int)pad) % s_) + s_) % s_, x0 = y0;
        g.iy0[r] = y0; g.ix0[r] = x0;
        g.ny[r] = (r < s_ && y0 < g.H) ? (g.H - y0 + s_ - 1) / s_ : 0;
        g.nx[r] = (r < s_ && x0 < g.W) ? (g.W - x0 + s_ - 1) / s_ : 0;
    }
    int64_t acc = 0;
    for (int c = 0; c < 4; ++c) {
        const int64_t rows = batch * (int64_t)g.ny[c >> 1] * g.nx[c & 1];
        acc += (rows + kDgRows - 1) / kDgRows;
        g.tiles[c] = acc;
    }
    if (acc <= 0 || batch * out_h * out_w * 64 >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;  // int offsets
    const unsigned grid = (unsigned)(acc < kDgGrid ? acc : kDgGrid);
    if ((g_conv1_bf16 & 4) && batch * out_h * out_w * 256 < ((int64_t)1 << 31)) {  // K27B (one buffer record for dY)
        if (g_conv1_bf16 & 8) {  // probe: 3 blocks per CU (<= 168 VGPRs)
            const unsigned g3 = (unsigned)(acc < 768 ? acc : 768);
            hipLaunchKernelGGL(conv_dgrad_s2k_bf16_kernel<3>, dim3(g3), dim3(256), 0, (hipStream_t)stream, dy, w, g, dx);
        } else {
            hipLaunchKernelGGL(conv_dgrad_s2k_bf16_kernel<2>, dim3(grid), dim3(256), 0, (hipStream_t)stream, dy, w, g,
                               dx);
        }
    } else
        hipLaunchKernelGGL(conv_dgrad_s2k_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, dy, w, g, dx);
    return xpa_launch_status();
}

XPA_API int64_t xpa_conv1_u8_wgrad_num_partials(void) { return kWgBlocks; }

XPA_API int xpa_conv1_u8_wgrad_act(int act, const float *dz, const float *y, float slope, const uint8_t *x,
                                   int64_t batch, int64_t height, int64_t width, int64_t channels, int64_t kernel,
                                   int64_t stride, int64_t pad, int64_t out_channels, float *partial,
                                   float *bias_partial, xpa_stream_t stream) {
    if (batch <= 0 || channels != 4 || kernel != 8 || out_channels != 32 || stride < 1 || pad < 0 || !dz || !x ||
        !partial || ((uintptr_t)x % 4) || height + 2 * pad < kernel || width + 2 * pad < kernel || act < -1 ||
        act > 2 || (act >= 0 && (!y || !bias_partial)))
        return (int)hipErrorInvalidValue;
    const int64_t OH = (height + 2 * pad - kernel) / stride + 1, OW = (width + 2 * pad - kernel) / stride + 1;
    const bool x2 = width % 2 == 0 && stride % 2 == 0 && pad % 2 == 0 && (uintptr_t)x % 8 == 0;
    hipStream_t s = (hipStream_t)stream;
    const bool bf = (g_conv1_bf16 & 2) && batch * OH * OW * 128 < ((int64_t)1 << 31) &&
                    batch * height * width * 4 < ((int64_t)1 << 31);  // K26B (one buffer record per operand)
#define XPA_WG(X_, A_)                                                                                             \
    if (bf)                                                                                                        \
        hipLaunchKernelGGL((conv1_u8_wgrad_bf16_kernel<X_, A_>), dim3(kWgBlocks), dim3(256), 0, s, dz,             \
                           (const unsigned *)x, batch * OH * OW, (int)height, (int)width, (int)OH, (int)OW,         \
                           (int)stride, (int)pad, partial, y, slope, bias_partial);                                 \
    else                                                                                                           \
        hipLaunchKernelGGL((conv1_u8_wgrad_kernel<X_, A_>), dim3(kWgBlocks), dim3(256), 0, s, dz,                  \
                           (const unsigned *)x, batch * OH * OW, (int)height, (int)width, (int)OH, (int)OW,         \
                           (int)stride, (int)pad, partial, y, slope, bias_partial)
#define XPA_WG_A(X_)                \
    if (act < 0) XPA_WG(X_, -1);    \
    else if (act == 0) XPA_WG(X_, 0); \
    else if (act == 1) XPA_WG(X_, 1); \
    else XPA_WG(X_, 2);
    if (x2) { XPA_WG_A(true) }
    else { XPA_WG_A(false) }
#undef XPA_WG_A
#undef XPA_WG
    return xpa_launch_status();
}

XPA_API int xpa_conv1_u8_wgrad(const float *dz, const uint8_t *x, int64_t batch, int64_t height, int64_t width,
                               int64_t channels, int64_t kernel, int64_t stride, int64_t pad, int64_t out_channels,
                               float *partial, xpa_stream_t stream) {
    return xpa_conv1_u8_wgrad_act(-1, dz, nullptr, 0.f, x, batch, height, width, channels, kernel, stride, pad,
                                  out_channels, partial, nullptr, stream);
}
