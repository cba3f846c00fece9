// K28 / K29 — generic NHWC convolutions of the CNN trunks (AC_CNN_Atari C3, Basic_CNN C5) as implicit GEMMs on the
// fp32 matrix cores (v_mfma_f32_32x32x2_f32: exact f32 fma chains), replacing every MIOpen call of the explicit CNN
// path (fused_cnn.py): the forward of the later conv blocks, their weight gradients and the stride-1 data gradient.
//
// Reference: cnn_block xuance/torch/utils/layers.py:27-57 (Conv2d(k, s, padding (k - s) // 2) + ReLU), AC_CNN_Atari /
// Basic_CNN xuance/torch/representations/cnn.py:5-93, and loss.backward() through them (a2c_learner.py:31-33,
// perdqn_learner.py:37-40).
//
// K28 xpa_conv_fwd / xpa_conv_dgrad: out[m, n] = sum_{tap, c} in[pixel(m, tap), c] W'[n, c, tap] over the output pixels
//   m = (b, oy, ox).  Forward: pixel = (oy S - P + ky, ox S - P + kx), W' = W, + bias + activation in the epilogue.
//   Data gradient (dY -> dX): pixel = ((oy + P - ky) / S, (ox + P - kx) / S) where divisible and inside the map (0
//   otherwise: for S = 2 three taps in four are masked — the generic form; the production stride-2 conv keeps K27),
//   W'[n = ci, c = co, tap] = W[co, ci, tap]; the epilogue can apply the PREVIOUS block's activation backward
//   (dz = dX * act'(y_prev), K22 folded in) and write that block's bias-gradient partials.
//   Block = 8 waves (512 threads), one per CU (the weight image takes up to 160 KiB of LDS): the whole W' staged once
//   as [tap][channel quad q][n][4] (one ds_read_b128 gives a lane the 4 channels of quad q for output n), then
//   persistent over contiguous ranges of 512-row blocks.  Wave = 64 rows (two 32-row m-tiles) x COUTP (one or two
//   32-column n-tiles); lane (h, i) owns row i of each m-tile and the channel quads 2j + h: a chunk (one tap, up to 4
//   quad pairs = 32 channels) is one 16-B load per (m-tile, quad pair) from a clamped address (the zero padding by
//   select), fed as 4 MFMAs' k = h against the matching weight quads; chunk k + 1 is requested before chunk k's MFMAs
//   (a register ring that runs on across row blocks).
// K29 xpa_conv_wgrad: dW[n, c, tap] = sum_m dz[m, n] in[pixel(m, tap), c] (the forward's pixel map): a long-K GEMM
//   over the rows, split over the grid (one partial [COUT, CIN, K, K] per block, summed in f64 by xpa_colsum_finalize
//   straight into the weight-gradient layout).  Wave = COUT x (TC column tiles of 16 (tap, channel) columns); every
//   wave of a block streams the block's rows four at a time (v_mfma_f32_16x16x4_f32, the MFMA's k = 4 rows: lane (kk, i)
//   loads dz[row 4q + kk, 16 nt + i] and in[pixel(row 4q + kk, tap_j), c_j] for its column j = i), two quads prefetched.
//   With act >= 0 the operand is g * act'(y) (the block's own activation backward folded in: K22 is not run) and wave 0
//   also writes the bias-gradient partials.
#include "xpa_common.h"
#include "s3_split.h"

namespace {

typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kIgThreads = 1024;         // 16 waves: 4 per SIMD (load latency hidden by the other waves)
constexpr int kIgMT = 1;                 // 32-row m-tiles per wave
constexpr int kIgRows = kIgThreads / 64 * 32 * kIgMT;  // rows per block step
constexpr int kIgLdsFloats = 40960;      // 160 KiB: the whole weight image
constexpr int kIgGrid = 256;             // one block per CU

template <int ACT>
__device__ __forceinline__ float ig_act(float z, float slope) {
    if (ACT == 1) return z > 0.f ? z : z * slope;
    if (ACT == 2) return tanhf(z);
    return z;
}

template <int ACT>
__device__ __forceinline__ float ig_grad(float d, float y, float slope) {  // d act / d z from the OUTPUT y
#pragma clang fp contract(off)  // as conv.hip's act_grad (K22): the same value whichever kernel forms it
    if (ACT == 1) return y > 0.f ? d : d * slope;
    if (ACT == 2) return d * (1.0f - y * y);
    return d;
}

struct IgArgs {
    const float *in;     // NHWC [B, IH, IW, CIN]
    int64_t in_bytes;    // < 2^31: the loads use 32-bit buffer offsets
    const float *w;      // torch layout: forward [COUT][CIN][K][K]; dgrad [CIN][COUT][K][K] (= the forward weight)
    const float *bias;   // forward: [COUT] (nullable)
    const float *yprev;  // dgrad: the previous block's output, NHWC like out (nullable: no activation backward)
    float *out;          // NHWC [B, OH, OW, COUT]
    float *bias_partial; // dgrad: [gridDim.x][COUT] (nullable)
    int64_t rows;        // B * OH * OW
    int64_t nblk;        // ceil(rows / kIgRows)
    int IH, IW, CIN, OH, OW, COUT, K, S, P;
    float slope;
};

// geometry of a lane's row in one m-tile (clamped past the end: every load address stays in bounds)
struct IgRow {
    int base;   // b * IH * IW (pixel index of the image)
    int oy, ox;
    bool ok;
};

template <int MODE>
__device__ __forceinline__ int ig_pixel(const IgArgs &a, const IgRow &r, int ky, int kx, bool &valid) {
    int iy, ix;
    if (MODE == 0) {
        iy = r.oy * a.S - a.P + ky;
        ix = r.ox * a.S - a.P + kx;
        valid = r.ok && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW;
    } else {
        const int ty = r.oy + a.P - ky, tx = r.ox + a.P - kx;
        iy = ty / a.S;
        ix = tx / a.S;
        valid = r.ok && ty >= 0 && tx >= 0 && iy * a.S == ty && ix * a.S == tx && iy < a.IH && ix < a.IW;
    }
    return valid ? r.base + iy * a.IW + ix : 0;
}

template <int CINP, int NT, int MODE, int ACT>
__global__ __launch_bounds__(kIgThreads, 1) void conv_igemm_kernel(IgArgs a) {
    constexpr int CQ = CINP / 4;                 // channel quads per tap
    constexpr int QPT = CINP / 8;                // quad pairs per tap
    constexpr int CJ = QPT < 4 ? QPT : 4;        // quad pairs per chunk
    constexpr int CPT = QPT / CJ;                // chunks per tap
    constexpr int COUTP = 32 * NT;
    __shared__ __attribute__((aligned(16))) float sB[kIgLdsFloats];
    const int t = threadIdx.x, lane = t & 63, h = lane >> 5, i = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int taps = a.K * a.K;
    const int nch = taps * CPT;
    // ---- the weight image [tap][q][n][4] ----
    const int img = taps * CQ * COUTP * 4;
    // 8 loads in flight per thread (a load-wait-store loop here costs ~36 serial L2 latencies per block)
    for (int e0 = t; e0 < img; e0 += 8 * kIgThreads) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int e = e0 + u * kIgThreads;
            const int cc = e & 3, n = (e >> 2) % COUTP, q = ((e >> 2) / COUTP) % CQ, tap = e / (4 * COUTP * CQ);
            const int c = 4 * q + cc, ky = tap / a.K, kx = tap - (tap / a.K) * a.K;
            v[u] = 0.f;
            if (e < img && n < a.COUT && c < a.CIN)
                v[u] = MODE == 0 ? a.w[((n * a.CIN + c) * a.K + ky) * a.K + kx]
                                 : a.w[((c * a.COUT + n) * a.K + ky) * a.K + kx];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (e0 + u * kIgThreads < img) sB[e0 + u * kIgThreads] = v[u];
    }
    __syncthreads();
    const int64_t g0 = a.nblk * blockIdx.x / gridDim.x, g1 = a.nblk * (blockIdx.x + 1) / gridDim.x;
    float bn[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bn[nt] = 0.f;
    if (MODE == 0 && a.bias) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) bn[nt] = 32 * nt + i < a.COUT ? a.bias[32 * nt + i] : 0.f;
    }
    float bsum[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bsum[nt] = 0.f;
    const int64_t ohw = (int64_t)a.OH * a.OW;
    auto geometry = [&](int64_t blk, IgRow (&rr)[kIgMT]) {
#pragma unroll
        for (int mt = 0; mt < kIgMT; ++mt) {
            const int64_t m = blk * kIgRows + wave * 32 * kIgMT + mt * 32 + i;
            const bool ok = m < a.rows;
            const int64_t mc = ok ? m : 0;
            const int64_t b = mc / ohw;
            const int rem = (int)(mc - b * ohw);
            rr[mt].oy = rem / a.OW;
            rr[mt].ox = rem - rr[mt].oy * a.OW;
            rr[mt].base = (int)(b * a.IH * a.IW);
            rr[mt].ok = ok;
        }
    };
    // A operand through a range-checked buffer descriptor: a padding tap or a ragged row gets an offset past the
    // record count and the hardware returns zeros, so no select sits between the load and its use and the wait for
    // chunk k + 1 lands after chunk k's MFMAs (a select right after the load would expose the whole load latency)
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(a.in), 0, (int)a.in_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, (int)(a.rows * a.COUT * 4),
                                                                          0x00020000);
    auto load_chunk = [&](f4v (&v)[kIgMT][CJ], const IgRow (&rr)[kIgMT], int k) {
        const int tap = k / CPT, jb = (k - tap * CPT) * CJ;
        const int ky = tap / a.K, kx = tap - (tap / a.K) * a.K;
#pragma unroll
        for (int mt = 0; mt < kIgMT; ++mt) {
            bool valid;
            const int pix = ig_pixel<MODE>(a, rr[mt], ky, kx, valid);
            const int off = valid ? pix * a.CIN * 4 : INT32_MIN;
#pragma unroll
            for (int j = 0; j < CJ; ++j) {
                const int q = 2 * (jb + j) + h;
                const int o = 4 * q < a.CIN ? off + 16 * q : INT32_MIN;
                v[mt][j] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rsrc, o, 0, 0));
            }
        }
    };
    if (g0 >= g1) return;
    IgRow cur[kIgMT], nxt[kIgMT];
    geometry(g0, cur);
    f4v va[kIgMT][CJ], vb[kIgMT][CJ];
    load_chunk(va, cur, 0);
    // The first chunk is waited for here, before the loop: with its loads still pending at the loop header the
    // compiler's wait for them (merged with the back edge) becomes vmcnt(0) at the first MFMA of EVERY chunk, which
    // drains the prefetch of chunk k + 1 too and exposes its whole latency.  Inside the loop the only wait is then at
    // the va <- vb copy after chunk k's MFMAs.
#pragma unroll
    for (int mt = 0; mt < kIgMT; ++mt)
#pragma unroll
        for (int j = 0; j < CJ; ++j) asm volatile("" ::"v"(va[mt][j]));
    for (int64_t blk = g0; blk < g1; ++blk) {
        const bool more = blk + 1 < g1;
        f32x16 acc[kIgMT][NT];
#pragma unroll
        for (int mt = 0; mt < kIgMT; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.f;
#pragma unroll 1
        for (int k = 0; k < nch; ++k) {
            // chunk k + 1 (or the next row block's chunk 0) requested before chunk k's MFMAs
            if (k + 1 < nch) {
                load_chunk(vb, cur, k + 1);
            } else if (more) {
                geometry(blk + 1, nxt);
                load_chunk(vb, nxt, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            const int tap = k / CPT, jb = (k - tap * CPT) * CJ;
#pragma unroll
            for (int j = 0; j < CJ; ++j) {
                const int q = 2 * (jb + j) + h;
                f4v b4[NT];
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    b4[nt] = *reinterpret_cast<const f4v *>(sB + ((tap * CQ + q) * COUTP + 32 * nt + i) * 4);
#pragma unroll
                for (int cc = 0; cc < 4; ++cc)
#pragma unroll
                    for (int mt = 0; mt < kIgMT; ++mt)
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt)
                            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(va[mt][j][cc], b4[nt][cc], acc[mt][nt],
                                                                             0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int mt = 0; mt < kIgMT; ++mt)
#pragma unroll
                for (int j = 0; j < CJ; ++j) {
                    va[mt][j] = vb[mt][j];
                    asm volatile("" ::"v"(va[mt][j]));
                }
        }
        // C/D map: row = (r & 3) + 8 (r >> 2) + 4 h of the m-tile, column n = 32 nt + i.  Buffer stores (and, for the
        // data gradient, loads of y_prev) with out-of-range offsets for ragged rows / padded columns: no branches, and
        // the 16 y_prev loads of an n-tile are all in flight before the first is used
#pragma unroll
        for (int mt = 0; mt < kIgMT; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const int n = 32 * nt + i;
                const int64_t m0 = blk * kIgRows + wave * 32 * kIgMT + mt * 32 + 4 * h;
                auto offset = [&](int r) -> int {
                    const int64_t m = m0 + (r & 3) + 8 * (r >> 2);
                    return m < a.rows && n < a.COUT ? (int)(m * a.COUT + n) * 4 : INT32_MIN;
                };
                if (MODE == 0) {
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        __builtin_amdgcn_raw_buffer_store_b32(
                            __builtin_bit_cast(unsigned, ig_act<ACT>(acc[mt][nt][r] + bn[nt], a.slope)), rout,
                            offset(r), 0, 0);
                } else {
#pragma unroll
                    for (int r0 = 0; r0 < 16; r0 += 8) {   // 8 y_prev loads in flight at a time
                        float yp[8];
                        if (ACT >= 0) {
#pragma unroll
                            for (int r = 0; r < 8; ++r) {
                                const int o = offset(r0 + r);
                                yp[r] = a.yprev[o != INT32_MIN ? o / 4 : 0];   // dropped rows: any valid address
                            }
                        }
#pragma unroll
                        for (int r = 0; r < 8; ++r) {
                            const int o = offset(r0 + r);
                            float v = acc[mt][nt][r0 + r];
                            if (ACT >= 0) v = ig_grad<ACT>(v, yp[r], a.slope);
                            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rout, o, 0, 0);
                            bsum[nt] += o != INT32_MIN ? v : 0.f;
                        }
                    }
                }
            }
        if (more) {
#pragma unroll
            for (int mt = 0; mt < kIgMT; ++mt) cur[mt] = nxt[mt];
        }
    }
    if (MODE == 1 && a.bias_partial) {
        // lane (h, i): column 32 nt + i over its rows; halves, then the 8 waves in a fixed order
        __syncthreads();   // every wave done with the weight image
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const float s = bsum[nt] + __shfl_xor(bsum[nt], 32, 64);
            if (h == 0) sB[wave * COUTP + 32 * nt + i] = s;
        }
        __syncthreads();
        if (t < a.COUT) {
            float s = 0.f;
            for (int w = 0; w < kIgThreads / 64; ++w) s += sB[w * COUTP + t];
            a.bias_partial[(int64_t)blockIdx.x * a.COUT + t] = s;
        }
    }
}

// ---- K29: weight gradient ------------------------------------------------------------------------------------------
// v_mfma_f32_16x16x4_f32 (k = 4 rows per instruction): lane (kk, i) supplies dz[row 4 s + kk][16 nt + i] (A) and
// in[pixel(row 4 s + kk, tap_j), c_j] (B, column j = 16 ct + i of the wave's tiles).  A wave holds TN x TC 16 x 16 tiles
// (TN = COUT / 16 row tiles, TC column tiles: 4 x 9 = 36 tiles = 144 accumulator registers at C3's conv3), so one load
// feeds TC (A) or TN (B) MFMAs: TN + TC 4-B loads per 4 rows and TN TC MFMAs (13 loads per 36 MFMAs at conv3).
constexpr int kWgGrid = 512;
constexpr int kWgMaxWaves = 16;

struct WgArgs {
    const float *g;      // NHWC [rows, COUT]: d loss / d output (after the activation when act < 0)
    const float *y;      // the block's forward output (act >= 0), NHWC like g
    const float *in;     // NHWC [B, IH, IW, CIN]
    int64_t in_bytes;    // < 2^31: the loads use 32-bit buffer offsets: the block's input
    float *partial;      // [gridDim.x][COUT][CIN][K][K]
    float *bias_partial; // [gridDim.x][COUT] (nullable; act >= 0)
    int64_t rows;
    int IH, IW, CIN, OH, OW, COUT, K, S, P, ncols;  // ncols = K K CIN
    float slope;
    // the LDS-slab form (conv_wgrad_lds_kernel): R output rows of one image per slab, nsl slabs per image; the x slab
    // [(R - 1) S + K][PW][CS] (zero-padded, CS = channel stride), then the dz slab [ceil4(R OW)][COUTS]
    int R, nsl, PW, CS, COUTS, xs_floats;
    int64_t nslabs;
};

template <int TN, int TC, int ACT>
__global__ __launch_bounds__(256, 2) void conv_wgrad_kernel(WgArgs a) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const int t = threadIdx.x, lane = t & 63, kk = lane >> 4, i = lane & 15;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int64_t quads = (a.rows + 3) / 4;
    const int64_t q0 = quads * blockIdx.x / gridDim.x, q1 = quads * (blockIdx.x + 1) / gridDim.x;
    // this lane's columns: (tap, channel) of column 16 ct + i of the wave's tiles
    int cky[TC], ckx[TC], cch[TC];
    bool cok[TC];
#pragma unroll
    for (int j = 0; j < TC; ++j) {
        const int gc = (wave * TC + j) * 16 + i;
        cok[j] = gc < a.ncols;
        const int gcc = cok[j] ? gc : 0;
        const int tap = gcc / a.CIN;
        cch[j] = gcc - tap * a.CIN;
        cky[j] = tap / a.K;
        ckx[j] = tap - cky[j] * a.K;
    }
    f4 acc[TN][TC];
#pragma unroll
    for (int nt = 0; nt < TN; ++nt)
#pragma unroll
        for (int j = 0; j < TC; ++j) acc[nt][j] = f4{0.f, 0.f, 0.f, 0.f};
    float bsum[TN];
#pragma unroll
    for (int nt = 0; nt < TN; ++nt) bsum[nt] = 0.f;
    // this lane's row 4 q + kk, tracked as (b, oy, ox)
    int64_t m = 4 * q0 + kk;
    const int64_t ohw = (int64_t)a.OH * a.OW;
    int64_t b = m / ohw;
    int rem = (int)(m - b * ohw);
    int oy = rem / a.OW, ox = rem - (rem / a.OW) * a.OW;
    constexpr int U = 2;
    float an[U][TN], xn[U][TC];
    // range-checked buffer loads (offset past the record count -> 0): no select between a load and its MFMA, so the
    // waits for group qq + U land after group qq's MFMAs; act'(0) x 0 = 0, so a dropped row contributes nothing
    const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.g), 0,
                                                                        (int)(a.rows * a.COUT * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(ACT >= 0 ? a.y : a.g), 0,
                                                                        (int)(a.rows * a.COUT * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.in), 0,
                                                                        (int)a.in_bytes, 0x00020000);
    float yn[U][TN];   // act >= 0: the block's output at the g rows, act' applied at use (not right after the load)
    auto load_group = [&](int64_t qq) {
        // the U rows' geometry first (the carry loop is control flow), then the loads as one straight-line run
        int go[U], gy[U], gx[U], gp[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool mv = qq + u < q1 && m < a.rows;
            go[u] = mv ? (int)m * a.COUT * 4 : INT32_MIN;
            gy[u] = mv ? oy * a.S - a.P : INT32_MIN / 2;   // an out-of-range row for every tap
            gx[u] = ox * a.S - a.P;
            gp[u] = (int)b * a.IH;
            m += 4;
            ox += 4;
            while (ox >= a.OW) {
                ox -= a.OW;
                if (++oy >= a.OH) {
                    oy = 0;
                    ++b;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int nt = 0; nt < TN; ++nt) {
                const int n = 16 * nt + i;
                const int o = n < a.COUT ? go[u] + 4 * n : INT32_MIN;
                an[u][nt] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, o, 0, 0));
                if (ACT >= 0) yn[u][nt] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ry, o, 0, 0));
            }
#pragma unroll
            for (int j = 0; j < TC; ++j) {
                const int iy = gy[u] + cky[j], ix = gx[u] + ckx[j];
                const bool inb = cok[j] && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW;
                const int o = inb ? (((gp[u] + iy) * a.IW + ix) * a.CIN + cch[j]) * 4 : INT32_MIN;
                xn[u][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, o, 0, 0));
            }
        }
    };
    if (q0 < q1) load_group(q0);
    for (int64_t qq = q0; qq < q1; qq += U) {
        float av[U][TN], xv[U][TC];
        // group qq's loads (issued one MFMA phase ago) are waited for HERE, before group qq + U's are issued: the
        // empty asm pins the wait to the copy (left to itself the compiler waits at the first MFMA with vmcnt(0),
        // draining the new group's loads too)
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int nt = 0; nt < TN; ++nt) {
                av[u][nt] = ACT >= 0 ? ig_grad<ACT>(an[u][nt], yn[u][nt], a.slope) : an[u][nt];
                asm volatile("" ::"v"(av[u][nt]));
            }
#pragma unroll
            for (int j = 0; j < TC; ++j) {
                xv[u][j] = xn[u][j];
                asm volatile("" ::"v"(xv[u][j]));
            }
        }
        if (qq + U < q1) load_group(qq + U);
        if (ACT >= 0 && wave == 0) {
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int nt = 0; nt < TN; ++nt) bsum[nt] += av[u][nt];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int nt = 0; nt < TN; ++nt)
#pragma unroll
                for (int j = 0; j < TC; ++j)
                    acc[nt][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][nt], xv[u][j], acc[nt][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
    // D of tile (nt, j): row n = 16 nt + 4 kk + r, column = this wave's column 16 ct + i -> weight layout [n][c][ky][kx]
    const int taps = a.K * a.K;
    float *pr = a.partial + (int64_t)blockIdx.x * a.COUT * a.ncols;
#pragma unroll
    for (int j = 0; j < TC; ++j) {
        if (!cok[j]) continue;
        const int col = cch[j] * taps + cky[j] * a.K + ckx[j];
#pragma unroll
        for (int nt = 0; nt < TN; ++nt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = 16 * nt + 4 * kk + r;
                if (n < a.COUT) pr[(int64_t)n * a.ncols + col] = acc[nt][j][r];
            }
    }
    if (ACT >= 0 && a.bias_partial && wave == 0) {
#pragma unroll
        for (int nt = 0; nt < TN; ++nt) {
            float s = bsum[nt];
            s += __shfl_xor(s, 16, 64);
            s += __shfl_xor(s, 32, 64);
            const int n = 16 * nt + i;
            if (kk == 0 && n < a.COUT) a.bias_partial[(int64_t)blockIdx.x * a.COUT + n] = s;
        }
    }
}

// K29 (LDS-slab form, the one every production shape takes): a block stages one slab — R output rows of one image —
// at a time: the input rows it reads, zero-padded, as xs[pr][pc][CS] (so no tap needs a bounds check), and its dz rows
// (act'(y) folded in, zero rows up to a multiple of 4) as dzs[p][COUTS].  CS and COUTS are padded so that the four
// 16-lane groups of a ds_read_b32 (four consecutive pixels) fall in different 16-bank quarters.  Then every operand is one
// ds_read_b32 at (pixel base + a per-lane column offset fixed for the whole kernel): per 4 pixels a wave issues TN + TC
// LDS reads and one add per B read, against TN x TC MFMAs, where the streaming form spent ~10 VALU per global load.
constexpr int kWsFloats = 19456;   // 76 KiB: two blocks per CU
bool g_wgrad_stream_only = false;

template <int TN, int TC, int ACT>
__global__ __launch_bounds__(256, 2) void conv_wgrad_lds_kernel(WgArgs a) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) float sm[kWsFloats];
    float *xs = sm;
    float *dzs = sm + a.xs_floats;
    const int t = threadIdx.x, lane = t & 63, kk = lane >> 4, i = lane & 15;
    const int nthr = blockDim.x;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    int coff[TC], cky[TC], ckx[TC], cch[TC];
    bool cok[TC];
#pragma unroll
    for (int j = 0; j < TC; ++j) {
        const int gc = (wave * TC + j) * 16 + i;
        cok[j] = gc < a.ncols;
        const int gcc = cok[j] ? gc : 0;
        const int tap = gcc / a.CIN;
        cch[j] = gcc - tap * a.CIN;
        cky[j] = tap / a.K;
        ckx[j] = tap - cky[j] * a.K;
        coff[j] = (cky[j] * a.PW + ckx[j]) * a.CS + cch[j];
    }
    f4 acc[TN][TC];
#pragma unroll
    for (int nt = 0; nt < TN; ++nt)
#pragma unroll
        for (int j = 0; j < TC; ++j) acc[nt][j] = f4{0.f, 0.f, 0.f, 0.f};
    float bsum[TN];
#pragma unroll
    for (int nt = 0; nt < TN; ++nt) bsum[nt] = 0.f;
    const int CQ = a.CIN / 4, NQ = a.COUT / 4;
    const int64_t ohw = (int64_t)a.OH * a.OW;
    for (int64_t z = blockIdx.x; z < a.nslabs; z += gridDim.x) {
        const int64_t b = z / a.nsl;
        const int oy0 = (int)(z - b * a.nsl) * a.R;
        const int rh = a.OH - oy0 < a.R ? a.OH - oy0 : a.R;
        const int np = rh * a.OW, np4 = (np + 3) & ~3;
        const int prh = (rh - 1) * a.S + a.K;
        __syncthreads();   // the previous slab's reads are done
        // staging: each thread's loads of a batch are all issued before its LDS writes (a load-wait-write loop costs one
        // memory latency per element, which at these slab sizes outweighs the slab's MFMAs)
        constexpr int XB = 6, DB = ACT >= 0 ? 2 : 4;
        const int nx = prh * a.PW * CQ;
        const int iy0 = oy0 * a.S - a.P;
        // (r03) every load unconditional from a clamped address, validity applied by select: under the bounds
        // branches hipcc waited vmcnt(0) at the joins — two or three serial round trips per batch instead of one
        for (int e0 = t; e0 < nx; e0 += XB * nthr) {
            f4 v[XB];
            bool ok[XB];
#pragma unroll
            for (int u = 0; u < XB; ++u) {
                const int e = e0 + u * nthr;
                const int c4 = e % CQ, pp = e / CQ, pc = pp % a.PW, pr = pp / a.PW;
                const int iy = iy0 + pr, ix = pc - a.P;
                ok[u] = e < nx && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW;
                const int64_t off = ok[u] ? ((b * a.IH + iy) * a.IW + ix) * a.CIN + 4 * c4 : 0;
                v[u] = *reinterpret_cast<const f4 *>(a.in + off);
            }
#pragma unroll
            for (int u = 0; u < XB; ++u) {
                const int e = e0 + u * nthr;
                const f4 zero = {0.f, 0.f, 0.f, 0.f};
                if (e < nx) *reinterpret_cast<f4 *>(xs + (e / CQ) * a.CS + 4 * (e % CQ)) = ok[u] ? v[u] : zero;
            }
        }
        const int nd = np4 * NQ;
        const int64_t row0 = b * ohw + (int64_t)oy0 * a.OW;
        for (int e0 = t; e0 < nd; e0 += DB * nthr) {
            f4 v[DB], yy[DB];
            bool ok[DB];
#pragma unroll
            for (int u = 0; u < DB; ++u) {
                const int e = e0 + u * nthr;
                const int n4 = e % NQ, p = e / NQ;
                ok[u] = e < nd && p < np;
                const int64_t o = ok[u] ? (row0 + p) * a.COUT + 4 * n4 : 0;
                v[u] = *reinterpret_cast<const f4 *>(a.g + o);
                yy[u] = f4{0.f, 0.f, 0.f, 0.f};
                if (ACT >= 0) yy[u] = *reinterpret_cast<const f4 *>(a.y + o);
            }
#pragma unroll
            for (int u = 0; u < DB; ++u) {
                const int e = e0 + u * nthr;
                const f4 zero = {0.f, 0.f, 0.f, 0.f};
                if (!ok[u]) {
                    v[u] = zero;
                    yy[u] = zero;
                }
                f4 w = v[u];
                if (ACT >= 0) {
                    w.x = ig_grad<ACT>(w.x, yy[u].x, a.slope);
                    w.y = ig_grad<ACT>(w.y, yy[u].y, a.slope);
                    w.z = ig_grad<ACT>(w.z, yy[u].z, a.slope);
                    w.w = ig_grad<ACT>(w.w, yy[u].w, a.slope);
                }
                if (e < nd) *reinterpret_cast<f4 *>(dzs + (e / NQ) * a.COUTS + 4 * (e % NQ)) = w;
            }
        }
        __syncthreads();
        // lane (kk, i) takes pixel 4 s + kk of the slab: (row oyr, column ox), advanced by 4 pixels per step
        int oyr = kk / a.OW, ox = kk - (kk / a.OW) * a.OW;
        float an[TN], xn[TC];
        auto load_quad = [&](int s) {
            const int p = 4 * s + kk;
            const int base = p < np ? (oyr * a.S * a.PW + ox * a.S) * a.CS : 0;   // dz row p >= np is 0
#pragma unroll
            for (int nt = 0; nt < TN; ++nt) an[nt] = dzs[p * a.COUTS + 16 * nt + i];
#pragma unroll
            for (int j = 0; j < TC; ++j) xn[j] = xs[base + coff[j]];
            ox += 4;
            while (ox >= a.OW) {
                ox -= a.OW;
                ++oyr;
            }
        };
        const int nq = np4 / 4;
        load_quad(0);
        for (int s = 0; s < nq; ++s) {
            float av[TN], xv[TC];
#pragma unroll
            for (int nt = 0; nt < TN; ++nt) {
                av[nt] = an[nt];
                asm volatile("" ::"v"(av[nt]));
            }
#pragma unroll
            for (int j = 0; j < TC; ++j) {
                xv[j] = xn[j];
                asm volatile("" ::"v"(xv[j]));
            }
            if (s + 1 < nq) load_quad(s + 1);
            if (ACT >= 0 && wave == 0) {
#pragma unroll
                for (int nt = 0; nt < TN; ++nt) bsum[nt] += av[nt];
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int nt = 0; nt < TN; ++nt)
#pragma unroll
                for (int j = 0; j < TC; ++j)
                    acc[nt][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[nt], xv[j], acc[nt][j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    const int taps = a.K * a.K;
    float *pr = a.partial + (int64_t)blockIdx.x * a.COUT * a.ncols;
#pragma unroll
    for (int j = 0; j < TC; ++j) {
        if (!cok[j]) continue;
        const int col = cch[j] * taps + cky[j] * a.K + ckx[j];
#pragma unroll
        for (int nt = 0; nt < TN; ++nt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = 16 * nt + 4 * kk + r;
                if (n < a.COUT) pr[(int64_t)n * a.ncols + col] = acc[nt][j][r];
            }
    }
    if (ACT >= 0 && a.bias_partial && wave == 0) {
#pragma unroll
        for (int nt = 0; nt < TN; ++nt) {
            float sm4 = bsum[nt];
            sm4 += __shfl_xor(sm4, 16, 64);
            sm4 += __shfl_xor(sm4, 32, 64);
            const int n = 16 * nt + i;
            if (kk == 0 && n < a.COUT) a.bias_partial[(int64_t)blockIdx.x * a.COUT + n] = sm4;
        }
    }
}

// channel stride with (S x stride) mod 64 in {16, 48}: four consecutive pixels in four different 16-bank quarters
int ws_pad(int need, int step) {
    for (int c = need; c < need + 64; c += 4)
        if ((step * c) % 64 == 16 || (step * c) % 64 == 48) return c;
    return need;
}

// ---- K28B (r05): K28 on the bf16 matrix cores ----------------------------------------------------------------------
// The same implicit GEMM (forward and data gradient, the same pixel maps, epilogues and buffer-record zero fill) with
// both f32 operands cut into their exact three-way bf16 split (s3_split.h) and six v_mfma_f32_32x32x16_bf16 products per
// 16-k step instead of eight v_mfma_f32_32x32x2_f32 — 192 against 512 matrix-core cycles per 16 k and 32 x 32 tile (K28
// measured 0.85 MFMA-busy: matrix-core bound).  k order: step s = (tap s / (CIN / 16), channels 16 (s % (CIN / 16)) ..
// + 15); lane half h feeds channels + 8 h .. + 7 (two adjacent 16-B quads of its row's pixel).  The weight image stays
// f32 in LDS as [tap][channel octet][n][8] (the three planes would not fit: 221 KiB at C3's conv3); each wave splits
// its B fragments per step (shared by its MT row tiles) and its A fragments per row tile.  Block = 8 waves (2 per SIMD,
// up to 256 VGPRs), one per CU, wave = MT x 32 rows x COUTP.  CIN must be a multiple of 16 (no channel padding).
template <int CIN, int NT, int MODE, int ACT, int MT>
__global__ __launch_bounds__(512, 1) void conv_igemm_bf16_kernel(IgArgs a) {
    constexpr int C8 = CIN / 8;
    constexpr int SPT = CIN / 16;
    constexpr int COUTP = 32 * NT;
    constexpr int kRowsB = 8 * 32 * MT;
    __shared__ __attribute__((aligned(16))) float sB[kIgLdsFloats];
    const int t = threadIdx.x, lane = t & 63, h = lane >> 5, i = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int taps = a.K * a.K;
    const int nst = taps * SPT;
    // ---- the weight image [tap][c8][n][8] (f32) ----
    const int img = taps * CIN * COUTP;
    for (int e0 = t; e0 < img; e0 += 8 * 512) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int e = e0 + u * 512;
            const int cc = e & 7, n = (e >> 3) % COUTP, c8 = ((e >> 3) / COUTP) % C8, tap = e / (8 * COUTP * C8);
            const int c = 8 * c8 + cc, ky = tap / a.K, kx = tap - (tap / a.K) * a.K;
            v[u] = 0.f;
            if (e < img && n < a.COUT)
                v[u] = MODE == 0 ? a.w[((n * CIN + c) * a.K + ky) * a.K + kx]
                                 : a.w[((c * a.COUT + n) * a.K + ky) * a.K + kx];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (e0 + u * 512 < img) sB[e0 + u * 512] = v[u];
    }
    __syncthreads();
    const int64_t nb = (a.rows + kRowsB - 1) / kRowsB;
    const int64_t g0 = nb * blockIdx.x / gridDim.x, g1 = nb * (blockIdx.x + 1) / gridDim.x;
    float bn[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bn[nt] = 0.f;
    if (MODE == 0 && a.bias) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) bn[nt] = 32 * nt + i < a.COUT ? a.bias[32 * nt + i] : 0.f;
    }
    float bsum[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bsum[nt] = 0.f;
    const int64_t ohw = (int64_t)a.OH * a.OW;
    auto geometry = [&](int64_t blk, IgRow (&rr)[MT]) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const int64_t m = blk * kRowsB + wave * 32 * MT + mt * 32 + i;
            const bool ok = m < a.rows;
            const int64_t mc = ok ? m : 0;
            const int64_t b = mc / ohw;
            const int rem = (int)(mc - b * ohw);
            rr[mt].oy = rem / a.OW;
            rr[mt].ox = rem - rr[mt].oy * a.OW;
            rr[mt].base = (int)(b * a.IH * a.IW);
            rr[mt].ok = ok;
        }
    };
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(a.in), 0, (int)a.in_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, (int)(a.rows * a.COUT * 4),
                                                                          0x00020000);
    auto load_step = [&](f4v (&v)[MT][2], const IgRow (&rr)[MT], int s) {
        const int tap = s / SPT, j = s - tap * SPT;
        const int ky = tap / a.K, kx = tap - (tap / a.K) * a.K;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            bool valid;
            const int pix = ig_pixel<MODE>(a, rr[mt], ky, kx, valid);
            const int off = valid ? (pix * CIN + 16 * j + 8 * h) * 4 : INT32_MIN;
#pragma unroll
            for (int q = 0; q < 2; ++q)
                v[mt][q] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rsrc, valid ? off + 16 * q
                                                                                               : INT32_MIN, 0, 0));
        }
    };
    if (g0 >= g1) return;
    IgRow cur[MT], nxt[MT];
    geometry(g0, cur);
    f4v va[MT][2], vb[MT][2];
    load_step(va, cur, 0);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int q = 0; q < 2; ++q) asm volatile("" ::"v"(va[mt][q]));
    for (int64_t blk = g0; blk < g1; ++blk) {
        const bool more = blk + 1 < g1;
        f32x16 acc[MT][NT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.f;
#pragma unroll 1
        for (int s = 0; s < nst; ++s) {
            if (s + 1 < nst) {
                load_step(vb, cur, s + 1);
            } else if (more) {
                geometry(blk + 1, nxt);
                load_step(vb, nxt, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            const int tap = s / SPT, j = s - tap * SPT;
            xpa_bf16x8 bh[NT], bm[NT], bl[NT];
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const f4v *bp = reinterpret_cast<const f4v *>(sB + ((tap * C8 + 2 * j + h) * COUTP + 32 * nt + i) * 8);
                const f4v b0 = bp[0], b1 = bp[1];
                xpa_split8(float4{b0[0], b0[1], b0[2], b0[3]}, float4{b1[0], b1[1], b1[2], b1[3]}, bh[nt], bm[nt],
                           bl[nt]);
            }
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                xpa_bf16x8 ah, am, al;
                xpa_split8(float4{va[mt][0][0], va[mt][0][1], va[mt][0][2], va[mt][0][3]},
                           float4{va[mt][1][0], va[mt][1][1], va[mt][1][2], va[mt][1][3]}, ah, am, al);
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = xpa_mfma_s3(ah, am, al, bh[nt], bm[nt], bl[nt], acc[mt][nt]);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    va[mt][q] = vb[mt][q];
                    asm volatile("" ::"v"(va[mt][q]));
                }
        }
        // K28's epilogue per m-tile (C/D map: row = (r & 3) + 8 (r >> 2) + 4 h, column n = 32 nt + i)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const int n = 32 * nt + i;
                const int64_t m0 = blk * kRowsB + wave * 32 * MT + mt * 32 + 4 * h;
                auto offset = [&](int r) -> int {
                    const int64_t m = m0 + (r & 3) + 8 * (r >> 2);
                    return m < a.rows && n < a.COUT ? (int)(m * a.COUT + n) * 4 : INT32_MIN;
                };
                if (MODE == 0) {
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        __builtin_amdgcn_raw_buffer_store_b32(
                            __builtin_bit_cast(unsigned, ig_act<ACT>(acc[mt][nt][r] + bn[nt], a.slope)), rout,
                            offset(r), 0, 0);
                } else {
#pragma unroll
                    for (int r0 = 0; r0 < 16; r0 += 8) {
                        float yp[8];
                        if (ACT >= 0) {
#pragma unroll
                            for (int r = 0; r < 8; ++r) {
                                const int o = offset(r0 + r);
                                yp[r] = a.yprev[o != INT32_MIN ? o / 4 : 0];
                            }
                        }
#pragma unroll
                        for (int r = 0; r < 8; ++r) {
                            const int o = offset(r0 + r);
                            float v = acc[mt][nt][r0 + r];
                            if (ACT >= 0) v = ig_grad<ACT>(v, yp[r], a.slope);
                            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rout, o, 0, 0);
                            bsum[nt] += o != INT32_MIN ? v : 0.f;
                        }
                    }
                }
            }
        if (more) {
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) cur[mt] = nxt[mt];
        }
    }
    if (MODE == 1 && a.bias_partial) {
        __syncthreads();
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const float s = bsum[nt] + __shfl_xor(bsum[nt], 32, 64);
            if (h == 0) sB[wave * COUTP + 32 * nt + i] = s;
        }
        __syncthreads();
        if (t < a.COUT) {
            float s = 0.f;
            for (int w = 0; w < 8; ++w) s += sB[w * COUTP + t];
            a.bias_partial[(int64_t)blockIdx.x * a.COUT + t] = s;
        }
    }
}

// r05: bit 0 = K28B (the bf16 matrix-core form where CIN is a multiple of 16), bit 1 = its 3-tile waves.  Off by
// default: 17-23 % faster per launch, but the C3 update's total GPU time came out unchanged (the kernels after it ran
// ~6 % slower: profiles/r05/r05k28b/)
int g_ig_form = 0;

template <int MODE, int ACT>
int ig_dispatch(const IgArgs &args, int cinp, int nt, hipStream_t s) {
    if ((g_ig_form & 1) && args.CIN % 16 == 0 && args.CIN == cinp) {   // K28B
        // MT = 2: 512-row block steps, so the data gradient's bias partials are K28's xpa_conv_dgrad_num_partials rows
        const int mt = (g_ig_form & 2) && MODE == 0 ? 3 : 2;
        const int64_t nb = (args.rows + 8 * 32 * mt - 1) / (8 * 32 * mt);
        const unsigned g = (unsigned)(nb < kIgGrid ? nb : kIgGrid);
#define XPA_IGB(C_, N_, M_) hipLaunchKernelGGL((conv_igemm_bf16_kernel<C_, N_, MODE, ACT, M_>), dim3(g), dim3(512), 0, s, args)
#define XPA_IGB_M(C_, N_) if (mt == 3) XPA_IGB(C_, N_, 3); else XPA_IGB(C_, N_, 2)
        if (nt == 1) {
            if (cinp == 16) { XPA_IGB_M(16, 1); } else if (cinp == 32) { XPA_IGB_M(32, 1); } else { XPA_IGB_M(64, 1); }
        } else {
            if (cinp == 16) { XPA_IGB_M(16, 2); } else if (cinp == 32) { XPA_IGB_M(32, 2); } else { XPA_IGB_M(64, 2); }
        }
#undef XPA_IGB_M
#undef XPA_IGB
        return xpa_launch_status();
    }
    const unsigned grid = (unsigned)(args.nblk < kIgGrid ? args.nblk : kIgGrid);
#define XPA_IG(C_, N_) hipLaunchKernelGGL((conv_igemm_kernel<C_, N_, MODE, ACT>), dim3(grid), dim3(kIgThreads), 0, s, args)
    if (nt == 1) {
        switch (cinp) {
            case 8: XPA_IG(8, 1); break;
            case 16: XPA_IG(16, 1); break;
            case 32: XPA_IG(32, 1); break;
            case 64: XPA_IG(64, 1); break;
            default: return (int)hipErrorInvalidValue;
        }
    } else {
        switch (cinp) {
            case 8: XPA_IG(8, 2); break;
            case 16: XPA_IG(16, 2); break;
            case 32: XPA_IG(32, 2); break;
            case 64: XPA_IG(64, 2); break;
            default: return (int)hipErrorInvalidValue;
        }
    }
#undef XPA_IG
    return xpa_launch_status();
}

// CINP = CIN rounded up to 8, 16, 32 or 64; NT = COUT rounded up to 32 / 32; the weight image must fit the LDS
bool ig_shape(int64_t cin, int64_t cout, int64_t k, int &cinp, int &nt) {
    if (cin < 1 || cin > 64 || cout < 1 || cout > 64 || k < 1 || cin % 4) return false;
    cinp = cin <= 8 ? 8 : cin <= 16 ? 16 : cin <= 32 ? 32 : 64;
    nt = cout <= 32 ? 1 : 2;
    return k * k * cinp * 32 * nt <= kIgLdsFloats;
}

}  // namespace

XPA_API int xpa_conv_igemm_ok(int64_t in_channels, int64_t out_channels, int64_t kernel) {
    int cinp, nt;
    return ig_shape(in_channels, out_channels, kernel, cinp, nt) ? 1 : 0;
}

// r05: K28's arithmetic — bit 0: K28B (bf16 matrix cores, six split products; taken where the GEMM's input channels
// are a multiple of 16), bit 1: K28B with 3 row tiles per wave (A/B); 0 = the fp32-MFMA K28.  mask < 0 only reads.
XPA_API int xpa_conv_igemm_form(int mask) {
    const int prev = g_ig_form;
    if (mask >= 0) g_ig_form = mask;
    return prev;
}

XPA_API int xpa_conv_fwd(int act, const float *x, int64_t batch, int64_t in_h, int64_t in_w, int64_t in_c,
                         const float *w, const float *bias, int64_t out_c, int64_t kernel, int64_t stride, int64_t pad,
                         float slope, float *y, xpa_stream_t stream) {
    int cinp, nt;
    if (batch <= 0 || in_h <= 0 || in_w <= 0 || stride < 1 || pad < 0 || act < 0 || act > 2 || !x || !w || !y ||
        !ig_shape(in_c, out_c, kernel, cinp, nt) || ((uintptr_t)x % 16))
        return (int)hipErrorInvalidValue;
    const int64_t OH = (in_h + 2 * pad - kernel) / stride + 1, OW = (in_w + 2 * pad - kernel) / stride + 1;
    if (OH < 1 || OW < 1 || batch * in_h * in_w * in_c * 4 >= ((int64_t)1 << 31) || batch * OH * OW >= ((int64_t)1 << 31))
        return (int)hipErrorInvalidValue;
    IgArgs a{};
    a.in = x; a.in_bytes = batch * in_h * in_w * in_c * 4; a.w = w; a.bias = bias; a.out = y;
    a.rows = batch * OH * OW; a.nblk = (a.rows + kIgRows - 1) / kIgRows;
    a.IH = (int)in_h; a.IW = (int)in_w; a.CIN = (int)in_c; a.OH = (int)OH; a.OW = (int)OW; a.COUT = (int)out_c;
    a.K = (int)kernel; a.S = (int)stride; a.P = (int)pad; a.slope = slope;
    hipStream_t s = (hipStream_t)stream;
    if (act == 0) return ig_dispatch<0, 0>(a, cinp, nt, s);
    if (act == 1) return ig_dispatch<0, 1>(a, cinp, nt, s);
    return ig_dispatch<0, 2>(a, cinp, nt, s);
}

XPA_API int64_t xpa_conv_dgrad_num_partials(int64_t batch, int64_t in_h, int64_t in_w) {
    const int64_t nblk = (batch * in_h * in_w + kIgRows - 1) / kIgRows;
    return nblk < kIgGrid ? nblk : kIgGrid;
}

XPA_API int xpa_conv_dgrad(const float *dy, int64_t batch, int64_t out_h, int64_t out_w, int64_t out_c,
                           const float *w, int64_t in_c, int64_t kernel, int64_t stride, int64_t pad, int64_t in_h,
                           int64_t in_w, int act_prev, const float *y_prev, float slope, float *dx, float *bias_partial,
                           xpa_stream_t stream) {
    int cinp, nt;
    // the GEMM's "input" is dY (out_c channels), its output dX (in_c channels)
    if (batch <= 0 || stride < 1 || stride > 2 || pad < 0 || act_prev < -1 || act_prev > 2 || !dy || !w || !dx ||
        !ig_shape(out_c, in_c, kernel, cinp, nt) || ((uintptr_t)dy % 16) ||
        out_h != (in_h + 2 * pad - kernel) / stride + 1 || out_w != (in_w + 2 * pad - kernel) / stride + 1 ||
        out_h < 1 || out_w < 1 || (act_prev >= 0 && !y_prev) ||
        batch * in_h * in_w * in_c >= ((int64_t)1 << 31) || batch * out_h * out_w * out_c * 4 >= ((int64_t)1 << 31))
        return (int)hipErrorInvalidValue;
    IgArgs a{};
    a.in = dy; a.in_bytes = batch * out_h * out_w * out_c * 4; a.w = w;
    a.yprev = act_prev >= 0 ? y_prev : nullptr; a.out = dx; a.bias_partial = bias_partial;
    a.rows = batch * in_h * in_w; a.nblk = (a.rows + kIgRows - 1) / kIgRows;
    a.IH = (int)out_h; a.IW = (int)out_w; a.CIN = (int)out_c; a.OH = (int)in_h; a.OW = (int)in_w; a.COUT = (int)in_c;
    a.K = (int)kernel; a.S = (int)stride; a.P = (int)pad; a.slope = slope;
    hipStream_t s = (hipStream_t)stream;
    if (act_prev < 0) return ig_dispatch<1, -1>(a, cinp, nt, s);
    if (act_prev == 0) return ig_dispatch<1, 0>(a, cinp, nt, s);
    if (act_prev == 1) return ig_dispatch<1, 1>(a, cinp, nt, s);
    return ig_dispatch<1, 2>(a, cinp, nt, s);
}

XPA_API int64_t xpa_conv_wgrad_num_partials(void) { return kWgGrid; }

// diagnostics / tests: 1 = always take the streaming K29 form (no LDS slabs)
XPA_API void xpa_conv_wgrad_force_stream(int on) { g_wgrad_stream_only = on != 0; }

XPA_API int xpa_conv_wgrad(int act, const float *g, const float *y, float slope, const float *x, int64_t batch,
                           int64_t in_h, int64_t in_w, int64_t in_c, int64_t out_c, int64_t kernel, int64_t stride,
                           int64_t pad, float *partial, float *bias_partial, xpa_stream_t stream) {
    if (batch <= 0 || in_h <= 0 || in_w <= 0 || in_c < 1 || out_c < 1 || out_c > 64 || kernel < 1 || stride < 1 ||
        pad < 0 || act < -1 || act > 2 || !g || !x || !partial || (act >= 0 && !y))
        return (int)hipErrorInvalidValue;
    const int64_t OH = (in_h + 2 * pad - kernel) / stride + 1, OW = (in_w + 2 * pad - kernel) / stride + 1;
    const int64_t ncols = kernel * kernel * in_c;
    const int tn = out_c <= 16 ? 1 : out_c <= 32 ? 2 : 4;
    // 16-column tiles over 4 waves (more waves only past 4 x 9 tiles): TC = ceil(tiles / 4), rounded to 2 / 4 / 8 / 9
    const int64_t nct = (ncols + 15) / 16;
    int tc = (int)((nct + 3) / 4);
    tc = tc <= 2 ? 2 : tc <= 4 ? 4 : tc <= 8 ? 8 : 9;
    const int64_t waves = (nct + tc - 1) / tc;
    if (OH < 1 || OW < 1 || waves > 4 || batch * in_h * in_w * in_c * 4 >= ((int64_t)1 << 31) ||
        batch * OH * OW * out_c * 4 >= ((int64_t)1 << 31))
        return (int)hipErrorInvalidValue;
    WgArgs a{};
    a.g = g; a.y = y; a.in = x; a.in_bytes = batch * in_h * in_w * in_c * 4;
    a.partial = partial; a.bias_partial = act >= 0 ? bias_partial : nullptr;
    a.rows = batch * OH * OW;
    a.IH = (int)in_h; a.IW = (int)in_w; a.CIN = (int)in_c; a.OH = (int)OH; a.OW = (int)OW; a.COUT = (int)out_c;
    a.K = (int)kernel; a.S = (int)stride; a.P = (int)pad; a.ncols = (int)ncols; a.slope = slope;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid(kWgGrid), block((unsigned)(64 * waves));
    // the LDS-slab form when a slab of at least one output row fits (and the f4 staging applies)
    bool slab = !g_wgrad_stream_only && in_c % 4 == 0 && out_c % 4 == 0 && (uintptr_t)x % 16 == 0 &&
                (uintptr_t)g % 16 == 0 && (act < 0 || (uintptr_t)y % 16 == 0);
    if (slab) {
        a.PW = (int)((OW - 1) * stride + kernel);
        a.CS = ws_pad((int)in_c, (int)stride);
        a.COUTS = ws_pad(16 * tn, 1);
        auto floats = [&](int64_t r) {
            const int64_t xs = (((r - 1) * stride + kernel) * a.PW * a.CS + 3) & ~(int64_t)3;
            return xs + ((r * OW + 3) & ~(int64_t)3) * a.COUTS;
        };
        int64_t r = OH;
        while (r >= 1 && floats(r) > kWsFloats) --r;
        slab = r >= 1;
        if (slab) {
            const int64_t nsl = (OH + r - 1) / r;
            a.R = (int)((OH + nsl - 1) / nsl);
            a.nsl = (int)nsl;
            a.nslabs = batch * nsl;
            a.xs_floats = (int)(((a.R - 1) * stride + kernel) * a.PW * a.CS + 3) & ~3;
        }
    }
#define XPA_WG(N_, C_, A_)                                                                           \
    if (slab) hipLaunchKernelGGL((conv_wgrad_lds_kernel<N_, C_, A_>), grid, block, 0, s, a);       \
    else hipLaunchKernelGGL((conv_wgrad_kernel<N_, C_, A_>), grid, block, 0, s, a)
#define XPA_WG_A(N_, C_)                 \
    if (act < 0) XPA_WG(N_, C_, -1);      \
    else if (act == 0) XPA_WG(N_, C_, 0); \
    else if (act == 1) XPA_WG(N_, C_, 1); \
    else XPA_WG(N_, C_, 2);
#define XPA_WG_C(N_)                                  \
    if (tc == 2) { XPA_WG_A(N_, 2) }                  \
    else if (tc == 4) { XPA_WG_A(N_, 4) }             \
    else if (tc == 8) { XPA_WG_A(N_, 8) }             \
    else { XPA_WG_A(N_, 9) }
    if (tn == 1) { XPA_WG_C(1) }
    else if (tn == 2) { XPA_WG_C(2) }
    else { XPA_WG_C(4) }
#undef XPA_WG_C
#undef XPA_WG_A
#undef XPA_WG
    return xpa_launch_status();
}
