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
//   straight into the weight-gradient layout).  Wave = COUTP x (CTW column tiles of 32 (tap, channel) columns); every
//   wave of a block streams the block's rows two at a time (the MFMA's k = the row pair: lane (h, i) loads dz[row 2p + h,
//   32 nt + i] and in[pixel(row 2p + h, tap_j), c_j] for its column j = i), four row pairs prefetched.  With act >= 0 the
//   operand is g * act'(y) (the block's own activation backward folded in: K22 is not run) and wave 0 also writes the
//   bias-gradient partials.
#include "xpa_common.h"

namespace {

typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kIgThreads = 512;
constexpr int kIgRows = 512;             // rows per block step (8 waves x 64)
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
    if (ACT == 1) return y > 0.f ? d : d * slope;
    if (ACT == 2) return d * (1.0f - y * y);
    return d;
}

struct IgArgs {
    const float *in;     // NHWC [B, IH, IW, CIN]
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
    for (int e = t; e < img; e += kIgThreads) {
        const int cc = e & 3, n = (e >> 2) % COUTP, q = ((e >> 2) / COUTP) % CQ, tap = e / (4 * COUTP * CQ);
        const int c = 4 * q + cc, ky = tap / a.K, kx = tap - (tap / a.K) * a.K;
        float v = 0.f;
        if (n < a.COUT && c < a.CIN)
            v = MODE == 0 ? a.w[((n * a.CIN + c) * a.K + ky) * a.K + kx] : a.w[((c * a.COUT + n) * a.K + ky) * a.K + kx];
        sB[e] = v;
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
    auto geometry = [&](int64_t blk, IgRow (&rr)[2]) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            const int64_t m = blk * kIgRows + wave * 64 + mt * 32 + i;
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
    auto load_chunk = [&](f4v (&v)[2][CJ], const IgRow (&rr)[2], int k) {
        const int tap = k / CPT, jb = (k - tap * CPT) * CJ;
        const int ky = tap / a.K, kx = tap - (tap / a.K) * a.K;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            bool valid;
            const int pix = ig_pixel<MODE>(a, rr[mt], ky, kx, valid);
            const float *p = a.in + (int64_t)pix * a.CIN;
#pragma unroll
            for (int j = 0; j < CJ; ++j) {
                const int q = 2 * (jb + j) + h;
                const bool qv = valid && 4 * q < a.CIN;
                const f4v d = *reinterpret_cast<const f4v *>(p + (qv ? 4 * q : 0));
                const f4v z = {0.f, 0.f, 0.f, 0.f};
                v[mt][j] = qv ? d : z;
            }
        }
    };
    if (g0 >= g1) return;
    IgRow cur[2], nxt[2];
    geometry(g0, cur);
    f4v va[2][CJ], vb[2][CJ];
    load_chunk(va, cur, 0);
    for (int64_t blk = g0; blk < g1; ++blk) {
        const bool more = blk + 1 < g1;
        f32x16 acc[2][NT];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
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
                    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt)
                            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(va[mt][j][cc], b4[nt][cc], acc[mt][nt],
                                                                             0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int j = 0; j < CJ; ++j) va[mt][j] = vb[mt][j];
        }
        // C/D map: row = (r & 3) + 8 (r >> 2) + 4 h of the m-tile, column n = 32 nt + i
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const int n = 32 * nt + i;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int64_t m = blk * kIgRows + wave * 64 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    if (m < a.rows && n < a.COUT) {
                        const int64_t o = m * a.COUT + n;
                        if (MODE == 0) {
                            a.out[o] = ig_act<ACT>(acc[mt][nt][r] + bn[nt], a.slope);
                        } else {
                            float v = acc[mt][nt][r];
                            if (ACT >= 0 && a.yprev) v = ig_grad<ACT>(v, a.yprev[o], a.slope);
                            a.out[o] = v;
                            bsum[nt] += v;
                        }
                    }
                }
            }
        if (more) {
            cur[0] = nxt[0];
            cur[1] = nxt[1];
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
constexpr int kWgGrid = 512;
constexpr int kWgMaxWaves = 8;

struct WgArgs {
    const float *g;      // NHWC [rows, COUT]: d loss / d output (after the activation when act < 0)
    const float *y;      // the block's forward output (act >= 0), NHWC like g
    const float *in;     // NHWC [B, IH, IW, CIN]: the block's input
    float *partial;      // [gridDim.x][COUT][CIN][K][K]
    float *bias_partial; // [gridDim.x][COUT] (nullable; act >= 0)
    int64_t rows;
    int IH, IW, CIN, OH, OW, COUT, K, S, P, ncols;  // ncols = K K CIN
    float slope;
};

template <int NTN, int CTW, int ACT>
__global__ __launch_bounds__(64 * kWgMaxWaves) void conv_wgrad_kernel(WgArgs a) {
    const int t = threadIdx.x, lane = t & 63, h = lane >> 5, i = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int64_t pairs = (a.rows + 1) / 2;
    const int64_t p0 = pairs * blockIdx.x / gridDim.x, p1 = pairs * (blockIdx.x + 1) / gridDim.x;
    // this lane's columns: (tap, channel) of column 32 ct + i of the wave's tiles
    int cky[CTW], ckx[CTW], cch[CTW];
    bool cok[CTW];
#pragma unroll
    for (int j = 0; j < CTW; ++j) {
        const int gc = (wave * CTW + j) * 32 + i;
        cok[j] = gc < a.ncols;
        const int gcc = cok[j] ? gc : 0;
        const int tap = gcc / a.CIN;
        cch[j] = gcc - tap * a.CIN;
        cky[j] = tap / a.K;
        ckx[j] = tap - cky[j] * a.K;
    }
    f32x16 acc[NTN][CTW];
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
        for (int j = 0; j < CTW; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[nt][j][r] = 0.f;
    float bsum[NTN];
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt) bsum[nt] = 0.f;
    // this lane's row 2 p + h, tracked as (b, oy, ox)
    int64_t m = 2 * p0 + h;
    const int64_t ohw = (int64_t)a.OH * a.OW;
    int64_t b = m / ohw;
    int rem = (int)(m - b * ohw);
    int oy = rem / a.OW, ox = rem - (rem / a.OW) * a.OW;
    constexpr int U = 4;
    float an[U][NTN], xn[U][CTW];
    auto load_group = [&](int64_t pp) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool mv = pp + u < p1 && m < a.rows;
            const int64_t mc = mv ? m : 0;
#pragma unroll
            for (int nt = 0; nt < NTN; ++nt) {
                const int n = 32 * nt + i;
                const bool ok = mv && n < a.COUT;
                const int64_t o = mc * a.COUT + (n < a.COUT ? n : 0);
                float v = a.g[o];
                if (ACT >= 0) v = ig_grad<ACT>(v, a.y[o], a.slope);
                an[u][nt] = ok ? v : 0.f;
            }
            const int pixb = (int)((mv ? b : 0) * a.IH);
#pragma unroll
            for (int j = 0; j < CTW; ++j) {
                const int iy = oy * a.S - a.P + cky[j], ix = ox * a.S - a.P + ckx[j];
                const bool inb = mv && cok[j] && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW;
                const float v = a.in[((int64_t)(pixb + (inb ? iy : 0)) * a.IW + (inb ? ix : 0)) * a.CIN + cch[j]];
                xn[u][j] = inb ? v : 0.f;
            }
            m += 2;
            ox += 2;
            while (ox >= a.OW) {
                ox -= a.OW;
                if (++oy >= a.OH) {
                    oy = 0;
                    ++b;
                }
            }
        }
    };
    if (p0 < p1) load_group(p0);
    for (int64_t pp = p0; pp < p1; pp += U) {
        float av[U][NTN], xv[U][CTW];
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int nt = 0; nt < NTN; ++nt) av[u][nt] = an[u][nt];
#pragma unroll
            for (int j = 0; j < CTW; ++j) xv[u][j] = xn[u][j];
        }
        if (pp + U < p1) load_group(pp + U);
        if (ACT >= 0 && wave == 0) {
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int nt = 0; nt < NTN; ++nt) bsum[nt] += av[u][nt];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
                for (int j = 0; j < CTW; ++j)
                    acc[nt][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u][nt], xv[u][j], acc[nt][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
    // D of tile (nt, j): row n = 32 nt + (r & 3) + 8 (r >> 2) + 4 h, column = this wave's column 32 ct + i -> the
    // weight layout [n][c][ky][kx]
    const int taps = a.K * a.K;
    float *pr = a.partial + (int64_t)blockIdx.x * a.COUT * a.ncols;
#pragma unroll
    for (int j = 0; j < CTW; ++j) {
        if (!cok[j]) continue;
        const int col = cch[j] * taps + cky[j] * a.K + ckx[j];
#pragma unroll
        for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = 32 * nt + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (n < a.COUT) pr[(int64_t)n * a.ncols + col] = acc[nt][j][r];
            }
    }
    if (ACT >= 0 && a.bias_partial && wave == 0) {
#pragma unroll
        for (int nt = 0; nt < NTN; ++nt) {
            const float s = bsum[nt] + __shfl_xor(bsum[nt], 32, 64);
            const int n = 32 * nt + i;
            if (h == 0 && n < a.COUT) a.bias_partial[(int64_t)blockIdx.x * a.COUT + n] = s;
        }
    }
}

template <int MODE, int ACT>
int ig_dispatch(const IgArgs &args, int cinp, int nt, hipStream_t s) {
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

XPA_API int xpa_conv_fwd(int act, const float *x, int64_t batch, int64_t in_h, int64_t in_w, int64_t in_c,
                         const float *w, const float *bias, int64_t out_c, int64_t kernel, int64_t stride, int64_t pad,
                         float slope, float *y, xpa_stream_t stream) {
    int cinp, nt;
    if (batch <= 0 || in_h <= 0 || in_w <= 0 || stride < 1 || pad < 0 || act < 0 || act > 2 || !x || !w || !y ||
        !ig_shape(in_c, out_c, kernel, cinp, nt) || ((uintptr_t)x % 16))
        return (int)hipErrorInvalidValue;
    const int64_t OH = (in_h + 2 * pad - kernel) / stride + 1, OW = (in_w + 2 * pad - kernel) / stride + 1;
    if (OH < 1 || OW < 1 || batch * in_h * in_w * in_c >= ((int64_t)1 << 31) || batch * OH * OW >= ((int64_t)1 << 31))
        return (int)hipErrorInvalidValue;
    IgArgs a{};
    a.in = x; a.w = w; a.bias = bias; a.out = y;
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
        batch * in_h * in_w * in_c >= ((int64_t)1 << 31) || batch * out_h * out_w * out_c >= ((int64_t)1 << 31))
        return (int)hipErrorInvalidValue;
    IgArgs a{};
    a.in = dy; a.w = w; a.yprev = act_prev >= 0 ? y_prev : nullptr; a.out = dx; a.bias_partial = bias_partial;
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

XPA_API int xpa_conv_wgrad(int act, const float *g, const float *y, float slope, const float *x, int64_t batch,
                           int64_t in_h, int64_t in_w, int64_t in_c, int64_t out_c, int64_t kernel, int64_t stride,
                           int64_t pad, float *partial, float *bias_partial, xpa_stream_t stream) {
    if (batch <= 0 || in_h <= 0 || in_w <= 0 || in_c < 1 || out_c < 1 || out_c > 64 || kernel < 1 || stride < 1 ||
        pad < 0 || act < -1 || act > 2 || !g || !x || !partial || (act >= 0 && !y))
        return (int)hipErrorInvalidValue;
    const int64_t OH = (in_h + 2 * pad - kernel) / stride + 1, OW = (in_w + 2 * pad - kernel) / stride + 1;
    const int64_t ncols = kernel * kernel * in_c;
    const int ntn = out_c <= 32 ? 1 : 2;
    // column tiles per wave: 3 when the tiles split evenly into <= 8 waves that way (conv3: 18 = 6 x 3), else 4
    const int64_t nct = (ncols + 31) / 32;
    const int ctw = (nct % 3 == 0 && nct / 3 <= kWgMaxWaves) ? 3 : 4;
    const int64_t waves = (nct + ctw - 1) / ctw;
    if (OH < 1 || OW < 1 || waves > kWgMaxWaves || batch * in_h * in_w * in_c >= ((int64_t)1 << 31) ||
        batch * OH * OW * out_c >= ((int64_t)1 << 31))
        return (int)hipErrorInvalidValue;
    WgArgs a{};
    a.g = g; a.y = y; a.in = x; a.partial = partial; a.bias_partial = act >= 0 ? bias_partial : nullptr;
    a.rows = batch * OH * OW;
    a.IH = (int)in_h; a.IW = (int)in_w; a.CIN = (int)in_c; a.OH = (int)OH; a.OW = (int)OW; a.COUT = (int)out_c;
    a.K = (int)kernel; a.S = (int)stride; a.P = (int)pad; a.ncols = (int)ncols; a.slope = slope;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid(kWgGrid), block((unsigned)(64 * waves));
#define XPA_WG(N_, C_, A_) hipLaunchKernelGGL((conv_wgrad_kernel<N_, C_, A_>), grid, block, 0, s, a)
#define XPA_WG_A(N_, C_)                 \
    if (act < 0) XPA_WG(N_, C_, -1);      \
    else if (act == 0) XPA_WG(N_, C_, 0); \
    else if (act == 1) XPA_WG(N_, C_, 1); \
    else XPA_WG(N_, C_, 2);
    if (ntn == 1) {
        if (ctw == 3) { XPA_WG_A(1, 3) } else { XPA_WG_A(1, 4) }
    } else {
        if (ctw == 3) { XPA_WG_A(2, 3) } else { XPA_WG_A(2, 4) }
    }
#undef XPA_WG_A
#undef XPA_WG
    return xpa_launch_status();
}
