// K40 — the update's f32 GEMMs on the bf16 matrix cores by a three-way split (gfx950).
//
// gfx950 has no xf32 MFMA: f32 operands run on v_mfma_f32_32x32x2_f32 at 64 FLOP/clk/SIMD (157.3 TF), 1/16 of the
// bf16 rate.  An f32 value splits EXACTLY into three bf16 values, x = hi + mid + lo (each the round-to-nearest bf16
// of what the previous ones leave; 3 x 8 significant bits = the f32 significand), so
//     a b = ah bh + (ah bm + am bh) + (am bm + ah bl + al bh) + [am bl + al bm + al bl]
// where the bracketed terms are below 2^-24 relative and are dropped.  Every kept product of two bf16 values is
// exact in f32 and v_mfma_f32_32x32x16_bf16 accumulates in f32, so a GEMM of the six products into one f32
// accumulator carries the f32 GEMM's error (one rounding of the running sum per 16-k group of each product, where the
// f32 MFMA rounds once per 2 k) at 6 x 16 / 16 = 6/16 of the f32 MFMA's cycles: 2.67x its arithmetic rate.
// tests/test_gpu_sgemm3.py holds it to the f32 MFMA GEMM's own error against an f64 product.
//
// Reference: the hidden layers' matmuls inside loss.backward() of PPOCLIP_Learner.update / A2C_Learner.update
// (ppoclip_learner.py:40-46, a2c_learner.py:33-39; torch f32 on the CPU): here the dX GEMM of the paired hidden layer,
// g = dz_pair [B, 512] . Wh_pair [512, 256] (fused_mlp.FusedActorCritic.loss_backward).
//
//   xpa_s3_split_b : B [K, N] (any strides) -> its three bf16 planes, laid out as the k loop's LDS image
//   xpa_s3_gemm    : C [M, 256] = A [M, K] (f32, row-major) . B (split), K % 16 == 0
//
// Mapping: 512 threads (8 waves), 256 rows per block, wave w owns rows [32 w, 32 w + 32) x all 256 columns (8
// accumulators of 32 x 32).  Per 16-k chunk a stage holds the A image (256 rows x 64 B of f32, K16's XOR-swizzled
// 16-B slots, DMA'd by each wave for its own rows) and the B image (3 planes x 256 columns x 32 B, one contiguous
// 24 KiB run of the split buffer); both arrive by LDS-DMA (global_load_lds_dwordx4) through a 3-stage ring with the
// counted vmcnt + one barrier per chunk of K16.  Each wave splits its A fragment (8 f32 per lane) in VALU and runs
// 8 x 6 MFMAs per chunk.  The k order inside a chunk is permuted (lane half h takes the quads h and h + 2 of its row,
// as K16) and the split kernel writes B's planes in that same order: any k order is exact as long as A and B agree.
#include "xpa_common.h"
#include "s3_split.h"

namespace {

typedef xpa_f32x16 f32x16;
typedef xpa_bf16x8 bf16x8;
typedef __attribute__((address_space(3))) char lds_char_t;

constexpr int kN = 256;                     // output columns (all of them per block)
constexpr int kKC = 16;                     // k per chunk (one bf16 MFMA k step)
constexpr int kBImg = 3 * kN * kKC * 2;     // bytes, 24 KiB
// K40 geometry: W waves of 32 rows (a block = 32 W rows x 256 columns), S ring stages (prefetch depth S - 1)
template <int W>
struct S3Geom {
    static constexpr int kRows = 32 * W;
    static constexpr int kAImg = kRows * kKC * 4;       // bytes: 16 KiB at W = 8
    static constexpr int kStage = kAImg + kBImg;
    static constexpr int kPer = kBImg / 1024 / W;       // B pieces per wave and chunk
    static constexpr int kDma = 2 + kPer;               // the vmcnt of one chunk in flight
    static_assert(kBImg % (1024 * W) == 0, "B image splits evenly over the waves");
};

__device__ __forceinline__ void glds16(const void *g, unsigned lds_wave_base) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(lds_wave_base)
                 : "memory", "m0");
}

// diagnostics only (tools/s3_ab.py --probe, xpa_s3_probe): 1 = no MFMAs (fragments still read / split), 2 = no operand
// loads (K40: no DMAs after the first two chunks; K41: no global loads — stale registers), 4 = one MFMA (hi x hi) per
// tile and k step instead of the six.  0 in production.
int g_s3_probe = 0;  // host side: selects the kernel instantiation
int g_pair_sa = 68;  // K41P: the actor's share of 128 slices (xpa_s3_wgrad_pair_tune)

// the k of element j of lane half h inside a 16-k chunk (quads h and h + 2)
__device__ __forceinline__ int kmap(int h, int j) { return 4 * h + j + (j >= 4 ? 4 : 0); }

// ---- B -> three planes -------------------------------------------------------------------------------------
// out (bf16): [K / 16 chunks][3 planes][8 column blocks][2 halves][32 columns][8]; element j of (chunk c, plane p,
// block cb, half h, column r) is plane p of B[16 c + kmap(h, j)][32 cb + r].  One thread per (c, n, h).
__global__ __launch_bounds__(256) void split_b_kernel(const float *__restrict__ b, int64_t K, int64_t sk, int64_t sn,
                                                      __bf16 *__restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t total = (K / kKC) * kN * 2;
    if (t >= total) return;
    const int h = (int)(t & 1);
    const int n = (int)((t >> 1) % kN);
    const int64_t c = (t >> 1) / kN;
    bf16x8 ph, pm, pl;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float x = b[(c * kKC + kmap(h, j)) * sk + (int64_t)n * sn];
        __bf16 a0, a1, a2;
        xpa_split3(x, a0, a1, a2);
        ph[j] = a0;
        pm[j] = a1;
        pl[j] = a2;
    }
    const int cb = n >> 5, r = n & 31;
    bf16x8 *o = reinterpret_cast<bf16x8 *>(out) + c * (3 * 8 * 64) + cb * 64 + h * 32 + r;
    o[0] = ph;
    o[8 * 64] = pm;
    o[16 * 64] = pl;
}

// up to 4 matrices split in one launch (the update's three per step: Wh_pair for dX, Wh_actor^T and Wh_critic^T for
// K16P): block y = matrix
// r05 (K42C): rows k >= rs_from[i] of matrix i scaled by rs_a[i] * rs_w[i][k - rs_from[i]] before the split (V =
// (1 - slope) diag(wc) Wh_c; rs_w null: no scale), and with cs_out the extra block row y = n_mat writes cs_out[j] =
// cs_slope * sum_c rs_w[c] B_i[rs_from + c][j] (f32 fma chain in c order) for the first scaled matrix i
struct SplitBatch {
    const float *b[4];
    int64_t k[4], sk[4], sn[4];
    __bf16 *out[4];
    const float *rs_w[4];
    float rs_a[4];
    int64_t rs_from[4];
    int64_t kv[4];   // rows k >= kv[i] are zero (r05: W0^T [376, 256] split as k = 384 for the C4 trunk forward)
    int n;
    float *cs_out;
    float cs_slope;
};
__global__ __launch_bounds__(256) void split_batch_kernel(SplitBatch sb) {
    const int i = blockIdx.y;
    if (i == sb.n) {   // cs: block b (< 8) owns columns 32 b .. + 31; 8 row groups of 32 threads, then the groups in order
        if (blockIdx.x >= 8) return;
        __shared__ float s_p[8][32];
        int m = 0;
        while (m < sb.n && sb.rs_w[m] == nullptr) ++m;
        const int col = 32 * (int)blockIdx.x + (threadIdx.x & 31), grp = threadIdx.x >> 5;
        const float *b = sb.b[m] + sb.rs_from[m] * sb.sk[m] + (int64_t)col * sb.sn[m];
        const float *w = sb.rs_w[m];
        const int64_t kc = sb.k[m] - sb.rs_from[m], sk = sb.sk[m];
        const int64_t c0 = grp * kc / 8, c1 = (grp + 1) * kc / 8;
        float acc = 0.f;
        int64_t c = c0;
        for (; c + 16 <= c1; c += 16) {   // 16 loads in flight, fma in row order
            float v[16], wv[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                v[u] = b[(c + u) * sk];
                wv[u] = w[c + u];
            }
#pragma unroll
            for (int u = 0; u < 16; ++u) acc = fmaf(wv[u], v[u], acc);
        }
        for (; c < c1; ++c) acc = fmaf(w[c], b[c * sk], acc);
        s_p[grp][threadIdx.x & 31] = acc;
        __syncthreads();
        if (grp == 0) {
            float sum = s_p[0][threadIdx.x];
#pragma unroll
            for (int g = 1; g < 8; ++g) sum += s_p[g][threadIdx.x];
            sb.cs_out[col] = sb.cs_slope * sum;
        }
        return;
    }
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t K = sb.k[i];
    if (t >= (K / kKC) * kN * 2) return;
    const float *b = sb.b[i];
    const int64_t sk = sb.sk[i], sn = sb.sn[i];
    const int h = (int)(t & 1);
    const int n = (int)((t >> 1) % kN);
    const int64_t c = (t >> 1) / kN;
    const float *rw = sb.rs_w[i];
    bf16x8 ph, pm, pl;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        __bf16 a0, a1, a2;
        const int64_t kk = c * kKC + kmap(h, j);
        float v = kk < sb.kv[i] ? b[kk * sk + (int64_t)n * sn] : 0.f;
        if (rw != nullptr && kk >= sb.rs_from[i]) v *= sb.rs_a[i] * rw[kk - sb.rs_from[i]];
        xpa_split3(v, a0, a1, a2);
        ph[j] = a0;
        pm[j] = a1;
        pl[j] = a2;
    }
    bf16x8 *o = reinterpret_cast<bf16x8 *>(sb.out[i]) + c * (3 * 8 * 64) + (n >> 5) * 64 + h * 32 + (n & 31);
    o[0] = ph;
    o[8 * 64] = pm;
    o[16 * 64] = pl;
}

// ---- the GEMM ---------------------------------------------------------------------------------------------
// chunk c's DMAs of wave w into the stage at LDS byte address st: A rows r0 + 32 w .. + 31 (two 16-row
// instructions, lane = (row, 16-B slot), slot p of row r holding k quad p ^ ((r >> 2) & 3)), then B's 1-KiB pieces
// 3 w .. 3 w + 2 of the chunk's 24 KiB.  Rows past M re-read row M - 1 (never stored).
template <int W>
__device__ __forceinline__ void issue(unsigned st, const float *__restrict__ a, int64_t lda,
                                      const __bf16 *__restrict__ bs, int64_t r0, int64_t M, int c, int lane,
                                      int wave) {
    using G = S3Geom<W>;
    const int rr = lane >> 2, p = lane & 3;
    const int q = p ^ ((rr >> 2) & 3);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        int64_t row = r0 + wave * 32 + i * 16 + rr;
        row = row < M ? row : M - 1;
        glds16(a + row * lda + c * kKC + 4 * q, st + (unsigned)((wave * 32 + i * 16) * kKC * 4));
    }
    const char *bsrc = reinterpret_cast<const char *>(bs) + (int64_t)c * kBImg;
#pragma unroll
    for (int j = 0; j < G::kPer; ++j) {
        const int piece = wave * G::kPer + j;
        glds16(bsrc + piece * 1024 + lane * 16, st + (unsigned)(G::kAImg + piece * 1024));
    }
}

// issue<W> with the lane's two A row pointers precomputed (r05, K40F: rows possibly through an index, ar_i = the row's
// base + 4 q, so no index load or address arithmetic sits in front of each chunk's DMAs)
template <int W>
__device__ __forceinline__ void issue_rows(unsigned st, const float *ar0, const float *ar1,
                                           const __bf16 *__restrict__ bs, int c, int lane, int wave) {
    using G = S3Geom<W>;
    glds16(ar0 + c * kKC, st + (unsigned)((wave * 32) * kKC * 4));
    glds16(ar1 + c * kKC, st + (unsigned)((wave * 32 + 16) * kKC * 4));
    const char *bsrc = reinterpret_cast<const char *>(bs) + (int64_t)c * kBImg;
#pragma unroll
    for (int j = 0; j < G::kPer; ++j) {
        const int piece = wave * G::kPer + j;
        glds16(bsrc + piece * 1024 + lane * 16, st + (unsigned)(G::kAImg + piece * 1024));
    }
}

// kvalid (wave-uniform, r06): A's columns >= kvalid of this chunk are zeroed before the split — K40F's row-index form
// reads the padded columns d .. kp - 1 of a row from the next buffer row, and 0 x a non-finite value there (the B rows
// of those columns are zero) would make this row's outputs NaN where the reference's are finite
template <int W, int PROBE>
__device__ __forceinline__ void chunk(const char *st, f32x16 (&acc)[8], int lane, int wave, int kvalid = kKC) {
    constexpr int kAImg = S3Geom<W>::kAImg;
    const int h = lane >> 5, i = lane & 31;
    const int sw = (i >> 2) & 3;
    const float *arow = reinterpret_cast<const float *>(st) + (wave * 32 + i) * kKC;
    float4 alo = *reinterpret_cast<const float4 *>(arow + 4 * (h ^ sw));
    float4 ahi = *reinterpret_cast<const float4 *>(arow + 4 * ((h + 2) ^ sw));
    if (kvalid < kKC) {   // the LDS position h ^ sw holds the row's logical quad h (issue_rows' swizzle)
        const int c0 = 4 * h, c1 = 4 * (h + 2);
        alo.x = c0 < kvalid ? alo.x : 0.f;
        alo.y = c0 + 1 < kvalid ? alo.y : 0.f;
        alo.z = c0 + 2 < kvalid ? alo.z : 0.f;
        alo.w = c0 + 3 < kvalid ? alo.w : 0.f;
        ahi.x = c1 < kvalid ? ahi.x : 0.f;
        ahi.y = c1 + 1 < kvalid ? ahi.y : 0.f;
        ahi.z = c1 + 2 < kvalid ? ahi.z : 0.f;
        ahi.w = c1 + 3 < kvalid ? ahi.w : 0.f;
    }
    bf16x8 ah, am, al;
    xpa_split8(alo, ahi, ah, am, al);
    const bf16x8 *bimg = reinterpret_cast<const bf16x8 *>(st + kAImg) + lane;
    if constexpr ((PROBE & 5) != 0) {
#pragma unroll
        for (int cb = 0; cb < 8; ++cb) {
            const bf16x8 bh = bimg[cb * 64], bm = bimg[(8 + cb) * 64], bl = bimg[(16 + cb) * 64];
            if constexpr ((PROBE & 1) != 0) asm volatile("" ::"v"(ah), "v"(am), "v"(al), "v"(bh), "v"(bm), "v"(bl));
            else acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[cb], 0, 0, 0);
            if constexpr ((PROBE & 1) == 0) asm volatile("" ::"v"(am), "v"(al), "v"(bm), "v"(bl));
        }
        return;
    }
#pragma unroll
    for (int cb = 0; cb < 8; ++cb)
        acc[cb] = xpa_mfma_s3(ah, am, al, bimg[cb * 64], bimg[(8 + cb) * 64], bimg[(16 + cb) * 64], acc[cb]);
}

// the 64 x 128 wave tile (W = 8 only): wave (wr = w & 3, wc = w >> 2) owns rows 64 wr .. + 63 x columns 128 wc ..
// + 127 (2 x 4 accumulators): per chunk 4 A + 12 B fragment reads per wave instead of 2 + 24 (the LDS reads of the
// 32 x 256 tile were one B image per wave)
__device__ __forceinline__ void chunk64(const char *st, f32x16 (&acc)[8], int lane, int wave) {
    constexpr int kAImg = S3Geom<8>::kAImg;
    const int h = lane >> 5, i = lane & 31;
    const int sw = (i >> 2) & 3;
    const int wr = wave & 3, wc = wave >> 2;
    bf16x8 ah[2], am[2], al[2];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
        const float *arow = reinterpret_cast<const float *>(st) + (wr * 64 + rt * 32 + i) * kKC;
        xpa_split8(*reinterpret_cast<const float4 *>(arow + 4 * (h ^ sw)),
                   *reinterpret_cast<const float4 *>(arow + 4 * ((h + 2) ^ sw)), ah[rt], am[rt], al[rt]);
    }
    const bf16x8 *bimg = reinterpret_cast<const bf16x8 *>(st + kAImg) + lane;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int cb = 4 * wc + j;
        const bf16x8 bh = bimg[cb * 64], bm = bimg[(8 + cb) * 64], bl = bimg[(16 + cb) * 64];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) acc[rt * 4 + j] = xpa_mfma_s3(ah[rt], am[rt], al[rt], bh, bm, bl, acc[rt * 4 + j]);
    }
}

// EPI (r05, K40F: the C4 trunk layer's forward): 0 = C = A B; 1 / 2 / 3 = C = act(A B + bias) with act identity /
// LeakyReLU (slope) / tanh, and with `sign` (EPI 1 / 2) the output's sign bits beside it (32 bytes per row, byte col bit
// cb = C[row, 32 cb + col] > 0: K42S's act' source, the layout xpa_thin_linear_act_fwd_gather_sign writes)
// K40G's activation-backward epilogue (r05, C3's fc data gradient = d conv3 output): the stored value is
// g act'(y) with y read at the output's own (row, column) (the previous block's output, same layout and row stride),
// and the block's column sums of it per channel (column mod C, C = 32 / 64) go to bpart[(problem x gridDim.x + row
// block) x C + channel] — K22 folded in
struct S3ActBwd {
    int act = -1;   // -1: none (a plain store)
    float slope = 0.f;
    int C = 64;
    float *bpart = nullptr;
};

template <int ACT>
__device__ __forceinline__ float s3_act_grad(float d, float y, float slope) {
#pragma clang fp contract(off)  // conv.hip's act_grad / igemm.hip's ig_grad: the same value as K22 writes
    if (ACT == 1) return y > 0.f ? d : d * slope;
    if (ACT == 2) return d * (1.0f - y * y);
    return d;
}

// the body of K40 for row block blk (s3_gemm_kernel: blk = blockIdx.x; s3_gemm_group_kernel: one of several
// problems per blockIdx.y).  AB >= 0 (EPI 0 only): the activation-backward epilogue above, y at the output's offsets
template <int W, int S, int PROBE, int T64, int EPI, int AB = -1>
__device__ __forceinline__ void s3_gemm_body(const float *__restrict__ a, int64_t lda, const __bf16 *__restrict__ bs,
                                             float *__restrict__ c, int64_t ldc, int64_t M, int nchunks,
                                             const float *__restrict__ bias, float slope,
                                             unsigned char *__restrict__ sign, const int64_t *__restrict__ ridx,
                                             int64_t blk, const float *__restrict__ yab = nullptr,
                                             const S3ActBwd *abp = nullptr, const float *__restrict__ wo = nullptr,
                                             const float *__restrict__ bo = nullptr) {
    using G = S3Geom<W>;
    // ONE LDS array (the DMA target; see head.hip)
    __shared__ __attribute__((aligned(16))) char lds[S * G::kStage];
    const unsigned base = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_char_t *)lds);
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int64_t r0 = blk * G::kRows;
    f32x16 acc[8];
#pragma unroll
    for (int cb = 0; cb < 8; ++cb)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[cb][r] = 0.f;
    // K40F (EPI != 0): the lane's two A rows resolved once (through ridx when given: the minibatch rows of the rollout
    // buffer, r05), rows past M re-reading row M - 1 as issue<W> does
    const float *ar[2] = {a, a};
    if constexpr (EPI != 0) {
        const int rr = lane >> 2, p = lane & 3;
        const int q = p ^ ((rr >> 2) & 3);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            int64_t row = r0 + wave * 32 + i * 16 + rr;
            row = row < M ? row : M - 1;
            if (ridx != nullptr) row = ridx[row];
            ar[i] = a + row * lda + 4 * q;
        }
    }
    auto issue_any = [&](unsigned st, int c) {
        if constexpr (EPI != 0) issue_rows<W>(st, ar[0], ar[1], bs, c, lane, wave);
        else issue<W>(st, a, lda, bs, r0, M, c, lane, wave);
    };
#pragma unroll
    for (int d = 0; d < S - 1; ++d)
        if (d < nchunks) issue_any(base + d * G::kStage, d);
#pragma unroll 1
    for (int ch = 0; ch < nchunks; ++ch) {
        // own DMAs of chunk ch landed (with 3 stages chunk ch + 1's may still fly), then every wave's: the stage
        // chunk ch + S - 1 refills was read by every wave in chunk ch - 1
        if (S == 3 && ch + 1 < nchunks) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(G::kDma) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        if (ch + S - 1 < nchunks && (PROBE & 2) == 0)
            issue_any(base + ((ch + S - 1) % S) * G::kStage, ch + S - 1);
        if constexpr (T64 != 0) chunk64(lds + (ch % S) * G::kStage, acc, lane, wave);
        else if constexpr (EPI != 0)   // K40F: through ridx the row ends at column lda (the buffer's row width)
            chunk<W, PROBE>(lds + (ch % S) * G::kStage, acc, lane, wave,
                            ridx != nullptr && lda - (int64_t)ch * kKC < kKC ? (int)(lda - (int64_t)ch * kKC) : kKC);
        else chunk<W, PROBE>(lds + (ch % S) * G::kStage, acc, lane, wave);
    }
    // C/D map of 32x32 MFMA: row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5), col = lane & 31
    const int h = lane >> 5, col = lane & 31;
    if constexpr (T64 != 0) {
        const int wr = wave & 3, wc = wave >> 2;
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t row = r0 + wr * 64 + rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (row < M) {
                    float *crow = c + row * ldc + 128 * wc + col;
#pragma unroll
                    for (int j = 0; j < 4; ++j) crow[j * 32] = acc[rt * 4 + j][r];
                }
            }
        return;
    }
    if constexpr (EPI >= 4) {
        // K40V (r06): the critic's value head in the epilogue — c[row] = act(z[row] + bias) . wo + bo[0] with act
        // identity / LeakyReLU (slope) / tanh for EPI 4 / 5 / 6: each lane's 8 columns in column-block order (one fmaf
        // chain), then the 32 lanes of its row half in a fixed butterfly; the hidden layer's output is never stored
        float bv[8], wv[8];
#pragma unroll
        for (int cb = 0; cb < 8; ++cb) {
            bv[cb] = bias[cb * 32 + col];
            wv[cb] = wo[cb * 32 + col];
        }
        const float b_out = bo[0];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float p = 0.f;
#pragma unroll
            for (int cb = 0; cb < 8; ++cb) {
                float x = acc[cb][r] + bv[cb];
                if constexpr (EPI == 5) x = x > 0.f ? x : x * slope;
                if constexpr (EPI == 6) x = tanhf(x);
                p = fmaf(x, wv[cb], p);
            }
#pragma unroll
            for (int o = 16; o > 0; o >>= 1) p += __shfl_xor(p, o, 64);
            const int64_t row = r0 + wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (col == 0 && row < M) c[row] = p + b_out;
        }
        return;
    }
    if constexpr (EPI != 0) {
        float bv[8];
#pragma unroll
        for (int cb = 0; cb < 8; ++cb) bv[cb] = bias[cb * 32 + col];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t row = r0 + wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (row < M) {
                float *crow = c + row * ldc + col;
                unsigned bits = 0u;
#pragma unroll
                for (int cb = 0; cb < 8; ++cb) {
                    float v = acc[cb][r] + bv[cb];
                    if constexpr (EPI == 2) v = v > 0.f ? v : v * slope;
                    if constexpr (EPI == 3) v = tanhf(v);
                    crow[cb * 32] = v;
                    bits |= (v > 0.f ? 1u : 0u) << cb;
                }
                if (EPI != 3 && sign != nullptr) sign[row * 32 + col] = (unsigned char)bits;
            }
        }
        return;
    }
    if constexpr (AB >= 0) {
        float s0 = 0.f, s1 = 0.f;   // channel col (even column blocks), 32 + col (odd; C = 32: both col)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t row = r0 + wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (row < M) {
                float *crow = c + row * ldc + col;
                const float *yrow = yab + row * ldc + col;
                float yv[8];
#pragma unroll
                for (int cb = 0; cb < 8; ++cb) yv[cb] = yrow[cb * 32];
#pragma unroll
                for (int cb = 0; cb < 8; ++cb) {
                    const float v = s3_act_grad<AB>(acc[cb][r], yv[cb], abp->slope);
                    crow[cb * 32] = v;
                    if (cb & 1) s1 += v;
                    else s0 += v;
                }
            }
        }
        s0 += __shfl_xor(s0, 32, 64);
        s1 += __shfl_xor(s1, 32, 64);
        __syncthreads();   // every wave is past the k loop: the LDS ring is free
        float *red = reinterpret_cast<float *>(lds);
        if (h == 0) {
            red[wave * 64 + col] = s0;
            red[wave * 64 + 32 + col] = s1;
        }
        __syncthreads();
        const int t = threadIdx.x;
        const int C = abp->C;
        if (t < C) {
            float tot = 0.f;
            for (int w = 0; w < W; ++w)
                tot += C == 64 ? red[w * 64 + t] : red[w * 64 + t] + red[w * 64 + 32 + t];
            abp->bpart[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * C + t] = tot;
        }
        return;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t row = r0 + wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row < M) {
            float *crow = c + row * ldc + col;
#pragma unroll
            for (int cb = 0; cb < 8; ++cb) crow[cb * 32] = acc[cb][r];
        }
    }
}

template <int W, int S, int PROBE, int T64 = 0, int EPI = 0>
__global__ __launch_bounds__(64 * W, 8 / W) void s3_gemm_kernel(const float *__restrict__ a, int64_t lda,
                                                               const __bf16 *__restrict__ bs, float *__restrict__ c,
                                                               int64_t ldc, int64_t M, int nchunks,
                                                               const float *__restrict__ bias = nullptr,
                                                               float slope = 0.f,
                                                               unsigned char *__restrict__ sign = nullptr,
                                                               const int64_t *__restrict__ ridx = nullptr) {
    s3_gemm_body<W, S, PROBE, T64, EPI>(a, lda, bs, c, ldc, M, nchunks, bias, slope, sign, ridx, blockIdx.x);
}

// K40V (r06): K40 with the value-head epilogue (EPI 4 / 5 / 6), v [M] out
template <int W, int EPI>
__global__ __launch_bounds__(64 * W, 8 / W) void s3_gemm_value_kernel(const float *__restrict__ a, int64_t lda,
                                                                     const __bf16 *__restrict__ bs,
                                                                     float *__restrict__ v, int64_t M, int nchunks,
                                                                     const float *__restrict__ bias, float slope,
                                                                     const float *__restrict__ wo,
                                                                     const float *__restrict__ bo) {
    s3_gemm_body<W, 3, 0, 0, EPI>(a, lda, bs, v, 1, M, nchunks, bias, slope, nullptr, nullptr, blockIdx.x, nullptr,
                                  nullptr, wo, bo);
}

// K40G (r05): up to kS3Groups independent K40 problems of one shape in one launch (blockIdx.y = the problem): the
// column blocks and k parts of a GEMM wider than 256 columns (C3's fc layer: [16384, 3136] x [3136, 512] forward in
// 2 column halves x 2 k halves, its data gradient in 13 column blocks) fill the chip where one K40 launch of M / 256
// blocks would not (64 blocks at 16 384 rows).
constexpr int kS3Groups = 32;
struct S3Group {
    const float *a[kS3Groups];
    const __bf16 *b[kS3Groups];
    float *c[kS3Groups];
    const float *y[kS3Groups];   // AB >= 0: the previous block's output at c[p]'s offsets
};

template <int AB>
__global__ __launch_bounds__(512, 1) void s3_gemm_group_kernel(S3Group g, int64_t lda, int64_t ldc, int64_t M,
                                                               int nchunks, S3ActBwd ab) {
    const int p = blockIdx.y;
    s3_gemm_body<8, 3, 0, 0, 0, AB>(g.a[p], lda, g.b[p], g.c[p], ldc, M, nchunks, nullptr, 0.f, nullptr, nullptr,
                                    blockIdx.x, g.y[p], &ab);
}

// K40R (r05): the rollout's paired hidden layer z [M, 512] = x [M, 256] . [B0 | B1] + bias (B0 / B1 = Wh_actor^T /
// Wh_critic^T, each split by xpa_s3_split_b into K40's chunk images) for the rollout's few rows (4096 at C2, where K40's
// 256-row blocks would leave all but 32 CUs idle and the f32 library GEMM took 15.5 us): 64-row x 128-column blocks
// (grid M / 64 x 4 column quarters: 256 at C2) of 4 waves, wave (wr = w & 1, wc = w >> 1) owning rows 32 wr .. + 31 x
// columns 64 wc .. + 63 of the block (2 accumulators); per 16-k chunk the block's A rows (4 KiB, K40's swizzled image)
// and its 12 KiB of B planes arrive by LDS-DMA through a 3-stage ring, one A and three B instructions per wave.  K40's
// products, product order and k order: every output is K40's (xpa_s3_gemm on the same half) + bias, bit for bit.
constexpr int kRRows = 64;
constexpr int kRAImg = kRRows * kKC * 4;   // 4 KiB
constexpr int kRBImg = 3 * 4 * 1024;       // 12 KiB: 3 planes x 4 column blocks
constexpr int kRStage = kRAImg + kRBImg;
// S ring stages of CPS 16-k chunks each (S - 1 stages requested ahead): one barrier per stage.  A chunk is only 384
// MFMA cycles per wave here (12 MFMAs), far less than an L2 round trip + a barrier, so several chunks ride one stage.
template <int S, int CPS>
__global__ __launch_bounds__(256, 1) void s3_gemm_r64_kernel(const float *__restrict__ a, int64_t lda,
                                                            const __bf16 *__restrict__ bs0,
                                                            const __bf16 *__restrict__ bs1, float *__restrict__ c,
                                                            int64_t ldc, int64_t M, int nchunks,
                                                            const float *__restrict__ bias) {
    constexpr int kSt = CPS * kRStage;
    __shared__ __attribute__((aligned(16))) char lds[S * kSt];
    const unsigned base = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_char_t *)lds);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int64_t r0 = (int64_t)blockIdx.x * kRRows;
    // XCD-aware rows (r05, M % 512 == 0): block bx (on XCD bx % 8, as gridDim.x is a multiple of 8) takes the 8-row
    // groups t = x + 8 (8 k + g), x = bx & 7, k = bx >> 3, g < 8 — the trunk launch wrote group t on XCD t % 8 = x, and
    // K14E reads it there (xcd_env); image row R = 8 g + j holds global row 8 t + j
    const bool xr = (M & 511) == 0;
    auto grow = [&](int R) -> int64_t {
        if (!xr) return r0 + R;
        const int64_t t = (int64_t)(blockIdx.x & 7) + 8 * (8 * (int64_t)(blockIdx.x >> 3) + (R >> 3));
        return 8 * t + (R & 7);
    };
    const int q = blockIdx.y;                       // column quarter of the 512
    const char *bsrc0 = reinterpret_cast<const char *>(q < 2 ? bs0 : bs1);
    const int coff = (q & 1) * 4;                   // first column block of the quarter inside its matrix
    const int nst = nchunks / CPS;                  // the caller checks nchunks % CPS == 0
    auto issue = [&](unsigned st, int stage) {
#pragma unroll
        for (int u = 0; u < CPS; ++u) {
            const int ch = stage * CPS + u;
            const unsigned sc = st + (unsigned)(u * kRStage);
            const int rr = lane >> 2, p = lane & 3;
            const int qq = p ^ ((rr >> 2) & 3);
            int64_t row = grow(wave * 16 + rr);
            row = row < M ? row : M - 1;
            glds16(a + row * lda + ch * kKC + 4 * qq, sc + (unsigned)(wave * 16 * kKC * 4));
            const char *bsrc = bsrc0 + (int64_t)ch * kBImg;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int piece = wave * 3 + k, plane = piece >> 2, j = piece & 3;
                glds16(bsrc + (plane * 8 + coff + j) * 1024 + lane * 16, sc + (unsigned)(kRAImg + piece * 1024));
            }
        }
    };
    f32x16 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
#pragma unroll
    for (int d = 0; d < S - 1; ++d)
        if (d < nst) issue(base + d * kSt, d);
    const int wr = wave & 1, wc = wave >> 1;
    const int h = lane >> 5, i = lane & 31, sw = (i >> 2) & 3;
    constexpr int kPerSt = 4 * CPS;   // DMA instructions per wave and stage
#pragma unroll 1
    for (int sg = 0; sg < nst; ++sg) {
        // own DMAs of stage sg landed (the `ahead` stages after it may fly), then every wave's; the slot stage
        // sg + S - 1 refills was read in stage sg - 1
        const int ahead = min(nst - 1 - sg, S - 2);
        if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * kPerSt) : "memory");
        else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(kPerSt) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        if (sg + S - 1 < nst) issue(base + ((sg + S - 1) % S) * kSt, sg + S - 1);
#pragma unroll
        for (int u = 0; u < CPS; ++u) {
            const char *st = lds + (sg % S) * kSt + u * kRStage;
            const float *arow = reinterpret_cast<const float *>(st) + (32 * wr + i) * kKC;
            bf16x8 ah, am, al;
            xpa_split8(*reinterpret_cast<const float4 *>(arow + 4 * (h ^ sw)),
                       *reinterpret_cast<const float4 *>(arow + 4 * ((h + 2) ^ sw)), ah, am, al);
            const bf16x8 *bimg = reinterpret_cast<const bf16x8 *>(st + kRAImg) + lane;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int cbl = 2 * wc + j;
                acc[j] = xpa_mfma_s3(ah, am, al, bimg[cbl * 64], bimg[(4 + cbl) * 64], bimg[(8 + cbl) * 64], acc[j]);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int col = q * 128 + (2 * wc + j) * 32 + i;
        const float bv = bias[col];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t row = grow(32 * wr + (r & 3) + 8 * (r >> 2) + 4 * h);
            if (row < M) c[row * ldc + col] = acc[j][r] + bv;
        }
    }
}

// K40T (r06): the rollout's trunk in K40R's launch — the block's 64 raw observation rows are normalised (clip((x -
// mean) / (sqrt(var) + 1e-8)), xpa_thin_linear_act_fwd_norm's arithmetic), their trunk layer act(x . W^T + b) is
// formed in the block (thread t <-> trunk column t = GEMM k index t, the same k-ascending fmaf chain as
// thin_fwd_norm_kernel, so h is that kernel's bit for bit) straight into a resident f32 A image of all 16 k chunks (K40R's
// swizzled layout), and the k loop streams only B's planes.  The trunk's h never reaches HBM; the 4 column-quarter
// blocks of a row tile each form it (4 x 64 x din x 256 FMAs, ~1 us of VALU before the first MFMA, overlapped with B's
// prefetch); the quarter-0 block writes the normalised rows to xn and the rollout buffer column.  Every z is K40R's on
// thin_fwd_norm's h, bit for bit.
template <int ACT>
__device__ __forceinline__ float trunk_act(float z, float slope) {
    if (ACT == 1) return z > 0.f ? z : z * slope;
    if (ACT == 2) return tanhf(z);
    return z;
}

constexpr int kTAImg = kRRows * kN * 4;   // 64 KiB: the block's h rows, all k chunks
// W's rows in LDS at this stride (d_in <= kTWst for the d_in-20 form: the whole K40T LDS then stays under 160 KiB)
template <int DMAX>
struct TrunkW { static constexpr int kSt = DMAX == 8 ? 8 : 18; };
template <int S, int CPS, int ACT, int DMAX, int PROBE = 0>
__global__ __launch_bounds__(256, 1) void s3_gemm_r64_trunk_kernel(
    const float *__restrict__ x, int64_t ldx, int din, const float *__restrict__ tw, const float *__restrict__ tb,
    float slope, const float *__restrict__ mean, const float *__restrict__ var, float clip, float *__restrict__ xn,
    int64_t ldn, float *__restrict__ col, int64_t col_ld, const xpa_cursor_t *__restrict__ cursor,
    const __bf16 *__restrict__ bs0, const __bf16 *__restrict__ bs1, float *__restrict__ c, int64_t ldc, int64_t M,
    const float *__restrict__ bias) {
    constexpr int kSt = CPS * kRBImg;
    constexpr int kNch = kN / kKC;
    constexpr int kWst = TrunkW<DMAX>::kSt;
    static_assert(kNch % CPS == 0 && (4 / CPS) * CPS == 4, "stages of CPS chunks, a trunk phase per 4 chunks");
    static_assert(DMAX % 2 == 0 && kWst % 2 == 0, "feature pairs");
    constexpr int kLds = kTAImg + S * kSt + kRRows * DMAX * 4 + kN * kWst * 4;
    static_assert(kLds <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) char lds[kLds];
    float *aimg = reinterpret_cast<float *>(lds);
    float *s_x = reinterpret_cast<float *>(lds + kTAImg + S * kSt);
    float *wl = s_x + kRRows * DMAX;
    const unsigned bbase = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_char_t *)lds) + kTAImg;
    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int64_t r0 = (int64_t)blockIdx.x * kRRows;
    const bool xr = (M & 511) == 0;   // K40R's XCD-aware row map
    auto grow = [&](int R) -> int64_t {
        if (!xr) return r0 + R;
        const int64_t tt = (int64_t)(blockIdx.x & 7) + 8 * (8 * (int64_t)(blockIdx.x >> 3) + (R >> 3));
        return 8 * tt + (R & 7);
    };
    const int q = blockIdx.y;
    const char *bsrc0 = reinterpret_cast<const char *>(q < 2 ? bs0 : bs1);
    const int coff = (q & 1) * 4;
    constexpr int nst = kNch / CPS;
    auto issue = [&](unsigned st, int stage) {
#pragma unroll
        for (int u = 0; u < CPS; ++u) {
            const int ch = stage * CPS + u;
            const char *bsrc = bsrc0 + (int64_t)ch * kBImg;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int piece = wave * 3 + k, plane = piece >> 2, j = piece & 3;
                glds16(bsrc + (plane * 8 + coff + j) * 1024 + lane * 16, st + (unsigned)(u * kRBImg + piece * 1024));
            }
        }
    };
#pragma unroll
    for (int d = 0; d < S - 1; ++d) issue(bbase + d * kSt, d);
    // W [256, din] into LDS (coalesced: a thread's own weights straight from global memory are 68-B strided across the
    // lanes, ~34 cache lines per load instruction) and the normalised rows into s_x; every load issued before the
    // first use (a rolled loop waited for each round trip in turn)
    {
        const int nw = kN * din;
        constexpr int kWPer = (kN * DMAX + 255) / 256;
        float wv[kWPer];
#pragma unroll
        for (int u = 0; u < kWPer; ++u) wv[u] = tw[min(t + 256 * u, nw - 1)];
        constexpr int kPer = (kRRows * DMAX + 255) / 256;
        float xv[kPer], mv[kPer], vv[kPer];
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int i = min(t + 256 * u, kRRows * DMAX - 1);
            const int R = i / DMAX, k = i - R * DMAX;
            const int64_t row = grow(R);
            const int kc = k < din ? k : 0;
            const int64_t rc = row < M ? row : M - 1;
            xv[u] = x[rc * ldx + kc];
            mv[u] = mean[kc];
            vv[u] = var[kc];
        }
#pragma unroll
        for (int u = 0; u < kWPer; ++u) {
            const int i = t + 256 * u;
            if (i < nw) wl[(i / din) * kWst + i % din] = wv[u];
        }
        const int64_t cof = col ? (int64_t)cursor->ptr * din : 0;
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int i = t + 256 * u;
            if (i >= kRRows * DMAX) break;
            const int R = i / DMAX, k = i - R * DMAX;
            const int64_t row = grow(R);
            const bool ok = k < din && row < M;
            float y = 0.f;
            if (ok) {
                const float sd = sqrtf(vv[u]);
                y = (xv[u] - mv[u]) / (sd + 1e-8f);
                y = fminf(fmaxf(y, -clip), clip);
                if (q == 0) {
                    xn[row * ldn + k] = y;
                    if (col) col[row * col_ld + cof + k] = y;
                }
            }
            s_x[((R >> 1) * DMAX + k) * 2 + (R & 1)] = y;   // row pairs: one float4 = features k, k + 1 of rows R, R + 1
        }
    }
    __syncthreads();
    // trunk phase p: the h columns 64 p .. 64 p + 63 = A chunks 4 p .. 4 p + 3, all 64 rows.  Lane (cq = lane & 15,
    // rq = lane >> 4) of wave w: columns 64 p + cq + 16 i (i < 4) of rows 16 w + 4 rq .. + 3 (two row pairs) — eight
    // independent v_pk_fma_f32 chains, each row's chain the k-ascending fmaf sequence of thin_fwd_norm_kernel (h is
    // that kernel's bit for bit).  Column cc lands at chunk cc / 16, logical quad (cc / 4) & 3 (stored at quad ^ sw(R)),
    // element cc & 3.  Phases 1-3 run inside the k loop, in the stages' DMA waits.
    typedef float f2 __attribute__((ext_vector_type(2)));
    const int cq = lane & 15, rq = lane >> 4;
    float bcs[4][4];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int i = 0; i < 4; ++i) bcs[p][i] = tb[64 * p + cq + 16 * i];
    auto trunk_phase = [&](int p) {
        if constexpr ((PROBE & 1) != 0) return;
        const int P0 = 8 * wave + 2 * rq;
        f2 acc[2][4];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[u][i] = f2{0.f, 0.f};
#pragma unroll
        for (int k = 0; k < DMAX; k += 2) {
            f2 wk[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const f2 wv = *reinterpret_cast<const f2 *>(wl + (64 * p + cq + 16 * i) * kWst + (k < kWst ? k : 0));
                wk[i] = f2{k < din ? wv.x : 0.f, k + 1 < din ? wv.y : 0.f};
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const float4 xv = *reinterpret_cast<const float4 *>(s_x + ((P0 + u) * DMAX + k) * 2);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    acc[u][i] = __builtin_elementwise_fma(f2{xv.x, xv.y}, f2{wk[i].x, wk[i].x}, acc[u][i]);
                    acc[u][i] = __builtin_elementwise_fma(f2{xv.z, xv.w}, f2{wk[i].y, wk[i].y}, acc[u][i]);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int cc = 64 * p + cq + 16 * i;
            float *dst = aimg + (cc >> 4) * (kRRows * kKC) + (cc & 3);
            const int lq = (cc >> 2) & 3;
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int R = 2 * (P0 + u) + e;
                    dst[R * kKC + 4 * (lq ^ ((R >> 2) & 3))] = trunk_act<ACT>(acc[u][i][e] + bcs[p][i], slope);
                }
        }
    };
    trunk_phase(0);
    if constexpr ((PROBE & 2) != 0) {   // diagnostics: the prologue alone (every prefetched DMA drained)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        return;
    }
    f32x16 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    const int wr = wave & 1, wc = wave >> 1;
    const int h = lane >> 5, i = lane & 31, sw = (i >> 2) & 3;
    constexpr int kPerSt = 3 * CPS;
    constexpr int kStPerPhase = 4 / CPS;
#pragma unroll 1
    for (int sg = 0; sg < nst; ++sg) {
        // own B DMAs of stage sg landed (the `ahead` stages after it may fly) and own LDS writes (the trunk phases)
        // done, then every wave's; the slot stage sg + S - 1 refills was read in stage sg - 1
        const int ahead = min(nst - 1 - sg, S - 2);
        switch (ahead) {
        case 5: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(5 * kPerSt) : "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(4 * kPerSt) : "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(3 * kPerSt) : "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(2 * kPerSt) : "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(kPerSt) : "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
        if (sg + S - 1 < nst) issue(bbase + ((sg + S - 1) % S) * kSt, sg + S - 1);
#pragma unroll
        for (int u = 0; u < CPS; ++u) {
            const int ch = sg * CPS + u;
            const char *st = lds + kTAImg + (sg % S) * kSt + u * kRBImg;
            const float *arow = aimg + ch * (kRRows * kKC) + (32 * wr + i) * kKC;
            bf16x8 ah, am, al;
            xpa_split8(*reinterpret_cast<const float4 *>(arow + 4 * (h ^ sw)),
                       *reinterpret_cast<const float4 *>(arow + 4 * ((h + 2) ^ sw)), ah, am, al);
            const bf16x8 *bimg = reinterpret_cast<const bf16x8 *>(st) + lane;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int cbl = 2 * wc + j;
                acc[j] = xpa_mfma_s3(ah, am, al, bimg[cbl * 64], bimg[(4 + cbl) * 64], bimg[(8 + cbl) * 64], acc[j]);
            }
        }
        // the next trunk phase while this stage's MFMAs run: phase p + 1 is first read at stage (p + 1) kStPerPhase,
        // at least one barrier (with its lgkmcnt(0)) later
        if (sg % kStPerPhase == 0 && sg / kStPerPhase + 1 < 4) trunk_phase(sg / kStPerPhase + 1);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int cl = q * 128 + (2 * wc + j) * 32 + i;
        const float bv = bias[cl];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t row = grow(32 * wr + (r & 3) + 8 * (r >> 2) + 4 * h);
            if (row < M) c[row * ldc + cl] = acc[j][r] + bv;
        }
    }
}

// K40W: K40 with the roles split over the waves (as K41W): waves 4-7 (producers) DMA the operands of chunk c + 2 (their
// own 32 A rows each + B's planes) and split chunk c + 1's A rows (own DMAs, so a vmcnt wait suffices) into the bf16
// planes of the stage, while waves 0-3 (consumers, one per SIMD, 32 rows x 256 columns each) read ready planes and run
// chunk c's 48 MFMAs; one barrier per chunk.  Stage: A planes [3][4 row blocks][64 lanes][16 B] (12 KiB), B planes
// (24 KiB), the raw A rows (8 KiB, K16's swizzled image); 3 stages, one 512-thread block per CU, persistent over
// 128-row tiles.  Products, their order and the k order are K40's: the output is K40's bit for bit.
constexpr int kWRows = 128;
constexpr int kWAPl = 3 * 4 * 1024;                 // A planes, bytes
constexpr int kWRaw = kWRows * kKC * 4;             // raw A rows, bytes
constexpr int kWStage = kWAPl + kBImg + kWRaw;      // 44 KiB
constexpr int kWDma = 2 + kBImg / 1024 / 4;         // per producer wave and chunk: 2 A rows + 6 B pieces

__device__ __forceinline__ void w_issue(unsigned st, const float *__restrict__ a, int64_t lda,
                                        const __bf16 *__restrict__ bs, int64_t r0, int64_t M, int c, int lane, int pw) {
    const int rr = lane >> 2, p = lane & 3;
    const int q = p ^ ((rr >> 2) & 3);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        int64_t row = r0 + pw * 32 + i * 16 + rr;
        row = row < M ? row : M - 1;
        glds16(a + row * lda + c * kKC + 4 * q, st + (unsigned)(kWAPl + kBImg + (pw * 32 + i * 16) * kKC * 4));
    }
    const char *bsrc = reinterpret_cast<const char *>(bs) + (int64_t)c * kBImg;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const int piece = pw * 6 + j;
        glds16(bsrc + piece * 1024 + lane * 16, st + (unsigned)(kWAPl + piece * 1024));
    }
}

// producer wave pw: split its 32 raw rows (lane (i, h): row 32 pw + i, quads h and h + 2) into the A planes
__device__ __forceinline__ void w_split(char *st, int lane, int pw) {
    const int h = lane >> 5, i = lane & 31;
    const int sw = (i >> 2) & 3;
    const float *arow = reinterpret_cast<const float *>(st + kWAPl + kBImg) + (pw * 32 + i) * kKC;
    bf16x8 ah, am, al;
    xpa_split8(*reinterpret_cast<const float4 *>(arow + 4 * (h ^ sw)),
               *reinterpret_cast<const float4 *>(arow + 4 * ((h + 2) ^ sw)), ah, am, al);
    bf16x8 *pl = reinterpret_cast<bf16x8 *>(st) + pw * 64 + lane;
    pl[0] = ah;
    pl[4 * 64] = am;
    pl[8 * 64] = al;
}

__device__ __forceinline__ void w_chunk(const char *st, f32x16 (&acc)[8], int lane, int cw) {
    const bf16x8 *pa = reinterpret_cast<const bf16x8 *>(st) + cw * 64 + lane;
    const bf16x8 ah = pa[0], am = pa[4 * 64], al = pa[8 * 64];
    const bf16x8 *bimg = reinterpret_cast<const bf16x8 *>(st + kWAPl) + lane;
#pragma unroll
    for (int cb = 0; cb < 8; ++cb)
        acc[cb] = xpa_mfma_s3(ah, am, al, bimg[cb * 64], bimg[(8 + cb) * 64], bimg[(16 + cb) * 64], acc[cb]);
}

__global__ __launch_bounds__(512, 1) void s3_gemm_ws_kernel(const float *__restrict__ a, int64_t lda,
                                                            const __bf16 *__restrict__ bs, float *__restrict__ c,
                                                            int64_t ldc, int64_t M, int nchunks) {
    __shared__ __attribute__((aligned(16))) char lds[3 * kWStage];
    const unsigned base = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_char_t *)lds);
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int64_t ntiles = (M + kWRows - 1) / kWRows;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t r0 = tile * kWRows;
        if (wave >= 4) {   // producers: 1 + nchunks barriers per tile, as the consumers
            const int pw = wave - 4;
            w_issue(base, a, lda, bs, r0, M, 0, lane, pw);
            if (nchunks > 1) {
                w_issue(base + kWStage, a, lda, bs, r0, M, 1, lane, pw);
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kWDma) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            w_split(lds, lane, pw);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll 1
            for (int ch = 0; ch < nchunks; ++ch) {
                if (ch + 2 < nchunks) {
                    w_issue(base + ((ch + 2) % 3) * kWStage, a, lda, bs, r0, M, ch + 2, lane, pw);
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kWDma) : "memory");   // chunk ch + 1 landed
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                if (ch + 1 < nchunks) w_split(lds + ((ch + 1) % 3) * kWStage, lane, pw);
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            }
            continue;
        }
        f32x16 acc[8];
#pragma unroll
        for (int cb = 0; cb < 8; ++cb)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[cb][r] = 0.f;
        asm volatile("s_barrier" ::: "memory");
#pragma unroll 1
        for (int ch = 0; ch < nchunks; ++ch) {
            w_chunk(lds + (ch % 3) * kWStage, acc, lane, wave);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
        const int h = lane >> 5, col = lane & 31;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t row = r0 + wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (row < M) {
                float *crow = c + row * ldc + col;
#pragma unroll
                for (int cb = 0; cb < 8; ++cb) crow[cb * 32] = acc[cb][r];
            }
        }
    }
}

// ---- K42: K40's dX GEMM with the representation's first layer backward in its epilogue ---------------------------
// g = dz . Wh_pair stays in the accumulators: dz1 = g * act'(h) (h = the layer's output, K13's act_g), db1 = the column
// sums of dz1 and dW1 = dz1^T x (x = the layer's input rows, d_in <= 32) per block, as K13's backward (thin.hip) does
// from a g in HBM — g is never stored (64 MiB less written and read per C2 update) and K13's backward launch is gone.
// dW1's product runs on the same split: the accumulator tile of a wave (column on the lane, rows in the registers) is
// the B operand of Y = x^T dz1 as it is (registers 8s .. 8s + 7 = the 8 k of k step s, cdna_hip_programming.md §3),
// x^T's fragment holds the same rows.  Per column block the 8 waves' Y [d_in x 32] meet in LDS and are added in wave
// order; one partial row per block (xpa_s3_gemm_trunk_bwd_num_partials), finalized by the caller's f64 column sums.
// K42S lookahead form (r04, xpa_s3_probe bit 128): a 4-stage ring, each wave splitting chunk c + 1's A fragment
// between chunk c's MFMA blocks (K41V's interleave), so the split no longer precedes the MFMAs of its own chunk
__device__ __forceinline__ void a_split(const char *st, int lane, int wave, bf16x8 &ah, bf16x8 &am, bf16x8 &al) {
    const int h = lane >> 5, i = lane & 31;
    const int sw = (i >> 2) & 3;
    const float *arow = reinterpret_cast<const float *>(st) + (wave * 32 + i) * kKC;
    xpa_split8(*reinterpret_cast<const float4 *>(arow + 4 * (h ^ sw)),
               *reinterpret_cast<const float4 *>(arow + 4 * ((h + 2) ^ sw)), ah, am, al);
}

__device__ __forceinline__ void chunk_la(const char *st, const char *st_next, f32x16 (&acc)[8], int lane, int wave,
                                         bf16x8 &ah, bf16x8 &am, bf16x8 &al) {
    constexpr int kAImg = S3Geom<8>::kAImg;
    const bf16x8 *bimg = reinterpret_cast<const bf16x8 *>(st + kAImg) + lane;
    bf16x8 nh, nm, nl;
#pragma unroll
    for (int cb = 0; cb < 8; ++cb) {
        acc[cb] = xpa_mfma_s3(ah, am, al, bimg[cb * 64], bimg[(8 + cb) * 64], bimg[(16 + cb) * 64], acc[cb]);
        if (cb == 1) a_split(st_next, lane, wave, nh, nm, nl);   // past the last chunk: a stale stage, unused
        __builtin_amdgcn_sched_barrier(0);
    }
    ah = nh;
    am = nm;
    al = nl;
}

// ---- PP (r05): the k loop as a ping-pong between the two waves of each SIMD ------------------------------------------
// K40 / K42 as written run both waves of a SIMD (w and w + 4) through the same chunk in lockstep: after each chunk
// barrier both split their A fragment and read their B fragments, then both issue their 48 MFMAs, so the matrix pipe
// idles through the first part and the VALU / LDS through the second (r04q probes: 84 us with no operand loads at all
// against ~45 us of MFMA time; the non-MFMA part alone 42 us — nothing overlapped).  Here the k loop is a sequence of
// phases, one block barrier each, and the halves (half = w >> 2) run one phase apart:
//     phase p, half h, q = p - h:  q even -> prep chunk q / 2 (its A fragment: 2 ds_read_b128 + the split in VALU)
//                                  q odd  -> compute chunk (q - 1) / 2 (48 MFMAs, B fragments read from the stage)
// so in every phase one wave of each SIMD issues MFMAs while its partner preps.  Chunk c's stage is read in phases 2c
// .. 2c + 2; chunk c + 3 refills it, issued at the start of phase 2c + 3 (each wave its own DMAs, as K40) and waited
// for (counted vmcnt + the barrier) at the end of phase 2c + 5, the phase before half 0 preps it.  Same products, same
// k order per accumulator as K40: the outputs are K40's bit for bit.
// the B fragments of column block cb + 1 are read while cb's six MFMAs run (one block ahead, sched_barrier-pinned:
// hipcc otherwise hoists all 24 reads, 96 VGPRs beside the 128 accumulators)
__device__ __forceinline__ void pp_compute(const char *st, f32x16 (&acc)[8], int lane, const bf16x8 &ah,
                                           const bf16x8 &am, const bf16x8 &al) {
    const bf16x8 *bimg = reinterpret_cast<const bf16x8 *>(st + S3Geom<8>::kAImg) + lane;
    bf16x8 bh = bimg[0], bm = bimg[8 * 64], bl = bimg[16 * 64];
#pragma unroll
    for (int cb = 0; cb < 8; ++cb) {
        bf16x8 nh, nm, nl;
        if (cb + 1 < 8) {
            nh = bimg[(cb + 1) * 64];
            nm = bimg[(9 + cb) * 64];
            nl = bimg[(17 + cb) * 64];
        }
        acc[cb] = xpa_mfma_s3(ah, am, al, bh, bm, bl, acc[cb]);
        __builtin_amdgcn_sched_barrier(0);
        if (cb + 1 < 8) {
            bh = nh;
            bm = nm;
            bl = nl;
        }
    }
}

__device__ __forceinline__ void pp_loop(unsigned base, const char *lds, const float *__restrict__ a, int64_t lda,
                                        const __bf16 *__restrict__ bs, int64_t r0, int64_t M, int nchunks, int lane,
                                        int wave, f32x16 (&acc)[8]) {
    using G = S3Geom<8>;
    const int N = nchunks;
    issue<8>(base, a, lda, bs, r0, M, 0, lane, wave);
    if (N > 1) {
        issue<8>(base + G::kStage, a, lda, bs, r0, M, 1, lane, wave);
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(G::kDma) : "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    // phase ends: even phases a bare barrier; odd phase 2m + 1 starts by issuing chunk m + 2 and ends once every
    // wave's chunk m + 1 landed.  Each half runs its own straight-line loop (no branch around the MFMAs: hipcc copied
    // and spilled the accumulators at the joins of a phase-indexed loop)
    auto end_even = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    auto start_odd = [&](int m) {
        if (m + 2 < N) issue<8>(base + ((m + 2) % 3) * G::kStage, a, lda, bs, r0, M, m + 2, lane, wave);
    };
    auto end_odd = [&](int m) {
        __builtin_amdgcn_sched_barrier(0);
        if (m + 2 < N) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(G::kDma) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    bf16x8 ah, am, al;
    if (wave < 4) {   // half 0: phase 2c preps chunk c, phase 2c + 1 computes it
#pragma unroll 1
        for (int c = 0; c < N; ++c) {
            a_split(lds + (c % 3) * G::kStage, lane, wave, ah, am, al);
            end_even();
            start_odd(c);
            pp_compute(lds + (c % 3) * G::kStage, acc, lane, ah, am, al);
            end_odd(c);
        }
        end_even();
    } else {          // half 1: one phase behind
        end_even();
        start_odd(0);
        a_split(lds, lane, wave, ah, am, al);
        end_odd(0);
#pragma unroll 1
        for (int c = 1; c < N; ++c) {
            pp_compute(lds + ((c - 1) % 3) * G::kStage, acc, lane, ah, am, al);
            end_even();
            start_odd(c);
            a_split(lds + (c % 3) * G::kStage, lane, wave, ah, am, al);
            end_odd(c);
        }
        pp_compute(lds + ((N - 1) % 3) * G::kStage, acc, lane, ah, am, al);
        end_even();
    }
}

// K40 with the ping-pong k loop (one 8-wave block per 256 rows, the 3-stage ring)
__global__ __launch_bounds__(512, 1) void s3_gemm_pp_kernel(const float *__restrict__ a, int64_t lda,
                                                            const __bf16 *__restrict__ bs, float *__restrict__ c,
                                                            int64_t ldc, int64_t M, int nchunks) {
    using G = S3Geom<8>;
    __shared__ __attribute__((aligned(16))) char lds[3 * G::kStage];
    const unsigned base = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_char_t *)lds);
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int64_t r0 = (int64_t)blockIdx.x * G::kRows;
    f32x16 acc[8];
#pragma unroll
    for (int cb = 0; cb < 8; ++cb)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[cb][r] = 0.f;
    pp_loop(base, lds, a, lda, bs, r0, M, nchunks, lane, wave, acc);
    const int h = lane >> 5, col = lane & 31;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t row = r0 + wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row < M) {
            float *crow = c + row * ldc + col;
#pragma unroll
            for (int cb = 0; cb < 8; ++cb) crow[cb * 32] = acc[cb][r];
        }
    }
}

template <int ACT>
__device__ __forceinline__ float tb_act_g(float h, float slope) {  // thin.hip act_g
    if (ACT == 1) return h > 0.f ? 1.f : slope;
    if (ACT == 2) return 1.0f - h * h;
    return 1.f;
}

// K42's epilogue (after the k loop, every wave done with the ring): dz1 = g * act'(h) in the accumulators, db1 and dW1
// partials of the block (row block blockIdx.x); lds: the ring's LDS, reused
template <int ACT, bool SIGN, bool DZ = false>
__device__ __forceinline__ void tb_epilogue(f32x16 (&acc)[8], char *lds, int64_t r0, int64_t M, int t, int lane,
                                            int wave, const float *__restrict__ hmat, int64_t ldh,
                                            const float *__restrict__ x, int64_t ldx, int din, float slope,
                                            float *__restrict__ p_dw, float *__restrict__ p_db,
                                            const unsigned *__restrict__ hsign, float *__restrict__ dz_out = nullptr,
                                            int64_t ld_out = 0) {
    // ---- dz1 = g * act'(h) in place (rows past M: 0)
    const int hh = lane >> 5, col = lane & 31;
    const int64_t wrow = r0 + wave * 32;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t row = wrow + (r & 3) + 8 * (r >> 2) + 4 * hh;
        const bool ok = row < M;
        if constexpr (SIGN) {   // byte col of the row: bit cb = h[row, 32 cb + col] > 0
            const unsigned bits = reinterpret_cast<const unsigned char *>(hsign + (ok ? row : 0) * 8)[col];
#pragma unroll
            for (int cb = 0; cb < 8; ++cb) {
                const float g = ACT == 1 ? (((bits >> cb) & 1u) ? 1.f : slope) : 1.f;
                acc[cb][r] = ok ? acc[cb][r] * g : 0.f;
            }
        } else {
            const float *hrow = hmat + (ok ? row : 0) * ldh + col;
#pragma unroll
            for (int cb = 0; cb < 8; ++cb) {
                const float hv = hrow[cb * 32];
                acc[cb][r] = ok ? acc[cb][r] * tb_act_g<ACT>(hv, slope) : 0.f;
            }
        }
    }
    if constexpr (DZ) {   // r05 (K42W, a wide trunk layer): dz1 stored for K41V's dW, db1 partials; no thin dW
        float *s_db = reinterpret_cast<float *>(lds);   // [8 waves][256]
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t row = wrow + (r & 3) + 8 * (r >> 2) + 4 * hh;
            if (row < M) {
                float *drow = dz_out + row * ld_out + col;
#pragma unroll
                for (int cb = 0; cb < 8; ++cb) drow[cb * 32] = acc[cb][r];
            }
        }
#pragma unroll
        for (int cb = 0; cb < 8; ++cb) {
            float cs = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) cs += acc[cb][r];
            cs += __shfl_xor(cs, 32, 64);
            if (hh == 0) s_db[wave * 256 + cb * 32 + col] = cs;
        }
        __syncthreads();
        if (t < 256) {
            float sum = s_db[t];
#pragma unroll
            for (int w = 1; w < 8; ++w) sum += s_db[w * 256 + t];
            p_db[(int64_t)blockIdx.x * 256 + t] = sum;
        }
        return;
    }
    // ---- x^T's fragments for the wave's 32 rows: lane (feature i, half hh), k step s element j = row rho(8 s + j, hh)
    bf16x8 xh[2], xm[2], xl[2];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int r = 8 * st + j;
            const int64_t row = wrow + (r & 3) + 8 * (r >> 2) + 4 * hh;
            const bool ok = row < M && col < din;
            const float xv = x[(row < M ? row : 0) * ldx + (col < din ? col : 0)];
            v[j] = ok ? xv : 0.f;
        }
        xpa_split8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), xh[st], xm[st], xl[st]);
    }
    float *s_y = reinterpret_cast<float *>(lds);                 // [8 waves][32 features][32 columns]
    float *s_db = reinterpret_cast<float *>(lds) + 8 * 32 * 32;  // [8 waves][256]
#pragma unroll   // unrolled: acc[cb] with a run-time cb put the accumulators in scratch (576 B, 2x the launch)
    for (int cb = 0; cb < 8; ++cb) {
        // db1: the wave's 32 rows of this column block (16 per lane half, then the two halves)
        float cs = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) cs += acc[cb][r];
        cs += __shfl_xor(cs, 32, 64);
        if (hh == 0) s_db[wave * 256 + cb * 32 + col] = cs;
        // Y = x^T dz1 over the wave's rows: two k steps of 16 rows
        f32x16 y;
#pragma unroll
        for (int r = 0; r < 16; ++r) y[r] = 0.f;
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = acc[cb][8 * st + j];
            bf16x8 gh, gm, gl;
            xpa_split8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), gh, gm, gl);
            y = xpa_mfma_s3(xh[st], xm[st], xl[st], gh, gm, gl, y);
        }
        // Y's rows are the features: lane (column, hh) holds features rho(r, hh)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = (r & 3) + 8 * (r >> 2) + 4 * hh;
            s_y[(wave * 32 + f) * 32 + col] = y[r];
        }
        __syncthreads();
        for (int e = t; e < din * 32; e += 512) {   // (feature, column) pairs: the 8 waves in order
            const int f = e >> 5, c = e & 31;
            float sum = s_y[f * 32 + c];
#pragma unroll
            for (int w = 1; w < 8; ++w) sum += s_y[(w * 32 + f) * 32 + c];
            p_dw[(int64_t)blockIdx.x * (256 * din) + (cb * 32 + c) * din + f] = sum;
        }
        __syncthreads();   // s_y reused by the next column block
    }
    if (t < 256) {
        float sum = s_db[t];
#pragma unroll
        for (int w = 1; w < 8; ++w) sum += s_db[w * 256 + t];
        p_db[(int64_t)blockIdx.x * 256 + t] = sum;
    }
}

// SIGN (r04, K42S): act' from the sign bits K16R's actor launch wrote (byte col of the row's 32: bit cb = h[row, 32 cb +
// col] > 0; LeakyReLU / identity only) instead of the 1 KiB h row — the same factor, 64 MiB less read per C2 update.
template <int ACT, bool SIGN = false, int LA = 0, bool DZ = false>
__global__ __launch_bounds__(512, 1) void s3_gemm_trunk_bwd_kernel(const float *__restrict__ a, int64_t lda,
                                                                   const __bf16 *__restrict__ bs, int64_t M,
                                                                   int nchunks, const float *__restrict__ hmat,
                                                                   int64_t ldh, const float *__restrict__ x,
                                                                   int64_t ldx, int din, float slope,
                                                                   float *__restrict__ p_dw, float *__restrict__ p_db,
                                                                   const unsigned *__restrict__ hsign = nullptr,
                                                                   float *__restrict__ dz_out = nullptr,
                                                                   int64_t ld_out = 0) {
    static_assert(!SIGN || ACT != 2, "sign bits carry act' of LeakyReLU / identity only");
    using G = S3Geom<8>;
    constexpr int kS = LA == 1 ? 4 : 3;   // ring stages (4 x 40 KiB = the whole 160 KiB with the lookahead)
    __shared__ __attribute__((aligned(16))) char lds[kS * G::kStage];
    const unsigned base = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_char_t *)lds);
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int64_t r0 = (int64_t)blockIdx.x * G::kRows;
    f32x16 acc[8];
#pragma unroll
    for (int cb = 0; cb < 8; ++cb)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[cb][r] = 0.f;
    if constexpr (LA == 2) {
        pp_loop(base, lds, a, lda, bs, r0, M, nchunks, lane, wave, acc);
    } else if constexpr (LA == 1) {
#pragma unroll
        for (int d = 0; d < 3; ++d)
            if (d < nchunks) issue<8>(base + d * G::kStage, a, lda, bs, r0, M, d, lane, wave);
        // chunk 0 landed (chunks 1, 2 may fly), everyone's; then its A fragment split
        if (nchunks >= 3) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * G::kDma) : "memory");
        else if (nchunks == 2) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(G::kDma) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        bf16x8 ah, am, al;
        a_split(lds, lane, wave, ah, am, al);
#pragma unroll 1
        for (int ch = 0; ch < nchunks; ++ch) {
            // chunk ch + 1 landed (ch + 2 may fly), everyone's; the stage chunk ch + 3 refills held chunk ch - 1,
            // whose B fragments every wave read in iteration ch - 1 (its A in ch - 2)
            if (ch + 2 < nchunks) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(G::kDma) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
            if (ch + 3 < nchunks) issue<8>(base + ((ch + 3) & 3) * G::kStage, a, lda, bs, r0, M, ch + 3, lane, wave);
            chunk_la(lds + (ch & 3) * G::kStage, lds + ((ch + 1) & 3) * G::kStage, acc, lane, wave, ah, am, al);
        }
    } else {
#pragma unroll
    for (int d = 0; d < 2; ++d)
        if (d < nchunks) issue<8>(base + d * G::kStage, a, lda, bs, r0, M, d, lane, wave);
#pragma unroll 1
    for (int ch = 0; ch < nchunks; ++ch) {
        if (ch + 1 < nchunks) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(G::kDma) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        if (ch + 2 < nchunks) issue<8>(base + ((ch + 2) % 3) * G::kStage, a, lda, bs, r0, M, ch + 2, lane, wave);
        chunk<8, 0>(lds + (ch % 3) * G::kStage, acc, lane, wave);
    }
    }
    __syncthreads();   // every wave done with the ring: the epilogue reuses its LDS
    tb_epilogue<ACT, SIGN, DZ>(acc, lds, r0, M, t, lane, wave, hmat, ldh, x, ldx, din, slope, p_dw, p_db, hsign,
                               dz_out, ld_out);
}

// ---- K42C (r05): K42S with the critic's half of dX factored -------------------------------------------------------
// The paired dX GEMM g = dz_pair . Wh_pair splits into the actor's half (dz_a . Wh_a: dz_a an f32 operand, six products)
// and the critic's: with the critic's hidden activation LeakyReLU (act' = slope + (1 - slope) m, m = [h_c > 0]) and its
// one output unit, dz_c[r, c] = dv[r] wc[c] act'(h_c[r, c]), so
//     (dz_c . Wh_c)[r, j] = dv[r] (sum_c m[r, c] V[c, j] + cs[j]),  V = (1 - slope) diag(wc) Wh_c,  cs = slope wc . Wh_c
// where m is exact in bf16 (0 / 1): the masked product takes THREE bf16 products (m V_lo, m V_mid, m V_hi; every one
// exact in f32, f32 accumulation), not six, and dz_c is never stored or read (the critic head writes the 32 B of
// sign bits and dv per row instead: xpa_head_gemm_s3q_critic_mask).  The k loop runs the critic's chunks first (split
// buffer chunks nca .. nca + ncc - 1: V's planes; A = the row's mask bits from LDS, no A DMA), scales the accumulators
// by dv[row] after adding cs, then the actor's chunks exactly as K42S (A = dz_a rows by LDS-DMA + the split).  The
// epilogue (the trunk layer's backward) is K42S's.
constexpr int kCMaskStride = 9;   // words per row of the LDS mask image (8 + 1: the 32 rows of a read hit 32 banks)
template <int ACT, bool DZ = false>
__global__ __launch_bounds__(512, 1) void s3_trunk_bwd_crit_kernel(
    const float *__restrict__ a, int64_t lda, const __bf16 *__restrict__ bs, int64_t M, int nca, int ncc,
    const unsigned *__restrict__ cmask, const float *__restrict__ cdv, const float *__restrict__ ccs,
    const float *__restrict__ x, int64_t ldx, int din, float slope, float *__restrict__ p_dw, float *__restrict__ p_db,
    const unsigned *__restrict__ hsign, float *__restrict__ dz_out = nullptr, int64_t ld_out = 0) {
    using G = S3Geom<8>;
    constexpr int kRing = 3 * G::kStage;
    constexpr int kMaskOff = kRing, kDvOff = kMaskOff + 256 * kCMaskStride * 4, kCsOff = kDvOff + 256 * 4;
    __shared__ __attribute__((aligned(16))) char lds[kCsOff + 256 * 4];
    const unsigned base = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_char_t *)lds);
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int64_t r0 = (int64_t)blockIdx.x * G::kRows;
    unsigned *s_mask = reinterpret_cast<unsigned *>(lds + kMaskOff);
    float *s_dv = reinterpret_cast<float *>(lds + kDvOff);
    float *s_cs = reinterpret_cast<float *>(lds + kCsOff);
    {   // the block's 256 mask rows (one uint4 per thread), dv rows and cs (rows past M: zeros)
        const int rr = t >> 1, q = t & 1;
        const int64_t row = r0 + rr;
        uint4 w = make_uint4(0u, 0u, 0u, 0u);
        if (row < M) w = *reinterpret_cast<const uint4 *>(cmask + row * 8 + 4 * q);
        unsigned *d = s_mask + rr * kCMaskStride + 4 * q;
        d[0] = w.x; d[1] = w.y; d[2] = w.z; d[3] = w.w;
        if (t < 256) {
            s_dv[t] = r0 + t < M ? cdv[r0 + t] : 0.f;
            s_cs[t] = ccs[t];
        }
    }
    __syncthreads();
    f32x16 acc[8];
#pragma unroll
    for (int cb = 0; cb < 8; ++cb)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[cb][r] = 0.f;
    const int N = nca + ncc;
    // processing index i -> split chunk: the critic's first
    auto chunk_of = [&](int i) { return i < ncc ? nca + i : i - ncc; };
    auto issue_i = [&](int i) {
        const unsigned st = base + (i % 3) * G::kStage;
        const int c = chunk_of(i);
        const int rr = lane >> 2, p = lane & 3;
        if (i >= ncc) {   // actor chunk: A rows by DMA (K40's swizzled image)
            const int q = p ^ ((rr >> 2) & 3);
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                int64_t row = r0 + wave * 32 + k * 16 + rr;
                row = row < M ? row : M - 1;
                glds16(a + row * lda + c * kKC + 4 * q, st + (unsigned)((wave * 32 + k * 16) * kKC * 4));
            }
        }
        const char *bsrc = reinterpret_cast<const char *>(bs) + (int64_t)c * kBImg;
#pragma unroll
        for (int j = 0; j < G::kPer; ++j) {
            const int piece = wave * G::kPer + j;
            glds16(bsrc + piece * 1024 + lane * 16, st + (unsigned)(G::kAImg + piece * 1024));
        }
    };
    // wait for every wave's DMAs of processing index i (i + 1's may still fly), then the barrier
    auto wait_i = [&](int i) {
        if (i + 1 >= N) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        else if (i + 1 >= ncc) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(G::kDma) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(G::kPer) : "memory");
    };
    issue_i(0);
    if (N > 1) issue_i(1);
    const int hh = lane >> 5, i32 = lane & 31;
    const unsigned *mrow = s_mask + (wave * 32 + i32) * kCMaskStride;
#pragma unroll 1
    for (int i = 0; i < ncc; ++i) {
        wait_i(i);
        if (i + 2 < N) issue_i(i + 2);
        // A = the 8 mask bits of the lane's row at k = 16 i + kmap(hh, j) (the split's k order), as bf16 0 / 1
        const unsigned wbits = mrow[i >> 1] >> (16 * (i & 1) + 4 * hh);
        unsigned pk[4];
#pragma unroll
        for (int pj = 0; pj < 4; ++pj) {
            const int j0 = 2 * pj, j1 = 2 * pj + 1;
            const int b0 = j0 < 4 ? j0 : j0 + 4, b1 = j1 < 4 ? j1 : j1 + 4;
            pk[pj] = (((wbits >> b0) & 1u) * 0x3F80u) | ((((wbits >> b1) & 1u) * 0x3F80u) << 16);
        }
        const bf16x8 am = __builtin_bit_cast(bf16x8, make_uint4(pk[0], pk[1], pk[2], pk[3]));
        const bf16x8 *bimg = reinterpret_cast<const bf16x8 *>(lds + (i % 3) * G::kStage + G::kAImg) + lane;
#pragma unroll
        for (int cb = 0; cb < 8; ++cb) {
            acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bimg[(16 + cb) * 64], acc[cb], 0, 0, 0);
            acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bimg[(8 + cb) * 64], acc[cb], 0, 0, 0);
            acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bimg[cb * 64], acc[cb], 0, 0, 0);
        }
    }
    {   // acc = dv[row] (acc + cs[col]): the critic's half of g
        const int col = lane & 31;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float dvr = s_dv[wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh];
#pragma unroll
            for (int cb = 0; cb < 8; ++cb) acc[cb][r] = dvr * (acc[cb][r] + s_cs[cb * 32 + col]);
        }
    }
#pragma unroll 1
    for (int i = ncc; i < N; ++i) {
        wait_i(i);
        if (i + 2 < N) issue_i(i + 2);
        chunk<8, 0>(lds + (i % 3) * G::kStage, acc, lane, wave);
    }
    __syncthreads();   // every wave done with the ring: the epilogue reuses its LDS
    tb_epilogue<ACT, true, DZ>(acc, lds, r0, M, t, lane, wave, nullptr, 0, x, ldx, din, slope, p_dw, p_db, hsign,
                               dz_out, ld_out);
}

// ---- K41: weight gradients dW = A^T B over the batch (K = rows), split-K -----------------------------------
// out[s] [M, 256] = A[rows of slice s]^T . B[rows of slice s], A [rows, M] (dz), B [rows, 256] (the layer input);
// the slices are summed by the caller (the learner's fixed-order f64 column-sum finalize), as the batched f32 GEMM
// it replaces.  Both operands are k-major (k = batch row), so they are staged through registers: per 32-row chunk a
// thread loads 8 k-strided values of one column for each of its 3 units (one A, two B: 512 + 1024 units of (column,
// k step, lane half) per chunk), splits them and writes the three bf16 fragments (16 B each) straight into the
// MFMA-ready LDS image [plane][column block][k step][64 lanes][16 B] — conflict-free ds_write_b128 / ds_read_b128.
// Block: 512 threads, a 128 x 256 tile of out[s]; wave w owns rows 64 (w & 1) .. + 63 x columns 64 (w >> 1) .. + 63
// (2 x 2 accumulators).  Two stages (72 KiB each): chunk c + 1's loads land in registers while chunk c's 48 MFMAs
// per wave run, one raw barrier per chunk (a __syncthreads would also wait for those loads: vmcnt counts both).
// Blocks of one slice sit on one XCD (blockIdx % 8 is the XCD), so the M / 128 tiles re-read B's rows from one L2.
constexpr int kWgM = 128;
constexpr int kWgKC = 32;
constexpr int kWgAImg = 3 * 4 * 2 * 1024;  // bytes: [3 planes][4 row blocks][2 k steps][64 lanes][16 B]
constexpr int kWgBImg = 3 * 8 * 2 * 1024;  // [3][8 column blocks][2][64][16 B]
constexpr int kWgStage = kWgAImg + kWgBImg;  // 72 KiB

struct WgUnits {
    float a[8], b0[8], b1[8];
};

// chunk at k0 (rows < kend): A unit (column ma, k step sa, half ha), B units (column nb, k step sb, halves 0 / 1)
__device__ __forceinline__ void wg_load(WgUnits &u, const float *__restrict__ A, int64_t lda, const float *__restrict__ B,
                                        int64_t ldb, int64_t k0, int64_t kend, int ma, int sa, int ha, int nb, int sb) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int64_t ra = k0 + 16 * sa + kmap(ha, j);
        const int64_t rb0 = k0 + 16 * sb + kmap(0, j), rb1 = k0 + 16 * sb + kmap(1, j);
        // rows past the slice re-read its last row (branch-free loads), then count as 0
        const float va = A[min(ra, kend - 1) * lda + ma];
        const float v0 = B[min(rb0, kend - 1) * ldb + nb], v1 = B[min(rb1, kend - 1) * ldb + nb];
        u.a[j] = ra < kend ? va : 0.f;
        u.b0[j] = rb0 < kend ? v0 : 0.f;
        u.b1[j] = rb1 < kend ? v1 : 0.f;
    }
}

__device__ __forceinline__ void wg_put(char *st, const float (&v)[8], int off) {
    bf16x8 h, m, l;
    xpa_split8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), h, m, l);
    *reinterpret_cast<bf16x8 *>(st + off) = h;
    *reinterpret_cast<bf16x8 *>(st + off + 8 * 1024 * ((off < kWgAImg) ? 1 : 2)) = m;  // plane stride
    *reinterpret_cast<bf16x8 *>(st + off + 16 * 1024 * ((off < kWgAImg) ? 1 : 2)) = l;
}

__device__ __forceinline__ void wg_store(char *st, const WgUnits &u, int ml, int sa, int ha, int nb, int sb) {
    // A image: plane stride 8 KiB ([4][2][64][16]), B image: 16 KiB ([8][2][64][16])
    wg_put(st, u.a, (((ml >> 5) * 2 + sa) * 64 + ha * 32 + (ml & 31)) * 16);
    wg_put(st, u.b0, kWgAImg + (((nb >> 5) * 2 + sb) * 64 + (nb & 31)) * 16);
    wg_put(st, u.b1, kWgAImg + (((nb >> 5) * 2 + sb) * 64 + 32 + (nb & 31)) * 16);
}

template <int PROBE>
__device__ __forceinline__ void wg_chunk(const char *st, f32x16 (&acc)[2][2], int lane, int wm, int wn) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        bf16x8 ah[2], am[2], al[2], bh[2], bm[2], bl[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const bf16x8 *pa = reinterpret_cast<const bf16x8 *>(st) + ((2 * wm + i) * 2 + s) * 64 + lane;
            ah[i] = pa[0];
            am[i] = pa[8 * 64];
            al[i] = pa[16 * 64];
            const bf16x8 *pb = reinterpret_cast<const bf16x8 *>(st + kWgAImg) + ((2 * wn + i) * 2 + s) * 64 + lane;
            bh[i] = pb[0];
            bm[i] = pb[16 * 64];
            bl[i] = pb[32 * 64];
        }
        if constexpr ((PROBE & 5) != 0) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if constexpr ((PROBE & 1) != 0)
                        asm volatile("" ::"v"(ah[i]), "v"(am[i]), "v"(al[i]), "v"(bh[j]), "v"(bm[j]), "v"(bl[j]));
                    else acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                    if constexpr ((PROBE & 1) == 0) asm volatile("" ::"v"(am[i]), "v"(al[i]), "v"(bm[j]), "v"(bl[j]));
                }
            continue;
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = xpa_mfma_s3(ah[i], am[i], al[i], bh[j], bm[j], bl[j], acc[i][j]);
    }
}

template <int PROBE>
__global__ __launch_bounds__(512, 1) void s3_wgrad_kernel(const float *__restrict__ A, int64_t lda,
                                                          const float *__restrict__ B, int64_t ldb, int64_t rows,
                                                          int64_t M, int slices, int64_t slice_rows,
                                                          float *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) char lds[2 * kWgStage];
    const int mtiles = (int)(M / kWgM);
    const int nblk = slices * mtiles;
    int L = blockIdx.x;
    if (nblk % 8 == 0) L = (blockIdx.x & 7) * (nblk >> 3) + (blockIdx.x >> 3);  // one slice's tiles on one XCD
    const int slice = L / mtiles, mt = L - slice * mtiles;
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int wm = wave & 1, wn = wave >> 1;
    const int ml = t & 127, sa = (t >> 7) & 1, ha = t >> 8, nb = t & 255, sb = t >> 8;
    const float *Am = A + (int64_t)mt * kWgM;
    const int64_t k0 = (int64_t)slice * slice_rows;
    const int64_t kend = min(rows, k0 + slice_rows);
    const int nch = kend > k0 ? (int)((kend - k0 + kWgKC - 1) / kWgKC) : 0;
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    WgUnits u;
    if (nch > 0) {
        wg_load(u, Am, lda, B, ldb, k0, kend, ml, sa, ha, nb, sb);
        wg_store(lds, u, ml, sa, ha, nb, sb);
        if (nch > 1) wg_load(u, Am, lda, B, ldb, k0 + kWgKC, kend, ml, sa, ha, nb, sb);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
        wg_chunk<PROBE>(lds + (c & 1) * kWgStage, acc, lane, wm, wn);
        if (c + 1 < nch) {
            // stage (c + 1) & 1 was last read in chunk c - 1, before the previous barrier
            wg_store(lds + ((c + 1) & 1) * kWgStage, u, ml, sa, ha, nb, sb);
            if (c + 2 < nch && (PROBE & 2) == 0)
                wg_load(u, Am, lda, B, ldb, k0 + (int64_t)(c + 2) * kWgKC, kend, ml, sa, ha, nb, sb);
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    float *o = out + ((int64_t)slice * M + (int64_t)mt * kWgM) * kN;
    const int h = lane >> 5, col = lane & 31;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = 64 * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
#pragma unroll
            for (int j = 0; j < 2; ++j) o[(int64_t)row * kN + 64 * wn + 32 * j + col] = acc[i][j][r];
        }
}

// K41W: the same product with the roles split over the waves of the block, so the staging and the MFMAs overlap by
// construction instead of alternating in every wave between the chunk barriers: waves 4-7 (producers) load chunk
// c + 2 into registers and split / write chunk c + 1 into the other stage while waves 0-3 (consumers, one per SIMD)
// run chunk c's MFMAs; one barrier per chunk hands the stage over.  Consumer w owns rows 64 (w & 1) .. + 63 x
// columns 128 (w >> 1) .. + 127 (2 x 4 accumulators).  A producer thread p stages 6 units per chunk: A (column
// p & 127, k step p >> 7, halves 0 / 1) and B (column p, k steps 0 / 1, halves 0 / 1).  Same LDS image, same products
// and k order per accumulator as K41: the outputs are K41's bit for bit.
__device__ __forceinline__ void wgw_load(float (&v)[6][8], const float *__restrict__ A, int64_t lda,
                                         const float *__restrict__ B, int64_t ldb, int64_t k0, int64_t kend, int p) {
    const int ma = p & 127, sa = p >> 7;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t ra = k0 + 16 * sa + kmap(h, j);
            const float va = A[min(ra, kend - 1) * lda + ma];
            v[h][j] = ra < kend ? va : 0.f;
        }
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int64_t rb = k0 + 16 * s + kmap(h, j);
                const float vb = B[min(rb, kend - 1) * ldb + p];
                v[2 + 2 * s + h][j] = rb < kend ? vb : 0.f;
            }
    }
}

__device__ __forceinline__ void wgw_store(char *st, const float (&v)[6][8], int p) {
    const int ma = p & 127, sa = p >> 7;
#pragma unroll
    for (int h = 0; h < 2; ++h) wg_put(st, v[h], (((ma >> 5) * 2 + sa) * 64 + h * 32 + (ma & 31)) * 16);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int h = 0; h < 2; ++h)
            wg_put(st, v[2 + 2 * s + h], kWgAImg + (((p >> 5) * 2 + s) * 64 + h * 32 + (p & 31)) * 16);
}

__device__ __forceinline__ void wgw_chunk(const char *st, f32x16 (&acc)[2][4], int lane, int wm, int wn) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        bf16x8 ah[2], am[2], al[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const bf16x8 *pa = reinterpret_cast<const bf16x8 *>(st) + ((2 * wm + i) * 2 + s) * 64 + lane;
            ah[i] = pa[0];
            am[i] = pa[8 * 64];
            al[i] = pa[16 * 64];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bf16x8 *pb = reinterpret_cast<const bf16x8 *>(st + kWgAImg) + ((4 * wn + j) * 2 + s) * 64 + lane;
            const bf16x8 bh = pb[0], bm = pb[16 * 64], bl = pb[32 * 64];
#pragma unroll
            for (int i = 0; i < 2; ++i) acc[i][j] = xpa_mfma_s3(ah[i], am[i], al[i], bh, bm, bl, acc[i][j]);
        }
    }
}

__global__ __launch_bounds__(512, 1) void s3_wgrad_ws_kernel(const float *__restrict__ A, int64_t lda,
                                                             const float *__restrict__ B, int64_t ldb, int64_t rows,
                                                             int64_t M, int slices, int64_t slice_rows,
                                                             float *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) char lds[2 * kWgStage];
    const int mtiles = (int)(M / kWgM);
    const int nblk = slices * mtiles;
    int L = blockIdx.x;
    if (nblk % 8 == 0) L = (blockIdx.x & 7) * (nblk >> 3) + (blockIdx.x >> 3);  // one slice's tiles on one XCD
    const int slice = L / mtiles, mt = L - slice * mtiles;
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const float *Am = A + (int64_t)mt * kWgM;
    const int64_t k0 = (int64_t)slice * slice_rows;
    const int64_t kend = min(rows, k0 + slice_rows);
    const int nch = kend > k0 ? (int)((kend - k0 + kWgKC - 1) / kWgKC) : 0;
    if (wave >= 4) {   // producers: the same barrier sequence as the consumers (1 + nch barriers)
        const int p = t - 256;
        float v[6][8];
        if (nch > 0) {
            wgw_load(v, Am, lda, B, ldb, k0, kend, p);
            wgw_store(lds, v, p);
            if (nch > 1) wgw_load(v, Am, lda, B, ldb, k0 + kWgKC, kend, p);
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll 1
        for (int c = 0; c < nch; ++c) {
            if (c + 1 < nch) {
                wgw_store(lds + ((c + 1) & 1) * kWgStage, v, p);
                if (c + 2 < nch) wgw_load(v, Am, lda, B, ldb, k0 + (int64_t)(c + 2) * kWgKC, kend, p);
            }
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
        return;
    }
    const int wm = wave & 1, wn = wave >> 1;
    f32x16 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    asm volatile("s_barrier" ::: "memory");
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
        wgw_chunk(lds + (c & 1) * kWgStage, acc, lane, wm, wn);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // done reading stage c & 1
    }
    float *o = out + ((int64_t)slice * M + (int64_t)mt * kWgM) * kN;
    const int h = lane >> 5, col = lane & 31;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = 64 * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
#pragma unroll
            for (int j = 0; j < 4; ++j) o[(int64_t)row * kN + 128 * wn + 32 * j + col] = acc[i][j][r];
        }
}

// K41V: K41 with vector staging and transposed fragment reads.  Each thread loads whole float4s of a row (k) of
// dz / x (6 dwordx4 per chunk instead of 24 k-strided dwords), splits them and writes the three bf16 planes k-major —
// [32 k rows][128 columns] tiles, 256-B rows XOR-swizzled by 16-B chunk (cdna_hip_programming.md T10 layout (b)) — with
// ds_write_b64; the MFMA fragments (8 consecutive k of one column) come back with ds_read_b64_tr_b16 (two per plane).
// Natural k order inside a step (lane half h: k 8h .. 8h + 7); the outputs carry K41's accuracy, not its bits.
constexpr int kVPlane = 32 * 128 * 2;                  // bytes of one [32][128] bf16 tile
constexpr int kVStage = 3 * kVPlane + 3 * 2 * kVPlane;  // A: 3 planes x 1 tile; B: 3 planes x 2 tiles = 72 KiB
typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

__device__ __forceinline__ int v_off(int row, int col) {   // byte offset of (row, col .. col + 3) in a [32][128] tile
    const int ch = col >> 3;
    return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) + 2 * (col & 7);
}

struct VUnits {
    float4 a[2], b[4];
    unsigned ok;   // bit u: unit u's row is inside the slice (a[0..1] = bits 0..1, b[0..3] = bits 2..5); applied at the
                   // split, not after the load, so no wait for the load sits in the loop body
};

__device__ __forceinline__ float4 v_zero_if(float4 v, bool keep) {
    return make_float4(keep ? v.x : 0.f, keep ? v.y : 0.f, keep ? v.z : 0.f, keep ? v.w : 0.f);
}

// s_idx (r05, K41V's row-index form): A's row r is row s_idx[r] of A (the slice's indices staged in LDS; B's rows
// are read directly)
__device__ __forceinline__ void v_load(VUnits &u, const float *__restrict__ A, int64_t lda, const float *__restrict__ B,
                                       int64_t ldb, int64_t k0, int64_t kend, int t,
                                       const int64_t *s_idx = nullptr) {
    unsigned ok = 0u;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int idx = t + 512 * j, k = idx >> 5, cq = idx & 31;
        const int64_t r = k0 + k;
        const int64_t rc = min(r, kend - 1);
        u.a[j] = *reinterpret_cast<const float4 *>(A + (s_idx != nullptr ? s_idx[rc] : rc) * lda + 4 * cq);
        ok |= (r < kend ? 1u : 0u) << j;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int idx = t + 512 * j, k = idx >> 6, nq = idx & 63;
        const int64_t r = k0 + k;
        u.b[j] = *reinterpret_cast<const float4 *>(B + min(r, kend - 1) * ldb + 4 * nq);
        ok |= (r < kend ? 1u : 0u) << (2 + j);
    }
    u.ok = ok;
}

// the three planes of 4 consecutive columns, each packed as 4 bf16 (8 B)
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void v_put(char *plane0, int plane_stride, int off, float4 v) {
    const float e[4] = {v.x, v.y, v.z, v.w};
    bf16x4 h, m, l;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        __bf16 a0, a1, a2;
        xpa_split3(e[j], a0, a1, a2);
        h[j] = a0;
        m[j] = a1;
        l[j] = a2;
    }
    *reinterpret_cast<bf16x4 *>(plane0 + off) = h;
    *reinterpret_cast<bf16x4 *>(plane0 + plane_stride + off) = m;
    *reinterpret_cast<bf16x4 *>(plane0 + 2 * plane_stride + off) = l;
}

__device__ __forceinline__ void v_store(char *st, const VUnits &u, int t) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int idx = t + 512 * j, k = idx >> 5, cq = idx & 31;
        v_put(st, kVPlane, v_off(k, 4 * cq), v_zero_if(u.a[j], (u.ok >> j) & 1u));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int idx = t + 512 * j, k = idx >> 6, n = 4 * (idx & 63);
        v_put(st + 3 * kVPlane, 2 * kVPlane, (n >> 7) * kVPlane + v_off(k, n & 127),
              v_zero_if(u.b[j], (u.ok >> (2 + j)) & 1u));
    }
}

__device__ __forceinline__ bf16x8 v_frag(const char *tile, int row0, int col) {
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s *)(tile + v_off(row0, col)));
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s *)(tile + v_off(row0 + 4, col)));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

__device__ __forceinline__ void v_chunk(const char *st, f32x16 (&acc)[2][2], int lane, int wm, int wn) {
    // lane 4q + p of 16-lane group g supplies row 8h + 4jj + q (h = g >> 1) and columns 16 (g & 1) + 4p .. + 3 of its
    // 32-column block; it receives column 16 (g & 1) + (lane & 15): the MFMA's lane map (row / column lane & 31, k 8h + j)
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3, h = lane >> 5;
    const int cofs = 16 * (g & 1) + 4 * p;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const int row0 = 16 * s + 8 * h + q;
        bf16x8 ah[2], am[2], al[2], bh[2], bm[2], bl[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int col = 32 * (2 * wm + i) + cofs;
            ah[i] = v_frag(st, row0, col);
            am[i] = v_frag(st + kVPlane, row0, col);
            al[i] = v_frag(st + 2 * kVPlane, row0, col);
            const int n = 32 * (2 * wn + i) + cofs;
            const char *bt = st + 3 * kVPlane + (n >> 7) * kVPlane;
            bh[i] = v_frag(bt, row0, n & 127);
            bm[i] = v_frag(bt + 2 * kVPlane, row0, n & 127);
            bl[i] = v_frag(bt + 4 * kVPlane, row0, n & 127);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = xpa_mfma_s3(ah[i], am[i], al[i], bh[j], bm[j], bl[j], acc[i][j]);
    }
}

// SCHED (r04, the default; probe bit 64 selects SCHED = 0): the loop body as ONE scheduling region (the next stage's split / stores and the chunk-after's
// loads unconditional: past the last chunk they rewrite the idle stage / re-read clamped rows) with
// sched_group_barrier placing ~5 VALU after each MFMA, so the split of chunk c + 1 issues inside chunk c's MFMA gaps
// (hipcc's own order: all 48 MFMAs, then ~250 VALU and the stores, with the matrix pipe idle — both waves of a SIMD
// reach that phase together after the chunk barrier).
// v_chunk with v_store's six float4 splits (each 3 ds_write_b64) placed one after each 6-MFMA accumulator block, in
// segments the scheduler may not merge (sched_barrier), and the second k step's fragment reads one segment in
__device__ __forceinline__ void v_frags(const char *st, int s, int lane, int wm, int wn, bf16x8 (&ah)[2],
                                        bf16x8 (&am)[2], bf16x8 (&al)[2], bf16x8 (&bh)[2], bf16x8 (&bm)[2],
                                        bf16x8 (&bl)[2]) {
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3, h = lane >> 5;
    const int cofs = 16 * (g & 1) + 4 * p;
    const int row0 = 16 * s + 8 * h + q;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int col = 32 * (2 * wm + i) + cofs;
        ah[i] = v_frag(st, row0, col);
        am[i] = v_frag(st + kVPlane, row0, col);
        al[i] = v_frag(st + 2 * kVPlane, row0, col);
        const int n = 32 * (2 * wn + i) + cofs;
        const char *bt = st + 3 * kVPlane + (n >> 7) * kVPlane;
        bh[i] = v_frag(bt, row0, n & 127);
        bm[i] = v_frag(bt + 2 * kVPlane, row0, n & 127);
        bl[i] = v_frag(bt + 4 * kVPlane, row0, n & 127);
    }
}

__device__ __forceinline__ void v_put_unit(char *nx, const VUnits &u, int t, int unit) {
    const bool keep = (u.ok >> unit) & 1u;
    if (unit < 2) {
        const int idx = t + 512 * unit, k = idx >> 5, cq = idx & 31;
        v_put(nx, kVPlane, v_off(k, 4 * cq), v_zero_if(u.a[unit], keep));
    } else {
        const int j = unit - 2, idx = t + 512 * j, k = idx >> 6, n = 4 * (idx & 63);
        v_put(nx + 3 * kVPlane, 2 * kVPlane, (n >> 7) * kVPlane + v_off(k, n & 127), v_zero_if(u.b[j], keep));
    }
}

// (and the loads of the chunk after next issued in segment 6, once the six units are split, so they fly during the
// last two MFMA blocks)
__device__ __forceinline__ void v_chunk_il(const char *st, char *nx, VUnits &u, f32x16 (&acc)[2][2], int lane, int wm,
                                           int wn, int t, const float *__restrict__ A, int64_t lda,
                                           const float *__restrict__ B, int64_t ldb, int64_t k_next, int64_t kend,
                                           const int64_t *s_idx = nullptr) {
    bf16x8 ah[2][2], am[2][2], al[2][2], bh[2][2], bm[2][2], bl[2][2];
    v_frags(st, 0, lane, wm, wn, ah[0], am[0], al[0], bh[0], bm[0], bl[0]);
#pragma unroll
    for (int seg = 0; seg < 8; ++seg) {
        const int s = seg >> 2, i = (seg >> 1) & 1, j = seg & 1;
        acc[i][j] = xpa_mfma_s3(ah[s][i], am[s][i], al[s][i], bh[s][j], bm[s][j], bl[s][j], acc[i][j]);
        if (seg < 6) v_put_unit(nx, u, t, seg);
        if (seg == 1) v_frags(st, 1, lane, wm, wn, ah[1], am[1], al[1], bh[1], bm[1], bl[1]);
        if (seg == 6) v_load(u, A, lda, B, ldb, k_next, kend, t, s_idx);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// IDX (r05): A's rows through aidx (the minibatch rows of the rollout buffer: C4's wide trunk dW without a gathered
// copy); the slice's indices are staged in LDS once (slice_rows <= kVIdxMax)
constexpr int kVIdxMax = 1536;   // 12 KiB beside the 144 KiB of stages
template <int SCHED = 0, bool IDX = false>
__global__ __launch_bounds__(512, 1) void s3_wgrad_v_kernel(const float *__restrict__ A, int64_t lda,
                                                            const float *__restrict__ B, int64_t ldb, int64_t rows,
                                                            int64_t M, int slices, int64_t slice_rows,
                                                            float *__restrict__ out,
                                                            const int64_t *__restrict__ aidx = nullptr) {
    __shared__ __attribute__((aligned(16))) char lds[2 * kVStage + (IDX ? kVIdxMax * 8 : 0)];
    const int mtiles = (int)(M / kWgM);
    const int nblk = slices * mtiles;
    int L = blockIdx.x;
    if (nblk % 8 == 0) L = (blockIdx.x & 7) * (nblk >> 3) + (blockIdx.x >> 3);  // one slice's tiles on one XCD
    const int slice = L / mtiles, mt = L - slice * mtiles;
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int wm = wave & 1, wn = wave >> 1;
    const float *Am = A + (int64_t)mt * kWgM;
    const int64_t k0 = (int64_t)slice * slice_rows;
    const int64_t kend = min(rows, k0 + slice_rows);
    const int nch = kend > k0 ? (int)((kend - k0 + kWgKC - 1) / kWgKC) : 0;
    const int64_t *s_idx = nullptr;   // IDX: s_idx[r] (r in [k0, kend)) = aidx[r], from LDS
    if constexpr (IDX) {
        int64_t *si = reinterpret_cast<int64_t *>(lds + 2 * kVStage);
        for (int64_t r = k0 + t; r < kend; r += 512) si[r - k0] = aidx[r];
        __syncthreads();
        s_idx = si - k0;
    }
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    VUnits u;
    if (nch > 0) {
        v_load(u, Am, lda, B, ldb, k0, kend, t, s_idx);
        v_store(lds, u, t);
        if (nch > 1) v_load(u, Am, lda, B, ldb, k0 + kWgKC, kend, t, s_idx);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
        if constexpr (!SCHED) v_chunk(lds + (c & 1) * kVStage, acc, lane, wm, wn);
        if constexpr (SCHED) {
            v_chunk_il(lds + (c & 1) * kVStage, lds + ((c + 1) & 1) * kVStage, u, acc, lane, wm, wn, t, Am, lda, B, ldb,
                       k0 + (int64_t)(c + 2) * kWgKC, kend, s_idx);
        } else if (c + 1 < nch) {
            v_store(lds + ((c + 1) & 1) * kVStage, u, t);
            if (c + 2 < nch) v_load(u, Am, lda, B, ldb, k0 + (int64_t)(c + 2) * kWgKC, kend, t, s_idx);
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    float *o = out + ((int64_t)slice * M + (int64_t)mt * kWgM) * kN;
    const int h = lane >> 5, col = lane & 31;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = 64 * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
#pragma unroll
            for (int j = 0; j < 2; ++j) o[(int64_t)row * kN + 64 * wn + 32 * j + col] = acc[i][j][r];
        }
}

// K41V-PP (r05): K41V's staging and fragments with the two waves of each SIMD one phase apart (K40 / K42's ping-pong):
// half 0 (waves 0-3) runs chunk c's MFMAs in phase 2c and stages its share of chunk c + 1 (its float4 units: the same
// thread-to-unit map as K41V, so each half writes half of the chunk's k rows) in phase 2c + 1; half 1 stages in 2c and
// computes in 2c + 1.  Chunk c + 1 is complete after phase 2c + 1; it reuses chunk c - 1's stage, which half 1 read
// last in phase 2c - 1.  One raw barrier per phase (lgkmcnt(0) first: the stage writes landed); each thread's global
// loads of chunk c + 2 are issued right after it stored its share of c + 1, two phases before their use.  Same
// fragments, products and order per accumulator as K41V's plain schedule: the same outputs bit for bit.
__global__ __launch_bounds__(512, 1) void s3_wgrad_pp_kernel(const float *__restrict__ A, int64_t lda,
                                                             const float *__restrict__ B, int64_t ldb, int64_t rows,
                                                             int64_t M, int slices, int64_t slice_rows,
                                                             float *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) char lds[2 * kVStage];
    const int mtiles = (int)(M / kWgM);
    const int nblk = slices * mtiles;
    int L = blockIdx.x;
    if (nblk % 8 == 0) L = (blockIdx.x & 7) * (nblk >> 3) + (blockIdx.x >> 3);  // one slice's tiles on one XCD
    const int slice = L / mtiles, mt = L - slice * mtiles;
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int wm = wave & 1, wn = wave >> 1;
    const float *Am = A + (int64_t)mt * kWgM;
    const int64_t k0 = (int64_t)slice * slice_rows;
    const int64_t kend = min(rows, k0 + slice_rows);
    const int nch = kend > k0 ? (int)((kend - k0 + kWgKC - 1) / kWgKC) : 0;
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    VUnits u;
    if (nch > 0) {
        v_load(u, Am, lda, B, ldb, k0, kend, t);
        v_store(lds, u, t);
        if (nch > 1) v_load(u, Am, lda, B, ldb, k0 + kWgKC, kend, t);
        bar();
        if (wave < 4) {
#pragma unroll 1
            for (int c = 0; c < nch; ++c) {
                v_chunk(lds + (c & 1) * kVStage, acc, lane, wm, wn);
                bar();
                if (c + 1 < nch) {
                    v_store(lds + ((c + 1) & 1) * kVStage, u, t);
                    if (c + 2 < nch) v_load(u, Am, lda, B, ldb, k0 + (int64_t)(c + 2) * kWgKC, kend, t);
                }
                bar();
            }
        } else {
#pragma unroll 1
            for (int c = 0; c < nch; ++c) {
                if (c + 1 < nch) {
                    v_store(lds + ((c + 1) & 1) * kVStage, u, t);
                    if (c + 2 < nch) v_load(u, Am, lda, B, ldb, k0 + (int64_t)(c + 2) * kWgKC, kend, t);
                }
                bar();
                v_chunk(lds + (c & 1) * kVStage, acc, lane, wm, wn);
                bar();
            }
        }
    }
    float *o = out + ((int64_t)slice * M + (int64_t)mt * kWgM) * kN;
    const int h = lane >> 5, col = lane & 31;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = 64 * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
#pragma unroll
            for (int j = 0; j < 2; ++j) o[(int64_t)row * kN + 64 * wn + 32 * j + col] = acc[i][j][r];
        }
}

// ---- K41P (r05): the paired hidden layer's weight gradient with the critic's half factored --------------------------
// dW_pair = dz_pair^T h splits into the actor's [256, 256] (dz_a^T h, K41V's six-product split, interleaved schedule) and
// the critic's: with dz_c[r, c] = dv[r] wc[c] (slope + (1 - slope) m[r, c]) (the critic head's one output unit,
// LeakyReLU hidden layer, m = [h_c > 0] from its sign bits),
//     dW_c[c, j] = wc[c] ((1 - slope) sum_r m[r, c] Y[r, j] + slope sum_r Y[r, j]),  Y = dv (.) h   (one f32 rounding)
// where m^T Y takes THREE bf16 products (m exact in bf16: m Y_lo, m Y_mid, m Y_hi) instead of six and dz_c is never
// read.  One launch: blocks [0, 2 sa) are the actor's (2 column tiles of 128 x sa slices), blocks [2 sa, 2 sa + 2 sc)
// the critic's (sc slices, ~2x the rows per slice: the same MFMA work per block); each critic block also forms its
// slice's column sums of Y (per-thread float4 over its staged rows, then the 8 waves in order) and writes its partial
// already as wc[c] ((1 - slope) P + slope colsum), so the caller's fixed-order slice sum gives dW_c.
struct CUnits {   // the critic's staging units: A = 4 mask bits per unit, B = Y rows (h float4 times dv of the row)
    unsigned abits[2];
    float4 b[4];
    float bdv[4];
    unsigned ok;
};

__device__ __forceinline__ void c_load(CUnits &u, const unsigned *__restrict__ cmask, const float *__restrict__ cdv,
                                       int mt, const float *__restrict__ B, int64_t ldb, int64_t k0, int64_t kend,
                                       int t) {
    unsigned ok = 0u;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int idx = t + 512 * j, k = idx >> 5, cq = idx & 31;
        const int64_t r = k0 + k;
        const int c = mt * kWgM + 4 * cq;
        u.abits[j] = cmask[min(r, kend - 1) * 8 + (c >> 5)] >> (c & 31);
        ok |= (r < kend ? 1u : 0u) << j;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int idx = t + 512 * j, k = idx >> 6, nq = idx & 63;
        const int64_t r = k0 + k;
        const int64_t rc = min(r, kend - 1);
        u.b[j] = *reinterpret_cast<const float4 *>(B + rc * ldb + 4 * nq);
        u.bdv[j] = cdv[rc];
        ok |= (r < kend ? 1u : 0u) << (2 + j);
    }
    u.ok = ok;
}

// unit `unit` of the critic's staging into stage nx (A: the hi plane only — m is 0 / 1 — B: the three planes of Y);
// ysum accumulates the thread's Y columns 4 (t & 63) .. + 3 over its rows
__device__ __forceinline__ void c_put_unit(char *nx, const CUnits &u, int t, int unit, float4 &ysum) {
    const bool keep = (u.ok >> unit) & 1u;
    if (unit < 2) {
        const int idx = t + 512 * unit, k = idx >> 5, cq = idx & 31;
        const unsigned bits = keep ? u.abits[unit] : 0u;
        const unsigned lo = ((bits & 1u) * 0x3F80u) | (((bits >> 1) & 1u) * 0x3F800000u);
        const unsigned hi = (((bits >> 2) & 1u) * 0x3F80u) | (((bits >> 3) & 1u) * 0x3F800000u);
        *reinterpret_cast<uint2 *>(nx + v_off(k, 4 * cq)) = make_uint2(lo, hi);
    } else {
        const int j = unit - 2, idx = t + 512 * j, k = idx >> 6, n = 4 * (idx & 63);
        const float d = u.bdv[j];
        float4 y = make_float4(d * u.b[j].x, d * u.b[j].y, d * u.b[j].z, d * u.b[j].w);
        y = v_zero_if(y, keep);
        ysum.x += y.x;
        ysum.y += y.y;
        ysum.z += y.z;
        ysum.w += y.w;
        v_put(nx + 3 * kVPlane, 2 * kVPlane, (n >> 7) * kVPlane + v_off(k, n & 127), y);
    }
}

// K41V's interleaved chunk for the critic: 8 segments of (3 MFMAs of one accumulator: m Y_lo, m Y_mid, m Y_hi) + one
// staging unit of the next stage; the second k step's fragments read in segment 1, the loads of the chunk after next
// in segment 6
__device__ __forceinline__ void c_chunk_il(const char *st, char *nx, CUnits &u, f32x16 (&acc)[2][2], int lane, int wm,
                                           int wn, int t, const unsigned *__restrict__ cmask,
                                           const float *__restrict__ cdv, int mt, const float *__restrict__ B,
                                           int64_t ldb, int64_t k_next, int64_t kend, float4 &ysum) {
    bf16x8 ah[2][2], am[2][2], al[2][2], bh[2][2], bm[2][2], bl[2][2];
    v_frags(st, 0, lane, wm, wn, ah[0], am[0], al[0], bh[0], bm[0], bl[0]);
#pragma unroll
    for (int seg = 0; seg < 8; ++seg) {
        const int s = seg >> 2, i = (seg >> 1) & 1, j = seg & 1;
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s][i], bl[s][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s][i], bm[s][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s][i], bh[s][j], acc[i][j], 0, 0, 0);
        if (seg < 6) c_put_unit(nx, u, t, seg, ysum);
        if (seg == 1) v_frags(st, 1, lane, wm, wn, ah[1], am[1], al[1], bh[1], bm[1], bl[1]);
        if (seg == 6) c_load(u, cmask, cdv, mt, B, ldb, k_next, kend, t);
        __builtin_amdgcn_sched_barrier(0);
    }
}

__global__ __launch_bounds__(512, 1) void s3_wgrad_pair_kernel(const float *__restrict__ A, int64_t lda,
                                                               const float *__restrict__ B, int64_t ldb, int64_t rows,
                                                               int sa, int64_t per_a, int sc, int64_t per_c,
                                                               const unsigned *__restrict__ cmask,
                                                               const float *__restrict__ cdv,
                                                               const float *__restrict__ cwc, float cslope,
                                                               float *__restrict__ out_a, float *__restrict__ out_c) {
    __shared__ __attribute__((aligned(16))) char lds[2 * kVStage];
    const int nblk = 2 * (sa + sc);
    int L = blockIdx.x;
    if (nblk % 8 == 0) L = (blockIdx.x & 7) * (nblk >> 3) + (blockIdx.x >> 3);   // a slice's 2 tiles on one XCD
    const bool crit = L >= 2 * sa;
    const int Lr = crit ? L - 2 * sa : L;
    const int slice = Lr >> 1, mt = Lr & 1;
    const int64_t per = crit ? per_c : per_a;
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int wm = wave & 1, wn = wave >> 1;
    const int64_t k0 = (int64_t)slice * per;
    const int64_t kend = min(rows, k0 + per);
    const int nch = kend > k0 ? (int)((kend - k0 + kWgKC - 1) / kWgKC) : 0;
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    float4 ysum = make_float4(0.f, 0.f, 0.f, 0.f);
    if (!crit) {   // K41V (interleaved schedule) on the actor's columns
        const float *Am = A + (int64_t)mt * kWgM;
        VUnits u;
        if (nch > 0) {
            v_load(u, Am, lda, B, ldb, k0, kend, t);
            v_store(lds, u, t);
            if (nch > 1) v_load(u, Am, lda, B, ldb, k0 + kWgKC, kend, t);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
#pragma unroll 1
        for (int c = 0; c < nch; ++c) {
            v_chunk_il(lds + (c & 1) * kVStage, lds + ((c + 1) & 1) * kVStage, u, acc, lane, wm, wn, t, Am, lda, B, ldb,
                       k0 + (int64_t)(c + 2) * kWgKC, kend);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
    } else {
        CUnits u;
        if (nch > 0) {
            c_load(u, cmask, cdv, mt, B, ldb, k0, kend, t);
#pragma unroll
            for (int unit = 0; unit < 6; ++unit) c_put_unit(lds, u, t, unit, ysum);
            if (nch > 1) c_load(u, cmask, cdv, mt, B, ldb, k0 + kWgKC, kend, t);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
#pragma unroll 1
        for (int c = 0; c < nch; ++c) {
            // past the last chunk the staging rewrites the idle stage from rows >= kend: zeros (ok bits), so the
            // column sums are unaffected
            c_chunk_il(lds + (c & 1) * kVStage, lds + ((c + 1) & 1) * kVStage, u, acc, lane, wm, wn, t, cmask, cdv, mt,
                       B, ldb, k0 + (int64_t)(c + 2) * kWgKC, kend, ysum);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
    }
    const int h = lane >> 5, col = lane & 31;
    if (!crit) {
        float *o = out_a + ((int64_t)slice * 256 + (int64_t)mt * kWgM) * kN;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = 64 * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
#pragma unroll
                for (int j = 0; j < 2; ++j) o[(int64_t)row * kN + 64 * wn + 32 * j + col] = acc[i][j][r];
            }
        return;
    }
    // the slice's column sums of Y: thread t holds columns 4 (t & 63) .. + 3 over the rows of its units; the 8 threads
    // of a column quad (t >> 6 = 0 .. 7) added in order
    float *s_ys = reinterpret_cast<float *>(lds);   // [8][256], the ring is free (every wave passed the last barrier)
    *reinterpret_cast<float4 *>(s_ys + (t >> 6) * 256 + 4 * (t & 63)) = ysum;
    __syncthreads();
    float *s_cs = s_ys + 8 * 256;   // [256]
    if (t < 256) {
        float sum = s_ys[t];
#pragma unroll
        for (int w = 1; w < 8; ++w) sum += s_ys[w * 256 + t];
        s_cs[t] = sum;
    }
    __syncthreads();
    float *o = out_c + ((int64_t)slice * 256 + (int64_t)mt * kWgM) * kN;
    const float a1 = 1.0f - cslope;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = 64 * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
            const float w = cwc[mt * kWgM + row];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int n = 64 * wn + 32 * j + col;
                o[(int64_t)row * kN + n] = w * (a1 * acc[i][j][r] + cslope * s_cs[n]);
            }
        }
}

}  // namespace

// the split-K slice count of xpa_s3_wgrad for this shape (the caller's workspace: slices x m x 256 floats)
XPA_API int64_t xpa_s3_wgrad_num_slices(int64_t rows, int64_t m) {
    if (rows <= 0 || m <= 0 || m % kWgM) return 0;
    int64_t s = 256 / (m / kWgM);
    s = s < 1 ? 1 : (s > 64 ? 64 : s);
    while (s > 1 && rows / s < 4 * kWgKC) s >>= 1;
    return s;
}

XPA_API int xpa_s3_wgrad(const float *a, int64_t lda, const float *b, int64_t ldb, int64_t rows, int64_t m, int64_t n,
                         int64_t slices, float *out, xpa_stream_t stream) {
    if (!a || !b || !out || rows <= 0 || m <= 0 || m % kWgM || n != kN || lda < m || ldb < n || slices < 1 ||
        slices > 4096)
        return (int)hipErrorInvalidValue;
    int64_t per = (rows + slices - 1) / slices;
    per = (per + kWgKC - 1) / kWgKC * kWgKC;
    const dim3 grid((unsigned)(slices * (m / kWgM))), block(512);
    // the production form is K41V (float4 staging; rows 16-B aligned); probe bits select the others: 8 K41W,
    // 32 or any of 1 / 2 / 4 the register-staged K41 (and its probes)
    const bool vec_ok = lda % 4 == 0 && ldb % 4 == 0 &&
                        ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) == 0;
    if (vec_ok && (g_s3_probe & (1 | 2 | 4 | 8 | 32)) == 0) {   // K41V (bit 64: without its interleaved schedule)
        if (g_s3_probe & 256)   // the ping-pong form (r05)
            s3_wgrad_pp_kernel<<<grid, block, 0, stream>>>(a, lda, b, ldb, rows, m, (int)slices, per, out);
        else if (g_s3_probe & 64)   // hipcc's own schedule (r04p: 115 us vs 104 interleaved at C2)
            s3_wgrad_v_kernel<0><<<grid, block, 0, stream>>>(a, lda, b, ldb, rows, m, (int)slices, per, out);
        else
            s3_wgrad_v_kernel<1><<<grid, block, 0, stream>>>(a, lda, b, ldb, rows, m, (int)slices, per, out);
        return xpa_launch_status();
    }
    if (g_s3_probe & 8) {   // the wave-specialised form (K41W)
        s3_wgrad_ws_kernel<<<grid, block, 0, stream>>>(a, lda, b, ldb, rows, m, (int)slices, per, out);
        return xpa_launch_status();
    }
    switch (g_s3_probe & 7) {
#define XPA_WG(P) case P: s3_wgrad_kernel<P><<<grid, block, 0, stream>>>(a, lda, b, ldb, rows, m, (int)slices, per, out); break;
        XPA_WG(1) XPA_WG(2) XPA_WG(3) XPA_WG(4) XPA_WG(6)
#undef XPA_WG
        default: s3_wgrad_kernel<0><<<grid, block, 0, stream>>>(a, lda, b, ldb, rows, m, (int)slices, per, out);
    }
    return xpa_launch_status();
}

// K41V over rows narrower than the row tiles (r06: C3's first fc layer, dW^T = flat^T g with flat [B, 3136]): m may exceed
// lda by < 128 — the last row tile reads past each row into the next (finite values of the same buffer) and, after the
// last row, into slack the caller guarantees readable (and finite); those output rows are garbage, dropped by the
// caller's finalize map.  No per-slice row limit (the rows are read in place, not through an index stage).
XPA_API int xpa_s3_wgrad_padded(const float *a, int64_t lda, const float *b, int64_t ldb, int64_t rows, int64_t m,
                                int64_t n, int64_t slices, float *out, xpa_stream_t stream) {
    if (!a || !b || !out || rows <= 0 || m <= 0 || m % kWgM || n != kN || lda < 4 || m > lda + kWgM || ldb < n ||
        slices < 1 || slices > 4096 || (lda & 3) || (ldb & 3) ||
        ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15))
        return (int)hipErrorInvalidValue;
    int64_t per = (rows + slices - 1) / slices;
    per = (per + kWgKC - 1) / kWgKC * kWgKC;
    const dim3 grid((unsigned)(slices * (m / kWgM))), block(512);
    s3_wgrad_v_kernel<1><<<grid, block, 0, stream>>>(a, lda, b, ldb, rows, m, (int)slices, per, out);
    return xpa_launch_status();
}

// K41V's row-index form (r05): A's row r is row aidx[r] of a (C4's trunk dW straight from the rollout buffer); m may
// exceed a's row width by < 128 (the last row tile reads past each row: the caller guarantees readable slack after the
// buffer's last row; those output rows are garbage and dropped by the caller's finalize map); rows per slice <= 1536
XPA_API int xpa_s3_wgrad_rows(const float *a, int64_t lda, const int64_t *aidx, const float *b, int64_t ldb,
                              int64_t rows, int64_t m, int64_t n, int64_t slices, float *out, xpa_stream_t stream) {
    if (!a || !aidx || !b || !out || rows <= 0 || m <= 0 || m % kWgM || n != kN || lda < 4 || m > lda + kWgM ||
        ldb < n || slices < 1 || slices > 4096 || (lda & 3) || (ldb & 3) ||
        ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15))
        return (int)hipErrorInvalidValue;
    int64_t per = (rows + slices - 1) / slices;
    per = (per + kWgKC - 1) / kWgKC * kWgKC;
    if (per > kVIdxMax) return (int)hipErrorInvalidValue;
    const dim3 grid((unsigned)(slices * (m / kWgM))), block(512);
    s3_wgrad_v_kernel<1, true><<<grid, block, 0, stream>>>(a, lda, b, ldb, rows, m, (int)slices, per, out, aidx);
    return xpa_launch_status();
}

// K41P (r05): slice counts of xpa_s3_wgrad_pair for `rows` (sa actor, sc critic slices; their rows per slice in
// per_a / per_c, multiples of 32): 2 (sa + sc) <= 256 blocks with ~2x the critic's rows per slice (3 products vs 6)
XPA_API int xpa_s3_wgrad_pair_slices(int64_t rows, int64_t *sa, int64_t *sc, int64_t *per_a, int64_t *per_c) {
    if (rows <= 0 || !sa || !sc || !per_a || !per_c) return (int)hipErrorInvalidValue;
    auto fit = [&](int64_t want, int64_t *s, int64_t *per) {
        int64_t n = want < 1 ? 1 : want;
        while (n > 1 && rows / n < 4 * kWgKC) n >>= 1;
        int64_t p = (rows + n - 1) / n;
        p = (p + kWgKC - 1) / kWgKC * kWgKC;
        *per = p;
        *s = (rows + p - 1) / p;
    };
    fit(g_pair_sa, sa, per_a);
    fit(128 - g_pair_sa, sc, per_c);
    return 0;
}

// the actor's share of K41P's 128 slice pairs (tuning: a critic chunk stages as many units as an actor chunk but runs
// half the MFMAs, so the balance sits between the MFMA ratio 85 / 43 and equal rows)
XPA_API int xpa_s3_wgrad_pair_tune(int sa_target) {
    if (sa_target < 8 || sa_target > 120) return (int)hipErrorInvalidValue;
    g_pair_sa = sa_target;
    return 0;
}

// dz_a [rows, 256] (row stride lda, the actor's half), h [rows, 256] (ldb), crit_mask [rows, 8] + crit_dv [rows]
// (xpa_head_gemm_s3q_critic_mask), crit_wc [256] (the critic's output weights), crit_slope (its hidden activation's):
// out_a [sa, 256, 256] (slices of dz_a^T h), out_c [sc, 256, 256] (slices of dW_c, wc and the slope term applied)
XPA_API int xpa_s3_wgrad_pair(const float *dz_a, int64_t lda, const float *h, int64_t ldb, int64_t rows,
                              const unsigned *crit_mask, const float *crit_dv, const float *crit_wc, float crit_slope,
                              int64_t sa, int64_t per_a, int64_t sc, int64_t per_c, float *out_a, float *out_c,
                              xpa_stream_t stream) {
    if (!dz_a || !h || !crit_mask || !crit_dv || !crit_wc || !out_a || !out_c || rows <= 0 || lda < 256 || ldb < 256 ||
        (lda & 3) || (ldb & 3) || ((reinterpret_cast<uintptr_t>(dz_a) | reinterpret_cast<uintptr_t>(h)) & 15) ||
        sa < 1 || sc < 1 || per_a % kWgKC || per_c % kWgKC || sa * per_a < rows || sc * per_c < rows ||
        2 * (sa + sc) > 4096)
        return (int)hipErrorInvalidValue;
    s3_wgrad_pair_kernel<<<dim3((unsigned)(2 * (sa + sc))), dim3(512), 0, stream>>>(
        dz_a, lda, h, ldb, rows, (int)sa, per_a, (int)sc, per_c, crit_mask, crit_dv, crit_wc, crit_slope, out_a, out_c);
    return xpa_launch_status();
}

XPA_API int xpa_s3_probe(int mask) {
    g_s3_probe = mask;
    return 0;
}

XPA_API int64_t xpa_s3_split_bytes(int64_t k, int64_t n) {
    return k * n * 3 * 2;
}

XPA_API int xpa_s3_split_batch_scaled(int n_mat, const float *const *b, const int64_t *k, const int64_t *sk,
                                      const int64_t *sn, void *const *out, const float *const *rs_w, const float *rs_a,
                                      const int64_t *rs_from, float *cs_out, float cs_slope, xpa_stream_t stream);
// n_mat <= 4 matrices B_i [k_i, 256] (element (r, c) at b_i[r sk_i + c sn_i]) split into out_i in one launch
XPA_API int xpa_s3_split_batch(int n_mat, const float *const *b, const int64_t *k, const int64_t *sk, const int64_t *sn,
                               void *const *out, xpa_stream_t stream) {
    return xpa_s3_split_batch_scaled(n_mat, b, k, sk, sn, out, nullptr, nullptr, nullptr, nullptr, 0.f, stream);
}

// xpa_s3_split_batch with per-matrix row scales (rs_w[i] nullable: rows k >= rs_from[i] times rs_a[i] * rs_w[i][k -
// rs_from[i]]) and, with cs_out, cs_out[j] = cs_slope * sum_c rs_w[c] B[rs_from + c][j] of the first scaled matrix
namespace {
int split_batch_impl(int n_mat, const float *const *b, const int64_t *k, const int64_t *kv, const int64_t *sk,
                     const int64_t *sn, void *const *out, const float *const *rs_w, const float *rs_a,
                     const int64_t *rs_from, float *cs_out, float cs_slope, xpa_stream_t stream) {
    if (n_mat < 1 || n_mat > 4 || !b || !k || !sk || !sn || !out) return (int)hipErrorInvalidValue;
    SplitBatch sb{};
    sb.n = n_mat;
    sb.cs_out = cs_out;
    sb.cs_slope = cs_slope;
    bool any_rs = false;
    for (int i = 0; i < n_mat; ++i) {
        sb.rs_w[i] = rs_w ? rs_w[i] : nullptr;
        sb.rs_a[i] = rs_w && rs_w[i] ? rs_a[i] : 1.f;
        sb.rs_from[i] = rs_w && rs_w[i] ? rs_from[i] : 0;
        if (sb.rs_w[i]) {
            if (sb.rs_from[i] < 0 || sb.rs_from[i] >= k[i]) return (int)hipErrorInvalidValue;
            any_rs = true;
        }
    }
    if (cs_out && !any_rs) return (int)hipErrorInvalidValue;
    int64_t kmax = 0;
    for (int i = 0; i < n_mat; ++i) {
        if (!b[i] || !out[i] || k[i] <= 0 || k[i] % kKC) return (int)hipErrorInvalidValue;
        sb.b[i] = b[i];
        sb.k[i] = k[i];
        sb.sk[i] = sk[i];
        sb.sn[i] = sn[i];
        sb.kv[i] = kv ? kv[i] : k[i];
        if (sb.kv[i] < 1 || sb.kv[i] > k[i] || (sb.rs_w[i] && sb.kv[i] != k[i])) return (int)hipErrorInvalidValue;
        sb.out[i] = static_cast<__bf16 *>(out[i]);
        kmax = k[i] > kmax ? k[i] : kmax;
    }
    const int64_t total = (kmax / kKC) * kN * 2;
    int64_t gx = (total + 255) / 256;
    if (cs_out && gx < 8) gx = 8;   // the cs row uses 8 blocks
    split_batch_kernel<<<dim3((unsigned)gx, (unsigned)(n_mat + (cs_out ? 1 : 0))), dim3(256), 0, stream>>>(sb);
    return xpa_launch_status();
}
}  // namespace

XPA_API int xpa_s3_split_batch_scaled(int n_mat, const float *const *b, const int64_t *k, const int64_t *sk,
                                      const int64_t *sn, void *const *out, const float *const *rs_w, const float *rs_a,
                                      const int64_t *rs_from, float *cs_out, float cs_slope, xpa_stream_t stream) {
    return split_batch_impl(n_mat, b, k, nullptr, sk, sn, out, rs_w, rs_a, rs_from, cs_out, cs_slope, stream);
}

// r05 (C4 trunk): xpa_s3_split_batch where matrix i holds kv[i] <= k[i] rows (element (r, c) at b_i[r sk_i + c sn_i],
// r < kv_i) and its planes cover k_i rows, rows kv_i .. k_i - 1 zero (a K that is not a multiple of 16 padded up)
XPA_API int xpa_s3_split_batch_padded(int n_mat, const float *const *b, const int64_t *k, const int64_t *kv,
                                      const int64_t *sk, const int64_t *sn, void *const *out, xpa_stream_t stream) {
    if (!kv) return (int)hipErrorInvalidValue;
    return split_batch_impl(n_mat, b, k, kv, sk, sn, out, nullptr, nullptr, nullptr, nullptr, 0.f, stream);
}

XPA_API int xpa_s3_split_b(const float *b, int64_t k, int64_t n, int64_t sk, int64_t sn, void *out,
                           xpa_stream_t stream) {
    if (!b || !out || k <= 0 || k % kKC != 0 || n != kN) return (int)hipErrorInvalidValue;
    const int64_t total = (k / kKC) * kN * 2;
    split_b_kernel<<<dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream>>>(b, k, sk, sn,
                                                                                    static_cast<__bf16 *>(out));
    return xpa_launch_status();
}

XPA_API int64_t xpa_s3_gemm_trunk_bwd_num_partials(int64_t rows) {
    return rows > 0 ? (rows + 255) / 256 : 0;
}

// K42: the dX GEMM g = dz . B (B split, k % 16 == 0, n = 256) and the first representation layer's backward on it:
// partial_dw [G, 256 * d_in] (W1's layout [256][d_in]) and partial_db [G, 256], G = xpa_s3_gemm_trunk_bwd_num_partials
XPA_API int xpa_s3_gemm_trunk_bwd(const float *dz, int64_t ldz, const void *b_split, int64_t k, const float *h,
                                  int64_t ldh, const float *x, int64_t ldx, int64_t rows, int64_t d_in, int act,
                                  float slope, float *partial_dw, float *partial_db, xpa_stream_t stream) {
    if (!dz || !b_split || !h || !x || !partial_dw || !partial_db || rows <= 0 || k <= 0 || k % kKC != 0 ||
        ldz < k || (ldz & 3) || (reinterpret_cast<uintptr_t>(dz) & 15) || ldh < kN || d_in < 1 || d_in > 32 ||
        ldx < d_in || act < 0 || act > 2 || k / kKC > (1 << 20))
        return (int)hipErrorInvalidValue;
    const dim3 grid((unsigned)xpa_s3_gemm_trunk_bwd_num_partials(rows)), block(512);
    const __bf16 *bs = static_cast<const __bf16 *>(b_split);
    const int nch = (int)(k / kKC);
#define XPA_TB(A_) s3_gemm_trunk_bwd_kernel<A_><<<grid, block, 0, stream>>>(dz, ldz, bs, rows, nch, h, ldh, x, ldx, \
                                                                          (int)d_in, slope, partial_dw, partial_db)
    if (act == 0) XPA_TB(0);
    else if (act == 1) XPA_TB(1);
    else XPA_TB(2);
#undef XPA_TB
    return xpa_launch_status();
}

// K42S: xpa_s3_gemm_trunk_bwd with act' from h's sign bits (xpa_head_gemm_s3r_actor's h_sign: 32 bytes per row, byte
// b bit j = h[row, 32 j + b] > 0) instead of h; act 0 (identity) or 1 (LeakyReLU / ReLU).  The same outputs bit for bit.
XPA_API int xpa_s3_gemm_trunk_bwd_sign(const float *dz, int64_t ldz, const void *b_split, int64_t k,
                                       const unsigned *h_sign, const float *x, int64_t ldx, int64_t rows,
                                       int64_t d_in, int act, float slope, float *partial_dw, float *partial_db,
                                       xpa_stream_t stream) {
    if (!dz || !b_split || !h_sign || !x || !partial_dw || !partial_db || rows <= 0 || k <= 0 || k % kKC != 0 ||
        ldz < k || (ldz & 3) || (reinterpret_cast<uintptr_t>(dz) & 15) || (reinterpret_cast<uintptr_t>(h_sign) & 15) ||
        d_in < 1 || d_in > 32 || ldx < d_in || act < 0 || act > 1 || k / kKC > (1 << 20))
        return (int)hipErrorInvalidValue;
    const dim3 grid((unsigned)xpa_s3_gemm_trunk_bwd_num_partials(rows)), block(512);
    const __bf16 *bs = static_cast<const __bf16 *>(b_split);
    const int nch = (int)(k / kKC);
    const bool la = (g_s3_probe & 128) != 0;   // the lookahead form (A/B)
    const bool pp = (g_s3_probe & 256) != 0;   // the ping-pong k loop (A/B)
    if (pp && act == 0)
        s3_gemm_trunk_bwd_kernel<0, true, 2><<<grid, block, 0, stream>>>(dz, ldz, bs, rows, nch, nullptr, 0, x, ldx,
                                                                          (int)d_in, slope, partial_dw, partial_db,
                                                                          h_sign);
    else if (pp)
        s3_gemm_trunk_bwd_kernel<1, true, 2><<<grid, block, 0, stream>>>(dz, ldz, bs, rows, nch, nullptr, 0, x, ldx,
                                                                          (int)d_in, slope, partial_dw, partial_db,
                                                                          h_sign);
    else if (act == 0 && la)
        s3_gemm_trunk_bwd_kernel<0, true, 1><<<grid, block, 0, stream>>>(dz, ldz, bs, rows, nch, nullptr, 0, x, ldx,
                                                                          (int)d_in, slope, partial_dw, partial_db,
                                                                          h_sign);
    else if (act == 0)
        s3_gemm_trunk_bwd_kernel<0, true><<<grid, block, 0, stream>>>(dz, ldz, bs, rows, nch, nullptr, 0, x, ldx,
                                                                       (int)d_in, slope, partial_dw, partial_db, h_sign);
    else if (la)
        s3_gemm_trunk_bwd_kernel<1, true, 1><<<grid, block, 0, stream>>>(dz, ldz, bs, rows, nch, nullptr, 0, x, ldx,
                                                                          (int)d_in, slope, partial_dw, partial_db,
                                                                          h_sign);
    else
        s3_gemm_trunk_bwd_kernel<1, true><<<grid, block, 0, stream>>>(dz, ldz, bs, rows, nch, nullptr, 0, x, ldx,
                                                                       (int)d_in, slope, partial_dw, partial_db, h_sign);
    return xpa_launch_status();
}

// K42C (r05): xpa_s3_gemm_trunk_bwd_sign with the critic's half of the paired dX factored (see s3_trunk_bwd_crit_kernel):
// dz_a [rows, k_a] (row stride ldz; the actor's half only), b_split = the split of [Wh_a; V] (k_a + k_c rows, V =
// (1 - slope_c) diag(wc) Wh_c: xpa_s3_split_batch with a row scale), crit_mask [rows, 8] u32 + crit_dv [rows] from
// xpa_head_gemm_s3q_critic_mask, crit_cs [256] = slope_c wc . Wh_c.  act 0 / 1 (the trunk layer's, from h_sign).
XPA_API int xpa_s3_gemm_trunk_bwd_crit(const float *dz_a, int64_t ldz, const void *b_split, int64_t k_a, int64_t k_c,
                                       const unsigned *crit_mask, const float *crit_dv, const float *crit_cs,
                                       const unsigned *h_sign, const float *x, int64_t ldx, int64_t rows, int64_t d_in,
                                       int act, float slope, float *partial_dw, float *partial_db, xpa_stream_t stream) {
    if (!dz_a || !b_split || !crit_mask || !crit_dv || !crit_cs || !h_sign || !x || !partial_dw || !partial_db ||
        rows <= 0 || k_a <= 0 || k_c <= 0 || k_a % kKC != 0 || k_c % kKC != 0 || k_c > 256 || ldz < k_a || (ldz & 3) ||
        (reinterpret_cast<uintptr_t>(dz_a) & 15) || (reinterpret_cast<uintptr_t>(h_sign) & 15) ||
        (reinterpret_cast<uintptr_t>(crit_mask) & 15) || d_in < 1 || d_in > 32 || ldx < d_in || act < 0 || act > 1 ||
        (k_a + k_c) / kKC > (1 << 20))
        return (int)hipErrorInvalidValue;
    const dim3 grid((unsigned)xpa_s3_gemm_trunk_bwd_num_partials(rows)), block(512);
    const __bf16 *bs = static_cast<const __bf16 *>(b_split);
    const int nca = (int)(k_a / kKC), ncc = (int)(k_c / kKC);
    if (act == 0)
        s3_trunk_bwd_crit_kernel<0><<<grid, block, 0, stream>>>(dz_a, ldz, bs, rows, nca, ncc, crit_mask, crit_dv,
                                                                 crit_cs, x, ldx, (int)d_in, slope, partial_dw,
                                                                 partial_db, h_sign);
    else
        s3_trunk_bwd_crit_kernel<1><<<grid, block, 0, stream>>>(dz_a, ldz, bs, rows, nca, ncc, crit_mask, crit_dv,
                                                                 crit_cs, x, ldx, (int)d_in, slope, partial_dw,
                                                                 partial_db, h_sign);
    return xpa_launch_status();
}

// K42W (r05, the C4 trunk layer): xpa_s3_gemm_trunk_bwd_sign for a representation layer too wide for the fused thin dW:
// dz_out [rows, 256] (row stride ld_out) = g . act'(h) from h's sign bits, and the db partials [G, 256]; the layer's
// dW comes from xpa_s3_wgrad on (x, dz_out)
XPA_API int xpa_s3_gemm_trunk_bwd_dz(const float *dz, int64_t ldz, const void *b_split, int64_t k,
                                     const unsigned *h_sign, int64_t rows, int act, float slope, float *dz_out,
                                     int64_t ld_out, float *partial_db, xpa_stream_t stream) {
    if (!dz || !b_split || !h_sign || !dz_out || !partial_db || rows <= 0 || k <= 0 || k % kKC != 0 || ldz < k ||
        (ldz & 3) || (reinterpret_cast<uintptr_t>(dz) & 15) || (reinterpret_cast<uintptr_t>(h_sign) & 15) ||
        ld_out < kN || act < 0 || act > 1 || k / kKC > (1 << 20))
        return (int)hipErrorInvalidValue;
    const dim3 grid((unsigned)xpa_s3_gemm_trunk_bwd_num_partials(rows)), block(512);
    const __bf16 *bs = static_cast<const __bf16 *>(b_split);
    const int nch = (int)(k / kKC);
    if (act == 0)
        s3_gemm_trunk_bwd_kernel<0, true, 0, true><<<grid, block, 0, stream>>>(dz, ldz, bs, rows, nch, nullptr, 0,
                                                                                nullptr, 0, 0, slope, nullptr,
                                                                                partial_db, h_sign, dz_out, ld_out);
    else
        s3_gemm_trunk_bwd_kernel<1, true, 0, true><<<grid, block, 0, stream>>>(dz, ldz, bs, rows, nch, nullptr, 0,
                                                                                nullptr, 0, 0, slope, nullptr,
                                                                                partial_db, h_sign, dz_out, ld_out);
    return xpa_launch_status();
}

// K42C's dz form (r05, the C4 trunk layer with the factored critic): xpa_s3_gemm_trunk_bwd_crit, its epilogue K42W's
XPA_API int xpa_s3_gemm_trunk_bwd_crit_dz(const float *dz_a, int64_t ldz, const void *b_split, int64_t k_a,
                                          int64_t k_c, const unsigned *crit_mask, const float *crit_dv,
                                          const float *crit_cs, const unsigned *h_sign, int64_t rows, int act,
                                          float slope, float *dz_out, int64_t ld_out, float *partial_db,
                                          xpa_stream_t stream) {
    if (!dz_a || !b_split || !crit_mask || !crit_dv || !crit_cs || !h_sign || !dz_out || !partial_db || rows <= 0 ||
        k_a <= 0 || k_c <= 0 || k_a % kKC != 0 || k_c % kKC != 0 || k_c > 256 || ldz < k_a || (ldz & 3) ||
        (reinterpret_cast<uintptr_t>(dz_a) & 15) || (reinterpret_cast<uintptr_t>(h_sign) & 15) ||
        (reinterpret_cast<uintptr_t>(crit_mask) & 15) || ld_out < kN || act < 0 || act > 1 ||
        (k_a + k_c) / kKC > (1 << 20))
        return (int)hipErrorInvalidValue;
    const dim3 grid((unsigned)xpa_s3_gemm_trunk_bwd_num_partials(rows)), block(512);
    const __bf16 *bs = static_cast<const __bf16 *>(b_split);
    const int nca = (int)(k_a / kKC), ncc = (int)(k_c / kKC);
    if (act == 0)
        s3_trunk_bwd_crit_kernel<0, true><<<grid, block, 0, stream>>>(dz_a, ldz, bs, rows, nca, ncc, crit_mask,
                                                                       crit_dv, crit_cs, nullptr, 0, 0, slope, nullptr,
                                                                       partial_db, h_sign, dz_out, ld_out);
    else
        s3_trunk_bwd_crit_kernel<1, true><<<grid, block, 0, stream>>>(dz_a, ldz, bs, rows, nca, ncc, crit_mask,
                                                                       crit_dv, crit_cs, nullptr, 0, 0, slope, nullptr,
                                                                       partial_db, h_sign, dz_out, ld_out);
    return xpa_launch_status();
}

// K40F (r05, the C4 trunk layer's forward): C [m, 256] = act(A [m, k] . B + bias), B split (k % 16 == 0; a layer
// width that is not a multiple of 16 goes in zero-padded: A's row pitch >= k with zero columns, B's planes from
// xpa_s3_split_batch_padded).  act 0 identity / 1 LeakyReLU (slope) / 2 tanh; sign_out (nullable, act 0 / 1): the
// output's sign bits, 32 bytes per row (K42W's act').
namespace {
int gemm_bias_act_impl(const float *a, int64_t lda, const int64_t *ridx, const void *b_split, float *c, int64_t ldc,
                       int64_t m, int64_t k, const float *bias, int act, float slope, unsigned *sign_out,
                       xpa_stream_t stream);
}

XPA_API int xpa_s3_gemm_bias_act(const float *a, int64_t lda, const void *b_split, float *c, int64_t ldc, int64_t m,
                                 int64_t k, const float *bias, int act, float slope, unsigned *sign_out,
                                 xpa_stream_t stream) {
    if (lda < k) return (int)hipErrorInvalidValue;
    return gemm_bias_act_impl(a, lda, nullptr, b_split, c, ldc, m, k, bias, act, slope, sign_out, stream);
}

// K40F's row-index form (r05): A's row r is row ridx[r] of a (the minibatch rows of the rollout buffer, no gathered
// copy).  k may exceed the row width (a zero-padded B: split with xpa_s3_split_batch_padded): the columns past the
// width then read the next row's first values (finite observations) or, for the buffer's last row, its allocation's
// zeroed tail, and meet zero rows of B — the caller guarantees k - width floats of readable, finite slack.
XPA_API int xpa_s3_gemm_bias_act_rows(const float *a, int64_t lda, const int64_t *ridx, const void *b_split, float *c,
                                      int64_t ldc, int64_t m, int64_t k, const float *bias, int act, float slope,
                                      unsigned *sign_out, xpa_stream_t stream) {
    if (!ridx || lda < 4 || k > lda + kKC) return (int)hipErrorInvalidValue;
    return gemm_bias_act_impl(a, lda, ridx, b_split, c, ldc, m, k, bias, act, slope, sign_out, stream);
}

namespace {
int gemm_bias_act_impl(const float *a, int64_t lda, const int64_t *ridx, const void *b_split, float *c, int64_t ldc,
                       int64_t m, int64_t k, const float *bias, int act, float slope, unsigned *sign_out,
                       xpa_stream_t stream) {
    if (!a || !b_split || !c || !bias || m <= 0 || k <= 0 || k % kKC != 0 || ldc < kN ||
        (reinterpret_cast<uintptr_t>(a) & 15) || (lda & 3) || act < 0 || act > 2 || (sign_out && act == 2) ||
        (reinterpret_cast<uintptr_t>(sign_out) & 15) || k / kKC > (1 << 20))
        return (int)hipErrorInvalidValue;
    const __bf16 *bs = static_cast<const __bf16 *>(b_split);
    const int nch = (int)(k / kKC);
    const dim3 grid((unsigned)((m + 255) / 256)), block(512);
    unsigned char *sg = reinterpret_cast<unsigned char *>(sign_out);
    if (act == 0)
        s3_gemm_kernel<8, 3, 0, 0, 1><<<grid, block, 0, stream>>>(a, lda, bs, c, ldc, m, nch, bias, slope, sg, ridx);
    else if (act == 1)
        s3_gemm_kernel<8, 3, 0, 0, 2><<<grid, block, 0, stream>>>(a, lda, bs, c, ldc, m, nch, bias, slope, sg, ridx);
    else
        s3_gemm_kernel<8, 3, 0, 0, 3><<<grid, block, 0, stream>>>(a, lda, bs, c, ldc, m, nch, bias, slope, nullptr,
                                                                  ridx);
    return xpa_launch_status();
}
}  // namespace

// K40V (r06): v [m] = act(a [m, k] . B + bias) . w_out + b_out[0] (act 0 identity / 1 LeakyReLU (slope) / 2 tanh; B
// split by xpa_s3_split_b, 256 columns): the critic of the rollout's deferred bootstrap rows up to its value in one
// launch, 64-row blocks (two waves of 32 rows x 256 columns) so a few thousand rows still spread over the chip
XPA_API int xpa_s3_gemm_value(const float *a, int64_t lda, const void *b_split, float *v, int64_t m, int64_t k,
                              const float *bias, int act, float slope, const float *w_out, const float *b_out,
                              xpa_stream_t stream) {
    if (!a || !b_split || !v || !bias || !w_out || !b_out || m <= 0 || k <= 0 || k % kKC != 0 || lda < k ||
        (reinterpret_cast<uintptr_t>(a) & 15) || (lda & 3) || act < 0 || act > 2 || k / kKC > (1 << 20) ||
        (m + 63) / 64 > 0x7fffffff)
        return (int)hipErrorInvalidValue;
    const __bf16 *bs = static_cast<const __bf16 *>(b_split);
    const int nch = (int)(k / kKC);
    const dim3 grid((unsigned)((m + 63) / 64)), block(128);
    hipStream_t s = (hipStream_t)stream;
    if (act == 0) s3_gemm_value_kernel<2, 4><<<grid, block, 0, s>>>(a, lda, bs, v, m, nch, bias, slope, w_out, b_out);
    else if (act == 1) s3_gemm_value_kernel<2, 5><<<grid, block, 0, s>>>(a, lda, bs, v, m, nch, bias, slope, w_out, b_out);
    else s3_gemm_value_kernel<2, 6><<<grid, block, 0, s>>>(a, lda, bs, v, m, nch, bias, slope, w_out, b_out);
    return xpa_launch_status();
}

// K40R (r05): z [m, 512] = x [m, 256] . [B0 | B1] + bias, B0 / B1 split by xpa_s3_split_b (k = 256): the rollout's
// paired hidden layer; each output is xpa_s3_gemm's + bias bit for bit
XPA_API int xpa_s3_gemm_rows_pair(const float *a, int64_t lda, const void *b0_split, const void *b1_split,
                                  const float *bias, float *c, int64_t ldc, int64_t m, xpa_stream_t stream) {
    if (!a || !b0_split || !b1_split || !bias || !c || m <= 0 || lda < kN || ldc < 2 * kN || (lda & 3) ||
        (reinterpret_cast<uintptr_t>(a) & 15) || (m + kRRows - 1) / kRRows > 0x7fffffff)
        return (int)hipErrorInvalidValue;
    const dim3 grid((unsigned)((m + kRRows - 1) / kRRows), 4);
    const __bf16 *b0 = static_cast<const __bf16 *>(b0_split), *b1 = static_cast<const __bf16 *>(b1_split);
    // forms (xpa_s3_probe, A/B): default 2 stages x 4 chunks; 512: 3 x 1 (a barrier per chunk); 1024: 3 x 2
    if (g_s3_probe & 512)
        s3_gemm_r64_kernel<3, 1><<<grid, dim3(256), 0, stream>>>(a, lda, b0, b1, c, ldc, m, kN / kKC, bias);
    else if (g_s3_probe & 1024)
        s3_gemm_r64_kernel<3, 2><<<grid, dim3(256), 0, stream>>>(a, lda, b0, b1, c, ldc, m, kN / kKC, bias);
    else
        s3_gemm_r64_kernel<2, 4><<<grid, dim3(256), 0, stream>>>(a, lda, b0, b1, c, ldc, m, kN / kKC, bias);
    return xpa_launch_status();
}

// K40T (r06): xpa_thin_linear_act_fwd_norm (d_out 256, d_in <= 20; h not stored) + xpa_s3_gemm_rows_pair in one launch
XPA_API int xpa_s3_gemm_rows_pair_trunk(int act, const float *x, int64_t ldx, int64_t d_in, const float *w,
                                        const float *b, float slope, const float *mean, const float *var, float clip,
                                        float *xn, int64_t ldn, float *col, int64_t col_ld, const xpa_cursor_t *cursor,
                                        const void *b0_split, const void *b1_split, const float *bias, float *c,
                                        int64_t ldc, int64_t m, xpa_stream_t stream) {
    if (!x || !w || !b || !mean || !var || !xn || !b0_split || !b1_split || !bias || !c || m <= 0 || d_in < 1 ||
        d_in > TrunkW<20>::kSt || act < 0 || act > 2 || ldx < d_in || ldn < d_in || ldc < 2 * kN ||
        (col && (!cursor || col_ld < d_in)) || (m + kRRows - 1) / kRRows > 0x7fffffff)
        return (int)hipErrorInvalidValue;
    const dim3 grid((unsigned)((m + kRRows - 1) / kRRows), 4);
    const __bf16 *b0 = static_cast<const __bf16 *>(b0_split), *b1 = static_cast<const __bf16 *>(b1_split);
    hipStream_t s = (hipStream_t)stream;
    const int din = (int)d_in;
#define XPA_K40T_P(A_, D_, P_)                                                                                        \
    s3_gemm_r64_trunk_kernel<3, 2, A_, D_, P_><<<grid, dim3(256), 0, s>>>(x, ldx, din, w, b, slope, mean, var, clip,  \
                                                                           xn, ldn, col, col_ld, cursor, b0, b1, c, ldc, \
                                                                           m, bias)
    // diagnostics (xpa_s3_probe, tools/k40t_probe.py; act 1, d_in 9-18): 4096 = no trunk FMAs, 8192 = the prologue
    // (loads, staging, trunk phase 0) alone
    if ((g_s3_probe & 12288) && act == 1 && din > 8) {
        if (g_s3_probe & 4096) XPA_K40T_P(1, 20, 1);
        else XPA_K40T_P(1, 20, 2);
        return xpa_launch_status();
    }
    if (din <= 8) {
        if (act == 0) XPA_K40T_P(0, 8, 0);
        else if (act == 1) XPA_K40T_P(1, 8, 0);
        else XPA_K40T_P(2, 8, 0);
    } else {
        if (act == 0) XPA_K40T_P(0, 20, 0);
        else if (act == 1) XPA_K40T_P(1, 20, 0);
        else XPA_K40T_P(2, 20, 0);
    }
#undef XPA_K40T_P
    return xpa_launch_status();
}

// K40G (r05): n (<= 32) problems c[p] [m, 256] = a[p] [m, k] . B[p] (split by xpa_s3_split_b), one lda / ldc / m / k,
// one launch (host pointer arrays)
XPA_API int xpa_s3_gemm_group(int n, const float *const *a, const void *const *b_split, float *const *c, int64_t lda,
                              int64_t ldc, int64_t m, int64_t k, xpa_stream_t stream) {
    if (n < 1 || n > kS3Groups || !a || !b_split || !c || m <= 0 || k <= 0 || k % kKC != 0 || lda < k || ldc < kN ||
        (lda & 3) || k / kKC > (1 << 20) || (m + 255) / 256 > 0x7fffffff)
        return (int)hipErrorInvalidValue;
    S3Group g{};
    for (int p = 0; p < n; ++p) {
        if (!a[p] || !b_split[p] || !c[p] || (reinterpret_cast<uintptr_t>(a[p]) & 15)) return (int)hipErrorInvalidValue;
        g.a[p] = a[p];
        g.b[p] = static_cast<const __bf16 *>(b_split[p]);
        g.c[p] = c[p];
    }
    s3_gemm_group_kernel<-1><<<dim3((unsigned)((m + 255) / 256), (unsigned)n), dim3(512), 0, stream>>>(
        g, lda, ldc, m, (int)(k / kKC), S3ActBwd{});
    return xpa_launch_status();
}

// K40G with the previous block's activation backward in the epilogue (r05): c[p] = (a[p] . B[p]) act'(y[p]) (act 0
// identity / 1 LeakyReLU(slope) from the output y / 2 tanh), and per (problem, row block) the column sums of c[p] per
// channel (column mod channels, channels 32 or 64; each c[p] must start at a multiple of `channels` columns of the
// layer) into bias_partial [n x ceil(m / 256)][channels] (xpa_s3_gemm_group_act_num_partials).  K22's output and
// bias partials in one launch; the stored values equal xpa_act_bwd_bias's dz bit for bit.
XPA_API int64_t xpa_s3_gemm_group_act_num_partials(int n, int64_t m) { return (int64_t)n * ((m + 255) / 256); }

XPA_API int xpa_s3_gemm_group_act(int n, const float *const *a, const void *const *b_split, float *const *c,
                                  const float *const *y, int64_t lda, int64_t ldc, int64_t m, int64_t k, int act,
                                  float slope, int64_t channels, float *bias_partial, xpa_stream_t stream) {
    if (n < 1 || n > kS3Groups || !a || !b_split || !c || !y || !bias_partial || m <= 0 || k <= 0 || k % kKC != 0 ||
        lda < k || ldc < kN || (lda & 3) || k / kKC > (1 << 20) || (m + 255) / 256 > 0x7fffffff || act < 0 || act > 2 ||
        (channels != 32 && channels != 64))
        return (int)hipErrorInvalidValue;
    S3Group g{};
    for (int p = 0; p < n; ++p) {
        if (!a[p] || !b_split[p] || !c[p] || !y[p] || (reinterpret_cast<uintptr_t>(a[p]) & 15))
            return (int)hipErrorInvalidValue;
        g.a[p] = a[p];
        g.b[p] = static_cast<const __bf16 *>(b_split[p]);
        g.c[p] = c[p];
        g.y[p] = y[p];
    }
    S3ActBwd ab;
    ab.act = act;
    ab.slope = slope;
    ab.C = (int)channels;
    ab.bpart = bias_partial;
    const dim3 grid((unsigned)((m + 255) / 256), (unsigned)n);
    if (act == 0) s3_gemm_group_kernel<0><<<grid, dim3(512), 0, stream>>>(g, lda, ldc, m, (int)(k / kKC), ab);
    else if (act == 1) s3_gemm_group_kernel<1><<<grid, dim3(512), 0, stream>>>(g, lda, ldc, m, (int)(k / kKC), ab);
    else s3_gemm_group_kernel<2><<<grid, dim3(512), 0, stream>>>(g, lda, ldc, m, (int)(k / kKC), ab);
    return xpa_launch_status();
}

XPA_API int xpa_s3_gemm(const float *a, int64_t lda, const void *b_split, float *c, int64_t ldc, int64_t m, int64_t k,
                        int64_t n, xpa_stream_t stream) {
    if (!a || !b_split || !c || m <= 0 || k <= 0 || k % kKC != 0 || n != kN || lda < k || ldc < n ||
        (reinterpret_cast<uintptr_t>(a) & 15) || (lda & 3) || k / kKC > (1 << 20))
        return (int)hipErrorInvalidValue;
    const __bf16 *bs = static_cast<const __bf16 *>(b_split);
    const int nch = (int)(k / kKC);
    // form (probe bits 8 / 16): 0 = one 8-wave block per CU with a 3-stage ring, 8 = two 4-wave blocks per CU, 2 stages,
    // 16 = the wave-specialised K40W
    if (g_s3_probe & 256) {   // the ping-pong k loop
        s3_gemm_pp_kernel<<<dim3((unsigned)((m + 255) / 256)), dim3(512), 0, stream>>>(a, lda, bs, c, ldc, m, nch);
        return xpa_launch_status();
    }
    if (g_s3_probe & 32) {   // the 64 x 128 wave tile
        s3_gemm_kernel<8, 3, 0, 1><<<dim3((unsigned)((m + 255) / 256)), dim3(512), 0, stream>>>(a, lda, bs, c, ldc, m,
                                                                                              nch);
        return xpa_launch_status();
    }
    if (g_s3_probe & 16) {
        const int64_t nt = (m + kWRows - 1) / kWRows;
        s3_gemm_ws_kernel<<<dim3((unsigned)(nt < 256 ? nt : 256)), dim3(512), 0, stream>>>(a, lda, bs, c, ldc, m, nch);
        return xpa_launch_status();
    }
    if (g_s3_probe & 8) {
        const dim3 grid((unsigned)((m + 127) / 128)), block(256);
        switch (g_s3_probe & 7) {
#define XPA_GM(P) case P: s3_gemm_kernel<4, 2, P><<<grid, block, 0, stream>>>(a, lda, bs, c, ldc, m, nch); break;
            XPA_GM(1) XPA_GM(2) XPA_GM(3) XPA_GM(4) XPA_GM(6)
#undef XPA_GM
            default: s3_gemm_kernel<4, 2, 0><<<grid, block, 0, stream>>>(a, lda, bs, c, ldc, m, nch);
        }
        return xpa_launch_status();
    }
    const dim3 grid((unsigned)((m + 255) / 256)), block(512);
    switch (g_s3_probe & 7) {
#define XPA_GM(P) case P: s3_gemm_kernel<8, 3, P><<<grid, block, 0, stream>>>(a, lda, bs, c, ldc, m, nch); break;
        XPA_GM(1) XPA_GM(2) XPA_GM(3) XPA_GM(4) XPA_GM(6)
#undef XPA_GM
        default: s3_gemm_kernel<8, 3, 0><<<grid, block, 0, stream>>>(a, lda, bs, c, ldc, m, nch);
    }
    return xpa_launch_status();
}
