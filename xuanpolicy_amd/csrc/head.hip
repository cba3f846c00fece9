// K12 — fused actor / critic head: hidden activation + output layer + PPO-Clip / A2C loss + backward,
// one pass per minibatch and head (gfx950).
//
// Replaces, for the MLP actor-critic (xuance/torch/policies/gaussian.py:8-51, categorical.py:16-58;
// mlp_block xuance/torch/utils/layers.py:8-24), the tail of the forward (activation of the last hidden
// layer, the output Linear), the loss of PPOCLIP_Learner.update / A2C_Learner.update
// (ppoclip_learner.py:32-44, a2c_learner.py:24-31, distributions.py:39-101) and the backward down to the
// hidden pre-activation (torch autograd in loss.backward(), ppoclip_learner.py:46).
//
// z and dz rows have stride ld (>= 256, multiple of 4: e.g. the halves of a [batch, 512] actor|critic
// pair).  Outputs: dz [batch, 256]; per-block partials dW_o [K*256], db_h [256], db_o [K] (reduced by
// xpa_colsum_finalize) and one row of the K2 loss-partials layout (surrogate, sq-err, entropy, clip
// count, value sum, dlogstd[K]; reduced by xpa_policy_loss_finalize).  The actor launch fills the actor
// columns, the critic launch the critic columns of the same partials array.
// HBM: reads z (4 B/elem), writes dz (4 B/elem): 2 KiB per row at H = 256, plus the per-row inputs.
#include "xpa_common.h"
#include "s3_split.h"

#ifndef XPA_HEAD_PROBE  // tools/head_probe.py builds variants with parts compiled out
#define XPA_HEAD_PROBE 0
#endif

namespace {

constexpr int kWaves = 4;
constexpr int kH = 256;  // hidden width handled
constexpr int kPartBase = 5;
constexpr int kHeadKMax = 18;  // largest head width of the fused head kernels (KMAX buckets 4 / 6 / 8 / 18)
constexpr float kLogSqrt2Pi = 0.91893853320467274178f;
constexpr float kHalfLog2PiPlusHalf = 1.41893853320467274178f;

template <int ACT>
__device__ __forceinline__ float act_f(float z, float slope) {
    if (ACT == 1) return z > 0.f ? z : z * slope;
    if (ACT == 2) return tanhf(z);
    return z;
}

template <int ACT>
__device__ __forceinline__ float act_g(float h, float slope) {  // d act / d z as a function of the output
    if (ACT == 1) return h > 0.f ? 1.f : slope;
    if (ACT == 2) return 1.0f - h * h;
    return 1.f;
}

__device__ __forceinline__ void adv_stats(const double *partials, int64_t n, int64_t batch, float *mean, float *inv,
                                          int tid) {
    if (tid < 64) {  // tid: the calling group's thread index (K16W's epilogue waves are not threads 0..63)
        // eight 16-B loads in flight per lane (n = 1024 partials at C2: 2 round trips instead of 16 at the start of
        // every block); each lane still adds its k = lane, lane + 64, ... in order
        double s = 0.0, q = 0.0;
        int64_t k = tid;
        for (; k + 7 * 64 < n; k += 8 * 64) {
            double2 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const double2 *>(partials + 2 * (k + 64 * u));
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s += v[u].x;
                q += v[u].y;
            }
        }
        for (; k < n; k += 64) {
            s += partials[2 * k];
            q += partials[2 * k + 1];
        }
        s = xpa_wave_sum(s);
        q = xpa_wave_sum(q);
        if (tid == 0) {
            const double m = s / (double)batch;
            const double var = fmax(q / (double)batch - m * m, 0.0);
            *mean = (float)m;
            *inv = (float)(1.0 / ((double)(float)sqrt(var) + 1e-8));
        }
    }
}

// Tiled formulation: a block walks tiles of kTile = 64 rows (grid-stride, next tile's z prefetched into
// registers while the current one is processed):
//   stage    256 threads load the [64 x 256] z tile coalesced (16-B loads), apply the activation and
//            store h into LDS (row stride kS = 260 floats);
//   phase 1  row owners: thread (wave q, lane r) dots h[r, 64q : 64q + 64] with the output weights
//            (wave-uniform scalar loads) -> per-quarter partials in LDS;
//   loss     wave 0, lane r: head[r] = sum of the 4 quarters + bias, the row's loss terms and d head
//            (once per row, no redundant lanes) -> LDS;
//   phase 2  column owners: thread c walks the tile's rows: dz[r, c] = (d_head[r] . w[:, c]) * act'(h),
//            accumulating dW_out[:, c] and db_hidden[c] in registers.
// LDS banks: phase-1 ds_read_b128 of lanes r = 16g..16g+15 start at dword 4r + c (mod 64): the 16-lane
// group covers the 64 banks once; phase-2 ds_read_b32 of consecutive columns hits consecutive banks.
typedef float f4v __attribute__((ext_vector_type(4)));
constexpr int kTile = 64;
constexpr int kS = 260;
constexpr int kGridMax = 512;  // 2 blocks per CU (77 KiB LDS each) x 256 CUs
// Blocks own the per-block partial rows blockIdx.x of p_dw / p_dbh / p_dbo / p_loss, which hold
// head_partials(batch) rows: a block beyond them must write nothing.  (r01: an uncommitted two-head
// experiment launched 13 tiles x 512 = 6656 blocks for B = 777; its blocks >= 13 skipped the tile loop and
// still wrote their partials in finish() — out of the buffers: HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION.)
__host__ __device__ constexpr int64_t head_partials(int64_t batch) {
    return (batch + kTile - 1) / kTile < kGridMax ? (batch + kTile - 1) / kTile : kGridMax;
}

struct HeadArgs {
    int64_t batch;
    int K;
    int64_t ld;
    const float *z;  // K12: hidden pre-activations; K16: the hidden layer's input x
    int64_t ldx;
    const float *Wh, *bh;  // K16: hidden layer weight [256, 256] and bias
    const float *W;
    const float *bias;
    float slope;
    const float *logstd;
    const int64_t *idx;
    int64_t n_rows;
    const float *act;
    const float *old_logp;
    const float *adv;
    const float *ret;
    const double *adv_partials;
    int64_t n_adv_partials;
    float clip_range, ent_coef, vf_coef;
    float *dz, *p_dw, *p_dbh, *p_dbo, *p_loss;
    int loss_width;
    // K16X: the trunk's first layer (gathered rows [batch, din] at ldxr, W0 [256, din], b0) and the h output
    const float *xr, *W0, *b0;
    int64_t ldxr, ldh;
    int din;
    float slope0;
    float *hout;
    unsigned *hmask;  // K16R: the trunk activations' sign bits [batch, 8 words] (actor; may be null)
    unsigned *cmask;  // r05: the critic's hidden sign bits [batch, 8 words] (HeadEpi::mask_out; may be null)
    float *cdv;       // r05: the critic's d loss / d v [batch] (may be null)
};

__device__ __forceinline__ void load_tile(float4 (&zq)[16], const float *__restrict__ z, int64_t ld, int64_t tile,
                                          int64_t batch) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int lin = i * 256 + (int)threadIdx.x;
        const int64_t row = tile * kTile + (lin >> 6);
        if (row < batch) {
            const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(z + row * ld) + (lin & 63));
            zq[i] = make_float4(v.x, v.y, v.z, v.w);
        } else {
            zq[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
}

__device__ int g_head_stagger = 0;   // r06: see head_gemm_kernel (xpa_head_stagger)

// dz stores: non-temporal (0, the default) or plain (1: xpa_head_store_probe, r04 A/B — the update's dz is read next by
// K41 and K42, and the 128 MiB of both halves fit the MALL)
__device__ int g_head_dz_plain = 0;

// ---- shared epilogue: everything after h = act(z) of a 64-row tile is in LDS ----------------------
// MODE: 0 Gaussian actor, 1 Categorical actor, 2 critic.  ALGO: 0 PPO, 1 A2C (actor only).
// NW: the waves running it (4: K12 / K16, all of the block; 2: K16W's epilogue waves).  Epilogue thread e (0 .. 64 NW)
// owns columns e + 64 NW j (j < CPT = 4 / NW) in phase 2; in phase 1 wave w owns the row quarters w 4/NW + i.  The
// arithmetic of every output is the same whichever NW runs it (each quarter / column is one sequential chain in the
// same order), so K16W reproduces K16 bit for bit.
// The steps have no barriers of their own: a kernel runs them in order with a block barrier between consecutive steps
// (the K12 / K16 wrapper `tile` does exactly that; K16W places them between its k-chunk barriers).
typedef float f2v __attribute__((ext_vector_type(2)));
template <int KMAX>
struct RowIn {  // epilogue wave 0, lane = row of the tile
    bool valid;
    bool masked;  // a batch row whose index is out of range (contributes nothing)
    float x, old, act[KMAX];
};

template <int MODE, int ALGO, int ACT, int KMAX, int NW = 4, bool QOK = true>
struct HeadEpi {
    static constexpr int KP = (KMAX + 3) & ~3;  // 16-B aligned d-head rows
    // phase-1 partials per pass: heads wider than 8 (C4's 17 / 18) go through s_part in two halves, so the K16 block
    // fits 80 KiB of LDS (2 blocks per CU; 90 KiB with all 18 at once)
    static constexpr int PH = KMAX > 8 ? (KMAX + 1) / 2 : KMAX;
    static constexpr int NPASS = (KMAX + PH - 1) / PH;
    static constexpr int NT = 64 * NW;      // epilogue threads
    static constexpr int CPT = 4 / NW;      // phase-2 columns per thread
    static constexpr int QPW = 4 / NW;      // phase-1 row quarters per wave
    // phase 2 (column t); dW_out accumulated in output pairs (v_pk_fma_f32: the same fused multiply-add per output,
    // half the VALU issues)
    static constexpr bool kPk = KMAX <= 8;  // the wide heads (C4) keep scalar accumulators (packed pairs spill there)
    static constexpr int KH2 = (KMAX + 1) / 2;
    // r06, phase 2 of the actor heads (KMAX <= 6, the whole block): thread e owns the 4 consecutive columns 4 (e & 63) ..
    // + 3 of rows r = e >> 6 (mod 4), so a wave reads a row of h with ONE ds_read_b128 per lane and writes its dz row as
    // ONE 1-KiB store (16 B per lane) instead of 64 B-strided 4-B ones; each dz value is the same arithmetic as before
    // (bit for bit), dW_out / db_hidden accumulate per wave and are summed over the 4 waves in a fixed order at finish
    // Register budget (2 blocks per CU: 256 VGPRs): the quad layout's 4-column accumulators live only through a tile's
    // epilogue (q_dw2 / q_dbh, zeroed in p2_quad, summed over the 4 waves into the one-column acc_dw2 / acc_dbh by
    // quad_flush), and its output weights are loaded per tile (16-B loads from L2): kept across the k loop they took the
    // K = 6 actor from 204 to 253 VGPRs and the K = 8 one into scratch
    // (QOK: the kernel allows it — K12 keeps its next tile's z prefetched in 64 VGPRs through the epilogue; KMAX <= 6:
    // the K = 8 bucket's packed accumulators and weights did not fit 256 VGPRs beside the rest)
    static constexpr bool kQuad = QOK && MODE != 2 && NW == 4 && KMAX <= 6;
    float wc[kQuad ? 1 : CPT][KMAX], acc_dw[CPT][kPk ? 1 : KMAX], acc_dbh[CPT];
    f2v acc_dw2[CPT][kPk ? KH2 : 1];
    f2v q_dw2[kQuad ? 4 : 1][KH2];
    float q_dbh[kQuad ? 4 : 1];
    __device__ __forceinline__ int col_of(int j) const { return e + NT * j; }
    // the wide heads (C4) keep the Gaussian's per-output variance / log-scale in LDS (s_stats[2 ..], written by
    // init_a): 36 registers fewer where the kernel sits at the 256-register cap of 2 blocks per CU
    static constexpr bool kLdsVar = KMAX > 8;
    static constexpr int kStatN = kLdsVar ? 2 + 2 * KMAX : 2;   // floats of s_stats
    float acc_dbo[KMAX], acc_dls[KMAX], var_[kLdsVar ? 1 : KMAX], logsc[kLdsVar ? 1 : KMAX];
    const float *s_var = nullptr;   // kLdsVar: 1 / var at s_var[o], log-scale at s_var[KMAX + o]
    float sum0, sum1, sum2, ent_const, inv_b, lo, hi, a_mean, a_inv, slope;
    float hd[KMAX];  // epilogue wave 0: the row's head outputs between the phase-1 passes and the loss
    int K, e;        // e: epilogue thread index
    // r05, the critic's factored backward (K16Q critic, xpa_head_gemm_s3q_critic_mask): mask_out (nullable) gets the
    // sign bits of the hidden activations, [batch][8] words, bit c & 31 of word c >> 5 = h[row, c] > 0; dv_out
    // (nullable) d loss / d v per row; dz_on = false skips the dz stores (db_hidden / dW_out are still accumulated)
    unsigned *mask_out = nullptr;
    float *dv_out = nullptr;
    bool dz_on = true;

    // W: output layer [K, 256]; s_stats: 2 floats of LDS.  init_a, a block barrier, then init_b.
    __device__ __forceinline__ void init_a(int e_, int K_in, const float *__restrict__ W,
                                           const float *__restrict__ logstd, const double *__restrict__ adv_partials,
                                           int64_t n_adv_partials, int64_t batch, float clip_range, float slope_,
                                           float *s_stats) {
        e = e_;
        K = MODE == 2 ? 1 : K_in;
        slope = slope_;
        if (MODE != 2 && adv_partials) {
            adv_stats(adv_partials, n_adv_partials, batch, s_stats, s_stats + 1, e);
        } else if (e == 0) {
            s_stats[0] = 0.f;
            s_stats[1] = 1.f;
        }
#pragma unroll
        for (int j = 0; j < (kQuad ? 1 : CPT); ++j)
#pragma unroll
            for (int o = 0; o < KMAX; ++o) wc[j][o] = (o < K && !kQuad) ? W[o * kH + col_of(j)] : 0.f;
#pragma unroll
        for (int o = 0; o < KMAX; ++o) {
            acc_dbo[o] = acc_dls[o] = 0.f;
            hd[o] = 0.f;
        }
#pragma unroll
        for (int o = 0; o < (kLdsVar ? 1 : KMAX); ++o) {
            var_[o] = 1.f;
            logsc[o] = 0.f;
        }
        if (kLdsVar && e < KMAX) {
            s_stats[2 + e] = 1.f;
            s_stats[2 + KMAX + e] = 0.f;
        }
#pragma unroll
        for (int j = 0; j < CPT; ++j) {
            if constexpr (kPk) {
#pragma unroll
                for (int o2 = 0; o2 < KH2; ++o2) acc_dw2[j][o2] = f2v{0.f, 0.f};
            } else {
#pragma unroll
                for (int o = 0; o < KMAX; ++o) acc_dw[j][o] = 0.f;
            }
            acc_dbh[j] = 0.f;
        }
        sum0 = sum1 = sum2 = ent_const = 0.f;
        if (MODE == 0) {
#pragma unroll
            for (int o = 0; o < KMAX; ++o) {
                const float sc = o < K ? expf(logstd[o]) : 1.f;
                const float ls = logf(sc);
                // r06: the reciprocal of the variance, so the per-row loss multiplies where it divided (three IEEE
                // divisions per output and row: ~half the loss's instructions); each product differs from the divide
                // by at most one rounding
                if constexpr (kLdsVar) {
                    if (e == o) {
                        s_stats[2 + o] = 1.0f / (sc * sc);
                        s_stats[2 + KMAX + o] = ls;
                    }
                } else {
                    var_[o] = 1.0f / (sc * sc);
                    logsc[o] = ls;
                }
                if (o < K) ent_const += kHalfLog2PiPlusHalf + ls;
            }
        }
        inv_b = 1.0f / (float)batch;
        lo = 1.0f - clip_range;
        hi = 1.0f + clip_range;
    }
    __device__ __forceinline__ void init_b(const float *s_stats) {
        a_mean = s_stats[0];
        a_inv = s_stats[1];
        s_var = s_stats + 2;
    }
    __device__ __forceinline__ float ivar_at(int o) const { return kLdsVar ? s_var[o] : var_[o]; }   // 1 / var
    __device__ __forceinline__ float logsc_at(int o) const { return kLdsVar ? s_var[KMAX + o] : logsc[o]; }

    __device__ __forceinline__ RowIn<KMAX> rows(int64_t tile, int64_t batch, const int64_t *__restrict__ idx,
                                                int64_t n_rows, const float *__restrict__ act,
                                                const float *__restrict__ old_logp, const float *__restrict__ adv,
                                                const float *__restrict__ ret) const {
        RowIn<KMAX> in;
        in.valid = false;
        in.masked = false;
        in.x = in.old = 0.f;
#pragma unroll
        for (int o = 0; o < KMAX; ++o) in.act[o] = 0.f;
        const int lane = e & 63;
        if (e < 64) {
            const int64_t b = tile * kTile + lane;
            if (b < batch) {
                const int64_t row = idx ? idx[b] : b;
                in.valid = row >= 0 && row < n_rows;
                in.masked = !in.valid;
                if (in.valid) {
                    if (MODE == 2) {
                        in.x = ret[row];
                    } else {
                        in.x = adv[row];
                        if (ALGO == 0) in.old = old_logp[row];
                        if (MODE == 0) {
#pragma unroll
                            for (int o = 0; o < KMAX; ++o)
                                if (o < K) in.act[o] = act[row * K + o];
                        } else {
                            in.act[0] = act[row];
                        }
                    }
                }
            }
        }
        return in;
    }

    // ---- phase 1, pass `pass`: partial dot products of outputs [pass PH, pass PH + PH), row = lane, quarter of
    // wave w's set.  Reads s_h (h of the tile, row stride kS), writes s_part.  Unconditional loads (rows o >= K re-read
    // row 0; their sums are never used): the scalar loads of a step issue together.  One fmaf chain per output and
    // quarter over its 64 columns in order.
    __device__ __forceinline__ void p1(int pass, const float *s_h, float (*s_part)[kTile][PH],
                                       const float *__restrict__ W) const {
        const int lane = e & 63;
        const int wave = __builtin_amdgcn_readfirstlane(e >> 6);
        const int o0 = pass * PH;
#pragma unroll
        for (int qi = 0; qi < QPW; ++qi) {
            const int quarter = wave * QPW + qi;
            float p[PH];
#pragma unroll
            for (int o = 0; o < PH; ++o) p[o] = 0.f;
            const float *hrow = s_h + lane * kS + quarter * 64;
            const float *wq = W + quarter * 64;
#pragma unroll 4
            for (int j = 0; j < 16; ++j) {
                const float4 hv = *reinterpret_cast<const float4 *>(hrow + 4 * j);
#pragma unroll
                for (int o = 0; o < PH; ++o) {
                    const int oo = o0 + o;
                    const float4 w4 = *reinterpret_cast<const float4 *>(wq + (oo < K ? oo : 0) * kH + 4 * j);
                    p[o] = fmaf(hv.x, w4.x, p[o]);
                    p[o] = fmaf(hv.y, w4.y, p[o]);
                    p[o] = fmaf(hv.z, w4.z, p[o]);
                    p[o] = fmaf(hv.w, w4.w, p[o]);
                }
            }
#pragma unroll
            for (int o = 0; o < PH; ++o) s_part[quarter][lane][o] = p[o];
        }
    }
    // epilogue wave 0 after a phase-1 pass: the head outputs of its row (the 4 quarters summed in a fixed order + bias)
    __device__ __forceinline__ void p1_sum(int pass, float (*s_part)[kTile][PH], const float *__restrict__ bias) {
        if (e >= 64) return;
        const int lane = e;
        const int o0 = pass * PH;
#pragma unroll
        for (int o = 0; o < PH; ++o)
            if (o0 + o < KMAX)
                hd[o0 + o] = o0 + o < K ? ((s_part[0][lane][o] + s_part[1][lane][o]) +
                                           (s_part[2][lane][o] + s_part[3][lane][o])) +
                                              bias[o0 + o]
                                        : 0.f;
    }

    // ---- loss: epilogue wave 0, one lane per row (after the last p1_sum); d head -> s_dh ----
    __device__ __forceinline__ void loss(float (*s_dh)[KP], const RowIn<KMAX> &in, float ent_coef, float vf_coef) {
#pragma clang fp contract(off)  // every product and sum rounded on its own: the same bits in every kernel inlining it
        if (e >= 64) return;
        const int lane = e;
        float dh_[KMAX];
#pragma unroll
        for (int o = 0; o < KMAX; ++o) dh_[o] = 0.f;
        if (in.valid) {
            if (MODE == 2) {
                const float diffv = hd[0] - in.x;
                sum0 += diffv * diffv;
                sum1 += hd[0];
                dh_[0] = vf_coef * 2.0f * diffv * inv_b;
                acc_dbo[0] += dh_[0];
            } else {
                const float A_n = (in.x - a_mean) * a_inv;
                float logp = 0.f, ent = 0.f, lse = 0.f;
                int ai = 0;
                float diff[KMAX];
                if (MODE == 0) {
#pragma unroll
                    for (int o = 0; o < KMAX; ++o) {
                        diff[o] = 0.f;
                        if (o < K) {
                            diff[o] = in.act[o] - hd[o];
                            logp += -(diff[o] * diff[o]) * (0.5f * ivar_at(o)) - logsc_at(o) - kLogSqrt2Pi;
                        }
                    }
                    ent = ent_const;
                } else {
                    float m = hd[0];
#pragma unroll
                    for (int o = 1; o < KMAX; ++o)
                        if (o < K) m = fmaxf(m, hd[o]);
                    float se = 0.f;
#pragma unroll
                    for (int o = 0; o < KMAX; ++o)
                        if (o < K) se += expf(hd[o] - m);
                    lse = m + logf(se);
                    ai = (int)in.act[0];
                    ai = ai < 0 ? 0 : (ai >= K ? K - 1 : ai);
#pragma unroll
                    for (int o = 0; o < KMAX; ++o) {
                        if (o < K) {
                            const float ln = hd[o] - lse;
                            ent -= expf(ln) * ln;
                            if (o == ai) logp = ln;
                        }
                    }
                }
                float dlogp;
                if (ALGO == 0) {
                    const float ratio = expf(logp - in.old);
                    const float cr = fminf(fmaxf(ratio, lo), hi);
                    const float s1 = cr * A_n, s2 = A_n * ratio;
                    sum0 += fminf(s1, s2);
                    const bool inr = (ratio >= lo) && (ratio <= hi);
                    const float g1 = inr ? A_n : 0.f;
                    const float w1 = (s1 < s2) ? 1.f : ((s1 == s2) ? 0.5f : 0.f);
                    const float w2 = (s2 < s1) ? 1.f : ((s1 == s2) ? 0.5f : 0.f);
                    dlogp = -inv_b * (w1 * g1 + w2 * A_n) * ratio;
                    sum2 += ((ratio < lo) || (ratio > hi)) ? 1.f : 0.f;
                } else {
                    sum0 += A_n * logp;
                    dlogp = -A_n * inv_b;
                }
                sum1 += ent;
                const float ec = ent_coef * inv_b;
#pragma unroll
                for (int o = 0; o < KMAX; ++o) {
                    if (o < K) {
                        if (MODE == 0) {
                            dh_[o] = dlogp * diff[o] * ivar_at(o);
                            acc_dls[o] += dlogp * (diff[o] * diff[o] * ivar_at(o) - 1.0f);
                        } else {
                            const float ln = hd[o] - lse;
                            const float p = expf(ln);
                            dh_[o] = dlogp * ((o == ai ? 1.f : 0.f) - p) + ec * p * (ln + ent);
                        }
                        acc_dbo[o] += dh_[o];
                    }
                }
            }
        }
        if (MODE == 0 && in.masked) {  // hand back the ent_coef / B the finalize subtracts for every row
#pragma unroll
            for (int o = 0; o < KMAX; ++o)
                if (o < K) acc_dls[o] += ent_coef * inv_b;
        }
        // the pad slots [KMAX, KP) too: phase 2 reads d head in float4s and, for KMAX = 1 (the critic), pairs slot 1
        // with a zero weight — LDS left over from an earlier kernel there (an Inf / NaN bit pattern) made 0 x NaN
        // dz rows (r04; tests/test_gpu_fused_mlp.py::test_head_gemm_kernels_vs_fp64_autograd after other kernels)
#pragma unroll
        for (int o = 0; o < KP; ++o) s_dh[lane][o] = o < KMAX ? dh_[o] : 0.f;
    }

    // ---- phase 2, rows [r0, r1) of the tile: column owner.  dz[r, c] = (d head[r] . w[:, c]) * act'(h[r, c]), dW_out
    // and db_hidden accumulated in registers; rows in groups of 4 (every LDS read of the group issued before the
    // arithmetic, the row order of the accumulations kept: bitwise the same sums as one row at a time).
    __device__ __forceinline__ void p2(const float *s_h, float (*s_dh)[KP], int64_t tile, int64_t batch, int r0, int r1,
                                       float *__restrict__ dz, int64_t ld, const float *__restrict__ W = nullptr) {
#if XPA_HEAD_PROBE == 5  // 5 = epilogue alone without phase 2
        r1 = r0;
#endif
        const int nr = (int)min((int64_t)r1, batch - tile * kTile);
        if constexpr (kQuad) {
            p2_quad(s_h, s_dh, tile, r0, nr, dz, ld, W);
            return;
        }
        unsigned mlo = 0u, mhi = 0u;   // mask_out: lane r of each wave ends with row r's two words of its 64 columns
        auto ballot_row = [&](int rr, float h) {
            if constexpr (CPT == 1) {
                if (mask_out != nullptr) {
                    const unsigned long long bl = __ballot(h > 0.f);
                    if ((e & 63) == rr) {
                        mlo = (unsigned)bl;
                        mhi = (unsigned)(bl >> 32);
                    }
                }
            }
        };
        f2v wc2[CPT][KH2];
#pragma unroll
        for (int j = 0; j < CPT; ++j)
#pragma unroll
            for (int o2 = 0; o2 < KH2; ++o2)
                wc2[j][o2] = f2v{wc[j][2 * o2], 2 * o2 + 1 < KMAX ? wc[j][2 * o2 + 1] : 0.f};
        int r = r0;
        constexpr int RG = 4;   // rows per group
        for (; r + RG <= nr; r += RG) {
            float hv[CPT][RG], gq[RG][KP];
#pragma unroll
            for (int u = 0; u < RG; ++u) {
#pragma unroll
                for (int j = 0; j < CPT; ++j) hv[j][u] = s_h[(r + u) * kS + e + NT * j];
#pragma unroll
                for (int q = 0; q < KP; q += 4) {
                    const float4 g4 = *reinterpret_cast<const float4 *>(&s_dh[r + u][q]);
                    gq[u][q] = g4.x;
                    gq[u][q + 1] = g4.y;
                    gq[u][q + 2] = g4.z;
                    gq[u][q + 3] = g4.w;
                }
            }
#pragma unroll
            for (int u = 0; u < RG; ++u) {
#pragma unroll
                for (int j = 0; j < CPT; ++j) col_row(j, hv[j][u], gq[u], wc2[j], dz + (tile * kTile + r + u) * ld);
                ballot_row(r + u, hv[0][u]);
            }
        }
        for (; r < nr; ++r) {
            float gq[KP];
#pragma unroll
            for (int q = 0; q < KP; ++q) gq[q] = s_dh[r][q];
#pragma unroll
            for (int j = 0; j < CPT; ++j) col_row(j, s_h[r * kS + e + NT * j], gq, wc2[j], dz + (tile * kTile + r) * ld);
            ballot_row(r, s_h[r * kS + e]);
        }
        if constexpr (CPT == 1) {
            // rows r0 .. nr of this call: lane r's words (rows past the batch: not stored)
            const int lr = e & 63;
            if (mask_out != nullptr && lr >= r0 && lr < nr) {
                unsigned *mrow = mask_out + (tile * kTile + lr) * 8 + 2 * (e >> 6);
                mrow[0] = mlo;
                mrow[1] = mhi;
            }
        }
    }
    // kQuad phase 2: rows r0 <= r < nr with r = wave (mod 4), 4 rows' LDS reads issued before their arithmetic
    __device__ __forceinline__ void p2_quad(const float *s_h, float (*s_dh)[KP], int64_t tile, int r0, int nr,
                                            float *__restrict__ dz, int64_t ld, const float *__restrict__ W) {
        const int w = e >> 6, l = e & 63;
        // wc2[j][o2] = (w[2 o2][4 l + j], w[2 o2 + 1][4 l + j]), loaded straight into place; rows o >= K re-read row 0
        // (finite) and their d head is 0 (loss() zeroes s_dh[.][o >= K]), so they add 0 to every chain.  r06: no select on
        // o < K — with one, hipcc put each row's load under a uniform branch with its own vmcnt(0) (KMAX serial L2 round
        // trips per tile); and no float4 staging array beside wc2 (its 4 KMAX registers made the kernel spill)
        f2v wc2[4][KH2];
#pragma unroll
        for (int o2 = 0; o2 < KH2; ++o2)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int oa = 2 * o2, ob = 2 * o2 + 1;
                const float a = W[(oa < K ? oa : 0) * kH + 4 * l + j];
                const float b = ob < KMAX ? W[(ob < K ? ob : 0) * kH + 4 * l + j] : 0.f;
                wc2[j][o2] = f2v{a, b};
            }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
            for (int o2 = 0; o2 < KH2; ++o2) q_dw2[j][o2] = f2v{0.f, 0.f};
            q_dbh[j] = 0.f;
        }
        int r = r0 + ((w - r0) & 3);
        constexpr int RG = 4;   // rows per group: r, r + 4, r + 8, r + 12
        for (; r + 4 * (RG - 1) < nr; r += 4 * RG) {
            float4 hv[RG];
            float gq[RG][KP];
#pragma unroll
            for (int u = 0; u < RG; ++u) {
                hv[u] = *reinterpret_cast<const float4 *>(s_h + (r + 4 * u) * kS + 4 * l);
#pragma unroll
                for (int q = 0; q < KP; q += 4) {
                    const float4 g4 = *reinterpret_cast<const float4 *>(&s_dh[r + 4 * u][q]);
                    gq[u][q] = g4.x;
                    gq[u][q + 1] = g4.y;
                    gq[u][q + 2] = g4.z;
                    gq[u][q + 3] = g4.w;
                }
            }
#pragma unroll
            for (int u = 0; u < RG; ++u) quad_row(hv[u], gq[u], wc2, dz + (tile * kTile + r + 4 * u) * ld);
        }
        for (; r < nr; r += 4) {
            float gq[KP];
#pragma unroll
            for (int q = 0; q < KP; ++q) gq[q] = s_dh[r][q];
            quad_row(*reinterpret_cast<const float4 *>(s_h + r * kS + 4 * l), gq, wc2, dz + (tile * kTile + r) * ld);
        }
    }
    __device__ __forceinline__ void quad_row(const float4 &h4, const float (&g)[KP], const f2v (&wc2)[4][KH2],
                                             float *__restrict__ dzrow) {
#pragma clang fp contract(off)
        const float hv[4] = {h4.x, h4.y, h4.z, h4.w};
        float dv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            // col_row's arithmetic per element: d head . w as one packed chain over the output pairs, then their sum
            f2v d2 = {0.f, 0.f};
#pragma unroll
            for (int o2 = 0; o2 < KH2; ++o2) d2 = __builtin_elementwise_fma(f2v{g[2 * o2], g[2 * o2 + 1]}, wc2[j][o2], d2);
            float d = d2.x + d2.y;
            const f2v hh = {hv[j], hv[j]};
#pragma unroll
            for (int o2 = 0; o2 < KH2; ++o2)
                q_dw2[j][o2] = __builtin_elementwise_fma(f2v{g[2 * o2], g[2 * o2 + 1]}, hh, q_dw2[j][o2]);
            d *= act_g<ACT>(hv[j], slope);
            dv[j] = d;
            q_dbh[j] += d;
        }
#if XPA_HEAD_PROBE != 4  // 4 = epilogue alone without the dz stores
        if (dz_on) {
            const f4v d4 = {dv[0], dv[1], dv[2], dv[3]};
            f4v *dst = reinterpret_cast<f4v *>(dzrow + 4 * (e & 63));
            if (g_head_dz_plain) *dst = d4;
            else __builtin_nontemporal_store(d4, dst);
        }
#endif
    }

    // kQuad, after phase 2 and a block barrier (s_h free): the 4 waves' 16-row partials of each column through LDS, summed
    // in wave order into column e's running dW_out / db_hidden; ends with a barrier (the LDS is the next tile's)
    __device__ __forceinline__ void quad_flush(float *s_red) {
        const int w = e >> 6, l = e & 63;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = 4 * l + j;
#pragma unroll
            for (int o2 = 0; o2 < KH2; ++o2) {
                s_red[(w * (2 * KH2 + 1) + 2 * o2) * kH + c] = q_dw2[j][o2].x;
                s_red[(w * (2 * KH2 + 1) + 2 * o2 + 1) * kH + c] = q_dw2[j][o2].y;
            }
            s_red[(w * (2 * KH2 + 1) + 2 * KH2) * kH + c] = q_dbh[j];
        }
        __syncthreads();
#pragma unroll
        for (int o2 = 0; o2 < KH2; ++o2) {
            f2v v = {s_red[(2 * o2) * kH + e], s_red[(2 * o2 + 1) * kH + e]};
#pragma unroll
            for (int ww = 1; ww < 4; ++ww)
                v += f2v{s_red[(ww * (2 * KH2 + 1) + 2 * o2) * kH + e], s_red[(ww * (2 * KH2 + 1) + 2 * o2 + 1) * kH + e]};
            acc_dw2[0][o2] += v;
        }
        float b = s_red[(2 * KH2) * kH + e];
#pragma unroll
        for (int ww = 1; ww < 4; ++ww) b += s_red[(ww * (2 * KH2 + 1) + 2 * KH2) * kH + e];
        acc_dbh[0] += b;
        __syncthreads();
    }

    __device__ __forceinline__ void col_row(int j, float h, const float (&g)[KP], const f2v (&wc2)[KH2],
                                            float *__restrict__ dzrow) {
#pragma clang fp contract(off)
        float d = 0.f;
        if constexpr (kPk) {
            // d head . w over the even and the odd outputs as one packed chain, then their sum (o >= K: s_dh and wc
            // are 0)
            f2v d2 = {0.f, 0.f};
#pragma unroll
            for (int o2 = 0; o2 < KH2; ++o2) d2 = __builtin_elementwise_fma(f2v{g[2 * o2], g[2 * o2 + 1]}, wc2[o2], d2);
            d = d2.x + d2.y;
            const f2v hh = {h, h};
#pragma unroll
            for (int o2 = 0; o2 < KH2; ++o2)  // KP >= 2 KH2: the pad slots of s_dh are 0
                acc_dw2[j][o2] = __builtin_elementwise_fma(f2v{g[2 * o2], g[2 * o2 + 1]}, hh, acc_dw2[j][o2]);
        } else {
#pragma unroll
            for (int o = 0; o < KMAX; ++o) {
                d += g[o] * wc[j][o];
                acc_dw[j][o] += g[o] * h;
            }
        }
        d *= act_g<ACT>(h, slope);
#if XPA_HEAD_PROBE != 4  // 4 = epilogue alone without the dz stores
        if (dz_on) {
            if (g_head_dz_plain) dzrow[e + NT * j] = d;   // A/B (xpa_head_store_probe): dz kept in the caches for K41 / K42
            else __builtin_nontemporal_store(d, dzrow + e + NT * j);
        }
#endif
        acc_dbh[j] += d;
    }

    // K12 / K16 (NW = 4, the whole block): phase 1 -> loss -> phase 2 with the block barriers between.  Starts with a
    // barrier (s_h complete), ends with one (s_h / s_dh free for the next tile).
    __device__ __forceinline__ void tile(const float *s_h, float (*s_part)[kTile][PH], float (*s_dh)[KP],
                                         const RowIn<KMAX> &in, int64_t tile, int64_t batch,
                                         const float *__restrict__ W, const float *__restrict__ bias,
                                         float *__restrict__ dz, int64_t ld, float ent_coef, float vf_coef) {
        __syncthreads();
        // unrolled: with a run-time pass (NPASS = 2, the wide heads) hd[pass PH + o] is a dynamic index and the whole
        // epilogue state went to scratch (r05: 600 B per lane, C4's actor head 196 us)
#pragma unroll
        for (int pass = 0; pass < NPASS; ++pass) {
            if (pass > 0) __syncthreads();  // wave 0 has read the previous pass
#if XPA_HEAD_PROBE != 10  // 10 = epilogue alone without phase 1
            p1(pass, s_h, s_part, W);
#endif
            __syncthreads();
#if XPA_HEAD_PROBE != 10
            p1_sum(pass, s_part, bias);
#endif
        }
#if XPA_HEAD_PROBE != 11  // 11 = epilogue alone without the loss
        loss(s_dh, in, ent_coef, vf_coef);
#endif
        __syncthreads();
        if (MODE == 2 && dv_out != nullptr && e < 64 && tile * kTile + e < batch) dv_out[tile * kTile + e] = s_dh[e][0];
        p2(s_h, s_dh, tile, batch, 0, kTile, dz, ld, W);
        __syncthreads();  // s_h / s_dh reused by the next tile
        if constexpr (kQuad) quad_flush(const_cast<float *>(s_h));
    }

    // Per-block partial row `blk`; with `zero_blk` >= 0 also a row of zeros (K16W: rows its grid does not own).
    __device__ __forceinline__ void finish(float *__restrict__ p_dw, float *__restrict__ p_dbh,
                                           float *__restrict__ p_dbo, float *__restrict__ p_loss, int loss_width,
                                           int64_t blk, int64_t zero_blk = -1) {
        const int lane = e & 63;
#pragma unroll
        for (int j = 0; j < CPT; ++j) {
            const int c = e + NT * j;
#pragma unroll
            for (int o = 0; o < KMAX; ++o)
                if (o < K) {
                    p_dw[(blk * K + o) * kH + c] = kPk ? acc_dw2[j][o >> 1][o & 1] : acc_dw[j][kPk ? 0 : o];
                    if (zero_blk >= 0) p_dw[(zero_blk * K + o) * kH + c] = 0.f;
                }
            p_dbh[blk * kH + c] = acc_dbh[j];
            if (zero_blk >= 0) p_dbh[zero_blk * kH + c] = 0.f;
        }
        if (e < 64) {
            sum0 = xpa_wave_sum(sum0);
            sum1 = xpa_wave_sum(sum1);
            sum2 = xpa_wave_sum(sum2);
#pragma unroll
            for (int o = 0; o < KMAX; ++o) {
                if (o < K) {
                    acc_dbo[o] = xpa_wave_sum(acc_dbo[o]);
                    if (MODE == 0) acc_dls[o] = xpa_wave_sum(acc_dls[o]);
                }
            }
            if (lane == 0) {
                float *prow = p_loss + blk * loss_width;
                if (MODE == 2) {
                    prow[1] = sum0;
                    prow[4] = sum1;
                } else {
                    prow[0] = sum0;
                    prow[2] = sum1;
                    prow[3] = sum2;
                }
                float *zrow = zero_blk >= 0 ? p_loss + zero_blk * loss_width : nullptr;
                if (zrow) {
                    if (MODE == 2) {
                        zrow[1] = 0.f;
                        zrow[4] = 0.f;
                    } else {
                        zrow[0] = zrow[2] = zrow[3] = 0.f;
                    }
                }
#pragma unroll
                for (int o = 0; o < KMAX; ++o) {
                    if (o < K) {
                        p_dbo[blk * K + o] = acc_dbo[o];
                        if (MODE == 0) prow[kPartBase + o] = acc_dls[o];
                        if (zrow) {
                            p_dbo[zero_blk * K + o] = 0.f;
                            if (MODE == 0) zrow[kPartBase + o] = 0.f;
                        }
                    }
                }
            }
        }
    }
};

#define XPA_HEAD_KERNEL_PARAMS                                                                                     \
    int64_t batch, int K_in, int64_t ld, const float *__restrict__ z, int64_t ldx, const float *__restrict__ Wh,   \
        const float *__restrict__ bh, const float *__restrict__ W, const float *__restrict__ bias, float slope,     \
        const float *__restrict__ logstd, const int64_t *__restrict__ idx, int64_t n_rows,                         \
        const float *__restrict__ act, const float *__restrict__ old_logp, const float *__restrict__ adv,          \
        const float *__restrict__ ret, const double *__restrict__ adv_partials, int64_t n_adv_partials,            \
        float clip_range, float ent_coef, float vf_coef, float *__restrict__ dz, float *__restrict__ p_dw,         \
        float *__restrict__ p_dbh, float *__restrict__ p_dbo, float *__restrict__ p_loss, int loss_width

// K12: z (the hidden pre-activations, row stride ld == ldx) streamed from HBM.
template <int MODE, int ALGO, int ACT, int KMAX>
__global__ __launch_bounds__(256, 2) void head_tile_kernel(XPA_HEAD_KERNEL_PARAMS) {
    using Epi = HeadEpi<MODE, ALGO, ACT, KMAX, 4, false>;
    __shared__ __attribute__((aligned(16))) float s_h[kTile * kS];
    __shared__ __attribute__((aligned(16))) float s_part[kWaves][kTile][Epi::PH];
    __shared__ __attribute__((aligned(16))) float s_dh[kTile][Epi::KP];
    __shared__ float s_stats[Epi::kStatN];
    const int t = threadIdx.x;
    const int64_t ntiles = (batch + kTile - 1) / kTile;
    if ((int64_t)blockIdx.x >= head_partials(batch)) return;  // no partial row of its own (see kGridMax)
    int64_t tile = blockIdx.x;
    float4 zq[16];
    load_tile(zq, z, ldx, tile, batch);
    Epi epi;
    epi.init_a(t, K_in, W, logstd, adv_partials, n_adv_partials, batch, clip_range, slope, s_stats);
    __syncthreads();
    epi.init_b(s_stats);
    for (; tile < ntiles; tile += gridDim.x) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {  // stage h = act(z)
            const int lin = i * 256 + t;
            float4 h;
            h.x = act_f<ACT>(zq[i].x, slope); h.y = act_f<ACT>(zq[i].y, slope);
            h.z = act_f<ACT>(zq[i].z, slope); h.w = act_f<ACT>(zq[i].w, slope);
            *reinterpret_cast<float4 *>(s_h + (lin >> 6) * kS + 4 * (lin & 63)) = h;
        }
        const RowIn<KMAX> in = epi.rows(tile, batch, idx, n_rows, act, old_logp, adv, ret);
        const int64_t next = tile + gridDim.x;
        if (next < ntiles) load_tile(zq, z, ldx, next, batch);  // in flight during the epilogue
        epi.tile(s_h, s_part, s_dh, in, tile, batch, W, bias, dz, ld, ent_coef, vf_coef);
    }
    epi.finish(p_dw, p_dbh, p_dbo, p_loss, loss_width, blockIdx.x);
}

// K16: the hidden layer's GEMM itself on the fp32 matrix cores, z = x Wh^T + bh for a [64 x 256] tile
// (v_mfma_f32_32x32x2_f32: exact f32 fma chains), then the K12 epilogue on the tile in LDS — z never
// goes to HBM.  Wave w owns columns [64w, 64w + 64) as 2 x 2 tiles of 32 x 32 (64 accumulator regs).
// Operands are staged by LDS-DMA (global_load_lds_dwordx4, no VGPR round trip) in chunks of 16 k
// through a 3-stage ring: chunk c + 2 is in flight while chunk c feeds the MFMAs, each wave waits only
// for its own chunk-c DMAs (counted vmcnt) before the one barrier per chunk.  A stage holds the A image
// (64 rows of x) and the B image (256 rows of Wh), every row 64 B = four 16-B slots, slot p of row r
// holding k quad q = p ^ ((r >> 2) & 3) — the swizzle is applied to the per-lane GLOBAL address (the DMA
// writes lane-linear), and makes the 16-lane groups of each ds_read_b128 cover the 16 slots of a bank
// row once.  Lane (i, h) reads quads h and h + 2 of its row; component s of quad q is k = 4q + s and is
// fed to the MFMA as its k = h: any k order is exact as long as A and B agree.
constexpr int kKin = 256;
constexpr int kKC = 16;
constexpr int kAImg = kTile * kKC;  // floats
constexpr int kBImg = kH * kKC;
constexpr int kStage = kAImg + kBImg;  // 20 KiB
constexpr int kStages = 3;
constexpr int kChunks = kKin / kKC;
static_assert(kStages * kStage <= kTile * kS, "operand stages share the epilogue tile");
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) char lds_char_t;

// One global_load_lds_dwordx4 (lane l's 16 B land at lds_wave_base + 16 l).  Issued from inline asm: the
// builtin form makes hipcc wait vmcnt(0) before every ds_read it cannot prove disjoint from an in-flight
// DMA — i.e. before each chunk's fragment reads, draining the ring; here the waits are the counted ones
// of the k-loop (and its last chunk waits vmcnt(0), so no compiler-counted wait after the loop is short).
__device__ __forceinline__ void glds16(const float *g, unsigned lds_wave_base) {
#if XPA_HEAD_PROBE == 6 || XPA_HEAD_PROBE == 9  // 6 = the GEMM without its operand DMAs (MFMA stream on stale LDS)
    asm volatile("" ::"v"(g), "s"(lds_wave_base) : "memory");
    return;
#endif
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(lds_wave_base)
                 : "memory", "m0");
}

// A chunk's 5 DMAs of wave w: A rows 16w .. 16w + 15, B rows 64w .. 64w + 63 (16 rows = 1 KiB each).
// st: LDS byte address of the stage.  Rows past the batch re-read the last row (results never used).
__device__ __forceinline__ void gemm_issue(unsigned st, const float *__restrict__ x, int64_t ldx,
                                           const float *__restrict__ Wh, int64_t r0, int64_t batch, int k0,
                                           int lane, int wave) {
    const int rr = lane >> 2, p = lane & 3;
    const int q = p ^ ((rr >> 2) & 3);  // (row >> 2) & 3 == (rr >> 2) & 3: row bases are multiples of 16
    int64_t grow = r0 + wave * 16 + rr;
    grow = grow < batch ? grow : batch - 1;
    glds16(x + grow * ldx + k0 + 4 * q, st + (unsigned)(wave * 16 * kKC * 4));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int row = wave * 64 + j * 16 + rr;
        glds16(Wh + row * kKin + k0 + 4 * q, st + (unsigned)((kAImg + (wave * 64 + j * 16) * kKC) * 4));
    }
}
constexpr int kDmaPerChunk = 5;  // per wave: the vmcnt count that leaves one chunk in flight

__device__ __forceinline__ void gemm_chunk(const float *st, f32x16 (&acc)[2][2], int lane, int wave) {
    const float *A = st, *B = st + kAImg;
    const int h = lane >> 5, i = lane & 31;
    const int sw = (i >> 2) & 3;
    const int olo = 4 * (h ^ sw), ohi = 4 * ((h + 2) ^ sw);
    float4 alo[2], ahi[2], blo[2], bhi[2];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
        const float *pa = A + (rt * 32 + i) * kKC;
        alo[rt] = *reinterpret_cast<const float4 *>(pa + olo);
        ahi[rt] = *reinterpret_cast<const float4 *>(pa + ohi);
    }
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
        const float *pb = B + (wave * 64 + ct * 32 + i) * kKC;
        blo[ct] = *reinterpret_cast<const float4 *>(pb + olo);
        bhi[ct] = *reinterpret_cast<const float4 *>(pb + ohi);
    }
#pragma unroll
    for (int s2 = 0; s2 < 8; ++s2) {
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            const float4 &av = s2 < 4 ? alo[rt] : ahi[rt];
            const float a = (s2 & 3) == 0 ? av.x : (s2 & 3) == 1 ? av.y : (s2 & 3) == 2 ? av.z : av.w;
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                const float4 &bv = s2 < 4 ? blo[ct] : bhi[ct];
                const float b = (s2 & 3) == 0 ? bv.x : (s2 & 3) == 1 ? bv.y : (s2 & 3) == 2 ? bv.z : bv.w;
                acc[rt][ct] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[rt][ct], 0, 0, 0);
            }
        }
    }
}

// K16S (r04): gemm_chunk's k step on the bf16 matrix cores by the three-way split (s3_split.h): the same LDS images
// and fragment reads, each wave splits its two A and two B fragments (8 f32 per lane each) in VALU and runs 4 x 6
// v_mfma_f32_32x32x16_bf16 (the element order j of a fragment is gemm_chunk's k order s2 — quads h, h + 2 — for A and
// B alike).  2.67x fewer matrix-core cycles per chunk than the 32 f32 MFMAs; the f32 GEMM's accuracy, not its bits.
__device__ __forceinline__ void gemm_chunk_s3(const float *st, f32x16 (&acc)[2][2], int lane, int wave) {
    const float *A = st, *B = st + kAImg;
    const int h = lane >> 5, i = lane & 31;
    const int sw = (i >> 2) & 3;
    const int olo = 4 * (h ^ sw), ohi = 4 * ((h + 2) ^ sw);
    xpa_bf16x8 ah[2], am[2], al[2], bh[2], bm[2], bl[2];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
        const float *pa = A + (rt * 32 + i) * kKC;
        xpa_split8(*reinterpret_cast<const float4 *>(pa + olo), *reinterpret_cast<const float4 *>(pa + ohi), ah[rt],
                   am[rt], al[rt]);
    }
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
        const float *pb = B + (wave * 64 + ct * 32 + i) * kKC;
        xpa_split8(*reinterpret_cast<const float4 *>(pb + olo), *reinterpret_cast<const float4 *>(pb + ohi), bh[ct],
                   bm[ct], bl[ct]);
    }
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
            acc[rt][ct] = xpa_mfma_s3(ah[rt], am[rt], al[rt], bh[ct], bm[ct], bl[ct], acc[rt][ct]);
}

// K16P (r04): K16S with Wh's three bf16 planes split once per update (xpa_s3_split_b of Wh^T, K40's layout: per 16-k
// chunk 24 KiB = [plane][column block][lane][16 B]) and DMA'd as they are, so the waves split only their A fragments.
// A chunk's stage is 4 KiB of A + 24 KiB of planes; two stages (56 KiB) fit the epilogue tile, so the ring is one
// chunk deep: chunk c + 1 is issued right after chunk c's barrier.
constexpr int kPStageB = 4096 + 24576;  // bytes
static_assert(2 * kPStageB <= kTile * kS * 4, "two K16P stages share the epilogue tile");
__device__ __forceinline__ void gemm_issue_p(unsigned st, const float *__restrict__ x, int64_t ldx,
                                             const char *__restrict__ wsp, int64_t r0, int64_t batch, int c, int lane,
                                             int wave) {
    const int rr = lane >> 2, p = lane & 3;
    const int q = p ^ ((rr >> 2) & 3);
    int64_t grow = r0 + wave * 16 + rr;
    grow = grow < batch ? grow : batch - 1;
    glds16(x + grow * ldx + c * kKC + 4 * q, st + (unsigned)(wave * 16 * kKC * 4));
#if XPA_HEAD_PROBE == 7  // 7 = K16P without its B-plane DMAs (A rows still staged)
    return;
#endif
    const char *src = wsp + (int64_t)c * 24576;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const int piece = wave * 6 + j;
        glds16(reinterpret_cast<const float *>(src + piece * 1024 + lane * 16), st + (unsigned)(4096 + piece * 1024));
    }
}
constexpr int kPDmaPerChunk = 7;

__device__ __forceinline__ void gemm_chunk_s3p(const char *st, f32x16 (&acc)[2][2], int lane, int wave) {
    const float *A = reinterpret_cast<const float *>(st);
    const int h = lane >> 5, i = lane & 31;
    const int sw = (i >> 2) & 3;
    const int olo = 4 * (h ^ sw), ohi = 4 * ((h + 2) ^ sw);
    xpa_bf16x8 ah[2], am[2], al[2];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
        const float *pa = A + (rt * 32 + i) * kKC;
#if XPA_HEAD_PROBE == 8 || XPA_HEAD_PROBE == 9  // 8 = K16P without the A split (f32 bits fed as bf16); 9 = also no DMAs
        const float4 lo = *reinterpret_cast<const float4 *>(pa + olo), hi = *reinterpret_cast<const float4 *>(pa + ohi);
        ah[rt] = __builtin_bit_cast(xpa_bf16x8, lo);
        am[rt] = __builtin_bit_cast(xpa_bf16x8, hi);
        al[rt] = __builtin_bit_cast(xpa_bf16x8, lo);
#else
        xpa_split8(*reinterpret_cast<const float4 *>(pa + olo), *reinterpret_cast<const float4 *>(pa + ohi), ah[rt],
                   am[rt], al[rt]);
#endif
    }
    const xpa_bf16x8 *bimg = reinterpret_cast<const xpa_bf16x8 *>(st + 4096) + lane;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
        const int cb = 2 * wave + ct;
        const xpa_bf16x8 bh = bimg[cb * 64], bm = bimg[(8 + cb) * 64], bl = bimg[(16 + cb) * 64];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) acc[rt][ct] = xpa_mfma_s3(ah[rt], am[rt], al[rt], bh, bm, bl, acc[rt][ct]);
    }
}

// K16Q (r04): K16P's operands with the waves tiled 2 x 2 over the [64 x 256] tile as 32 rows x 128 columns each
// (row tile wave & 1, column blocks 4 (wave >> 1) .. + 3) instead of 64 rows x 64 columns: each wave splits ONE A
// fragment per chunk (K16P: both row tiles, so every A value was split by all 4 waves) and reads 4 B column blocks'
// planes (ds_read_b128, no VALU).  Every output's accumulation chain is K16P's: bit for bit the same dz / partials.
__device__ __forceinline__ void gemm_chunk_s3q(const char *st, f32x16 (&acc)[2][2], int lane, int wave) {
    const float *A = reinterpret_cast<const float *>(st);
    const int h = lane >> 5, i = lane & 31;
    const int sw = (i >> 2) & 3;
    const float *pa = A + ((wave & 1) * 32 + i) * kKC;
    xpa_bf16x8 ah, am, al;
#if XPA_HEAD_PROBE == 8 || XPA_HEAD_PROBE == 9 || XPA_HEAD_PROBE == 12  // the A split's cost: f32 bits fed as bf16
    {
        const float4 lo = *reinterpret_cast<const float4 *>(pa + 4 * (h ^ sw)),
                     hi = *reinterpret_cast<const float4 *>(pa + 4 * ((h + 2) ^ sw));
        ah = __builtin_bit_cast(xpa_bf16x8, lo);
        am = __builtin_bit_cast(xpa_bf16x8, hi);
        al = __builtin_bit_cast(xpa_bf16x8, lo);
    }
#else
    xpa_split8(*reinterpret_cast<const float4 *>(pa + 4 * (h ^ sw)),
               *reinterpret_cast<const float4 *>(pa + 4 * ((h + 2) ^ sw)), ah, am, al);
#endif
    const xpa_bf16x8 *bimg = reinterpret_cast<const xpa_bf16x8 *>(st + 4096) + lane;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int cb = 4 * (wave >> 1) + j;
        acc[j >> 1][j & 1] = xpa_mfma_s3(ah, am, al, bimg[cb * 64], bimg[(8 + cb) * 64], bimg[(16 + cb) * 64],
                                         acc[j >> 1][j & 1]);
    }
}

// K16R (r04): K16P with the A operand (the trunk activations h) formed in the k loop instead of read from HBM:
// h = act(x W0^T + b0) for the tile's 64 rows, the representation's one thin layer (K13's Linear(d_in <= 20, 256) +
// activation, its fmaf chain over the zero-padded inputs: the same bits as K13's h).  Thread t owns row t >> 2 of
// the tile and slot p = t & 3 of the chunk's swizzled A image (k quad q = p ^ ((row >> 2) & 3), gemm_issue_p's
// layout), so per 16-k chunk it forms 4 values (80 FMAs from its x row in registers and 4 W0 rows in LDS) and writes
// them with one ds_write_b128 where the DMA would have landed them.  W0 / b0 are staged per tile beside the two
// operand stages (the epilogue reuses that LDS).  The actor launch also writes h (K41's operand) and its sign bits
// (K42's act' for LeakyReLU / identity); K13 only gathers the minibatch rows (64 MiB of h writes and 192 MiB of h
// reads fewer per C2 update).
constexpr int kRW = 20;                                   // W0 row stride in LDS (= kTrunkDMax, zero padded)
constexpr int kROff = 2 * kPStageB;                       // bytes: W0 then b0 after the two stages
constexpr int kREnd = kROff + (kH * kRW + kH) * 4;       // 78848 B
__device__ __forceinline__ void gemm_issue_b(unsigned st, const char *__restrict__ wsp, int c, int lane, int wave) {
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const int piece = wave * 6 + j;
        glds16(reinterpret_cast<const float *>(wsp + (int64_t)c * 24576 + piece * 1024 + lane * 16),
               st + (unsigned)(4096 + piece * 1024));
    }
}

// lane p of a row's 4 lanes (a DPP quad) holds x[4 i + p] in xq[i]: x[k] = quad broadcast of xq[k >> 2] from lane
// k & 3 (folded into the FMAs as DPP operands), 5 VGPRs instead of 20 for the row
__device__ __forceinline__ float quad_bcast(float v, int j) {
    const int ctrl = j * 0x55;   // quad_perm [j, j, j, j]
    int r;
    switch (j) {
        case 0: r = __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x00, 0xF, 0xF, false); break;
        case 1: r = __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x55, 0xF, 0xF, false); break;
        case 2: r = __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xAA, 0xF, 0xF, false); break;
        default: r = __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xFF, 0xF, 0xF, false); break;
    }
    (void)ctrl;
    return __builtin_bit_cast(float, r);
}

template <int ACT>
__device__ __forceinline__ void trunk_chunk(char *st, const float *s_w0, const float (&xq)[kRW / 4], int c, int q,
                                            float slope0, float4 &hq) {
    const int k0 = 16 * c + 4 * q;
    const float4 bq = *reinterpret_cast<const float4 *>(s_w0 + kH * kRW + k0);
    float hv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float *wr = s_w0 + (k0 + j) * kRW;
        float a0 = 0.f;
#pragma unroll
        for (int i = 0; i < kRW / 4; ++i) {
            const float4 w4 = *reinterpret_cast<const float4 *>(wr + 4 * i);
            a0 = fmaf(quad_bcast(xq[i], 0), w4.x, a0);
            a0 = fmaf(quad_bcast(xq[i], 1), w4.y, a0);
            a0 = fmaf(quad_bcast(xq[i], 2), w4.z, a0);
            a0 = fmaf(quad_bcast(xq[i], 3), w4.w, a0);
        }
        const float b = j == 0 ? bq.x : j == 1 ? bq.y : j == 2 ? bq.z : bq.w;
        hv[j] = act_f<ACT>(a0 + b, slope0);
    }
    hq = make_float4(hv[0], hv[1], hv[2], hv[3]);
    *reinterpret_cast<float4 *>(st + 16 * threadIdx.x) = hq;
}

// K16X prologue (r03): the representation's first layer (K13's Linear(d_in <= 20, 256) + activation, bit for bit
// its fmaf chain over the zero-padded inputs) for the tile's rows, from the minibatch's gathered observation rows;
// thread t = column t; h goes to HBM (the backward's copy) with plain stores, so the k loop's A-operand DMAs right
// after read it from L2.  s_x: [64][DMAX] floats of LDS (the operand ring's space, free until the first DMA).
// Ends with every store drained and a block barrier.
constexpr int kTrunkDMax = 20;
template <int ACT>
__device__ __forceinline__ void trunk_prologue(float *s_x, const float *__restrict__ xr, int64_t ldxr, int din,
                                               const float *__restrict__ W0, const float *__restrict__ b0,
                                               float slope0, float *__restrict__ hout, int64_t ldh, int64_t r0,
                                               int64_t batch) {
    constexpr int DMAX = kTrunkDMax;
    const int t = threadIdx.x;
    float w0[DMAX];
#pragma unroll
    for (int k = 0; k < DMAX; ++k) w0[k] = W0[t * din + (k < din ? k : 0)];
#pragma unroll
    for (int k = 0; k < DMAX; ++k) w0[k] = k < din ? w0[k] : 0.f;
    const float b0c = b0[t];
    for (int e = t; e < kTile * DMAX; e += 256) {
        const int r = e / DMAX, k = e - r * DMAX;
        const int64_t row = r0 + r < batch ? r0 + r : batch - 1;
        const float v = xr[row * ldxr + (k < din ? k : 0)];
        s_x[e] = (k < din && r0 + r < batch) ? v : 0.f;
    }
    __syncthreads();
    const int nr = (int)min((int64_t)kTile, batch - r0);
    for (int r = 0; r < nr; ++r) {
        const float *xrow = s_x + r * DMAX;
        float a0 = 0.f;
#pragma unroll
        for (int k = 0; k < DMAX; k += 4) {
            const float4 xv = *reinterpret_cast<const float4 *>(xrow + k);
            a0 = fmaf(xv.x, w0[k], a0);
            a0 = fmaf(xv.y, w0[k + 1], a0);
            a0 = fmaf(xv.z, w0[k + 2], a0);
            a0 = fmaf(xv.w, w0[k + 3], a0);
        }
        hout[(r0 + r) * ldh + t] = act_f<ACT>(a0 + b0c, slope0);
    }
    xpa_drain();      // this block's h rows are in L2 before any wave's DMA reads them
    __syncthreads();  // (and every wave is done with s_x before the ring overwrites it)
}

// TRUNK (K16X, r03): the prologue above forms the tile's A rows (h) first; z / ldx are then ignored and the k loop
// reads A from hout / ldh.
template <int MODE, int ALGO, int ACT, int KMAX, bool TRUNK = false, int S3 = 0>
__global__ __launch_bounds__(256, 2) void head_gemm_kernel(XPA_HEAD_KERNEL_PARAMS, const float *__restrict__ xr = nullptr,
                                                           int64_t ldxr = 0, int din = 0,
                                                           const float *__restrict__ W0 = nullptr,
                                                           const float *__restrict__ b0 = nullptr, float slope0 = 0.f,
                                                           float *__restrict__ hout = nullptr, int64_t ldh = 0,
                                                           unsigned *__restrict__ hmask = nullptr,
                                                           unsigned *__restrict__ cmask = nullptr,
                                                           float *__restrict__ cdv = nullptr) {
    using Epi = HeadEpi<MODE, ALGO, ACT, KMAX>;
    // ONE LDS array (a second __shared__ object beside the DMA target can make hipcc wait vmcnt(0) before
    // every chunk's ds_reads): operand stages / h tile, then the epilogue's partials, d head and stats.
    constexpr int kPartOff = kTile * kS, kDhOff = kPartOff + kWaves * kTile * Epi::PH;
    constexpr int kStatsOff = kDhOff + kTile * Epi::KP;
    constexpr int kStatsEnd = kStatsOff + (Epi::kStatN > 4 ? Epi::kStatN : 4);
    static_assert(KMAX <= 8 || kStatsEnd * 4 <= 81920, "wide heads: 2 blocks per CU");
    constexpr int kLdsBase = S3 == 3 && kREnd / 4 > kStatsEnd ? kREnd / 4 : kStatsEnd;
    // K16Q (r06): the hidden bias staged once per launch past everything else (the h conversion's bias reads, 4 per
    // lane and tile, were serial L2 round trips after the k loop)
    static_assert(kLdsBase * 4 <= 81920, "2 blocks per CU");
    constexpr bool kBhLds = S3 == 4 && (kLdsBase + kH) * 4 <= 81920;   // the widest heads have no 1 KiB to spare
    constexpr int kBhOff = kLdsBase, kLdsFloats = kLdsBase + (kBhLds ? kH : 0);
    __shared__ __attribute__((aligned(16))) float lds[kLdsFloats];
    float *smem = lds;
    auto s_part = reinterpret_cast<float(*)[kTile][Epi::PH]>(lds + kPartOff);
    auto s_dh = reinterpret_cast<float(*)[Epi::KP]>(lds + kDhOff);
    float *s_stats = lds + kStatsOff;
    const unsigned lds_base = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_char_t *)lds);
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int64_t ntiles = (batch + kTile - 1) / kTile;
    if ((int64_t)blockIdx.x >= head_partials(batch)) return;  // no partial row of its own (see kGridMax)
    // r06 (xpa_head_stagger, A/B): the second wave of resident blocks (blockIdx >= 256: the second block slot of each CU)
    // starts g_head_stagger x ~0.85 us late, so that its k loop runs beside the first block's epilogue instead of in
    // phase with it (both blocks' GEMMs sharing the matrix cores, then both epilogues sharing the VALU).  0: off.
    if (g_head_stagger > 0 && blockIdx.x >= 256)
        for (int i = 0; i < g_head_stagger; ++i) __builtin_amdgcn_s_sleep(32);
    Epi epi;
    epi.init_a(t, K_in, W, logstd, adv_partials, n_adv_partials, batch, clip_range, slope, s_stats);
    epi.mask_out = cmask;
    epi.dv_out = cdv;
    epi.dz_on = dz != nullptr;
    if constexpr (kBhLds) lds[kBhOff + t] = bh[t];   // kH == 256 == blockDim.x
    __syncthreads();
    epi.init_b(s_stats);
    const float bh0 = bh[wave * 64 + (lane & 31)], bh1 = bh[wave * 64 + 32 + (lane & 31)];
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t r0 = tile * kTile;
        // the rows' inputs load before the k loop (their latency hidden behind it) — for the wide heads (C4) after it:
        // act[18] live across the k loop pushed the kernel past 256 registers (r05: 608 B of scratch per lane)
        RowIn<KMAX> in;
        if constexpr (KMAX <= 8) in = epi.rows(tile, batch, idx, n_rows, act, old_logp, adv, ret);
        f32x16 acc[2][2];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[rt][ct][r] = 0.f;
        __syncthreads();  // the previous tile's epilogue is done with smem
        const float *xa = z;
        int64_t lda = ldx;
        if constexpr (TRUNK) {
            trunk_prologue<ACT>(smem, xr, ldxr, din, W0, b0, slope0, hout, ldh, r0, batch);
            xa = hout;
            lda = ldh;
        }
#if XPA_HEAD_PROBE != 2 && XPA_HEAD_PROBE != 4 && XPA_HEAD_PROBE != 5 && XPA_HEAD_PROBE != 10 && XPA_HEAD_PROBE != 11  // tools/head_probe.py: 2 = epilogue alone (4, 5, 10, 11: parts of it)
        if constexpr (S3 == 3) {   // K16R: B as K16P, A formed from the gathered rows (see trunk_chunk)
            const char *wsp = reinterpret_cast<const char *>(Wh);
            float *s_w0 = reinterpret_cast<float *>(reinterpret_cast<char *>(smem) + kROff);
            gemm_issue_b(lds_base, wsp, 0, lane, wave);
            for (int e = t; e < kH * kRW; e += 256) {
                const int cc = e / kRW, k = e - cc * kRW;
                s_w0[e] = k < din ? W0[cc * din + k] : 0.f;
            }
            s_w0[kH * kRW + t] = b0[t];
            // rows past the batch form (and the actor writes) row batch - 1's values again: the same bits, so the
            // stores need no predicate and every wave issues the same count (the counted waits below)
            const int rr = t >> 2, q = (t & 3) ^ ((rr >> 2) & 3);
            const int64_t xrow = r0 + rr < batch ? r0 + rr : batch - 1;
            float xv[kRW / 4];
#pragma unroll
            for (int i = 0; i < kRW / 4; ++i) {
                const int k = 4 * i + (t & 3);
                const float v = xr[xrow * ldxr + (k < din ? k : 0)];
                xv[i] = k < din ? v : 0.f;
            }
            __syncthreads();   // W0 / b0 staged (and chunk 0's planes landed)
            float *hrow = hout != nullptr ? hout + xrow * ldh + 4 * q : nullptr;
            // sign bits, K42S's lane order: byte b of a row's 32 bytes holds bit j = h[row, 32 j + b] > 0, so this
            // thread's 4 columns 16 c + 4 q + i (i < 4) of every chunk of parity P land in bytes 16 P + 4 q + i, bit c / 2
            unsigned sgn[2] = {0u, 0u};
            auto form = [&](int c) {
                float4 hq;
                trunk_chunk<ACT>(reinterpret_cast<char *>(smem) + (c & 1) * kPStageB, s_w0, xv, c, q, slope0, hq);
                if (hrow != nullptr) {
                    *reinterpret_cast<float4 *>(hrow + 16 * c) = hq;
                    const unsigned sh = (unsigned)(c >> 1);
                    const unsigned add = ((hq.x > 0.f ? 1u : 0u) << sh) | ((hq.y > 0.f ? 1u : 0u) << (8 + sh)) |
                                         ((hq.z > 0.f ? 1u : 0u) << (16 + sh)) | ((hq.w > 0.f ? 1u : 0u) << (24 + sh));
                    if (c & 1) sgn[1] |= add;
                    else sgn[0] |= add;
                }
            };
            form(0);
#pragma unroll 1
            for (int c = 0; c < kChunks; ++c) {
                // chunk c's planes landed (the store of chunk c's h, issued after them, may still fly) and every
                // wave wrote its A image; chunk c - 1's stage is free
                if (hrow != nullptr) asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)\n\ts_barrier" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
                if (c + 1 < kChunks) gemm_issue_b(lds_base + ((c + 1) & 1) * kPStageB, wsp, c + 1, lane, wave);
#if XPA_HEAD_PROBE != 3
                gemm_chunk_s3p(reinterpret_cast<const char *>(smem) + (c & 1) * kPStageB, acc, lane, wave);
#endif
                if (c + 1 < kChunks) form(c + 1);
            }
            if (hrow != nullptr && hmask != nullptr) {
                hmask[xrow * 8 + q] = sgn[0];
                hmask[xrow * 8 + 4 + q] = sgn[1];
            }
        } else if constexpr (S3 == 2 || S3 == 4) {   // K16P / K16Q: Wh arrives as its three bf16 planes (the split buffer)
            const char *wsp = reinterpret_cast<const char *>(Wh);
            gemm_issue_p(lds_base, xa, lda, wsp, r0, batch, 0, lane, wave);
#pragma unroll 1
            for (int c = 0; c < kChunks; ++c) {
                // own chunk-c DMAs landed, then every wave's; chunk c - 1's stage (the one c + 1 refills) was read
                asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
                if (c + 1 < kChunks)
                    gemm_issue_p(lds_base + ((c + 1) & 1) * kPStageB, xa, lda, wsp, r0, batch, c + 1, lane, wave);
#if XPA_HEAD_PROBE != 3
                if constexpr (S3 == 4) gemm_chunk_s3q(reinterpret_cast<const char *>(smem) + (c & 1) * kPStageB, acc, lane, wave);
                else gemm_chunk_s3p(reinterpret_cast<const char *>(smem) + (c & 1) * kPStageB, acc, lane, wave);
#endif
            }
        } else {
        gemm_issue(lds_base, xa, lda, Wh, r0, batch, 0, lane, wave);
        gemm_issue(lds_base + kStage * 4, xa, lda, Wh, r0, batch, kKC, lane, wave);
#pragma unroll 1
        for (int c = 0; c < kChunks; ++c) {
            // own DMAs of chunk c landed (chunk c + 1's may still fly), then every wave's: chunk c is in
            // LDS and chunk c - 1's stage — the one chunk c + 2 refills — has been read by all waves
            if (c + 1 < kChunks) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(kDmaPerChunk) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
            if (c + 2 < kChunks)
                gemm_issue(lds_base + ((c + 2) % kStages) * kStage * 4, xa, lda, Wh, r0, batch, (c + 2) * kKC, lane,
                           wave);
#if XPA_HEAD_PROBE != 3  // 3 = operand staging alone
            if constexpr (S3 == 1) gemm_chunk_s3(smem + (c % kStages) * kStage, acc, lane, wave);
            else gemm_chunk(smem + (c % kStages) * kStage, acc, lane, wave);
#endif
        }
        }
        __syncthreads();  // every wave done with the stages before the h tile overwrites them
#endif
        // h = act(z + bh) into the tile image: C/D map row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5), col = lane & 31
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                // K16Q: acc[a][b] is column block 2 a + b of the wave's 128 columns, rows of row tile wave & 1
                const int col = S3 == 4 ? (wave >> 1) * 128 + (2 * rt + ct) * 32 + (lane & 31)
                                        : wave * 64 + ct * 32 + (lane & 31);
                const float bc = kBhLds ? lds[kBhOff + col] : S3 == 4 ? bh[col] : ct ? bh1 : bh0;
                const int row0 = S3 == 4 ? (wave & 1) * 32 : rt * 32;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = row0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    smem[row * kS + col] = act_f<ACT>(acc[rt][ct][r] + bc, slope);
                }
            }
#if XPA_HEAD_PROBE == 1 || XPA_HEAD_PROBE == 3 || XPA_HEAD_PROBE == 6 || XPA_HEAD_PROBE == 12  // the GEMM alone: keep its result live
        __syncthreads();
        if (r0 + (t >> 2) < batch) dz[(r0 + (t >> 2)) * ld + (t & 3)] = smem[(t >> 2) * kS + (t & 3)];
#else
        if constexpr (KMAX > 8) in = epi.rows(tile, batch, idx, n_rows, act, old_logp, adv, ret);
        epi.tile(smem, s_part, s_dh, in, tile, batch, W, bias, dz, ld, ent_coef, vf_coef);
#endif
    }
    epi.finish(p_dw, p_dbh, p_dbo, p_loss, loss_width, blockIdx.x);
}

// K16W (r04): K16 with its waves specialised, one 512-thread block per CU persistent over 64-row tiles, so that the
// K12 epilogue of tile n runs on other waves WHILE the matrix cores compute tile n + 1 (K16 runs them one after the
// other inside a block; its two co-resident blocks overlap them only by chance).
//   waves 0-3 (G): tile n + 1's hidden GEMM exactly as K16 (wave g: columns 64g .. 64g + 63 as 2 x 2 32x32 tiles,
//                  v_mfma_f32_32x32x2_f32, the same k order), then h = act(z + bh) into the h tile;
//   waves 4-5 (E): the K12 epilogue of tile n on the h tile, split into barrier-separated steps (phase-1 passes, their
//                  sums + the loss, phase 2 in 8-row slices) that fit between the GEMM's k-chunk barriers;
//   waves 6-7 (D): only the operand DMAs of the 3-stage ring (chunk q + 2 right after the barrier of chunk q, 10
//                  global_load_lds_dwordx4 per wave and chunk), so their hand-counted vmcnt sees no other memory op.
// One block barrier per k chunk (the D waves' vmcnt for chunk q before it), two per tile for the h hand-off.  The
// chunk sequence runs on across a block's tiles, so the next tile's first chunks are in flight during the last ones.
// Every output is K16's arithmetic (shared gemm_chunk and HeadEpi; NW = 2 only changes which thread runs a chain):
// bit for bit K16's dz and partials (tests/test_gpu_fused_mlp.py).  KMAX <= 8 (the E waves' state beside G's
// accumulators must fit 256 VGPRs); wider heads (C4's A = 17) keep K16.
constexpr int kWsGridMax = 256;  // one block per CU
constexpr int kWsP2Split = 8;    // phase-2 slices per tile (8 rows each)
constexpr int kWsStages = 4;     // operand ring: chunk q + 3 is issued during chunk q (3 chunks of DMA flight time)
constexpr int kWsDma = 10;       // DMAs per D wave and chunk
// diagnostics (tools/k16w_ab.py --probe): bit 0 the E waves skip the epilogue steps, bit 1 the G waves skip their MFMAs
// (and the h write), bit 2 the D waves issue no DMAs; every barrier stays.  0 in production.
__device__ int g_ws_probe = 0;
__host__ __device__ constexpr int64_t head_ws_grid(int64_t batch) {
    return (batch + kTile - 1) / kTile < kWsGridMax ? (batch + kTile - 1) / kTile : kWsGridMax;
}

template <int MODE, int ALGO, int ACT, int KMAX>
__global__ __launch_bounds__(512, 1) void head_gemm_ws_kernel(XPA_HEAD_KERNEL_PARAMS) {
    static_assert(KMAX <= 8, "K16W: heads up to 8 wide");
    using Epi = HeadEpi<MODE, ALGO, ACT, KMAX, 2>;
    constexpr int kHOff = kWsStages * kStage;  // the ring, then the h tile (both live at once here)
    constexpr int kPartOff = kHOff + kTile * kS;
    constexpr int kDhOff = kPartOff + kWaves * kTile * Epi::PH;
    constexpr int kStatsOff = kDhOff + kTile * Epi::KP;
    static_assert((kStatsOff + 4) * 4 <= 160 * 1024, "K16W: one block per CU");
    constexpr int kSteps = 2 * Epi::NPASS + kWsP2Split;  // E's steps per tile
    static_assert(kSteps <= kChunks, "the epilogue steps fit between the GEMM's chunk barriers");
    __shared__ __attribute__((aligned(16))) float lds[kStatsOff + 4];
    float *smem = lds;
    float *s_h = lds + kHOff;
    auto s_part = reinterpret_cast<float(*)[kTile][Epi::PH]>(lds + kPartOff);
    auto s_dh = reinterpret_cast<float(*)[Epi::KP]>(lds + kDhOff);
    float *s_stats = lds + kStatsOff;
    const unsigned lds_base = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_char_t *)lds);
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const bool is_g = wave < 4, is_e = wave == 4 || wave == 5, is_d = wave >= 6;
    const int64_t ntiles = (batch + kTile - 1) / kTile;
    const int64_t G = gridDim.x, blk = blockIdx.x;
    if (blk >= ntiles) return;  // the grid is at most the tile count (head_ws_grid): never taken
    const int64_t my_tiles = (ntiles - 1 - blk) / G + 1;
    const int64_t nchunks = my_tiles * kChunks;
    const int probe = __builtin_amdgcn_readfirstlane(g_ws_probe);
    // Each role runs its own copy of the period / chunk loop (so the allocator sees G's accumulators and E's epilogue
    // state in disjoint branches); every copy executes the same barrier sequence: per period, one per chunk (or per
    // epilogue step in the last period) and the two of the h hand-off.
    Epi epi;
    if (is_e) epi.init_a(t - 256, K_in, W, logstd, adv_partials, n_adv_partials, batch, clip_range, slope, s_stats);
    __syncthreads();  // s_stats; no DMA in flight yet
    if (is_g) {
        const float bh0 = bh[wave * 64 + (lane & 31)], bh1 = bh[wave * 64 + 32 + (lane & 31)];
#pragma unroll 1
        for (int64_t i = 0; i <= my_tiles; ++i) {
            const bool gemm = i < my_tiles;
            f32x16 acc[2][2];
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[rt][ct][r] = 0.f;
            const int nph = gemm ? kChunks : kSteps;
#pragma unroll 1
            for (int c = 0; c < nph; ++c) {
                asm volatile("s_barrier" ::: "memory");
                if (gemm && !(probe & 2)) gemm_chunk(smem + ((i * kChunks + c) % kWsStages) * kStage, acc, lane, wave);
            }
            asm volatile("s_barrier" ::: "memory");  // X: the E waves are done with the h tile of tile i - 1
            if (gemm && !(probe & 2)) {
                // h = act(z + bh) into the h tile: C/D map row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5), col = lane & 31
#pragma unroll
                for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                    for (int ct = 0; ct < 2; ++ct) {
                        const int col = wave * 64 + ct * 32 + (lane & 31);
                        const float bc = ct ? bh1 : bh0;
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const int row = rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                            s_h[row * kS + col] = act_f<ACT>(acc[rt][ct][r] + bc, slope);
                        }
                    }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
            asm volatile("s_barrier" ::: "memory");  // Y: the h tile of tile i is complete
        }
    } else if (is_e) {
        epi.init_b(s_stats);
        RowIn<KMAX> in_cur = {}, in_nxt = {};
#pragma unroll 1
        for (int64_t i = 0; i <= my_tiles; ++i) {  // period i: the epilogue of the block's tile i - 1
            const bool gemm = i < my_tiles, epil = i > 0;
            const int64_t tile_e = blk + (i - 1) * G;
            if (gemm) in_nxt = epi.rows(blk + i * G, batch, idx, n_rows, act, old_logp, adv, ret);  // used next period
            const int nph = gemm ? kChunks : kSteps;
#pragma unroll 1
            for (int c = 0; c < nph; ++c) {
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // the previous step's LDS writes done
                if (!epil || c >= kSteps || (probe & 1)) continue;
                if (c < 2 * Epi::NPASS) {
                    const int pass = c >> 1;
                    if ((c & 1) == 0) {
                        epi.p1(pass, s_h, s_part, W);
                    } else {
                        epi.p1_sum(pass, s_part, bias);
                        if (pass == Epi::NPASS - 1) epi.loss(s_dh, in_cur, ent_coef, vf_coef);
                    }
                } else {
                    const int sl = c - 2 * Epi::NPASS;
                    epi.p2(s_h, s_dh, tile_e, batch, sl * (kTile / kWsP2Split), (sl + 1) * (kTile / kWsP2Split), dz,
                           ld);
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // X
            asm volatile("s_barrier" ::: "memory");                           // Y
            in_cur = in_nxt;
        }
        const int64_t np = head_partials(batch);
        epi.finish(p_dw, p_dbh, p_dbo, p_loss, loss_width, blk, blk + G < np ? blk + G : -1);
    } else {  // D: wave d issues the A / B rows K16's waves 2d and 2d + 1 would
        const int d = wave - 6;
        const bool dma = !(probe & 4);
        auto issue = [&](int64_t q) {
            if (!dma) return;
            const int64_t tile = blk + (q / kChunks) * G;
            const unsigned st = lds_base + (unsigned)((q % kWsStages) * kStage * 4);
            gemm_issue(st, z, ldx, Wh, tile * kTile, batch, (int)(q % kChunks) * kKC, lane, 2 * d);
            gemm_issue(st, z, ldx, Wh, tile * kTile, batch, (int)(q % kChunks) * kKC, lane, 2 * d + 1);
        };
        constexpr int L = kWsStages - 1;  // chunks in flight ahead of the one being consumed
        for (int64_t q = 0; q < L && q < nchunks; ++q) issue(q);
#pragma unroll 1
        for (int64_t i = 0; i <= my_tiles; ++i) {
            const bool gemm = i < my_tiles;
            const int nph = gemm ? kChunks : kSteps;
#pragma unroll 1
            for (int c = 0; c < nph; ++c) {
                const int64_t q = i * kChunks + c;
                // own DMAs of chunk q landed (the up to L - 1 chunks issued after it may still fly), then the barrier:
                // chunk q is in LDS for every wave and stage (q + L) % kWsStages — chunk q - 1's — has been read
                const int64_t after = gemm ? (q + L - 1 < nchunks ? L - 1 : nchunks - 1 - q) : 0;
                if (after >= 2) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * kWsDma) : "memory");
                else if (after == 1) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(kWsDma) : "memory");
                else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
                if (gemm && q + L < nchunks) issue(q + L);
            }
            asm volatile("s_barrier" ::: "memory");  // X
            asm volatile("s_barrier" ::: "memory");  // Y
        }
    }
}

}  // namespace

#ifndef XPA_HEAD_KERNELS_ONLY  // tools/_probe: include the kernels alone and instantiate one
XPA_API int64_t xpa_head_fused_num_partials(int64_t batch) {
    return head_partials(batch);
}

namespace {
#define XPA_HEAD_ARGS(a) a.batch, a.K, a.ld, a.z, a.ldx, a.Wh, a.bh, a.W, a.bias, a.slope, a.logstd, a.idx, a.n_rows, a.act, a.old_logp, a.adv, a.ret, a.adv_partials, a.n_adv_partials, a.clip_range, a.ent_coef, a.vf_coef, a.dz, a.p_dw, a.p_dbh, a.p_dbo, a.p_loss, a.loss_width
// KIND: 0 K12 (z from HBM), 1 K16 (hidden GEMM inside), 2 K16X (trunk layer + hidden GEMM inside), 3 K16W,
// 4 K16S (K16 with the hidden GEMM on the bf16 matrix cores by the three-way split), 5 K16P (K16S with Wh pre-split),
// 6 K16R (K16P with h formed from the gathered rows in the k loop), 7 K16Q (K16P with 32 x 128 wave tiles)
template <int KIND, int MODE, int ALGO, int ACT, int KMAX>
void launch_one(const HeadArgs &a, hipStream_t s) {
    const dim3 grid((unsigned)xpa_head_fused_num_partials(a.batch)), block(256);
    if constexpr (KIND == 3) {
        if constexpr (KMAX <= 8)
            hipLaunchKernelGGL((head_gemm_ws_kernel<MODE, ALGO, ACT, KMAX>), dim3((unsigned)head_ws_grid(a.batch)),
                               dim3(512), 0, s, XPA_HEAD_ARGS(a));
    } else if constexpr (KIND == 4)
        hipLaunchKernelGGL((head_gemm_kernel<MODE, ALGO, ACT, KMAX, false, 1>), grid, block, 0, s, XPA_HEAD_ARGS(a),
                           nullptr, (int64_t)0, 0, nullptr, nullptr, 0.f, nullptr, (int64_t)0, nullptr);
    else if constexpr (KIND == 5)
        hipLaunchKernelGGL((head_gemm_kernel<MODE, ALGO, ACT, KMAX, false, 2>), grid, block, 0, s, XPA_HEAD_ARGS(a),
                           nullptr, (int64_t)0, 0, nullptr, nullptr, 0.f, nullptr, (int64_t)0, nullptr);
    else if constexpr (KIND == 2)
        hipLaunchKernelGGL((head_gemm_kernel<MODE, ALGO, ACT, KMAX, true>), grid, block, 0, s, XPA_HEAD_ARGS(a), a.xr,
                           a.ldxr, a.din, a.W0, a.b0, a.slope0, a.hout, a.ldh, nullptr);
    else if constexpr (KIND == 7)
        hipLaunchKernelGGL((head_gemm_kernel<MODE, ALGO, ACT, KMAX, false, 4>), grid, block, 0, s, XPA_HEAD_ARGS(a),
                           nullptr, (int64_t)0, 0, nullptr, nullptr, 0.f, nullptr, (int64_t)0, nullptr, a.cmask, a.cdv);
    else if constexpr (KIND == 6)
        hipLaunchKernelGGL((head_gemm_kernel<MODE, ALGO, ACT, KMAX, false, 3>), grid, block, 0, s, XPA_HEAD_ARGS(a),
                           a.xr, a.ldxr, a.din, a.W0, a.b0, a.slope0, a.hout, a.ldh, a.hmask);
    else if constexpr (KIND == 1)
        hipLaunchKernelGGL((head_gemm_kernel<MODE, ALGO, ACT, KMAX, false>), grid, block, 0, s, XPA_HEAD_ARGS(a),
                           nullptr, (int64_t)0, 0, nullptr, nullptr, 0.f, nullptr, (int64_t)0, nullptr);
    else
        hipLaunchKernelGGL((head_tile_kernel<MODE, ALGO, ACT, KMAX>), grid, block, 0, s, XPA_HEAD_ARGS(a));
}

template <int KIND, int MODE, int ALGO, int KMAX>
void launch_act(const HeadArgs &a, int act_code, hipStream_t s) {
    if (act_code == 0) launch_one<KIND, MODE, ALGO, 0, KMAX>(a, s);
    else if (act_code == 1) launch_one<KIND, MODE, ALGO, 1, KMAX>(a, s);
    else launch_one<KIND, MODE, ALGO, 2, KMAX>(a, s);
}

template <int KIND, int MODE, int ALGO>
void launch_head(const HeadArgs &a, int act_code, hipStream_t s) {
    if constexpr (MODE == 2) launch_act<KIND, MODE, ALGO, 1>(a, act_code, s);
    else if (a.K <= 4) launch_act<KIND, MODE, ALGO, 4>(a, act_code, s);  // KMAX = smallest of 4 / 6 / 8 >= K
    else if (a.K <= 6) launch_act<KIND, MODE, ALGO, 6>(a, act_code, s);
    else if (a.K <= 8) launch_act<KIND, MODE, ALGO, 8>(a, act_code, s);
    else if constexpr (KIND != 2 && KIND != 3 && KIND != 6)
        launch_act<KIND, MODE, ALGO, 18>(a, act_code, s);  // C4 (A = 17), 18-way
}
#undef XPA_HEAD_ARGS

template <int KIND>
int actor_entry(int algo, int dist, int act_code, HeadArgs &a, hipStream_t s) {
    if (dist == XPA_DIST_GAUSSIAN) {
        if (algo == XPA_ALGO_PPO) launch_head<KIND, 0, 0>(a, act_code, s);
        else launch_head<KIND, 0, 1>(a, act_code, s);
    } else {
        if (algo == XPA_ALGO_PPO) launch_head<KIND, 1, 0>(a, act_code, s);
        else launch_head<KIND, 1, 1>(a, act_code, s);
    }
    return xpa_launch_status();
}

int check_actor(int algo, int dist, int act_code, int64_t batch, int64_t act_dim, int64_t hidden, const float *w,
                const float *b, const float *logstd, int64_t n_rows, const int64_t *idx, const float *act,
                const float *old_logp, const float *adv, const float *dz, const float *partial_dw,
                const float *partial_db_hidden, const float *partial_db_out, const float *loss_partials,
                int64_t loss_width) {
    if (batch <= 0 || hidden != kH || act_dim < 1 || act_dim > kHeadKMax || act_code < 0 || act_code > 2 || !w || !b ||
        !act || !adv || !dz || !partial_dw || !partial_db_hidden || !partial_db_out || !loss_partials ||
        loss_width < kPartBase + act_dim || n_rows <= 0 || (!idx && n_rows < batch))
        return (int)hipErrorInvalidValue;
    if ((algo != XPA_ALGO_PPO && algo != XPA_ALGO_A2C) || (dist != XPA_DIST_GAUSSIAN && dist != XPA_DIST_CATEGORICAL))
        return (int)hipErrorInvalidValue;
    if ((dist == XPA_DIST_GAUSSIAN && !logstd) || (algo == XPA_ALGO_PPO && !old_logp) ||
        (dist == XPA_DIST_CATEGORICAL && act_dim < 2))
        return (int)hipErrorInvalidValue;
    if ((uintptr_t)w % 16 || (uintptr_t)dz % 16) return (int)hipErrorInvalidValue;   // r06: 16-B dz row stores (kQuad)
    return 0;
}
}  // namespace

XPA_API int xpa_head_fused_actor(int algo, int dist, int act_code, int64_t batch, int64_t act_dim, int64_t hidden,
                                 int64_t ld, const float *z, const float *w, const float *b, float slope, const float *logstd,
                                 const int64_t *idx, int64_t n_rows, const float *act, const float *old_logp,
                                 const float *adv, const double *adv_partials, int64_t n_adv_partials,
                                 float clip_range, float ent_coef, float *dz, float *partial_dw,
                                 float *partial_db_hidden, float *partial_db_out, float *loss_partials,
                                 int64_t loss_width, xpa_stream_t stream) {
    int rc = check_actor(algo, dist, act_code, batch, act_dim, hidden, w, b, logstd, n_rows, idx, act, old_logp, adv, dz,
                         partial_dw, partial_db_hidden, partial_db_out, loss_partials, loss_width);
    if (rc) return rc;
    if (!z || (uintptr_t)z % 16 || ld < kH || ld % 4) return (int)hipErrorInvalidValue;
    HeadArgs a{};
    a.batch = batch; a.K = (int)act_dim; a.ld = ld; a.z = z; a.ldx = ld; a.W = w; a.bias = b; a.slope = slope;
    a.logstd = logstd; a.idx = idx; a.n_rows = n_rows; a.act = act; a.old_logp = old_logp; a.adv = adv;
    a.ret = nullptr; a.adv_partials = adv_partials; a.n_adv_partials = n_adv_partials; a.clip_range = clip_range;
    a.ent_coef = ent_coef; a.vf_coef = 0.f; a.dz = dz; a.p_dw = partial_dw; a.p_dbh = partial_db_hidden;
    a.p_dbo = partial_db_out; a.p_loss = loss_partials; a.loss_width = (int)loss_width;
    return actor_entry<0>(algo, dist, act_code, a, (hipStream_t)stream);
}

XPA_API int xpa_head_fused_critic(int act_code, int64_t batch, int64_t hidden, int64_t ld, const float *z, const float *w,
                                  const float *b, float slope, const int64_t *idx, int64_t n_rows, const float *ret,
                                  float vf_coef, float *dz, float *partial_dw, float *partial_db_hidden,
                                  float *partial_db_out, float *loss_partials, int64_t loss_width,
                                  xpa_stream_t stream) {
    if (batch <= 0 || hidden != kH || act_code < 0 || act_code > 2 || !z || !w || !b || !ret || !dz || !partial_dw ||
        !partial_db_hidden || !partial_db_out || !loss_partials || loss_width < kPartBase || n_rows <= 0 ||
        (!idx && n_rows < batch))
        return (int)hipErrorInvalidValue;
    if (((uintptr_t)z | (uintptr_t)w) % 16 || ld < kH || ld % 4) return (int)hipErrorInvalidValue;
    HeadArgs a{};
    a.batch = batch; a.K = 1; a.ld = ld; a.z = z; a.ldx = ld; a.W = w; a.bias = b; a.slope = slope; a.idx = idx;
    a.n_rows = n_rows; a.ret = ret; a.vf_coef = vf_coef; a.dz = dz; a.p_dw = partial_dw; a.p_dbh = partial_db_hidden;
    a.p_dbo = partial_db_out; a.p_loss = loss_partials; a.loss_width = (int)loss_width;
    launch_head<0, 2, 0>(a, act_code, (hipStream_t)stream);
    return xpa_launch_status();
}

namespace {
#define XPA_GEMM_ACTOR_PARAMS                                                                                          \
    int algo, int dist, int act_code, int64_t batch, int64_t act_dim, int64_t hidden, const float *x, int64_t ldx,  \
        const float *w_hidden, const float *b_hidden, int64_t ld_dz, const float *w, const float *b, float slope,   \
        const float *logstd, const int64_t *idx, int64_t n_rows, const float *act, const float *old_logp,           \
        const float *adv, const double *adv_partials, int64_t n_adv_partials, float clip_range, float ent_coef,     \
        float *dz, float *partial_dw, float *partial_db_hidden, float *partial_db_out, float *loss_partials,        \
        int64_t loss_width, xpa_stream_t stream
#define XPA_GEMM_ACTOR_ARGS                                                                                            \
    algo, dist, act_code, batch, act_dim, hidden, x, ldx, w_hidden, b_hidden, ld_dz, w, b, slope, logstd, idx, n_rows, \
        act, old_logp, adv, adv_partials, n_adv_partials, clip_range, ent_coef, dz, partial_dw, partial_db_hidden,   \
        partial_db_out, loss_partials, loss_width, stream
#define XPA_GEMM_CRITIC_PARAMS                                                                                         \
    int act_code, int64_t batch, int64_t hidden, const float *x, int64_t ldx, const float *w_hidden,                \
        const float *b_hidden, int64_t ld_dz, const float *w, const float *b, float slope, const int64_t *idx,      \
        int64_t n_rows, const float *ret, float vf_coef, float *dz, float *partial_dw, float *partial_db_hidden,     \
        float *partial_db_out, float *loss_partials, int64_t loss_width, xpa_stream_t stream
#define XPA_GEMM_CRITIC_ARGS                                                                                           \
    act_code, batch, hidden, x, ldx, w_hidden, b_hidden, ld_dz, w, b, slope, idx, n_rows, ret, vf_coef, dz,         \
        partial_dw, partial_db_hidden, partial_db_out, loss_partials, loss_width, stream

// the hidden-GEMM head kernels' entries (KIND 1 K16, 3 K16W, 4 K16S): same arguments, same outputs
template <int KIND>
int gemm_actor_entry(XPA_GEMM_ACTOR_PARAMS) {
    int rc = check_actor(algo, dist, act_code, batch, act_dim, hidden, w, b, logstd, n_rows, idx, act, old_logp, adv, dz,
                         partial_dw, partial_db_hidden, partial_db_out, loss_partials, loss_width);
    if (rc) return rc;
    if ((KIND == 3 && act_dim > 8) || !x || !w_hidden || !b_hidden || ((uintptr_t)x | (uintptr_t)w_hidden) % 16 ||
        ldx < kKin || ldx % 4 || ld_dz < kH || ld_dz % 4)   // r06: 16-B dz row stores (kQuad)
        return (int)hipErrorInvalidValue;
    HeadArgs a{};
    a.batch = batch; a.K = (int)act_dim; a.ld = ld_dz; a.z = x; a.ldx = ldx; a.Wh = w_hidden; a.bh = b_hidden;
    a.W = w; a.bias = b; a.slope = slope; a.logstd = logstd; a.idx = idx; a.n_rows = n_rows; a.act = act;
    a.old_logp = old_logp; a.adv = adv; a.ret = nullptr; a.adv_partials = adv_partials;
    a.n_adv_partials = n_adv_partials; a.clip_range = clip_range; a.ent_coef = ent_coef; a.vf_coef = 0.f; a.dz = dz;
    a.p_dw = partial_dw; a.p_dbh = partial_db_hidden; a.p_dbo = partial_db_out; a.p_loss = loss_partials;
    a.loss_width = (int)loss_width;
    return actor_entry<KIND>(algo, dist, act_code, a, (hipStream_t)stream);
}

template <int KIND>
int gemm_critic_entry(XPA_GEMM_CRITIC_PARAMS, unsigned *cmask = nullptr, float *cdv = nullptr) {
    if (batch <= 0 || hidden != kH || act_code < 0 || act_code > 2 || !x || !w_hidden || !b_hidden || !w || !b ||
        !ret || (!dz && !(cmask && cdv)) || !partial_dw || !partial_db_hidden || !partial_db_out || !loss_partials ||
        loss_width < kPartBase || n_rows <= 0 || (!idx && n_rows < batch))
        return (int)hipErrorInvalidValue;
    if ((cmask || cdv) && (KIND != 7 || (uintptr_t)cmask % 8)) return (int)hipErrorInvalidValue;
    if (((uintptr_t)x | (uintptr_t)w_hidden | (uintptr_t)w) % 16 || ldx < kKin || ldx % 4 || ld_dz < kH)
        return (int)hipErrorInvalidValue;
    HeadArgs a{};
    a.batch = batch; a.K = 1; a.ld = ld_dz; a.z = x; a.ldx = ldx; a.Wh = w_hidden; a.bh = b_hidden; a.W = w;
    a.bias = b; a.slope = slope; a.idx = idx; a.n_rows = n_rows; a.ret = ret; a.vf_coef = vf_coef; a.dz = dz;
    a.p_dw = partial_dw; a.p_dbh = partial_db_hidden; a.p_dbo = partial_db_out; a.p_loss = loss_partials;
    a.loss_width = (int)loss_width;
    a.cmask = cmask; a.cdv = cdv;
    launch_head<KIND, 2, 0>(a, act_code, (hipStream_t)stream);
    return xpa_launch_status();
}
}  // namespace

XPA_API int xpa_head_gemm_actor(XPA_GEMM_ACTOR_PARAMS) { return gemm_actor_entry<1>(XPA_GEMM_ACTOR_ARGS); }
XPA_API int xpa_head_gemm_critic(XPA_GEMM_CRITIC_PARAMS) { return gemm_critic_entry<1>(XPA_GEMM_CRITIC_ARGS); }
// K16S: the same arguments and outputs; the hidden GEMM at the f32 GEMM's accuracy, not K16's bits
XPA_API int xpa_head_gemm_s3_actor(XPA_GEMM_ACTOR_PARAMS) { return gemm_actor_entry<4>(XPA_GEMM_ACTOR_ARGS); }
XPA_API int xpa_head_gemm_s3_critic(XPA_GEMM_CRITIC_PARAMS) { return gemm_critic_entry<4>(XPA_GEMM_CRITIC_ARGS); }
// K16P: as K16S with w_hidden = the split buffer of Wh^T (xpa_s3_split_b(Wh, 256, 256, 1, 256, ...))
XPA_API int xpa_head_gemm_s3p_actor(XPA_GEMM_ACTOR_PARAMS) { return gemm_actor_entry<5>(XPA_GEMM_ACTOR_ARGS); }
XPA_API int xpa_head_gemm_s3p_critic(XPA_GEMM_CRITIC_PARAMS) { return gemm_critic_entry<5>(XPA_GEMM_CRITIC_ARGS); }
// K16Q: K16P's arguments and outputs bit for bit, the waves tiled 32 x 128 (one A fragment split per wave and chunk)
XPA_API int xpa_head_gemm_s3q_actor(XPA_GEMM_ACTOR_PARAMS) { return gemm_actor_entry<7>(XPA_GEMM_ACTOR_ARGS); }
XPA_API int xpa_head_gemm_s3q_critic(XPA_GEMM_CRITIC_PARAMS) { return gemm_critic_entry<7>(XPA_GEMM_CRITIC_ARGS); }
// r05: K16Q critic for the factored critic backward: also writes the hidden activations' sign bits (mask [batch][8]
// u32, bit c & 31 of word c >> 5 = h[row, c] > 0) and d loss / d v per row (dv [batch]); dz may be null (not stored:
// K41V / K42S then take the critic's half from mask, dv and the output weights)
XPA_API int xpa_head_gemm_s3q_critic_mask(XPA_GEMM_CRITIC_PARAMS, unsigned *mask, float *dv) {
    if (!mask || !dv) return (int)hipErrorInvalidValue;
    return gemm_critic_entry<7>(XPA_GEMM_CRITIC_ARGS, mask, dv);
}

// K16W entries: xpa_head_gemm_actor / _critic's arguments and outputs (the same partial-row count, rows the grid does
// not own written as zeros); act_dim <= 8.
XPA_API int64_t xpa_head_gemm_ws_grid(int64_t batch) {
    return head_ws_grid(batch);
}

// Test support: fill every CU's LDS with NaN bit patterns (one 160 KiB block per CU, twice over), so that a kernel
// launched next that reads LDS it did not write sees a NaN instead of whatever the previous kernel left (usually
// finite).  tests/test_gpu_fused_mlp.py runs the head kernels behind it.
__global__ __launch_bounds__(1024) void lds_poison_kernel() {
    __shared__ unsigned lds[40960];
    for (int i = threadIdx.x; i < 40960; i += 1024) lds[i] = 0xFFFFFFFFu;
    __syncthreads();
    if (lds[(threadIdx.x * 37) % 40960] == 0u) lds[0] = 1u;  // keep the stores
}
XPA_API int xpa_lds_poison(xpa_stream_t stream) {
    lds_poison_kernel<<<dim3(512), dim3(1024), 0, (hipStream_t)stream>>>();
    return xpa_launch_status();
}

XPA_API int xpa_head_store_probe(int plain) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_head_dz_plain), &plain, sizeof(int));
}

// r06 A/B: the K16 heads' second-slot blocks start n x ~0.85 us late (see head_gemm_kernel); 0 = off (the default)
XPA_API int xpa_head_stagger(int n) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_head_stagger), &n, sizeof(int));
}

// diagnostics only (tools/k16w_ab.py --probe): see g_ws_probe
XPA_API int xpa_head_gemm_ws_probe(int mask) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_ws_probe), &mask, sizeof(int));
}

XPA_API int xpa_head_gemm_ws_actor(XPA_GEMM_ACTOR_PARAMS) { return gemm_actor_entry<3>(XPA_GEMM_ACTOR_ARGS); }
XPA_API int xpa_head_gemm_ws_critic(XPA_GEMM_CRITIC_PARAMS) { return gemm_critic_entry<3>(XPA_GEMM_CRITIC_ARGS); }
#undef XPA_GEMM_ACTOR_PARAMS
#undef XPA_GEMM_ACTOR_ARGS
#undef XPA_GEMM_CRITIC_PARAMS
#undef XPA_GEMM_CRITIC_ARGS

namespace {
int check_trunk(int64_t d_in, const float *x_rows, int64_t ld_rows, const float *w_in, const float *b_in,
                const float *w_hidden, const float *b_hidden, int64_t ld_dz) {
    if (d_in < 1 || d_in > kTrunkDMax || !x_rows || ld_rows < d_in || !w_in || !b_in || !w_hidden || !b_hidden ||
        (uintptr_t)w_hidden % 16 || ld_dz < kH || ld_dz % 4)
        return (int)hipErrorInvalidValue;
    return 0;
}
}  // namespace

XPA_API int xpa_head_gemm_trunk_actor(int algo, int dist, int act_code, int64_t batch, int64_t act_dim, int64_t hidden,
                                      const float *x_rows, int64_t ld_rows, int64_t d_in, const float *w_in,
                                      const float *b_in, float slope_in, float *h_out, int64_t ld_h,
                                      const float *w_hidden, const float *b_hidden, int64_t ld_dz, const float *w,
                                      const float *b, float slope, const float *logstd, const int64_t *idx,
                                      int64_t n_rows, const float *act, const float *old_logp, const float *adv,
                                      const double *adv_partials, int64_t n_adv_partials, float clip_range,
                                      float ent_coef, float *dz, float *partial_dw, float *partial_db_hidden,
                                      float *partial_db_out, float *loss_partials, int64_t loss_width,
                                      xpa_stream_t stream) {
    int rc = check_actor(algo, dist, act_code, batch, act_dim, hidden, w, b, logstd, n_rows, idx, act, old_logp, adv, dz,
                         partial_dw, partial_db_hidden, partial_db_out, loss_partials, loss_width);
    if (rc) return rc;
    rc = check_trunk(d_in, x_rows, ld_rows, w_in, b_in, w_hidden, b_hidden, ld_dz);
    if (rc) return rc;
    if (act_dim > 8 || !h_out || (uintptr_t)h_out % 16 || ld_h < kH || ld_h % 4) return (int)hipErrorInvalidValue;
    HeadArgs a{};
    a.batch = batch; a.K = (int)act_dim; a.ld = ld_dz; a.z = nullptr; a.ldx = kKin; a.Wh = w_hidden; a.bh = b_hidden;
    a.W = w; a.bias = b; a.slope = slope; a.logstd = logstd; a.idx = idx; a.n_rows = n_rows; a.act = act;
    a.old_logp = old_logp; a.adv = adv; a.ret = nullptr; a.adv_partials = adv_partials;
    a.n_adv_partials = n_adv_partials; a.clip_range = clip_range; a.ent_coef = ent_coef; a.vf_coef = 0.f; a.dz = dz;
    a.p_dw = partial_dw; a.p_dbh = partial_db_hidden; a.p_dbo = partial_db_out; a.p_loss = loss_partials;
    a.loss_width = (int)loss_width;
    a.xr = x_rows; a.ldxr = ld_rows; a.din = (int)d_in; a.W0 = w_in; a.b0 = b_in; a.slope0 = slope_in;
    a.hout = h_out; a.ldh = ld_h;
    return actor_entry<2>(algo, dist, act_code, a, (hipStream_t)stream);
}

XPA_API int xpa_head_gemm_trunk_critic(int act_code, int64_t batch, int64_t hidden, const float *x_rows,
                                       int64_t ld_rows, int64_t d_in, const float *w_in, const float *b_in,
                                       float slope_in, float *h_out, int64_t ld_h, const float *w_hidden,
                                       const float *b_hidden, int64_t ld_dz, const float *w, const float *b,
                                       float slope, const int64_t *idx, int64_t n_rows, const float *ret,
                                       float vf_coef, float *dz, float *partial_dw, float *partial_db_hidden,
                                       float *partial_db_out, float *loss_partials, int64_t loss_width,
                                       xpa_stream_t stream) {
    if (batch <= 0 || hidden != kH || act_code < 0 || act_code > 2 || !w || !b || !ret || !dz || !partial_dw ||
        !partial_db_hidden || !partial_db_out || !loss_partials || loss_width < kPartBase || n_rows <= 0 ||
        (!idx && n_rows < batch) || (uintptr_t)w % 16)
        return (int)hipErrorInvalidValue;
    int rc = check_trunk(d_in, x_rows, ld_rows, w_in, b_in, w_hidden, b_hidden, ld_dz);
    if (rc) return rc;
    if (!h_out || (uintptr_t)h_out % 16 || ld_h < kH || ld_h % 4) return (int)hipErrorInvalidValue;
    HeadArgs a{};
    a.batch = batch; a.K = 1; a.ld = ld_dz; a.z = nullptr; a.ldx = kKin; a.Wh = w_hidden; a.bh = b_hidden; a.W = w;
    a.bias = b; a.slope = slope; a.idx = idx; a.n_rows = n_rows; a.ret = ret; a.vf_coef = vf_coef; a.dz = dz;
    a.p_dw = partial_dw; a.p_dbh = partial_db_hidden; a.p_dbo = partial_db_out; a.p_loss = loss_partials;
    a.loss_width = (int)loss_width;
    a.xr = x_rows; a.ldxr = ld_rows; a.din = (int)d_in; a.W0 = w_in; a.b0 = b_in; a.slope0 = slope_in;
    a.hout = h_out; a.ldh = ld_h;
    launch_head<2, 2, 0>(a, act_code, (hipStream_t)stream);
    return xpa_launch_status();
}
// K16R entries: xpa_head_gemm_s3p_*'s outputs (w_hidden = the split buffer of Wh^T) with the hidden layer's input h
// formed inside from the gathered minibatch rows x_rows [batch, d_in <= 20] (the representation's one thin layer:
// w_in [256, d_in], b_in, the heads' activation with slope_in) — K13's h bit for bit.  The actor also writes h
// (h_out [batch, >= 256] at ld_h) and, when h_sign is given, its sign bits: byte b of row r's 32 bytes (h_sign + 8 r)
// bit j = h[r, 32 j + b] > 0 (xpa_s3_gemm_trunk_bwd_sign's act', one byte per lane there).  act_dim <= 8.
XPA_API int xpa_head_gemm_s3r_actor(int algo, int dist, int act_code, int64_t batch, int64_t act_dim, int64_t hidden,
                                    const float *x_rows, int64_t ld_rows, int64_t d_in, const float *w_in,
                                    const float *b_in, float slope_in, float *h_out, int64_t ld_h, unsigned *h_sign,
                                    const void *w_hidden, const float *b_hidden, int64_t ld_dz, const float *w,
                                    const float *b, float slope, const float *logstd, const int64_t *idx,
                                    int64_t n_rows, const float *act, const float *old_logp, const float *adv,
                                    const double *adv_partials, int64_t n_adv_partials, float clip_range,
                                    float ent_coef, float *dz, float *partial_dw, float *partial_db_hidden,
                                    float *partial_db_out, float *loss_partials, int64_t loss_width,
                                    xpa_stream_t stream) {
    int rc = check_actor(algo, dist, act_code, batch, act_dim, hidden, w, b, logstd, n_rows, idx, act, old_logp, adv, dz,
                         partial_dw, partial_db_hidden, partial_db_out, loss_partials, loss_width);
    if (rc) return rc;
    const float *whp = static_cast<const float *>(w_hidden);
    rc = check_trunk(d_in, x_rows, ld_rows, w_in, b_in, whp, b_hidden, ld_dz);
    if (rc) return rc;
    if (act_dim > 8 || !h_out || (uintptr_t)h_out % 16 || ld_h < kH || ld_h % 4) return (int)hipErrorInvalidValue;
    HeadArgs a{};
    a.batch = batch; a.K = (int)act_dim; a.ld = ld_dz; a.z = nullptr; a.ldx = kKin; a.Wh = whp; a.bh = b_hidden;
    a.W = w; a.bias = b; a.slope = slope; a.logstd = logstd; a.idx = idx; a.n_rows = n_rows; a.act = act;
    a.old_logp = old_logp; a.adv = adv; a.ret = nullptr; a.adv_partials = adv_partials;
    a.n_adv_partials = n_adv_partials; a.clip_range = clip_range; a.ent_coef = ent_coef; a.vf_coef = 0.f; a.dz = dz;
    a.p_dw = partial_dw; a.p_dbh = partial_db_hidden; a.p_dbo = partial_db_out; a.p_loss = loss_partials;
    a.loss_width = (int)loss_width;
    a.xr = x_rows; a.ldxr = ld_rows; a.din = (int)d_in; a.W0 = w_in; a.b0 = b_in; a.slope0 = slope_in;
    a.hout = h_out; a.ldh = ld_h; a.hmask = h_sign;
    return actor_entry<6>(algo, dist, act_code, a, (hipStream_t)stream);
}

XPA_API int xpa_head_gemm_s3r_critic(int act_code, int64_t batch, int64_t hidden, const float *x_rows,
                                     int64_t ld_rows, int64_t d_in, const float *w_in, const float *b_in,
                                     float slope_in, const void *w_hidden, const float *b_hidden, int64_t ld_dz,
                                     const float *w, const float *b, float slope, const int64_t *idx, int64_t n_rows,
                                     const float *ret, float vf_coef, float *dz, float *partial_dw,
                                     float *partial_db_hidden, float *partial_db_out, float *loss_partials,
                                     int64_t loss_width, xpa_stream_t stream) {
    if (batch <= 0 || hidden != kH || act_code < 0 || act_code > 2 || !w || !b || !ret || !dz || !partial_dw ||
        !partial_db_hidden || !partial_db_out || !loss_partials || loss_width < kPartBase || n_rows <= 0 ||
        (!idx && n_rows < batch) || (uintptr_t)w % 16)
        return (int)hipErrorInvalidValue;
    const float *whp = static_cast<const float *>(w_hidden);
    int rc = check_trunk(d_in, x_rows, ld_rows, w_in, b_in, whp, b_hidden, ld_dz);
    if (rc) return rc;
    HeadArgs a{};
    a.batch = batch; a.K = 1; a.ld = ld_dz; a.z = nullptr; a.ldx = kKin; a.Wh = whp; a.bh = b_hidden; a.W = w;
    a.bias = b; a.slope = slope; a.idx = idx; a.n_rows = n_rows; a.ret = ret; a.vf_coef = vf_coef; a.dz = dz;
    a.p_dw = partial_dw; a.p_dbh = partial_db_hidden; a.p_dbo = partial_db_out; a.p_loss = loss_partials;
    a.loss_width = (int)loss_width;
    a.xr = x_rows; a.ldxr = ld_rows; a.din = (int)d_in; a.W0 = w_in; a.b0 = b_in; a.slope0 = slope_in;
    a.hout = nullptr; a.ldh = 0; a.hmask = nullptr;
    launch_head<6, 2, 0>(a, act_code, (hipStream_t)stream);
    return xpa_launch_status();
}
#endif  // XPA_HEAD_KERNELS_ONLY
