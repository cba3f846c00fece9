// K30 — one small-MLP PPO-Clip / A2C update in ONE launch (C1: CartPole-v1, 8 envs x 128 steps, [64] nets,
// 128-row minibatches), gfx950.
//
// Replaces, for an actor-critic whose representation is one mlp_block and whose actor / critic are one hidden
// mlp_block + an output Linear (xuance/torch/representations/mlp.py:21-51, policies/categorical.py:16-58,
// utils/layers.py:8-24), everything one PPOCLIP_Learner.update / A2C_Learner.update does for one minibatch
// (ppoclip_learner.py:24-65, a2c_learner.py:19-50): the minibatch gather (memory_tools.py:230-243 with the adv
// normalisation), the forward, the loss (Categorical log-prob / entropy, clipped surrogate, value MSE), the
// backward through every layer, clip_grad_norm_ and Adam (with the learning rate / Adam step from the device
// schedule of xpa_clip_adam_step_sched).  At 128 rows x 64 hidden units the whole update is ~7 MFLOP: split over
// ~25 launches it was bound by their latency (~105 us per update); here one workgroup of 512 threads keeps every
// activation in LDS and the update takes one launch.
//
// Layout: activations transposed, [feature][batch] with row stride S = BP + 4 (BP = batch rounded up to 32).
// Every product (the five forward layers, the five weight gradients, the two data gradients) is a set of 32 x 32
// tiles on v_mfma_f32_32x32x2_f32 (exact f32 fma chains), one wave per tile, operands read straight from the LDS
// images with per-operand strides (the first form, VALU 4 x 4 register tiles, was bound by its LDS round trips:
// 95 us per update at C1, 222 k cycles of which 41 k in the output layers alone).  In-place reuse: h1 / h2 become
// dh1 / dh2 once the output layers' weight gradients are formed, h0 becomes dh0 once the hidden ones' are.
// Arithmetic of the loss and of the clip + Adam step: exactly K2's per-row formulas (loss.hip) and K9's (optim.hip).
#include "xpa_common.h"

namespace {

constexpr int kSmThreads = 512;
constexpr int kSmWaves = kSmThreads / 64;
constexpr int kSmLds = 40704;   // floats (159 KiB: the rest of the 160 KiB holds the reduction scratch)
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int ACT>
__device__ __forceinline__ float sm_act(float z, float slope) {
    if (ACT == 1) return z > 0.f ? z : z * slope;
    if (ACT == 2) return tanhf(z);
    return z;
}
template <int ACT>
__device__ __forceinline__ float sm_grad(float y, float slope) {   // d act / d z from the output y
    if (ACT == 1) return y > 0.f ? 1.f : slope;
    if (ACT == 2) return 1.f - y * y;
    return 1.f;
}

// One 32 x 32 tile D[m][n] = sum_{k < kred} A(m, k) B(k, n) with A(m, k) = pa[k ak + m am], B(k, n) = pb[k bk + n bn]
// (LDS), rows m >= mvalid / columns n >= nvalid of the operands read as 0.  Lane (i, h) feeds A(i, k + h) and
// B(k + h, i); D element r of lane (i, h) is D[(r & 3) + 8 (r >> 2) + 4 h][i].
__device__ __forceinline__ f32x16 sm_tile(const float *pa, int am, int ak, int mvalid, const float *pb, int bk, int bn,
                                          int nvalid, int kred) {
    const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
    const bool av = i < mvalid, bv = i < nvalid;
    const float *qa = pa + (av ? i : 0) * am + h * ak, *qb = pb + (bv ? i : 0) * bn + h * bk;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    // 8 k-steps per group: the 16 operand reads issued before the group's MFMAs (a plain loop ran load, wait,
    // MFMA per k-step: one LDS round trip per MFMA)
    int k = 0;
    for (; k + 16 <= kred; k += 16) {
        float x[8], y[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            x[u] = qa[(k + 2 * u) * ak];
            y[u] = qb[(k + 2 * u) * bk];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av ? x[u] : 0.f, bv ? y[u] : 0.f, acc, 0, 0, 0);
    }
    for (; k < kred; k += 2) {
        const float x = qa[k * ak], y = qb[k * bk];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av ? x : 0.f, bv ? y : 0.f, acc, 0, 0, 0);
    }
    return acc;
}
__device__ __forceinline__ int sm_row(int r) { return (r & 3) + 8 * (r >> 2) + 4 * ((threadIdx.x & 63) >> 5); }

#define XPA_SM_STAMP(i_)                                                                                  \
    do {                                                                                                  \
        if (a.stamps && t == 0 && blockIdx.x == 0) a.stamps[i_] = (int64_t)__builtin_amdgcn_s_memtime(); \
    } while (0)

template <int ACT, int ALGO>
__global__ __launch_bounds__(kSmThreads, 1) void small_mlp_update_kernel(XpaSmallMlpArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[kSmLds];
    __shared__ double s_red[kSmWaves * 6];
    __shared__ float s_stat[4];
    __shared__ float s_coef, s_step, s_inv;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, li = lane & 31;
    // Split form (G = gridDim.x > 1): workgroup g takes minibatch rows [32 g, 32 g + 32) and writes its partial
    // weight / bias gradients (sums over its rows) into grad_part[g] at the flat buffer's offsets and its loss sums
    // into loss_part[g]; small_mlp_finalize_kernel then sums the partials in g order, clips and steps Adam.  The
    // advantage moments are over the whole minibatch in every workgroup.
    const int G = gridDim.x, gi = blockIdx.x;
    const int Btot = a.batch;
    const int r0 = G > 1 ? 32 * gi : 0;
    const int B = G > 1 ? min(32, Btot - r0) : Btot;   // this workgroup's rows
    const int64_t *idx = a.idx + r0;
    auto gp = [&](float *p) -> float * { return G > 1 ? a.grad_part + (int64_t)gi * a.n + (p - a.grad) : p; };
    const int BP = (B + 31) & ~31, S = BP + 4;
    const int D = a.d_in, DP = (a.d_in + 3) & ~3, H0 = a.h0, H1 = a.h1, H2 = a.h2, K = a.k, KP = (a.k + 3) & ~3;
    const int MB = BP / 32;
    const float slope = a.slope;
    // ---- LDS carve (offsets multiples of 4 floats) ----
    float *xT = lds;                       // [DP][S]
    float *h0T = xT + DP * S;              // [H0][S]  -> dh0
    float *h1T = h0T + H0 * S;             // [H1][S]  -> dh1
    float *h2T = h1T + H1 * S;             // [H2][S]  -> dh2
    float *dlT = h2T + H2 * S;             // [KP][S]  d logits (rows >= K zero)
    float *dvT = dlT + KP * S;             // [4][S]   d v in row 0
    float *W0T = dvT + 4 * S;              // [DP][H0]
    // W1T / W2T: row stride H1 + 1 / H2 + 1, so that the coalesced (source-order) staging writes are conflict-free
    const int H1P = H1 + 1, H2P = H2 + 1;
    float *W1T = W0T + DP * H0;            // [H0][H1P], after the forward W1 row-major [H1][H0]
    float *W2T = W1T + H0 * H1P;           // [H0][H2P], after the forward W2 row-major [H2][H0] (at W1T + H1 H0)
    float *WaT = W2T + H0 * H2P;           // [H1][KP]
    float *Wcv = WaT + H1 * KP;            // [H2]
    float *b0s = Wcv + H2, *b1s = b0s + H0, *b2s = b1s + H1, *bas = b2s + H2, *bcs = bas + KP;
    float *rowf = bcs + 4;                 // action, old_logp, adv, ret: [4][BP]
    float *logit = rowf + 4 * BP;          // [BP][KP]
    float *vrow = logit + BP * KP;         // [BP]
    XPA_SM_STAMP(0);
    // ---- staging: two global round trips in all — the row indices with every weight load, then the rows ----
    // (five dependent load / store rounds took ~21 k cycles before)
    const int n0 = H0 * D, na = K * H1, nm = n0 + na + H2 + H0 + H1 + H2 + K + 1;   // W0 | Wa | Wc | biases
    const int nw1 = H0 * H1, nw2 = H0 * H2;
    const bool fast = nm <= 2 * kSmThreads && nw1 <= 8 * kSmThreads && nw2 <= 8 * kSmThreads && BP <= kSmThreads &&
                      Btot <= kSmThreads;
    float adv_all = 0.f;   // split form: the advantage of minibatch row t (the moments are over every row)
    // element e of the small-tensor range: its source (loads) and LDS destination (stores)
    auto msrc_of = [&](int e, int &off) -> const float * {
        if (e < n0) { off = e; return a.W0; }
        if ((e -= n0) < na) { off = e; return a.Wa; }
        if ((e -= na) < H2) { off = e; return a.Wc; }
        if ((e -= H2) < H0) { off = e; return a.b0; }
        if ((e -= H0) < H1) { off = e; return a.b1; }
        if ((e -= H1) < H2) { off = e; return a.b2; }
        if ((e -= H2) < K) { off = e; return a.ba; }
        off = 0;
        return a.bc;
    };
    auto mdst_of = [&](int e) -> float * {
        if (e < n0) return W0T + (e % D) * H0 + e / D;
        if ((e -= n0) < na) return WaT + (e % H1) * KP + e / H1;
        if ((e -= na) < H2) return Wcv + e;
        if ((e -= H2) < H0) return b0s + e;
        if ((e -= H0) < H1) return b1s + e;
        if ((e -= H1) < H2) return b2s + e;
        if ((e -= H2) < K) return bas + e;
        return bcs;
    };
    if (fast) {
        const bool rb = t < BP && t < B;
        int64_t row = rb ? idx[t] : 0;
        const bool ra = G > 1 && t < Btot;
        const int64_t rowa = ra ? a.idx[t] : 0;
        float vm[2], v1[8], v2[8];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            int off;
            const float *src = msrc_of(t + u * kSmThreads, off);
            vm[u] = t + u * kSmThreads < nm ? src[off] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {   // source order: coalesced loads (see stage_T below)
            const int e1 = t + u * kSmThreads;
            v1[u] = e1 < nw1 ? a.W1[e1] : 0.f;
            v2[u] = e1 < nw2 ? a.W2[e1] : 0.f;
        }
        // the rows (second round trip)
        const bool valid = rb && row >= 0 && row < a.n_rows;
        const int64_t rc = valid ? row : 0;
        float xo[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) xo[i] = i < D ? a.obs[rc * a.obs_ld + i] : 0.f;
        const float act_v = a.actions[rc], lp_v = a.old_logp ? a.old_logp[rc] : 0.f, av = a.adv[rc], rt = a.ret[rc];
        if (ra && rowa >= 0 && rowa < a.n_rows) adv_all = a.adv[rowa];
        // LDS stores
#pragma unroll
        for (int u = 0; u < 2; ++u)
            if (t + u * kSmThreads < nm) *mdst_of(t + u * kSmThreads) = vm[u];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int e1 = t + u * kSmThreads;
            if (e1 < nw1) W1T[(e1 % H0) * H1P + e1 / H0] = v1[u];
            if (e1 < nw2) W2T[(e1 % H0) * H2P + e1 / H0] = v2[u];
        }
        if (t < BP) {
#pragma unroll
            for (int i = 0; i < 32; ++i)
                if (i < DP) xT[i * S + t] = valid ? xo[i] : 0.f;
            rowf[0 * BP + t] = valid ? act_v : 0.f;
            rowf[1 * BP + t] = valid ? lp_v : 0.f;
            rowf[2 * BP + t] = valid ? av : 0.f;
            rowf[3 * BP + t] = valid ? rt : 0.f;
        }
    } else {
    {
        // the small tensors as one virtual range: W0 [H0][D] | Wa [K][H1] | Wc [H2] | b0 | b1 | b2 | ba | bc
        const int n0 = H0 * D, na = K * H1, nm = n0 + na + H2 + H0 + H1 + H2 + K + 1;
        for (int e0 = t; e0 < nm; e0 += 4 * kSmThreads) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                int e = e0 + u * kSmThreads;
                const float *src = a.bc;
                int off = 0;
                if (e < n0) { src = a.W0; off = e; }
                else if ((e -= n0) < na) { src = a.Wa; off = e; }
                else if ((e -= na) < H2) { src = a.Wc; off = e; }
                else if ((e -= H2) < H0) { src = a.b0; off = e; }
                else if ((e -= H0) < H1) { src = a.b1; off = e; }
                else if ((e -= H1) < H2) { src = a.b2; off = e; }
                else if ((e -= H2) < K) { src = a.ba; off = e; }
                v[u] = e0 + u * kSmThreads < nm ? src[off] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                int e = e0 + u * kSmThreads;
                if (e >= nm) continue;
                if (e < n0) { W0T[(e % D) * H0 + e / D] = v[u]; continue; }
                if ((e -= n0) < na) { WaT[(e % H1) * KP + e / H1] = v[u]; continue; }
                if ((e -= na) < H2) { Wcv[e] = v[u]; continue; }
                if ((e -= H2) < H0) { b0s[e] = v[u]; continue; }
                if ((e -= H0) < H1) { b1s[e] = v[u]; continue; }
                if ((e -= H1) < H2) { b2s[e] = v[u]; continue; }
                if ((e -= H2) < K) { bas[e] = v[u]; continue; }
                bcs[0] = v[u];
            }
        }
        // zero pads: W0T rows D .. DP, WaT columns K .. KP, ba K .. KP
        for (int e = t; e < (DP - D) * H0; e += kSmThreads) W0T[D * H0 + e] = 0.f;
        for (int e = t; e < H1 * (KP - K); e += kSmThreads) WaT[(e / (KP - K)) * KP + K + e % (KP - K)] = 0.f;
        for (int e = K + t; e < KP; e += kSmThreads) bas[e] = 0.f;
        // W1 [H1][H0] -> W1T [H0][H1P], W2 likewise: 8 loads per thread in flight, walked in source order (coalesced:
        // a destination-order gather made every lane of a wave touch its own cache line) and written with the odd
        // row stride H1P (consecutive lanes -> consecutive banks; with stride H1 every lane hit one bank)
        auto stage_T = [&](const float *src, int rows, int cols, float *dst, int ldd) {
            const int n = rows * cols;
            for (int e0 = t; e0 < n; e0 += 8 * kSmThreads) {
                float v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int e = e0 + u * kSmThreads;
                    v[u] = e < n ? src[e] : 0.f;
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int e = e0 + u * kSmThreads;
                    if (e < n) dst[(e % cols) * ldd + e / cols] = v[u];
                }
            }
        };
        stage_T(a.W1, H1, H0, W1T, H1P);
        stage_T(a.W2, H2, H0, W2T, H2P);
    }
    double adv_s0 = 0.0, adv_q0 = 0.0;
    for (int b = t; b < BP; b += kSmThreads) {
        const bool ok = b < B;
        const int64_t row = ok ? idx[b] : 0;
        const bool valid = ok && row >= 0 && row < a.n_rows;
        const int64_t rc = valid ? row : 0;
        float xo[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) xo[i] = i < D ? a.obs[rc * a.obs_ld + i] : 0.f;
        const float act_v = a.actions[rc], lp_v = a.old_logp ? a.old_logp[rc] : 0.f, av = a.adv[rc], rt = a.ret[rc];
#pragma unroll
        for (int i = 0; i < 32; ++i)
            if (i < DP) xT[i * S + b] = valid ? xo[i] : 0.f;
        rowf[0 * BP + b] = valid ? act_v : 0.f;
        rowf[1 * BP + b] = valid ? lp_v : 0.f;
        rowf[2 * BP + b] = valid ? av : 0.f;
        rowf[3 * BP + b] = valid ? rt : 0.f;
        if (ok) {   // the minibatch advantage moments (K4's (sum, sumsq) in f64) over the batch rows
            const double ad = valid ? (double)av : 0.0;
            adv_s0 += ad;
            adv_q0 += ad * ad;
        }
    }
    }
    for (int e = t; e < (DP - D) * H0; e += kSmThreads) W0T[D * H0 + e] = 0.f;
    for (int e = t; e < H1 * (KP - K); e += kSmThreads) WaT[(e / (KP - K)) * KP + K + e % (KP - K)] = 0.f;
    for (int e = K + t; e < KP; e += kSmThreads) bas[e] = 0.f;
    __syncthreads();   // the rows' advantages are in LDS
    double adv_s = 0.0, adv_q = 0.0;
    if (G == 1) {
        for (int b = t; b < B; b += kSmThreads) {   // the minibatch advantage moments (K4's (sum, sumsq) in f64)
            const double ad = (double)rowf[2 * BP + b];
            adv_s += ad;
            adv_q += ad * ad;
        }
    } else if (fast) {
        if (t < Btot) {   // the same per-row terms, from the rows' advantages loaded with the staging
            const double ad = (double)adv_all;
            adv_s += ad;
            adv_q += ad * ad;
        }
    } else {
        for (int b = t; b < Btot; b += kSmThreads) {
            const int64_t row = a.idx[b];
            const double ad = (row >= 0 && row < a.n_rows) ? (double)a.adv[row] : 0.0;
            adv_s += ad;
            adv_q += ad * ad;
        }
    }
    for (int e = t; e < 4 * S; e += kSmThreads) dvT[e] = 0.f;
    for (int e = t; e < KP * S; e += kSmThreads) dlT[e] = 0.f;
    adv_s = xpa_wave_sum(adv_s);
    adv_q = xpa_wave_sum(adv_q);
    if (lane == 0) {
        s_red[w] = adv_s;
        s_red[kSmWaves + w] = adv_q;
    }
    __syncthreads();
    if (t == 0) {
        double s = 0.0, q = 0.0;
        for (int i = 0; i < kSmWaves; ++i) {
            s += s_red[i];
            q += s_red[kSmWaves + i];
        }
        if (a.use_advnorm) {   // memory_tools.py:241-242, the arithmetic of loss.hip adv_moments
            const double mean = s / (double)Btot;
            const double var = fmax(q / (double)Btot - mean * mean, 0.0);
            s_stat[0] = (float)mean;
            s_stat[1] = (float)(1.0 / ((double)(float)sqrt(var) + 1e-8));
        } else {
            s_stat[0] = 0.f;
            s_stat[1] = 1.f;
        }
    }
    XPA_SM_STAMP(1);
    // ---- forward: h0 = act(x W0^T + b0), then h1 / h2 from h0 ----
    for (int tl = w; tl < MB * (H0 / 32); tl += kSmWaves) {
        const int b0 = 32 * (tl % MB), j0 = 32 * (tl / MB);
        const f32x16 acc = sm_tile(xT + b0, 1, S, 32, W0T + j0, H0, 1, 32, DP);
#pragma unroll
        for (int r = 0; r < 16; ++r)
            h0T[(j0 + li) * S + b0 + sm_row(r)] = sm_act<ACT>(acc[r] + b0s[j0 + li], slope);
    }
    __syncthreads();
    {
        const int n1 = MB * (H1 / 32), n2 = MB * (H2 / 32);
        for (int tl = w; tl < n1 + n2; tl += kSmWaves) {
            const bool two = tl >= n1;
            const int q = two ? tl - n1 : tl, b0 = 32 * (q % MB), j0 = 32 * (q / MB);
            const int HOP = two ? H2P : H1P;
            const float *WT = two ? W2T : W1T, *bb = two ? b2s : b1s;
            float *outT = two ? h2T : h1T;
            const f32x16 acc = sm_tile(h0T + b0, 1, S, 32, WT + j0, HOP, 1, 32, H0);
#pragma unroll
            for (int r = 0; r < 16; ++r)
                outT[(j0 + li) * S + b0 + sm_row(r)] = sm_act<ACT>(acc[r] + bb[j0 + li], slope);
        }
    }
    __syncthreads();
    XPA_SM_STAMP(2);
    // output layers: logits [BP][KP] from h1, v [BP] from h2
    for (int tl = w; tl < 2 * MB; tl += kSmWaves) {
        const bool val = tl >= MB;
        const int b0 = 32 * (val ? tl - MB : tl);
        const f32x16 acc = val ? sm_tile(h2T + b0, 1, S, 32, Wcv, 1, 0, 1, H2)
                               : sm_tile(h1T + b0, 1, S, 32, WaT, KP, 1, KP, H1);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int b = b0 + sm_row(r);
            if (val) {
                if (li == 0) vrow[b] = acc[r] + bcs[0];
            } else if (li < KP) {
                logit[b * KP + li] = acc[r] + bas[li];
            }
        }
    }
    __syncthreads();
    XPA_SM_STAMP(3);
    // ---- loss, one thread per row (K2's categorical arithmetic) ----
    const float inv_b = 1.0f / (float)Btot;
    float surr = 0.f, sqe = 0.f, ent = 0.f, clipc = 0.f, vsum = 0.f;
    const float mean_a = s_stat[0], inv_a = s_stat[1];
    for (int b = t; b < B; b += kSmThreads) {
        const int64_t row = idx[b];
        if (!(row >= 0 && row < a.n_rows)) continue;   // out-of-range index: zero gradient (dlT / dvT stay 0)
        const float *zr = logit + b * KP;
        const float A_n = (rowf[2 * BP + b] - mean_a) * inv_a;
        const float vb = vrow[b];
        const float diffv = vb - rowf[3 * BP + b];
        sqe += diffv * diffv;
        vsum += vb;
        dvT[b] = a.vf_coef * 2.0f * diffv * inv_b;
        float m = zr[0];
        for (int k = 1; k < K; ++k) m = fmaxf(m, zr[k]);
        float se = 0.f;
        for (int k = 0; k < K; ++k) se += expf(zr[k] - m);
        const float lse = m + logf(se);
        int ai = (int)rowf[b];
        ai = ai < 0 ? 0 : (ai >= K ? K - 1 : ai);
        const float logp = zr[ai] - lse;
        float H = 0.f;
        for (int k = 0; k < K; ++k) {
            const float ln = zr[k] - lse;
            H -= expf(ln) * ln;
        }
        ent += H;
        float dlogp;
        if (ALGO == XPA_ALGO_PPO) {
            const float ratio = expf(logp - rowf[BP + b]);
            const float lo = 1.0f - a.clip_range, hi = 1.0f + a.clip_range;
            const float cr = fminf(fmaxf(ratio, lo), hi);
            const float s1 = cr * A_n, s2 = A_n * ratio;
            surr += fminf(s1, s2);
            const bool inr = (ratio >= lo) && (ratio <= hi);
            const float g1 = inr ? A_n : 0.f;
            const float w1 = (s1 < s2) ? 1.f : ((s1 == s2) ? 0.5f : 0.f);
            const float w2 = (s2 < s1) ? 1.f : ((s1 == s2) ? 0.5f : 0.f);
            dlogp = -inv_b * (w1 * g1 + w2 * A_n) * ratio;
            clipc += ((ratio < lo) || (ratio > hi)) ? 1.f : 0.f;
        } else {
            surr += A_n * logp;
            dlogp = -A_n * inv_b;
        }
        const float ec = a.ent_coef * inv_b;
        for (int k = 0; k < K; ++k) {
            const float ln = zr[k] - lse;
            const float p = expf(ln);
            dlT[k * S + b] = dlogp * ((k == ai ? 1.f : 0.f) - p) + ec * p * (ln + H);
        }
    }
    {
        const float vals[5] = {surr, sqe, ent, clipc, vsum};
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            const float r = xpa_wave_sum(vals[q]);
            if (lane == 0) s_red[q * kSmWaves + w] = (double)r;
        }
    }
    __syncthreads();
    if (t == 0 && G > 1) {   // split form: this workgroup's loss sums (finalized by small_mlp_finalize_kernel)
        for (int q = 0; q < 5; ++q) {
            double tq = 0.0;
            for (int i = 0; i < kSmWaves; ++i) tq += s_red[q * kSmWaves + i];
            a.loss_part[gi * 8 + q] = tq;
        }
    }
    if (t == 0 && G == 1) {
        double tot[5];
        for (int q = 0; q < 5; ++q) {
            tot[q] = 0.0;
            for (int i = 0; i < kSmWaves; ++i) tot[q] += s_red[q * kSmWaves + i];
        }
        const double Bd = (double)B;
        const double actor = -tot[0] / Bd, critic = tot[1] / Bd, entropy = tot[2] / Bd;
        a.scalars[XPA_OUT_ACTOR_LOSS] = (float)actor;
        a.scalars[XPA_OUT_CRITIC_LOSS] = (float)critic;
        a.scalars[XPA_OUT_ENTROPY] = (float)entropy;
        a.scalars[XPA_OUT_LOSS] = (float)(actor - (double)a.ent_coef * entropy + (double)a.vf_coef * critic);
        a.scalars[XPA_OUT_CLIP_RATIO] = ALGO == XPA_ALGO_PPO ? (float)(tot[3] / Bd) : 0.f;
        a.scalars[XPA_OUT_VALUE_MEAN] = (float)(tot[4] / Bd);
    }
    XPA_SM_STAMP(4);
    // ---- backward ----
    double sq = 0.0;   // this thread's share of |grad|^2
    // the hidden weights row-major ([j][i], over the transposed forward copies) for dh0: loads issued now, stored
    // below (the forward is the last reader of the transposed images)
    {
        const int n1 = H1 * H0, n2 = H2 * H0;
        for (int e0 = t; e0 < n1 + n2; e0 += 8 * kSmThreads) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = e0 + u * kSmThreads;
                v[u] = e < n1 ? a.W1[e] : (e < n1 + n2 ? a.W2[e - n1] : 0.f);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = e0 + u * kSmThreads;
                if (e < n1 + n2) W1T[e] = v[u];   // W2T == W1T + H0 H1: the W2 block follows contiguously
            }
        }
    }
    // output layers' weight gradients: gWa [K][H1] = dl^T h1, gWc [H2] = dv^T h2
    for (int tl = w; tl < H1 / 32 + H2 / 32; tl += kSmWaves) {
        const bool val = tl >= H1 / 32;
        const int j0 = 32 * (val ? tl - H1 / 32 : tl);
        const f32x16 acc = val ? sm_tile(dvT, S, 1, 1, h2T + j0 * S, 1, S, 32, BP)
                               : sm_tile(dlT, S, 1, KP, h1T + j0 * S, 1, S, 32, BP);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = sm_row(r);
            if (val ? m == 0 : m < K) {
                const float g = acc[r];
                if (val) gp(a.gWc)[j0 + li] = g;
                else gp(a.gWa)[m * H1 + j0 + li] = g;
                sq += (double)g * g;
            }
        }
    }
    __syncthreads();
    XPA_SM_STAMP(5);
    // dh1 = (dl Wa) act'(h1) on MFMA, dh2 = dv wc act'(h2) elementwise: in place over h1 / h2
    for (int tl = w; tl < MB * (H1 / 32); tl += kSmWaves) {
        const int b0 = 32 * (tl % MB), j0 = 32 * (tl / MB);
        const f32x16 acc = sm_tile(dlT + b0, 1, S, 32, WaT + j0 * KP, 1, KP, 32, KP);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float *p = h1T + (j0 + li) * S + b0 + sm_row(r);
            *p = acc[r] * sm_grad<ACT>(*p, slope);
        }
    }
    for (int e = t; e < H2 * BP; e += kSmThreads) {
        const int j = e / BP, b = e % BP;
        float *p = h2T + j * S + b;
        *p = dvT[b] * Wcv[j] * sm_grad<ACT>(*p, slope);
    }
    __syncthreads();
    XPA_SM_STAMP(6);
    // hidden layers' weight gradients: gW1 [H1][H0] = dh1^T h0, gW2 [H2][H0] = dh2^T h0
    {
        const int n1 = (H1 / 32) * (H0 / 32), n2 = (H2 / 32) * (H0 / 32);
        for (int tl = w; tl < n1 + n2; tl += kSmWaves) {
            const bool two = tl >= n1;
            const int q = two ? tl - n1 : tl, j0 = 32 * (q % ((two ? H2 : H1) / 32)), i0 = 32 * (q / ((two ? H2 : H1) / 32));
            const f32x16 acc = sm_tile((two ? h2T : h1T) + j0 * S, S, 1, 32, h0T + i0 * S, 1, S, 32, BP);
            float *gW = gp(two ? a.gW2 : a.gW1);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float g = acc[r];
                gW[(j0 + sm_row(r)) * H0 + i0 + li] = g;
                sq += (double)g * g;
            }
        }
    }
    __syncthreads();
    XPA_SM_STAMP(7);
    // dh0 = (dh1 W1 + dh2 W2) act'(h0), in place over h0
    for (int tl = w; tl < MB * (H0 / 32); tl += kSmWaves) {
        const int b0 = 32 * (tl % MB), i0 = 32 * (tl / MB);
        f32x16 acc = sm_tile(h1T + b0, 1, S, 32, W1T + i0, H0, 1, 32, H1);
        const f32x16 acc2 = sm_tile(h2T + b0, 1, S, 32, W1T + H1 * H0 + i0, H0, 1, 32, H2);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float *p = h0T + (i0 + li) * S + b0 + sm_row(r);
            *p = (acc[r] + acc2[r]) * sm_grad<ACT>(*p, slope);
        }
    }
    __syncthreads();
    XPA_SM_STAMP(8);
    // first layer's weight gradient gW0 [H0][D] = dh0^T x, and every bias gradient (row sums over the batch)
    for (int tl = w; tl < H0 / 32; tl += kSmWaves) {
        const int i0 = 32 * tl;
        const f32x16 acc = sm_tile(h0T + i0 * S, S, 1, 32, xT, 1, S, DP, BP);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (li < D) {
                const float g = acc[r];
                gp(a.gW0)[(i0 + sm_row(r)) * D + li] = g;
                sq += (double)g * g;
            }
        }
    }
    {
        // bias gradients: one thread per output feature, its row summed with 16-B reads (BP % 32 == 0)
        const int nr = H0 + H1 + H2 + K + 1;
        for (int f = t; f < nr; f += kSmThreads) {
            const float *src;
            float *dst;
            if (f < H0) { src = h0T + f * S; dst = gp(a.gb0) + f; }
            else if (f < H0 + H1) { src = h1T + (f - H0) * S; dst = gp(a.gb1) + f - H0; }
            else if (f < H0 + H1 + H2) { src = h2T + (f - H0 - H1) * S; dst = gp(a.gb2) + f - H0 - H1; }
            else if (f < H0 + H1 + H2 + K) { src = dlT + (f - H0 - H1 - H2) * S; dst = gp(a.gba) + f - H0 - H1 - H2; }
            else { src = dvT; dst = gp(a.gbc); }
            float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
            for (int b = 0; b < BP; b += 4) {
                const float4 v = *reinterpret_cast<const float4 *>(src + b);
                s0 += v.x;
                s1 += v.y;
                s2 += v.z;
                s3 += v.w;
            }
            const float s = (s0 + s1) + (s2 + s3);
            *dst = s;
            sq += (double)s * s;
        }
    }
    XPA_SM_STAMP(9);
    if (G > 1) return;   // the split form's partials are done: small_mlp_finalize_kernel sums, clips and steps
    // ---- clip_grad_norm_ + Adam over the flat buffers (K9's arithmetic, schedule at the device cursor) ----
    sq = xpa_wave_sum(sq);
    if (lane == 0) s_red[w] = sq;
    __syncthreads();   // also orders every gradient store of the block before the flat-buffer reads below
    if (t == 0) {
        double s = 0.0;
        for (int i = 0; i < kSmWaves; ++i) s += s_red[i];
        const float total = (float)sqrt(s);
        float coef = 1.0f;
        if (a.max_norm >= 0.f) coef = fminf(a.max_norm / (total + 1e-6f), 1.0f);
        s_coef = coef;
        if (a.total_norm_out) *a.total_norm_out = total;
        int k = a.cursor[0];
        if (k >= a.n_sched) {
            a.cursor[2] = 1;
            k = a.n_sched - 1;
        }
        s_step = a.sched[2 * k];
        s_inv = a.sched[2 * k + 1];
    }
    __syncthreads();
    const float coef = s_coef, step_size = s_step, inv_bc2_sqrt = s_inv;
    const float b1 = a.beta1, b2 = a.beta2, eps = a.eps;
    // 16-B accesses, 4 float4 of each stream in flight per thread (the flat buffers are 16-B aligned, n % 4 == 0
    // is checked on the host)
    const int64_t n4 = a.n / 4;
    float4 *p4 = reinterpret_cast<float4 *>(a.param), *g4 = reinterpret_cast<float4 *>(a.grad);
    float4 *m4 = reinterpret_cast<float4 *>(a.exp_avg), *v4 = reinterpret_cast<float4 *>(a.exp_avg_sq);
    for (int64_t i0 = t; i0 < n4; i0 += 4 * kSmThreads) {
        float4 P[4], G[4], M[4], V[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = i0 + u * kSmThreads < n4 ? i0 + u * kSmThreads : n4 - 1;
            P[u] = p4[i];
            G[u] = g4[i];
            M[u] = m4[i];
            V[u] = v4[i];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            float *pp = &P[u].x, *gg = &G[u].x, *mm = &M[u].x, *vv = &V[u].x;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                float g = gg[c] * coef, m = mm[c], v = vv[c];
                m = m + (1.0f - b1) * (g - m);
                v = b2 * v + (1.0f - b2) * g * g;
                const float denom = sqrtf(v) * inv_bc2_sqrt + eps;
                pp[c] = pp[c] - step_size * (m / denom);
                gg[c] = g;
                mm[c] = m;
                vv[c] = v;
            }
            if (i0 + u * kSmThreads < n4) {
                const int64_t i = i0 + u * kSmThreads;
                p4[i] = P[u];
                g4[i] = G[u];
                m4[i] = M[u];
                v4[i] = V[u];
            }
        }
    }
    XPA_SM_STAMP(10);
    if (t == 0) a.cursor[0] = a.cursor[0] + 1;
}

// Split form's second launch: the loss scalars from the workgroups' loss sums, the gradient as the sum of the
// workgroups' partials in workgroup order (written to the flat gradient buffer), clip_grad_norm_ and Adam — K30's
// tail arithmetic.
template <int ALGO>
__global__ __launch_bounds__(kSmThreads, 1) void small_mlp_finalize_kernel(XpaSmallMlpArgs a) {
    __shared__ double s_red[kSmWaves];
    __shared__ float s_coef, s_step, s_inv;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int G = a.n_groups;
    if (t == 0) {
        double tot[5];
        for (int q = 0; q < 5; ++q) {
            tot[q] = 0.0;
            for (int g = 0; g < G; ++g) tot[q] += a.loss_part[g * 8 + q];
        }
        const double Bd = (double)a.batch;
        const double actor = -tot[0] / Bd, critic = tot[1] / Bd, entropy = tot[2] / Bd;
        a.scalars[XPA_OUT_ACTOR_LOSS] = (float)actor;
        a.scalars[XPA_OUT_CRITIC_LOSS] = (float)critic;
        a.scalars[XPA_OUT_ENTROPY] = (float)entropy;
        a.scalars[XPA_OUT_LOSS] = (float)(actor - (double)a.ent_coef * entropy + (double)a.vf_coef * critic);
        a.scalars[XPA_OUT_CLIP_RATIO] = ALGO == XPA_ALGO_PPO ? (float)(tot[3] / Bd) : 0.f;
        a.scalars[XPA_OUT_VALUE_MEAN] = (float)(tot[4] / Bd);
    }
    const int64_t n4 = a.n / 4;
    const float4 *part4 = reinterpret_cast<const float4 *>(a.grad_part);
    float4 *p4 = reinterpret_cast<float4 *>(a.param), *g4 = reinterpret_cast<float4 *>(a.grad);
    float4 *m4 = reinterpret_cast<float4 *>(a.exp_avg), *v4 = reinterpret_cast<float4 *>(a.exp_avg_sq);
    const float b1 = a.beta1, b2 = a.beta2, eps = a.eps;
    // Adam's element update (K9's arithmetic): gg is the unclipped gradient in, the clipped one out
    auto adam4 = [&](float4 &P, float4 &Gr, float4 &M, float4 &V, float coef, float step_size, float inv_bc2_sqrt) {
        float *pp = &P.x, *gg = &Gr.x, *mm = &M.x, *vv = &V.x;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            float g = gg[c] * coef, m = mm[c], v = vv[c];
            m = m + (1.0f - b1) * (g - m);
            v = b2 * v + (1.0f - b2) * g * g;
            const float denom = sqrtf(v) * inv_bc2_sqrt + eps;
            pp[c] = pp[c] - step_size * (m / denom);
            gg[c] = g;
            mm[c] = m;
            vv[c] = v;
        }
    };
    // Every element's partials, parameter and moments loaded in ONE round trip before the norm (the norm only scales
    // the gradient): up to kFinJ float4 elements per thread held in registers.
    constexpr int kFinJ = 6;
    const bool regs = n4 <= (int64_t)kFinJ * kSmThreads && G <= 4;
    double sq = 0.0;
    float4 Sg[kFinJ], Pp[kFinJ], Mm[kFinJ], Vv[kFinJ];
    if (regs) {
        float4 Q[kFinJ][4];
#pragma unroll
        for (int j = 0; j < kFinJ; ++j) {
            const int64_t i0 = t + (int64_t)j * kSmThreads;
            const int64_t i = i0 < n4 ? i0 : n4 - 1;
#pragma unroll
            for (int g = 0; g < 4; ++g)
                if (g < G) Q[j][g] = part4[(int64_t)g * n4 + i];
            Pp[j] = p4[i];
            Mm[j] = m4[i];
            Vv[j] = v4[i];
        }
#pragma unroll
        for (int j = 0; j < kFinJ; ++j) {
            float4 sg = Q[j][0];
#pragma unroll
            for (int g = 1; g < 4; ++g)
                if (g < G) {
                    sg.x += Q[j][g].x;
                    sg.y += Q[j][g].y;
                    sg.z += Q[j][g].z;
                    sg.w += Q[j][g].w;
                }
            Sg[j] = sg;
            if (t + (int64_t)j * kSmThreads < n4) {
                sq += (double)sg.x * sg.x;
                sq += (double)sg.y * sg.y;
                sq += (double)sg.z * sg.z;
                sq += (double)sg.w * sg.w;
            }
        }
    } else {
        for (int64_t i0 = t; i0 < n4; i0 += 2 * kSmThreads) {
            float4 P[2][16];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int64_t i = i0 + u * kSmThreads < n4 ? i0 + u * kSmThreads : n4 - 1;
#pragma unroll
                for (int g = 0; g < 16; ++g)
                    if (g < G) P[u][g] = part4[(int64_t)g * n4 + i];
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                float4 sg = P[u][0];
#pragma unroll
                for (int g = 1; g < 16; ++g)
                    if (g < G) {
                        sg.x += P[u][g].x;
                        sg.y += P[u][g].y;
                        sg.z += P[u][g].z;
                        sg.w += P[u][g].w;
                    }
                if (i0 + u * kSmThreads < n4) {
                    g4[i0 + u * kSmThreads] = sg;
                    sq += (double)sg.x * sg.x;
                    sq += (double)sg.y * sg.y;
                    sq += (double)sg.z * sg.z;
                    sq += (double)sg.w * sg.w;
                }
            }
        }
    }
    sq = xpa_wave_sum(sq);
    if (lane == 0) s_red[w] = sq;
    __syncthreads();   // also orders the two-pass form's gradient stores before its Adam pass's reads
    if (t == 0) {
        double s = 0.0;
        for (int i = 0; i < kSmWaves; ++i) s += s_red[i];
        const float total = (float)sqrt(s);
        float coef = 1.0f;
        if (a.max_norm >= 0.f) coef = fminf(a.max_norm / (total + 1e-6f), 1.0f);
        s_coef = coef;
        if (a.total_norm_out) *a.total_norm_out = total;
        int k = a.cursor[0];
        if (k >= a.n_sched) {
            a.cursor[2] = 1;
            k = a.n_sched - 1;
        }
        s_step = a.sched[2 * k];
        s_inv = a.sched[2 * k + 1];
    }
    __syncthreads();
    const float coef = s_coef, step_size = s_step, inv_bc2_sqrt = s_inv;
    if (regs) {
#pragma unroll
        for (int j = 0; j < kFinJ; ++j) {
            const int64_t i = t + (int64_t)j * kSmThreads;
            adam4(Pp[j], Sg[j], Mm[j], Vv[j], coef, step_size, inv_bc2_sqrt);
            if (i < n4) {
                p4[i] = Pp[j];
                g4[i] = Sg[j];
                m4[i] = Mm[j];
                v4[i] = Vv[j];
            }
        }
    } else {
        for (int64_t i0 = t; i0 < n4; i0 += 4 * kSmThreads) {
            float4 P[4], Gr[4], M[4], V[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t i = i0 + u * kSmThreads < n4 ? i0 + u * kSmThreads : n4 - 1;
                P[u] = p4[i];
                Gr[u] = g4[i];
                M[u] = m4[i];
                V[u] = v4[i];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                adam4(P[u], Gr[u], M[u], V[u], coef, step_size, inv_bc2_sqrt);
                if (i0 + u * kSmThreads < n4) {
                    const int64_t i = i0 + u * kSmThreads;
                    p4[i] = P[u];
                    g4[i] = Gr[u];
                    m4[i] = M[u];
                    v4[i] = V[u];
                }
            }
        }
    }
    if (t == 0) a.cursor[0] = a.cursor[0] + 1;
}

}  // namespace

XPA_API int64_t xpa_small_mlp_lds_floats(int64_t batch, int64_t d_in, int64_t h0, int64_t h1, int64_t h2, int64_t k) {
    const int64_t BP = (batch + 31) & ~31, S = BP + 4, DP = (d_in + 3) & ~3, KP = (k + 3) & ~3;
    return DP * S + (h0 + h1 + h2) * S + KP * S + 4 * S + DP * h0 + h0 * (h1 + 1) + h0 * (h2 + 1) + h1 * KP + h2 + h0 +
           h1 + h2 +
           KP + 4 + 4 * BP + BP * KP + BP;
}

XPA_API int xpa_small_mlp_update(const XpaSmallMlpArgs *args, xpa_stream_t stream) {
    if (!args) return (int)hipErrorInvalidValue;
    const XpaSmallMlpArgs &a = *args;
    if (a.batch < 1 || a.d_in < 1 || a.d_in > 32 || a.h0 < 32 || a.h1 < 32 || a.h2 < 32 || a.h0 % 32 || a.h1 % 32 ||
        a.h2 % 32 || a.h0 > 256 || a.h1 > 256 || a.h2 > 256 || a.k < 2 || a.k > 16 || a.act_code < 0 || a.act_code > 2 ||
        (a.algo != XPA_ALGO_PPO && a.algo != XPA_ALGO_A2C) || (a.algo == XPA_ALGO_PPO && !a.old_logp) || !a.obs ||
        !a.idx || !a.actions || !a.adv || !a.ret || !a.param || !a.grad || !a.exp_avg || !a.exp_avg_sq || !a.sched ||
        !a.cursor || a.n_sched < 1 || !a.scalars || a.n < 1 || !a.W0 || !a.b0 || !a.W1 || !a.b1 || !a.W2 || !a.b2 ||
        !a.Wa || !a.ba || !a.Wc || !a.bc || !a.gW0 || !a.gb0 || !a.gW1 || !a.gb1 || !a.gW2 || !a.gb2 || !a.gWa ||
        !a.gba || !a.gWc || !a.gbc || a.n % 4 ||
        ((uintptr_t)a.param | (uintptr_t)a.grad | (uintptr_t)a.exp_avg | (uintptr_t)a.exp_avg_sq) % 16)
        return (int)hipErrorInvalidValue;
    const int G = a.n_groups < 1 ? 1 : a.n_groups;
    if (G > 1 && (G > 16 || G != (a.batch + 31) / 32 || !a.grad_part || !a.loss_part || (uintptr_t)a.grad_part % 16))
        return (int)hipErrorInvalidValue;
    if (xpa_small_mlp_lds_floats(G > 1 ? 32 : a.batch, a.d_in, a.h0, a.h1, a.h2, a.k) > kSmLds)
        return (int)hipErrorInvalidValue;
    hipStream_t s = (hipStream_t)stream;
#define XPA_SM(A_, G_) hipLaunchKernelGGL((small_mlp_update_kernel<A_, G_>), dim3(G), dim3(kSmThreads), 0, s, a)
    if (a.algo == XPA_ALGO_PPO) {
        if (a.act_code == 0) XPA_SM(0, XPA_ALGO_PPO);
        else if (a.act_code == 1) XPA_SM(1, XPA_ALGO_PPO);
        else XPA_SM(2, XPA_ALGO_PPO);
    } else {
        if (a.act_code == 0) XPA_SM(0, XPA_ALGO_A2C);
        else if (a.act_code == 1) XPA_SM(1, XPA_ALGO_A2C);
        else XPA_SM(2, XPA_ALGO_A2C);
    }
#undef XPA_SM
    if (G > 1) {
        if (a.algo == XPA_ALGO_PPO)
            hipLaunchKernelGGL((small_mlp_finalize_kernel<XPA_ALGO_PPO>), dim3(1), dim3(kSmThreads), 0, s, a);
        else
            hipLaunchKernelGGL((small_mlp_finalize_kernel<XPA_ALGO_A2C>), dim3(1), dim3(kSmThreads), 0, s, a);
    }
    return xpa_launch_status();
}
