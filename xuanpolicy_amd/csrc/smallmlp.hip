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
// Layout: activations transposed, [feature][batch] with row stride BPS = BP + 4 (BP = batch rounded up to 4; the
// +4 puts consecutive feature rows 4 banks apart, so the 16 rows a wave reads in a tile step are conflict-free).
// Forward tiles: a thread owns 4 output features x 4 rows and walks the input features (one ds_read_b128 of the
// input rows, one of the transposed weights, 16 FMAs).  Weight gradients: a thread owns 4 x 4 (out, in) and walks
// the rows 4 at a time (8 ds_read_b128, 64 FMAs).  In-place reuse: h1 / h2 become dh1 / dh2 once the output layers'
// weight gradients are formed, h0 becomes dh0 once the hidden layers' weight gradients are formed.
// Arithmetic of the loss and of the clip + Adam step: exactly K2's per-row formulas (loss.hip) and K9's (optim.hip).
#include "xpa_common.h"

namespace {

constexpr int kSmThreads = 512;
constexpr int kSmWaves = kSmThreads / 64;
constexpr int kSmLds = 40704;   // floats (159 KiB: the rest of the 160 KiB holds the reduction scratch)

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

// outT[j][b] = act(bias[j] + sum_i inT[i][b] WT[i][j]),  j < HO, b < BP (row stride S, WT row stride HO)
template <int ACT>
__device__ void sm_fwd(const float *inT, int HI, const float *WT, const float *bias, int HO, float *outT, int BP,
                       int S, float slope) {
    const int tj = HO / 4, tb = BP / 4;
    for (int t = threadIdx.x; t < tj * tb; t += kSmThreads) {
        const int j0 = 4 * (t % tj), b0 = 4 * (t / tj);
        float acc[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[r][c] = 0.f;
#pragma unroll 4
        for (int i = 0; i < HI; ++i) {
            const float4 x = *reinterpret_cast<const float4 *>(inT + i * S + b0);
            const float4 w = *reinterpret_cast<const float4 *>(WT + i * HO + j0);
            const float xv[4] = {x.x, x.y, x.z, x.w}, wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) acc[r][c] = fmaf(xv[c], wv[r], acc[r][c]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float4 o;
            o.x = sm_act<ACT>(acc[r][0] + bias[j0 + r], slope);
            o.y = sm_act<ACT>(acc[r][1] + bias[j0 + r], slope);
            o.z = sm_act<ACT>(acc[r][2] + bias[j0 + r], slope);
            o.w = sm_act<ACT>(acc[r][3] + bias[j0 + r], slope);
            *reinterpret_cast<float4 *>(outT + (j0 + r) * S + b0) = o;
        }
    }
}

// gW[j][i] = sum_b dT[j][b] inT[i][b] (j < JO rows and i < IV columns written, JP / HI padded to 4), gb[j] =
// sum_b dT[j][b]; b < BP (padding rows of dT are 0).  Written to global in torch's [out][in] layout ([JO][IV]);
// squares summed into sq (per thread, f64).
__device__ void sm_wgrad(const float *dT, int JO, int JP, const float *inT, int HI, int IV, int BP, int S, float *gW,
                         float *gb, double &sq) {
    const int tj = JP / 4, ti = HI / 4;
    for (int t = threadIdx.x; t < tj * ti; t += kSmThreads) {
        const int j0 = 4 * (t % tj), i0 = 4 * (t / tj);
        float acc[4][4], bs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[r][c] = 0.f;
#pragma unroll 2
        for (int b = 0; b < BP; b += 4) {
            float4 d[4], x[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) d[r] = *reinterpret_cast<const float4 *>(dT + (j0 + r) * S + b);
#pragma unroll
            for (int c = 0; c < 4; ++c) x[c] = *reinterpret_cast<const float4 *>(inT + (i0 + c) * S + b);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    float a = acc[r][c];
                    a = fmaf(d[r].x, x[c].x, a);
                    a = fmaf(d[r].y, x[c].y, a);
                    a = fmaf(d[r].z, x[c].z, a);
                    a = fmaf(d[r].w, x[c].w, a);
                    acc[r][c] = a;
                }
                if (i0 == 0) bs[r] += (d[r].x + d[r].y) + (d[r].z + d[r].w);
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (j0 + r >= JO) continue;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                if (i0 + c >= IV) continue;
                gW[(j0 + r) * IV + i0 + c] = acc[r][c];
                sq += (double)acc[r][c] * acc[r][c];
            }
            if (i0 == 0) {
                gb[j0 + r] = bs[r];
                sq += (double)bs[r] * bs[r];
            }
        }
    }
}

#define XPA_SM_STAMP(i_)                                                                  \
    do {                                                                                  \
        if (a.stamps && t == 0) a.stamps[i_] = (int64_t)__builtin_amdgcn_s_memtime();     \
    } while (0)

template <int ACT, int ALGO>
__global__ __launch_bounds__(kSmThreads, 1) void small_mlp_update_kernel(XpaSmallMlpArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[kSmLds];
    __shared__ double s_red[kSmWaves * 6];
    __shared__ float s_stat[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int B = a.batch, BP = (B + 3) & ~3, S = BP + 4;
    const int D = a.d_in, DP = (a.d_in + 3) & ~3, H0 = a.h0, H1 = a.h1, H2 = a.h2, K = a.k, KP = (a.k + 3) & ~3;
    // ---- LDS carve (offsets multiples of 4 floats) ----
    float *xT = lds;                       // [DP][S]
    float *h0T = xT + DP * S;              // [H0][S]  -> dh0
    float *h1T = h0T + H0 * S;             // [H1][S]  -> dh1
    float *h2T = h1T + H1 * S;             // [H2][S]  -> dh2
    float *dlT = h2T + H2 * S;             // [KP][S]  d logits (rows >= K zero)
    float *dvT = dlT + KP * S;             // [4][S]   d v in row 0, rows 1-3 zero
    float *W0T = dvT + 4 * S;              // [DP][H0]
    float *W1T = W0T + DP * H0;            // [H0][H1]
    float *W2T = W1T + H0 * H1;            // [H0][H2]
    float *WaT = W2T + H0 * H2;            // [H1][KP]
    float *WcT = WaT + H1 * KP;            // [H2][4]  (column 0)
    float *bias = WcT + H2 * 4;            // b0 | b1 | b2 | ba (KP) | bc (4)
    float *b0s = bias, *b1s = b0s + H0, *b2s = b1s + H1, *bas = b2s + H2, *bcs = bas + KP;
    float *rowf = bcs + 4;                 // act, old_logp, adv, ret: [4][BP]
    float *logit = rowf + 4 * BP;          // [BP][KP] (row-major, the loss reads its row)
    float *vrow = logit + BP * KP;         // [BP]
    XPA_SM_STAMP(0);
    // ---- stage the weights (transposed), biases, the minibatch rows through idx ----
    // coalesced reads of the row-major torch weights, 8 loads in flight per thread, scattered LDS writes (a
    // load-wait-store loop costs one global latency per element: ~30 us of this kernel at C1 before)
    auto stage_T = [&](const float *src, int rows, int cols, float *dst, int ldd, int col_limit) {
        // dst[c * ldd + r] = src[r * cols + c] for r < rows, c < cols (c >= col_limit: 0)
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
                if (e < n) {
                    const int r = e / cols, c = e - (e / cols) * cols;
                    dst[c * ldd + r] = c < col_limit ? v[u] : 0.f;
                }
            }
        }
    };
    stage_T(a.W0, H0, D, W0T, H0, D);               // W0 [H0][D] -> W0T [D][H0] (rows D .. DP zeroed below)
    for (int e = t; e < (DP - D) * H0; e += kSmThreads) W0T[D * H0 + e] = 0.f;
    stage_T(a.W1, H1, H0, W1T, H1, H0);             // W1 [H1][H0] -> W1T [H0][H1]
    stage_T(a.W2, H2, H0, W2T, H2, H0);             // W2 [H2][H0] -> W2T [H0][H2]
    for (int e = t; e < H1 * KP; e += kSmThreads) WaT[e] = 0.f;
    for (int e = t; e < H2 * 4; e += kSmThreads) WcT[e] = 0.f;
    __syncthreads();
    stage_T(a.Wa, K, H1, WaT, KP, H1);              // Wa [K][H1] -> WaT [H1][KP]
    stage_T(a.Wc, 1, H2, WcT, 4, H2);               // Wc [1][H2] -> WcT [H2][4] column 0
    for (int e = t; e < H0; e += kSmThreads) b0s[e] = a.b0[e];
    for (int e = t; e < H1; e += kSmThreads) b1s[e] = a.b1[e];
    for (int e = t; e < H2; e += kSmThreads) b2s[e] = a.b2[e];
    for (int e = t; e < KP; e += kSmThreads) bas[e] = e < K ? a.ba[e] : 0.f;
    if (t < 4) bcs[t] = t == 0 ? a.bc[0] : 0.f;
    double adv_s = 0.0, adv_q = 0.0;
    for (int b = t; b < BP; b += kSmThreads) {
        const bool ok = b < B;
        const int64_t row = ok ? a.idx[b] : 0;
        const bool valid = ok && row >= 0 && row < a.n_rows;
        const int64_t rc = valid ? row : 0;
        for (int i = 0; i < DP; ++i) xT[i * S + b] = valid && i < D ? a.obs[rc * a.obs_ld + i] : 0.f;
        const float av = valid ? a.adv[rc] : 0.f;
        rowf[0 * BP + b] = valid ? a.actions[rc] : 0.f;
        rowf[1 * BP + b] = valid && a.old_logp ? a.old_logp[rc] : 0.f;
        rowf[2 * BP + b] = av;
        rowf[3 * BP + b] = valid ? a.ret[rc] : 0.f;
        if (ok) {   // the minibatch advantage moments (K4's (sum, sumsq) in f64), over the batch rows
            adv_s += (double)av;
            adv_q += (double)av * av;
        }
    }
    // rows BP .. S of every [feature][S] array are never read; zero the padded dvT rows 1-3 and dlT rows >= K
    for (int e = t; e < 4 * S; e += kSmThreads) dvT[e] = 0.f;
    for (int e = t; e < KP * S; e += kSmThreads) dlT[e] = 0.f;
    {
        adv_s = xpa_wave_sum(adv_s);
        adv_q = xpa_wave_sum(adv_q);
        if (lane == 0) {
            s_red[w] = adv_s;
            s_red[kSmWaves + w] = adv_q;
        }
    }
    __syncthreads();
    if (t == 0) {
        double s = 0.0, q = 0.0;
        for (int i = 0; i < kSmWaves; ++i) {
            s += s_red[i];
            q += s_red[kSmWaves + i];
        }
        if (a.use_advnorm) {   // memory_tools.py:241-242, the arithmetic of loss.hip adv_moments
            const double mean = s / (double)B;
            const double var = fmax(q / (double)B - mean * mean, 0.0);
            s_stat[0] = (float)mean;
            s_stat[1] = (float)(1.0 / ((double)(float)sqrt(var) + 1e-8));
        } else {
            s_stat[0] = 0.f;
            s_stat[1] = 1.f;
        }
    }
    XPA_SM_STAMP(1);
    // ---- forward ----
    sm_fwd<ACT>(xT, DP, W0T, b0s, H0, h0T, BP, S, a.slope);
    __syncthreads();
    sm_fwd<ACT>(h0T, H0, W1T, b1s, H1, h1T, BP, S, a.slope);
    sm_fwd<ACT>(h0T, H0, W2T, b2s, H2, h2T, BP, S, a.slope);
    __syncthreads();
    XPA_SM_STAMP(2);
    // output layers: one thread per row (logits from h1, value from h2)
    for (int b = t; b < BP; b += kSmThreads) {
        float z[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) z[k] = 0.f;
        float vv = 0.f;
        for (int j = 0; j < H1; ++j) {
            const float h = h1T[j * S + b];
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (k < KP) z[k] = fmaf(h, WaT[j * KP + k], z[k]);
        }
        for (int j = 0; j < H2; ++j) vv = fmaf(h2T[j * S + b], WcT[j * 4], vv);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (k < KP) logit[b * KP + k] = z[k] + bas[k];
        vrow[b] = vv + bcs[0];
    }
    __syncthreads();
    XPA_SM_STAMP(3);
    // ---- loss, one thread per row (K2's categorical arithmetic) ----
    const float inv_b = 1.0f / (float)B;
    float surr = 0.f, sqe = 0.f, ent = 0.f, clipc = 0.f, vsum = 0.f;
    const float mean_a = s_stat[0], inv_a = s_stat[1];
    for (int b = t; b < B; b += kSmThreads) {
        const int64_t row = a.idx[b];
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
    if (t == 0) {
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
    sm_wgrad(dlT, K, KP, h1T, H1, H1, BP, S, a.gWa, a.gba, sq);   // output layers (they still read h1 / h2)
    sm_wgrad(dvT, 1, 4, h2T, H2, H2, BP, S, a.gWc, a.gbc, sq);
    __syncthreads();
    XPA_SM_STAMP(5);
    // dh1 = (dlogits Wa) act'(h1), dh2 = dv wc act'(h2): in place over h1 / h2
    for (int e = t; e < H1 * BP; e += kSmThreads) {
        const int j = e / BP, b = e % BP;
        float g = 0.f;
        for (int k = 0; k < K; ++k) g = fmaf(dlT[k * S + b], WaT[j * KP + k], g);
        float *p = h1T + j * S + b;
        *p = g * sm_grad<ACT>(*p, a.slope);
    }
    for (int e = t; e < H2 * BP; e += kSmThreads) {
        const int j = e / BP, b = e % BP;
        float *p = h2T + j * S + b;
        *p = dvT[b] * WcT[j * 4] * sm_grad<ACT>(*p, a.slope);
    }
    __syncthreads();
    XPA_SM_STAMP(6);
    sm_wgrad(h1T, H1, H1, h0T, H0, H0, BP, S, a.gW1, a.gb1, sq);   // hidden layers (read h0)
    sm_wgrad(h2T, H2, H2, h0T, H0, H0, BP, S, a.gW2, a.gb2, sq);
    // the hidden weights row-major ([j][i], over the transposed forward copies) for dh0's 16-B weight reads
    auto copy8 = [&](const float *src, float *dst, int n) {
        for (int e0 = t; e0 < n; e0 += 8 * kSmThreads) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = e0 + u * kSmThreads < n ? src[e0 + u * kSmThreads] : 0.f;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (e0 + u * kSmThreads < n) dst[e0 + u * kSmThreads] = v[u];
        }
    };
    copy8(a.W1, W1T, H1 * H0);
    copy8(a.W2, W2T, H2 * H0);
    __syncthreads();
    XPA_SM_STAMP(7);
    // dh0 = (dh1 W1 + dh2 W2) act'(h0), in place over h0: thread tile 4 features x 4 rows
    {
        const int ti = H0 / 4, tb = BP / 4;
        for (int q = t; q < ti * tb; q += kSmThreads) {
            const int i0 = 4 * (q % ti), b0 = 4 * (q / ti);
            float acc[4][4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) acc[r][c] = 0.f;
            for (int j = 0; j < H1; ++j) {
                const float4 d = *reinterpret_cast<const float4 *>(h1T + j * S + b0);
                const float4 wq = *reinterpret_cast<const float4 *>(W1T + j * H0 + i0);   // W1[j][i0 .. i0 + 3]
                const float dv[4] = {d.x, d.y, d.z, d.w}, wr[4] = {wq.x, wq.y, wq.z, wq.w};
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc[r][c] = fmaf(dv[c], wr[r], acc[r][c]);
            }
            for (int j = 0; j < H2; ++j) {
                const float4 d = *reinterpret_cast<const float4 *>(h2T + j * S + b0);
                const float4 wq = *reinterpret_cast<const float4 *>(W2T + j * H0 + i0);   // W2[j][i0 .. i0 + 3]
                const float dv[4] = {d.x, d.y, d.z, d.w}, wr[4] = {wq.x, wq.y, wq.z, wq.w};
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc[r][c] = fmaf(dv[c], wr[r], acc[r][c]);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float4 *p = reinterpret_cast<float4 *>(h0T + (i0 + r) * S + b0);
                float4 y = *p;
                y.x = acc[r][0] * sm_grad<ACT>(y.x, a.slope);
                y.y = acc[r][1] * sm_grad<ACT>(y.y, a.slope);
                y.z = acc[r][2] * sm_grad<ACT>(y.z, a.slope);
                y.w = acc[r][3] * sm_grad<ACT>(y.w, a.slope);
                // padding rows b >= B: their dh1 / dh2 are 0 (dlT / dvT are 0 there), so dh0 is 0 too
                *p = y;
            }
        }
    }
    __syncthreads();
    XPA_SM_STAMP(8);
    sm_wgrad(h0T, H0, H0, xT, DP, D, BP, S, a.gW0, a.gb0, sq);   // first layer ([H0][D]: padding columns dropped)
    XPA_SM_STAMP(9);
    // ---- clip_grad_norm_ + Adam over the flat buffers (K9's arithmetic, schedule at the device cursor) ----
    sq = xpa_wave_sum(sq);
    if (lane == 0) s_red[w] = sq;
    __syncthreads();   // also orders every gradient store of the block before the flat-buffer reads below
    __shared__ float s_coef, s_step, s_inv;
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

}  // namespace

XPA_API int64_t xpa_small_mlp_lds_floats(int64_t batch, int64_t d_in, int64_t h0, int64_t h1, int64_t h2, int64_t k) {
    const int64_t BP = (batch + 3) & ~3, S = BP + 4, DP = (d_in + 3) & ~3, KP = (k + 3) & ~3;
    return DP * S + (h0 + h1 + h2) * S + KP * S + 4 * S + DP * h0 + h0 * h1 + h0 * h2 + h1 * KP + h2 * 4 + h0 + h1 +
           h2 + KP + 4 + 4 * BP + BP * KP + BP;
}

XPA_API int xpa_small_mlp_update(const XpaSmallMlpArgs *args, xpa_stream_t stream) {
    if (!args) return (int)hipErrorInvalidValue;
    const XpaSmallMlpArgs &a = *args;
    if (a.batch < 1 || a.d_in < 1 || a.h0 < 4 || a.h1 < 4 || a.h2 < 4 || a.h0 % 4 || a.h1 % 4 || a.h2 % 4 ||
        a.h0 > 256 || a.h1 > 256 || a.h2 > 256 || a.k < 2 || a.k > 16 || a.act_code < 0 || a.act_code > 2 ||
        (a.algo != XPA_ALGO_PPO && a.algo != XPA_ALGO_A2C) || (a.algo == XPA_ALGO_PPO && !a.old_logp) || !a.obs ||
        !a.idx || !a.actions || !a.adv || !a.ret || !a.param || !a.grad || !a.exp_avg || !a.exp_avg_sq || !a.sched ||
        !a.cursor || a.n_sched < 1 || !a.scalars || a.n < 1 || !a.W0 || !a.b0 || !a.W1 || !a.b1 || !a.W2 || !a.b2 ||
        !a.Wa || !a.ba || !a.Wc || !a.bc || !a.gW0 || !a.gb0 || !a.gW1 || !a.gb1 || !a.gW2 || !a.gb2 || !a.gWa ||
        !a.gba || !a.gWc || !a.gbc || a.n % 4 ||
        ((uintptr_t)a.param | (uintptr_t)a.grad | (uintptr_t)a.exp_avg | (uintptr_t)a.exp_avg_sq) % 16)
        return (int)hipErrorInvalidValue;
    if (xpa_small_mlp_lds_floats(a.batch, a.d_in, a.h0, a.h1, a.h2, a.k) > kSmLds) return (int)hipErrorInvalidValue;
    hipStream_t s = (hipStream_t)stream;
#define XPA_SM(A_, G_) hipLaunchKernelGGL((small_mlp_update_kernel<A_, G_>), dim3(1), dim3(kSmThreads), 0, s, a)
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
    return xpa_launch_status();
}
