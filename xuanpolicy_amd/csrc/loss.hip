// K2 — fused PPO-Clip / A2C policy + value + entropy loss, forward and backward, one minibatch (gfx950).
//
// Replaces (reference paths):
//   PPOCLIP_Learner.update loss     xuance/torch/learners/policy_gradient/ppoclip_learner.py:32-44
//   A2C_Learner.update loss         xuance/torch/learners/policy_gradient/a2c_learner.py:24-31
//   DiagGaussian/Categorical        xuance/torch/utils/distributions.py:39-101 (torch Normal / Categorical)
//   per-minibatch adv-norm          xuance/common/memory_tools.py:241-242
// One thread per sample: reads the policy head row (mu or logits), its value, and — through the
// minibatch permutation idx — act/old_logp/adv/ret straight from the [n_envs, horizon] buffer (no
// gathered copies), writes d loss/d head and d loss/d v, and one row of block partial sums
// (surrogate, squared error, entropy, clip count, value, d loss/d logstd[A]).  The partials are
// reduced in a fixed order by xpa_policy_loss_finalize (no float atomics -> bit-reproducible).
// Closed-form gradients follow torch autograd's tie rules: clamp passes the
// gradient on [1-eps, 1+eps] inclusive; minimum() splits an exact tie half/half.
// HBM-bound elementwise work: Gaussian 4(3A+5) B/sample, Categorical 4(2K+6) B/sample.
#include "xpa_common.h"
#include "loss_finalize.h"

namespace {

constexpr int kLossThreads = 256;
constexpr int kLossWaves = kLossThreads / 64;
constexpr int kPartBase = 5;  // surrogate, sq-err, entropy, clip count, value
constexpr int kMaxAct = 64;
constexpr float kLogSqrt2Pi = 0.91893853320467274178f;  // log(sqrt(2*pi))
constexpr float kHalfLog2PiPlusHalf = 1.41893853320467274178f;  // 0.5 + 0.5*log(2*pi)

__device__ __forceinline__ void adv_moments(const double *partials, int64_t n_partials, int64_t batch,
                                            float *s_mean, float *s_inv) {
    // Wave 0 reduces the gather kernel's (sum, sumsq) rows in a fixed order.
    if (threadIdx.x < 64) {
        double s = 0.0, q = 0.0;
        int64_t k = threadIdx.x;
        for (; k + 7 * 64 < n_partials; k += 8 * 64) {  // 8 x 16-B loads in flight, added in k order
            double2 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const double2 *>(partials + 2 * (k + 64 * u));
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s += v[u].x;
                q += v[u].y;
            }
        }
        for (; k < n_partials; k += 64) {
            s += partials[2 * k];
            q += partials[2 * k + 1];
        }
        s = xpa_wave_sum(s);
        q = xpa_wave_sum(q);
        if (threadIdx.x == 0) {
            const double mean = s / (double)batch;
            const double var = fmax(q / (double)batch - mean * mean, 0.0);
            *s_mean = (float)mean;
            *s_inv = (float)(1.0 / ((double)(float)sqrt(var) + 1e-8));
        }
    }
}

// Grid-stride form: at most kLossMaxBlocks blocks (8 per CU), each thread walks rows b, b + grid * 256, ...
// accumulating its loss terms (and, Gaussian, its d logstd terms: KM registers, KM >= A) before ONE block
// reduction — the per-block prologue (exp/log of logstd, the adv moments) and the reduction are paid once
// per ~B / 2048 rows instead of once per 256.  Per-row arithmetic (d_head, d_v) is unchanged.
constexpr int64_t kLossMaxBlocks = 2048;

template <int DIST, int ALGO, int KM>
__global__ __launch_bounds__(kLossThreads) void policy_loss_kernel(
    int64_t batch, int A, const float *__restrict__ head, const float *__restrict__ logstd,
    const float *__restrict__ v, const int64_t *__restrict__ idx, int64_t n_rows, const float *__restrict__ act,
    const float *__restrict__ old_logp, const float *__restrict__ adv, const float *__restrict__ ret,
    const double *__restrict__ adv_partials, int64_t n_adv_partials, float clip_range, float vf_coef,
    float ent_coef, float *__restrict__ d_head, float *__restrict__ d_v, float *__restrict__ partials, int width) {
    __shared__ float s_scale[kMaxAct], s_logscale[kMaxAct], s_var[kMaxAct];
    __shared__ float s_ent;
    __shared__ float s_mean, s_inv;
    __shared__ float s_red[(kPartBase + kMaxAct) * kLossWaves];

    const int tid = threadIdx.x;
    if (DIST == XPA_DIST_GAUSSIAN) {
        for (int a = tid; a < A; a += kLossThreads) {
            const float sc = expf(logstd[a]);   // std = logstd.exp() (gaussian.py:29)
            s_scale[a] = sc;
            s_logscale[a] = logf(sc);           // Normal.log_prob uses scale.log()
            s_var[a] = sc * sc;
        }
    }
    if (adv_partials) {
        adv_moments(adv_partials, n_adv_partials, batch, &s_mean, &s_inv);
    } else if (tid == 0) {
        s_mean = 0.f;
        s_inv = 1.f;
    }
    __syncthreads();
    if (DIST == XPA_DIST_GAUSSIAN && tid == 0) {
        float e = 0.f;
        for (int a = 0; a < A; ++a) e += kHalfLog2PiPlusHalf + s_logscale[a];
        s_ent = e;
    }
    __syncthreads();
    const float inv_b = 1.0f / (float)batch;
    const float mean_a = s_mean, inv_a = s_inv;
    // var / log scale are read from LDS where used (wave-uniform broadcast reads): held in registers they
    // cost 2 KM VGPRs and the occupancy that goes with them
    const float *var_r = s_var, *logsc_r = s_logscale;
    const float ent_g = DIST == XPA_DIST_GAUSSIAN ? s_ent : 0.f;

    float surr_t = 0.f, sq_t = 0.f, ent_t = 0.f, clip_t = 0.f, vv_t = 0.f;
    float dls_t[KM];
#pragma unroll
    for (int a = 0; a < KM; ++a) dls_t[a] = 0.f;

    // Gaussian, KM <= 20: the tile's head rows (and act rows when they are read in order) are staged through
    // LDS with 16-B loads and d_head leaves through LDS with 16-B stores — the rows are A floats (24 B at
    // A = 6), so per-thread row accesses would be 4-B loads strided by the row (a TA-bound pattern).
    // d_head is written in place over the tile's head rows (each thread reads its own mu row before it
    // writes its d mu row at the same LDS address): two row images per block, 16 KiB at KM = 8.
    constexpr bool kStage = DIST == XPA_DIST_GAUSSIAN && KM <= 20;
    constexpr int kQ = kStage ? (KM * kLossThreads / 4 + kLossThreads - 1) / kLossThreads : 1;  // float4 / thread
    __shared__ __attribute__((aligned(16))) float s_rows[kStage ? 2 * kLossThreads * KM : 4];
    const bool stage = kStage && (((uintptr_t)head | (uintptr_t)d_head) % 16 == 0) && (A % 4 == 0 || true);
    const bool stage_act = stage && idx == nullptr && ((uintptr_t)act % 16 == 0);
    const int64_t ntiles = (batch + kLossThreads - 1) / kLossThreads;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t b = tile * kLossThreads + tid;
        const int64_t t0 = tile * kLossThreads;
        const int nt = (int)(batch - t0 < kLossThreads ? batch - t0 : kLossThreads);  // rows in this tile
        float *s_mu = s_rows, *s_x = s_rows + kLossThreads * KM, *s_dm = s_rows;
        // this row's scalars are requested before the tile staging (one HBM round trip for both).  Every load
        // of the tile is unconditional, from a clamped (always valid) address, and selected afterwards: a load
        // under a lane-divergent branch made hipcc wait for it (vmcnt(0)) at the branch's join.
        const int64_t bc = b < batch ? b : batch - 1;
        const int64_t row = b < batch ? (idx ? idx[bc] : bc) : -1;
        const bool valid = row >= 0 && row < n_rows;
        const int64_t rc = valid ? row : 0;
        float p_adv = adv[rc], p_v = v[bc], p_ret = ret[rc], p_old = ALGO == XPA_ALGO_PPO ? old_logp[rc] : 0.f;
        if (stage) {
            const int n = nt * A;  // floats of the tile's rows (contiguous in head / act)
            const float *gm = head + t0 * A, *gx = act + t0 * A;
            const int n4 = (t0 * A) % 4 == 0 ? n / 4 : 0;  // 16-B aligned tile start: vector part
            // every 16-B load of the tile is issued before the first LDS write (one round trip per tile)
            float4 hq[kQ], xq[kQ];
            if (n4 > 0) {  // block-uniform
                const float4 *gm4 = reinterpret_cast<const float4 *>(gm);
                const float4 *gx4 = reinterpret_cast<const float4 *>(stage_act ? gx : gm);
#pragma unroll
                for (int j = 0; j < kQ; ++j) {
                    const int i = tid + j * kLossThreads;
                    const int ic = i < n4 ? i : n4 - 1;
                    hq[j] = gm4[ic];
                    xq[j] = gx4[ic];
                }
            }
            __syncthreads();  // the previous tile's d_head is out of LDS
#pragma unroll
            for (int j = 0; j < kQ; ++j) {
                const int i = tid + j * kLossThreads;
                if (i < n4) {
                    reinterpret_cast<float4 *>(s_mu)[i] = hq[j];
                    if (stage_act) reinterpret_cast<float4 *>(s_x)[i] = xq[j];
                }
            }
            for (int i = 4 * n4 + tid; i < n; i += kLossThreads) {
                s_mu[i] = gm[i];
                if (stage_act) s_x[i] = gx[i];
            }
            __syncthreads();
        }
        if (b >= batch) {
            if (stage) goto store_tile;
            continue;
        }
        {
        if (!valid) {  // out-of-range index: zero gradient, no contribution
            d_v[b] = 0.f;
            // the finalize subtracts ent_coef (= ent_coef / B per row) from d logstd for every row of the
            // batch: a masked row hands its share back, so it contributes nothing there either
            if (DIST == XPA_DIST_GAUSSIAN)
                for (int a = 0; a < KM; ++a)
                    if (a < A) dls_t[a] += ent_coef * inv_b;
            if (stage)
                for (int a = 0; a < A; ++a) s_dm[tid * A + a] = 0.f;
            else
                for (int a = 0; a < A; ++a) d_head[b * A + a] = 0.f;
            if (stage) goto store_tile;
            continue;
        }
        const float A_n = (p_adv - mean_a) * inv_a;
        const float vb = p_v;
        const float diffv = vb - p_ret;
        sq_t += diffv * diffv;
        vv_t += vb;
        d_v[b] = vf_coef * 2.0f * diffv * inv_b;
        float logp = 0.f, lse = 0.f, H = 0.f;
        int ai = 0;
        float diff_r[KM];
        if (DIST == XPA_DIST_GAUSSIAN) {
            const float *mu = stage ? s_mu + tid * A : head + b * A;
            const float *x = stage_act ? s_x + tid * A : act + row * A;
#pragma unroll
            for (int a = 0; a < KM; ++a) {
                diff_r[a] = 0.f;
                if (a < A) {
                    diff_r[a] = x[a] - mu[a];
                    logp += -(diff_r[a] * diff_r[a]) / (2.0f * var_r[a]) - logsc_r[a] - kLogSqrt2Pi;
                }
            }
            ent_t += ent_g;
        } else {
            const float *z = head + b * A;
            float m = z[0];
            for (int k = 1; k < A; ++k) m = fmaxf(m, z[k]);
            float se = 0.f;
            for (int k = 0; k < A; ++k) se += expf(z[k] - m);
            lse = m + logf(se);
            ai = (int)act[row];
            // Deliberate divergence: torch's Categorical.log_prob raises on an action outside [0, A); the kernel
            // clamps it (a bounded read instead of a fault). The device rollout only writes in-range actions, and
            // the drop-in learner validates host-supplied categorical actions before the launch (learners.py).
            ai = ai < 0 ? 0 : (ai >= A ? A - 1 : ai);
            logp = z[ai] - lse;
            for (int k = 0; k < A; ++k) {
                const float ln = z[k] - lse;
                H -= expf(ln) * ln;
            }
            ent_t += H;
        }
        float dlogp;
        if (ALGO == XPA_ALGO_PPO) {
            const float ratio = expf(logp - p_old);
            const float lo = 1.0f - clip_range, hi = 1.0f + clip_range;
            const float cr = fminf(fmaxf(ratio, lo), hi);
            const float s1 = cr * A_n;
            const float s2 = A_n * ratio;
            surr_t += fminf(s1, s2);
            const bool inr = (ratio >= lo) && (ratio <= hi);
            const float g1 = inr ? A_n : 0.f;
            const float w1 = (s1 < s2) ? 1.f : ((s1 == s2) ? 0.5f : 0.f);
            const float w2 = (s2 < s1) ? 1.f : ((s1 == s2) ? 0.5f : 0.f);
            dlogp = -inv_b * (w1 * g1 + w2 * A_n) * ratio;
            clip_t += ((ratio < lo) || (ratio > hi)) ? 1.f : 0.f;
        } else {
            surr_t += A_n * logp;
            dlogp = -A_n * inv_b;
        }
        if (DIST == XPA_DIST_GAUSSIAN) {
            float *dm = stage ? s_dm + tid * A : d_head + b * A;
#pragma unroll
            for (int a = 0; a < KM; ++a) {
                if (a < A) {
                    dm[a] = dlogp * diff_r[a] / var_r[a];
                    dls_t[a] += dlogp * (diff_r[a] * diff_r[a] / var_r[a] - 1.0f);
                }
            }
        } else {
            const float *z = head + b * A;
            float *dz = d_head + b * A;
            const float ec = ent_coef * inv_b;
            for (int k = 0; k < A; ++k) {
                const float ln = z[k] - lse;
                const float p = expf(ln);
                const float oh = (k == ai) ? 1.f : 0.f;
                dz[k] = dlogp * (oh - p) + ec * p * (ln + H);
            }
        }
        }
    store_tile:
        if (stage) {  // the tile's d_head rows: LDS -> HBM with 16-B stores
            __syncthreads();
            const int n = nt * A;
            float *gd = d_head + t0 * A;
            const int n4 = (t0 * A) % 4 == 0 ? n / 4 : 0;
            for (int i = tid; i < n4; i += kLossThreads)
                reinterpret_cast<float4 *>(gd)[i] = reinterpret_cast<const float4 *>(s_dm)[i];
            for (int i = 4 * n4 + tid; i < n; i += kLossThreads) gd[i] = s_dm[i];
        }
    }
    // Block partial sums: every value is wave-reduced by shuffles into its own LDS slot row, then ONE
    // barrier and a fixed-order sum over the waves (deterministic, no per-value barriers).
    const int w = tid >> 6;
    const bool lane0 = (tid & 63) == 0;
    {
        const float r0 = xpa_wave_sum(surr_t), r1 = xpa_wave_sum(sq_t), r2 = xpa_wave_sum(ent_t);
        const float r3 = xpa_wave_sum(clip_t), r4 = xpa_wave_sum(vv_t);
        if (lane0) {
            s_red[0 * kLossWaves + w] = r0;
            s_red[1 * kLossWaves + w] = r1;
            s_red[2 * kLossWaves + w] = r2;
            s_red[3 * kLossWaves + w] = r3;
            s_red[4 * kLossWaves + w] = r4;
        }
    }
    if (DIST == XPA_DIST_GAUSSIAN) {
#pragma unroll
        for (int a = 0; a < KM; ++a) {
            if (a < A) {
                const float g = xpa_wave_sum(dls_t[a]);
                if (lane0) s_red[(kPartBase + a) * kLossWaves + w] = g;
            }
        }
    }
    __syncthreads();
    const int nvals = kPartBase + (DIST == XPA_DIST_GAUSSIAN ? A : 0);
    float *prow = partials + (int64_t)blockIdx.x * width;
    for (int j = tid; j < nvals; j += kLossThreads) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < kLossWaves; ++k) s += s_red[j * kLossWaves + k];
        prow[j] = s;
    }
}

typedef __attribute__((address_space(3))) char lds_char_t;

// One global_load_lds_dwordx4: lane l's 16 B land at LDS byte lds_wave_base + 16 l (M0 = the wave's base).
// Inline asm: the builtin form makes hipcc insert vmcnt(0) before LDS reads it cannot prove disjoint.
__device__ __forceinline__ void lds_dma16(const float *g, unsigned lds_wave_base) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(lds_wave_base)
                 : "memory", "m0");
}

// Streaming form of K2 for Gaussian heads (A <= KM <= 20, 16-B aligned head / d_head; the drop-in learners'
// case and the flushed sweep): the tile body is straight-line — every load unconditional from a clamped
// address, validity applied by selects, stores the only predicated work — so the only memory waits are the
// one per tile before the LDS staging writes.  (In the generic kernel, loads under lane-divergent branches
// made hipcc put vmcnt(0) at the joins, which on gfx9 also waits for every store still in flight: two to
// three serialised HBM round trips per tile.)  Same arithmetic, same partial layout as policy_loss_kernel.
// IDX: rows come through the minibatch permutation (act rows gathered per thread) or in order (act staged).
template <int ALGO, int KM, bool IDX>
__global__ __launch_bounds__(kLossThreads, 8) void policy_loss_gauss_kernel(
    int64_t batch, int A, const float *__restrict__ head, const float *__restrict__ logstd,
    const float *__restrict__ v, const int64_t *__restrict__ idx, int64_t n_rows, const float *__restrict__ act,
    const float *__restrict__ old_logp, const float *__restrict__ adv, const float *__restrict__ ret,
    const double *__restrict__ adv_partials, int64_t n_adv_partials, float clip_range, float vf_coef,
    float ent_coef, float *__restrict__ d_head, float *__restrict__ d_v, float *__restrict__ partials, int width) {
    static_assert(KM % 4 == 0, "the row images are whole float4 per thread");
    constexpr int kQ = KM / 4;  // float4 per thread per image
    __shared__ float s_var[KM], s_logscale[KM];
    __shared__ float s_ent, s_mean, s_inv;
    __shared__ float s_red[(kPartBase + KM) * kLossWaves];
    // ONE LDS array for the DMA targets (a second __shared__ object beside a DMA target can make hipcc wait
    // vmcnt(0) before LDS reads it cannot prove disjoint): head rows (then d_head in place), act rows
    __shared__ __attribute__((aligned(16))) float s_img[(IDX ? 1 : 2) * kLossThreads * KM];
    float *s_mu = s_img, *s_x = s_img + kLossThreads * KM;
    const unsigned lds_mu = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_char_t *)s_img);
    const unsigned lds_x = lds_mu + (unsigned)(kLossThreads * KM * 4);
    const int tid = threadIdx.x;
    for (int a = tid; a < A; a += kLossThreads) {
        const float sc = expf(logstd[a]);  // std = logstd.exp() (gaussian.py:29)
        s_logscale[a] = logf(sc);          // Normal.log_prob uses scale.log()
        s_var[a] = sc * sc;
    }
    if (adv_partials) {
        adv_moments(adv_partials, n_adv_partials, batch, &s_mean, &s_inv);
    } else if (tid == 0) {
        s_mean = 0.f;
        s_inv = 1.f;
    }
    __syncthreads();
    if (tid == 0) {
        float e = 0.f;
        for (int a = 0; a < A; ++a) e += kHalfLog2PiPlusHalf + s_logscale[a];
        s_ent = e;
    }
    __syncthreads();
    const float inv_b = 1.0f / (float)batch;
    const float mean_a = s_mean, inv_a = s_inv, ent_g = s_ent;
    const float lo = 1.0f - clip_range, hi = 1.0f + clip_range;
    float surr_t = 0.f, sq_t = 0.f, ent_t = 0.f, clip_t = 0.f, vv_t = 0.f;
    float dls_t[KM];
#pragma unroll
    for (int a = 0; a < KM; ++a) dls_t[a] = 0.f;
    const int64_t ntiles = (batch + kLossThreads - 1) / kLossThreads;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        __syncthreads();  // the previous tile's d_head is out of LDS
        const int64_t t0 = tile * kLossThreads, b = t0 + tid;
        const int nt = (int)(batch - t0 < kLossThreads ? batch - t0 : kLossThreads);  // rows in this tile
        const bool inb = tid < nt;
        const int64_t bc = inb ? b : batch - 1;
        const int64_t row = IDX ? idx[bc] : bc;
        const bool valid = inb && row >= 0 && row < n_rows;
        const int64_t rc = valid ? row : 0;
        const float p_adv = adv[rc], p_v = v[bc], p_ret = ret[rc];
        const float p_old = ALGO == XPA_ALGO_PPO ? old_logp[rc] : 0.f;
        const int n = nt * A;                      // floats of the tile's rows (t0 * A is a multiple of 4)
        const int n4 = n / 4;
        // The row images go global -> LDS by DMA (global_load_lds_dwordx4: no VGPR staging, nothing for the
        // compiler to serialise); float4 i = tid + 256 j lands at byte 16 i of its image, i.e. wave w's
        // instruction j fills the KiB (4 j + w) lane-linearly.  Slots past the tile's rows take clamped copies
        // (unread); a tile shorter than one float4 (the last, at most) reads tile 0's first floats instead.
        const int64_t q0 = n4 > 0 ? t0 * A : 0;
        const float *gm = head + q0, *gx = IDX ? head + q0 : act + q0;
        const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
#pragma unroll
        for (int j = 0; j < kQ; ++j) {
            const int i = tid + j * kLossThreads;
            const int ic = i < n4 ? i : (n4 > 0 ? n4 - 1 : 0);
            const unsigned slot = (unsigned)((4 * j + wv) * 1024);
            lds_dma16(gm + 4 * ic, lds_mu + slot);
            if (!IDX) lds_dma16(gx + 4 * ic, lds_x + slot);
        }
        float xr[KM];
        if (IDX) {  // act row of this sample through the permutation
#pragma unroll
            for (int a = 0; a < KM; ++a) xr[a] = a < A ? act[rc * A + a] : 0.f;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMAs (and this row's scalars) have landed
        for (int i = 4 * n4 + tid; i < n; i += kLossThreads) {  // the last tile's ragged end
            s_mu[i] = head[t0 * A + i];
            if (!IDX) s_x[i] = act[t0 * A + i];
        }
        __syncthreads();
        const float A_n = (p_adv - mean_a) * inv_a;
        const float diffv = p_v - p_ret;
        float logp = 0.f, diff_r[KM];
#pragma unroll
        for (int a = 0; a < KM; ++a) {
            diff_r[a] = 0.f;
            if (a < A) {
                const float x = IDX ? xr[a] : s_x[tid * A + a];
                diff_r[a] = x - s_mu[tid * A + a];
                logp += -(diff_r[a] * diff_r[a]) / (2.0f * s_var[a]) - s_logscale[a] - kLogSqrt2Pi;
            }
        }
        float dlogp, surr, clipped = 0.f;
        if (ALGO == XPA_ALGO_PPO) {
            const float ratio = expf(logp - p_old);
            const float cr = fminf(fmaxf(ratio, lo), hi);
            const float s1 = cr * A_n;
            const float s2 = A_n * ratio;
            surr = fminf(s1, s2);
            const bool inr = (ratio >= lo) && (ratio <= hi);
            const float g1 = inr ? A_n : 0.f;
            const float w1 = (s1 < s2) ? 1.f : ((s1 == s2) ? 0.5f : 0.f);
            const float w2 = (s2 < s1) ? 1.f : ((s1 == s2) ? 0.5f : 0.f);
            dlogp = -inv_b * (w1 * g1 + w2 * A_n) * ratio;
            clipped = ((ratio < lo) || (ratio > hi)) ? 1.f : 0.f;
        } else {
            surr = A_n * logp;
            dlogp = -A_n * inv_b;
        }
        surr_t += valid ? surr : 0.f;
        clip_t += valid ? clipped : 0.f;
        sq_t += valid ? diffv * diffv : 0.f;
        vv_t += valid ? p_v : 0.f;
        ent_t += valid ? ent_g : 0.f;
        // a masked row (invalid index) hands back the ent_coef / B the finalize subtracts for every row
        const float dls_masked = inb ? ent_coef * inv_b : 0.f;
#pragma unroll
        for (int a = 0; a < KM; ++a) {
            if (a < A) {
                const float dm = dlogp * diff_r[a] / s_var[a];
                dls_t[a] += valid ? dlogp * (diff_r[a] * diff_r[a] / s_var[a] - 1.0f) : dls_masked;
                if (inb) s_mu[tid * A + a] = valid ? dm : 0.f;
            }
        }
        if (inb) d_v[b] = valid ? vf_coef * 2.0f * diffv * inv_b : 0.f;
        __syncthreads();  // the tile's d_head rows: LDS -> HBM with 16-B stores
        float4 *gd4 = reinterpret_cast<float4 *>(d_head + t0 * A);
#pragma unroll
        for (int j = 0; j < kQ; ++j) {
            const int i = tid + j * kLossThreads;
            if (i < n4) gd4[i] = reinterpret_cast<const float4 *>(s_mu)[i];
        }
        for (int i = 4 * n4 + tid; i < n; i += kLossThreads) d_head[t0 * A + i] = s_mu[i];
    }
    const int w = tid >> 6;
    const bool lane0 = (tid & 63) == 0;
    {
        const float r0 = xpa_wave_sum(surr_t), r1 = xpa_wave_sum(sq_t), r2 = xpa_wave_sum(ent_t);
        const float r3 = xpa_wave_sum(clip_t), r4 = xpa_wave_sum(vv_t);
        if (lane0) {
            s_red[0 * kLossWaves + w] = r0;
            s_red[1 * kLossWaves + w] = r1;
            s_red[2 * kLossWaves + w] = r2;
            s_red[3 * kLossWaves + w] = r3;
            s_red[4 * kLossWaves + w] = r4;
        }
    }
#pragma unroll
    for (int a = 0; a < KM; ++a) {
        if (a < A) {
            const float g = xpa_wave_sum(dls_t[a]);
            if (lane0) s_red[(kPartBase + a) * kLossWaves + w] = g;
        }
    }
    __syncthreads();
    const int nvals = kPartBase + A;
    float *prow = partials + (int64_t)blockIdx.x * width;
    for (int j = tid; j < nvals; j += kLossThreads) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < kLossWaves; ++k) s += s_red[j * kLossWaves + k];
        prow[j] = s;
    }
}

__global__ __launch_bounds__(256) void policy_loss_finalize_kernel(XpaLossFinalizeArgs args, double *sq_out) {
    __shared__ double tot[kPartBase];
    __shared__ float s_dls[kMaxAct];
    xpa_loss_finalize_body(args, sq_out, tot, s_dls);
}

}  // namespace

XPA_API int64_t xpa_loss_num_partials(int64_t batch) {
    const int64_t blocks = (batch + kLossThreads - 1) / kLossThreads;
    return blocks < kLossMaxBlocks ? blocks : kLossMaxBlocks;
}

XPA_API int64_t xpa_loss_partial_width(int64_t act_dim) { return kPartBase + act_dim; }

XPA_API int xpa_policy_loss_fwd_bwd(int algo, int dist, int64_t batch, int64_t act_dim, const float *head,
                                    const float *logstd, const float *v, const int64_t *idx, int64_t n_rows,
                                    const float *act,
                                    const float *old_logp, const float *adv, const float *ret,
                                    const double *adv_partials, int64_t n_adv_partials, float clip_range,
                                    float vf_coef, float ent_coef, float *d_head, float *d_v, float *partials,
                                    xpa_stream_t stream) {
    if (batch <= 0 || act_dim <= 0 || act_dim > kMaxAct) return (int)hipErrorInvalidValue;
    if (algo != XPA_ALGO_PPO && algo != XPA_ALGO_A2C) return (int)hipErrorInvalidValue;
    if (dist != XPA_DIST_GAUSSIAN && dist != XPA_DIST_CATEGORICAL) return (int)hipErrorInvalidValue;
    if (dist == XPA_DIST_CATEGORICAL && act_dim < 2) return (int)hipErrorInvalidValue;
    if (!head || !v || !act || !adv || !ret || !d_head || !d_v || !partials) return (int)hipErrorInvalidValue;
    if (n_rows <= 0 || (!idx && n_rows < batch)) return (int)hipErrorInvalidValue;
    if (dist == XPA_DIST_GAUSSIAN && !logstd) return (int)hipErrorInvalidValue;
    if (algo == XPA_ALGO_PPO && !old_logp) return (int)hipErrorInvalidValue;
    const int64_t blocks = xpa_loss_num_partials(batch);
    if (blocks > 0x7fffffffLL) return (int)hipErrorInvalidValue;
    const int width = (int)xpa_loss_partial_width(act_dim);
    const int A = (int)act_dim;
    hipStream_t s = (hipStream_t)stream;
#define XPA_LOSS_LAUNCH(D_, A_, KM_)                                                                              \
    hipLaunchKernelGGL((policy_loss_kernel<D_, A_, KM_>), dim3((unsigned)blocks), dim3(kLossThreads), 0, s, batch,  \
                       A, head, logstd, v, idx, n_rows, act, old_logp, adv, ret, adv_partials, n_adv_partials,       \
                       clip_range, vf_coef, ent_coef, d_head, d_v, partials, width)
#define XPA_LOSS_GAUSS(A_)                                                \
    if (A <= 8) XPA_LOSS_LAUNCH(XPA_DIST_GAUSSIAN, A_, 8);                \
    else if (A <= 20) XPA_LOSS_LAUNCH(XPA_DIST_GAUSSIAN, A_, 20);         \
    else XPA_LOSS_LAUNCH(XPA_DIST_GAUSSIAN, A_, kMaxAct);
    const bool streaming = dist == XPA_DIST_GAUSSIAN && A <= 20 && batch * A >= 4 &&
                           ((uintptr_t)head | (uintptr_t)d_head) % 16 == 0 &&
                           (idx != nullptr || (uintptr_t)act % 16 == 0);
#define XPA_LOSS_STREAM(A_, KM_, I_)                                                                              \
    hipLaunchKernelGGL((policy_loss_gauss_kernel<A_, KM_, I_>), dim3((unsigned)blocks), dim3(kLossThreads), 0, s,    \
                       batch, A, head, logstd, v, idx, n_rows, act, old_logp, adv, ret, adv_partials, n_adv_partials, \
                       clip_range, vf_coef, ent_coef, d_head, d_v, partials, width)
#define XPA_LOSS_STREAM_I(A_, KM_)               \
    if (idx) XPA_LOSS_STREAM(A_, KM_, true);     \
    else XPA_LOSS_STREAM(A_, KM_, false);
#define XPA_LOSS_STREAM_K(A_)                          \
    if (A <= 4) { XPA_LOSS_STREAM_I(A_, 4) }           \
    else if (A <= 8) { XPA_LOSS_STREAM_I(A_, 8) }      \
    else { XPA_LOSS_STREAM_I(A_, 20) }
    if (streaming) {
        if (algo == XPA_ALGO_PPO) { XPA_LOSS_STREAM_K(XPA_ALGO_PPO) }
        else { XPA_LOSS_STREAM_K(XPA_ALGO_A2C) }
    } else if (dist == XPA_DIST_GAUSSIAN) {
        if (algo == XPA_ALGO_PPO) { XPA_LOSS_GAUSS(XPA_ALGO_PPO) }
        else { XPA_LOSS_GAUSS(XPA_ALGO_A2C) }
    } else {
        if (algo == XPA_ALGO_PPO) XPA_LOSS_LAUNCH(XPA_DIST_CATEGORICAL, XPA_ALGO_PPO, 1);
        else XPA_LOSS_LAUNCH(XPA_DIST_CATEGORICAL, XPA_ALGO_A2C, 1);
    }
#undef XPA_LOSS_STREAM_K
#undef XPA_LOSS_STREAM_I
#undef XPA_LOSS_STREAM
#undef XPA_LOSS_GAUSS
#undef XPA_LOSS_LAUNCH
    return xpa_launch_status();
}

XPA_API int xpa_policy_loss_finalize_sq(int algo, int dist, int64_t batch, int64_t act_dim, const float *partials,
                                        int64_t n_partials, float vf_coef, float ent_coef, float *scalars,
                                        float *d_logstd, double *sq_out, xpa_stream_t stream) {
    if (batch <= 0 || act_dim <= 0 || act_dim > kMaxAct || n_partials <= 0 || !partials || !scalars)
        return (int)hipErrorInvalidValue;
    if (dist == XPA_DIST_GAUSSIAN && !d_logstd) return (int)hipErrorInvalidValue;
    const XpaLossFinalizeArgs args{algo, dist, batch, (int)act_dim, partials, n_partials,
                                   (int)xpa_loss_partial_width(act_dim), vf_coef, ent_coef, scalars, d_logstd};
    hipLaunchKernelGGL(policy_loss_finalize_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, args, sq_out);
    return xpa_launch_status();
}

XPA_API int xpa_policy_loss_finalize(int algo, int dist, int64_t batch, int64_t act_dim, const float *partials,
                                     int64_t n_partials, float vf_coef, float ent_coef, float *scalars,
                                     float *d_logstd, xpa_stream_t stream) {
    return xpa_policy_loss_finalize_sq(algo, dist, batch, act_dim, partials, n_partials, vf_coef, ent_coef, scalars,
                                       d_logstd, nullptr, stream);
}
