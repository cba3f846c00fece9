// Deterministic reduction of the loss partials (K2 / K12 / K16 layout: surrogate, sq-err, entropy, clip
// count, value sum, d logstd[A] per row) into the loss scalars and d logstd — the body of
// xpa_policy_loss_finalize, shared with the batched column-sum finalize that runs it as one extra block.
#pragma once
#include "xpa_common.h"

struct XpaLossFinalizeArgs {
    int algo, dist;
    int64_t batch;
    int A;
    const float *partials;
    int64_t n_partials;
    int width;
    float vf_coef, ent_coef;
    float *scalars, *d_logstd;
};

constexpr int kXpaLossPartBase = 5;
constexpr int kXpaLossMaxAct = 64;

// Every thread of the block calls it (blockDim.x a multiple of 64).  sq_out (nullable): sum of d_logstd^2, written
// through (sc1) for a ticketed hand-off in the same launch.  s_tot / s_dls: LDS.
__device__ inline void xpa_loss_finalize_body(const XpaLossFinalizeArgs &a, double *sq_out, double *s_tot,
                                              float *s_dls) {
    const int ncols = kXpaLossPartBase + (a.dist == XPA_DIST_GAUSSIAN ? a.A : 0);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // every wave of the block takes columns (r03: the batched finalize's 16-wave block sums C2's 11 columns in one
    // pass — one memory round trip — instead of three passes of 4 waves)
    const int nw = (int)(blockDim.x >> 6);
    {
        for (int j = w; j < ncols; j += nw) {  // one wave per column, fixed lane order -> deterministic
            double s = 0.0;
            int64_t k = lane;
            for (; k + 7 * 64 < a.n_partials; k += 8 * 64) {  // 8 loads in flight, added in k order
                float v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = a.partials[(k + 64 * u) * a.width + j];
#pragma unroll
                for (int u = 0; u < 8; ++u) s += (double)v[u];
            }
            for (; k < a.n_partials; k += 64) s += (double)a.partials[k * a.width + j];
            s = xpa_wave_sum(s);
            if (lane == 0) {
                if (j < kXpaLossPartBase) s_tot[j] = s;
                else a.d_logstd[j - kXpaLossPartBase] = s_dls[j - kXpaLossPartBase] = (float)(s - (double)a.ent_coef);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && sq_out) {  // this gradient's share of the clip norm (xpa_clip_adam_step_partials)
        double q = 0.0;
        if (a.dist == XPA_DIST_GAUSSIAN)
            for (int k = 0; k < a.A; ++k) q += (double)s_dls[k] * (double)s_dls[k];
        xpa_store_agent(sq_out, q);
    }
    if (threadIdx.x == 0) {
        const double B = (double)a.batch;
        const double actor = -s_tot[0] / B;
        const double critic = s_tot[1] / B;
        const double entropy = s_tot[2] / B;
        a.scalars[XPA_OUT_ACTOR_LOSS] = (float)actor;
        a.scalars[XPA_OUT_CRITIC_LOSS] = (float)critic;
        a.scalars[XPA_OUT_ENTROPY] = (float)entropy;
        a.scalars[XPA_OUT_LOSS] = (float)(actor - (double)a.ent_coef * entropy + (double)a.vf_coef * critic);
        a.scalars[XPA_OUT_CLIP_RATIO] = a.algo == XPA_ALGO_PPO ? (float)(s_tot[3] / B) : 0.f;
        a.scalars[XPA_OUT_VALUE_MEAN] = (float)(s_tot[4] / B);
    }
}
