// K19 — PER-DQN TD target / loss / gradient / priorities in one launch (BASELINE.json configs[4]).
//
// Replaces the tensor algebra of PerDQN_Learner.update (xuance/torch/learners/qlearning_family/
// perdqn_learner.py:23-30, 48) between the two Q-network forwards and the backward:
//   y_b = r_b + (gamma * (1 - d_b)) * max_a' targetQ[b, a']        (f32, torch's operation order)
//   p_b = evalQ[b, act_b],  loss = mean((p - y)^2)                   (F.mse_loss)
//   dQ[b, a] = 2 (p_b - y_b) / B at a = act_b, 0 elsewhere           (d loss / d evalQ)
//   td_abs_b = |y_b - p_b|                                           (the new PER priorities, kept on device:
//                                                                      xpa_per_update_priorities reads them)
// One block walks the batch (B = 2048 at C5; the reduction for loss and mean(p) is a fixed-order f64 block
// sum, so the scalars are bit-reproducible).  Latency-bound: B (2A + 4) floats in, B (A + 1) out.
// Actions are float-coded indices (the buffer stores them as float32, memory_tools.py); out-of-range values are
// clamped into [0, A) (F.one_hot would raise) and counted into *err when err is given.
#include "xpa_common.h"

namespace {
constexpr int kDqnThreads = 1024;

__global__ __launch_bounds__(kDqnThreads) void dqn_td_kernel(int64_t B, int A, const float *__restrict__ evalQ,
                                                              int64_t ld_eval, const float *__restrict__ targetQ,
                                                              int64_t ld_tgt, const float *__restrict__ act,
                                                              const float *__restrict__ rew,
                                                              const float *__restrict__ term, float gamma,
                                                              float *__restrict__ dQ, int64_t ld_dq,
                                                              float *__restrict__ td_abs, float *__restrict__ scalars,
                                                              int *__restrict__ err) {
#pragma clang fp contract(off)  // torch CPU's separate roundings of the product and the sum
    __shared__ double s_red[2][kDqnThreads / 64];
    const int tid = threadIdx.x;
    const float inv_b2 = 2.0f / (float)B;
    double sq = 0.0, ps = 0.0;
    int bad = 0;
    for (int64_t b = tid; b < B; b += kDqnThreads) {
        const float *tq = targetQ + b * ld_tgt;
        float m = tq[0];
        for (int a = 1; a < A; ++a) m = fmaxf(m, tq[a]);
        const float y = rew[b] + (gamma * (1.0f - term[b])) * m;
        int ai = (int)act[b];
        if (ai < 0 || ai >= A) {
            ++bad;
            ai = ai < 0 ? 0 : A - 1;
        }
        const float p = evalQ[b * ld_eval + ai];
        const float d = p - y;
        float *dq = dQ + b * ld_dq;
        for (int a = 0; a < A; ++a) dq[a] = a == ai ? inv_b2 * d : 0.0f;
        td_abs[b] = fabsf(y - p);
        sq += (double)d * (double)d;
        ps += (double)p;
    }
    sq = xpa_wave_sum(sq);
    ps = xpa_wave_sum(ps);
    if ((tid & 63) == 0) {
        s_red[0][tid >> 6] = sq;
        s_red[1][tid >> 6] = ps;
    }
    if (err && bad) atomicAdd(err, bad);
    __syncthreads();
    if (tid == 0) {
        double a0 = 0.0, a1 = 0.0;
        for (int w = 0; w < kDqnThreads / 64; ++w) {
            a0 += s_red[0][w];
            a1 += s_red[1][w];
        }
        scalars[0] = (float)(a0 / (double)B);  // Qloss
        scalars[1] = (float)(a1 / (double)B);  // predictQ mean
    }
}
}  // namespace

XPA_API int xpa_dqn_td_loss(int64_t batch, int64_t n_actions, const float *evalQ, int64_t ld_eval,
                            const float *targetQ, int64_t ld_tgt, const float *act, const float *rew,
                            const float *term, float gamma, float *dQ, int64_t ld_dq, float *td_abs, float *scalars,
                            int32_t *err, xpa_stream_t stream) {
    if (batch <= 0 || n_actions <= 0 || n_actions > 4096 || !evalQ || !targetQ || !act || !rew || !term || !dQ ||
        !td_abs || !scalars || ld_eval < n_actions || ld_tgt < n_actions || ld_dq < n_actions)
        return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(dqn_td_kernel, dim3(1), dim3(kDqnThreads), 0, (hipStream_t)stream, batch, (int)n_actions, evalQ,
                       ld_eval, targetQ, ld_tgt, act, rew, term, gamma, dQ, ld_dq, td_abs, scalars, err);
    return xpa_launch_status();
}
