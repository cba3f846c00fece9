// Fused global-norm gradient clipping + Adam over flat fp32 buffers (gfx950).
//
// Replaces, per learner update, torch.nn.utils.clip_grad_norm_ + torch.optim.Adam.step as called by
// PPOCLIP_Learner.update / A2C_Learner.update (xuance/torch/learners/policy_gradient/ppoclip_learner.py:47-49,
// a2c_learner.py:34-35) with the optimizer the runner builds (Adam(eps=1e-5), xuance/torch/runners/
// runner_drl.py:71).  Semantics follow torch: total_norm = ||g||_2 over all parameters,
// coef = min(max_norm / (total_norm + 1e-6), 1); g *= coef; then Adam:
//   m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2;  p -= (lr / bc1) m / (sqrt(v) / sqrt(bc2) + eps).
// max_norm < 0 means "no clipping" (use_grad_clip False); max_norm = 0 clips to zero as torch does.
// Two launches: K_a per-block sum of squares (f64, fixed order), K_b every block re-reduces those
// partials (deterministic, no atomics), scales g in place and applies the Adam update with 16-B
// accesses.  HBM-bound: 4 B read (K_a) + 4x4 B read + 4x4 B write... per parameter (p, g, m, v).
#include "xpa_common.h"

namespace {

constexpr int kOptThreads = 256;
constexpr int kMaxNormBlocks = 512;

__global__ __launch_bounds__(kOptThreads) void grad_sqnorm_kernel(const float *__restrict__ g, int64_t n,
                                                                  double *__restrict__ partials) {
    __shared__ double s_red[kOptThreads / 64];
    double acc = 0.0;
    const int64_t n4 = n / 4;
    const float4 *g4 = reinterpret_cast<const float4 *>(g);
    for (int64_t i = (int64_t)blockIdx.x * kOptThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kOptThreads) {
        const float4 x = g4[i];
        acc += (double)x.x * x.x + (double)x.y * x.y + (double)x.z * x.z + (double)x.w * x.w;
    }
    for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * kOptThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kOptThreads)
        acc += (double)g[i] * g[i];
    acc = xpa_block_sum(acc, s_red, kOptThreads / 64);
    if (threadIdx.x == 0) partials[blockIdx.x] = acc;
}

__device__ __forceinline__ void adam1(float &p, float &g, float &m, float &v, float coef, float b1, float b2,
                                      float step_size, float inv_bc2_sqrt, float eps) {
    g *= coef;
    m = m + (1.0f - b1) * (g - m);  // exp_avg.lerp_(grad, 1 - beta1)
    v = b2 * v + (1.0f - b2) * g * g;
    const float denom = sqrtf(v) * inv_bc2_sqrt + eps;
    p = p - step_size * (m / denom);
}

__global__ __launch_bounds__(kOptThreads) void clip_adam_kernel(float *__restrict__ p, float *__restrict__ g,
                                                                float *__restrict__ m, float *__restrict__ v, int64_t n,
                                                                const double *__restrict__ partials, int n_partials,
                                                                float max_norm, float b1, float b2, float step_size,
                                                                float inv_bc2_sqrt, float eps,
                                                                float *__restrict__ norm_out,
                                                                const float *__restrict__ sched, int n_sched,
                                                                int *__restrict__ cursor) {
    __shared__ float s_coef, s_step, s_inv;
    if (threadIdx.x < 64) {
        double s = 0.0;
        for (int k = threadIdx.x; k < n_partials; k += 64) s += partials[k];
        s = xpa_wave_sum(s);
        if (threadIdx.x == 0) {
            const float total = (float)sqrt(s);
            // max_norm < 0: no clipping; max_norm >= 0 clips exactly like clip_grad_norm_ (0 zeroes g)
            float coef = 1.0f;
            if (max_norm >= 0.f) coef = fminf(max_norm / (total + 1e-6f), 1.0f);
            s_coef = coef;
            if (blockIdx.x == 0 && norm_out) *norm_out = total;
            s_step = step_size;
            s_inv = inv_bc2_sqrt;
            if (sched) {
                // device schedule (step_size, 1/sqrt(bc2)) of update cursor[0]; an index past the table is clamped
                // and flagged in cursor[2]
                int k = __hip_atomic_load(cursor, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (k >= n_sched) {
                    if (blockIdx.x == 0) cursor[2] = 1;
                    k = n_sched - 1;
                }
                s_step = sched[2 * k];
                s_inv = sched[2 * k + 1];
            }
        }
    }
    __syncthreads();
    const float coef = s_coef;
    step_size = s_step;
    inv_bc2_sqrt = s_inv;
    if (sched && threadIdx.x == 0) {
        // every block has read cursor[0]: the last one to take a ticket advances it for the next update's launch
        const int t = __hip_atomic_fetch_add(cursor + 1, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (t == (int)gridDim.x - 1) {
            cursor[1] = 0;
            __hip_atomic_fetch_add(cursor, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    const int64_t n4 = n / 4;
    float4 *p4 = reinterpret_cast<float4 *>(p);
    float4 *g4 = reinterpret_cast<float4 *>(g);
    float4 *m4 = reinterpret_cast<float4 *>(m);
    float4 *v4 = reinterpret_cast<float4 *>(v);
    for (int64_t i = (int64_t)blockIdx.x * kOptThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kOptThreads) {
        float4 pp = p4[i], gg = g4[i], mm = m4[i], vv = v4[i];
        adam1(pp.x, gg.x, mm.x, vv.x, coef, b1, b2, step_size, inv_bc2_sqrt, eps);
        adam1(pp.y, gg.y, mm.y, vv.y, coef, b1, b2, step_size, inv_bc2_sqrt, eps);
        adam1(pp.z, gg.z, mm.z, vv.z, coef, b1, b2, step_size, inv_bc2_sqrt, eps);
        adam1(pp.w, gg.w, mm.w, vv.w, coef, b1, b2, step_size, inv_bc2_sqrt, eps);
        p4[i] = pp; g4[i] = gg; m4[i] = mm; v4[i] = vv;
    }
    for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * kOptThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kOptThreads) {
        float pp = p[i], gg = g[i], mm = m[i], vv = v[i];
        adam1(pp, gg, mm, vv, coef, b1, b2, step_size, inv_bc2_sqrt, eps);
        p[i] = pp; g[i] = gg; m[i] = mm; v[i] = vv;
    }
}

inline int64_t norm_blocks(int64_t n) {
    int64_t b = (n / 4 + kOptThreads - 1) / kOptThreads;
    if (b < 1) b = 1;
    return b > kMaxNormBlocks ? kMaxNormBlocks : b;
}

}  // namespace

XPA_API int64_t xpa_grad_norm_num_partials(int64_t n) { return norm_blocks(n); }

// The clip + Adam step from squared-norm partials the gradient producers already wrote (the batched
// column-sum finalize's per-tile partials and the loss finalize's d logstd share, world size 1): the norm
// pass over the flat gradient is skipped.  sq_partials: n_sq doubles whose sum is |grad|^2.
XPA_API int xpa_clip_adam_step_partials(float *param, float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
                                        const double *sq_partials, int64_t n_sq, float max_norm, float lr,
                                        float beta1, float beta2, float eps, int64_t step, float *total_norm_out,
                                        xpa_stream_t stream) {
    if (n <= 0 || step < 1 || !param || !grad || !exp_avg || !exp_avg_sq || !sq_partials || n_sq <= 0 ||
        n_sq > 0x7fffffff)
        return (int)hipErrorInvalidValue;
    if (((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16)
        return (int)hipErrorInvalidValue;
    const double bc1 = 1.0 - pow((double)beta1, (double)step);
    const double bc2 = 1.0 - pow((double)beta2, (double)step);
    const float step_size = (float)((double)lr / bc1);
    const float inv_bc2_sqrt = (float)(1.0 / sqrt(bc2));
    int64_t ab = (n / 4 + kOptThreads - 1) / kOptThreads;
    if (ab < 1) ab = 1;
    if (ab > 2048) ab = 2048;
    hipLaunchKernelGGL(clip_adam_kernel, dim3((unsigned)ab), dim3(kOptThreads), 0, (hipStream_t)stream, param, grad,
                       exp_avg, exp_avg_sq, n, sq_partials, (int)n_sq, max_norm, beta1, beta2, step_size,
                       inv_bc2_sqrt, eps, total_norm_out, nullptr, 0, nullptr);
    return xpa_launch_status();
}

XPA_API int xpa_clip_adam_step(float *param, float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
                               double *norm_partials, float max_norm, float lr, float beta1, float beta2, float eps,
                               int64_t step, float *total_norm_out, xpa_stream_t stream) {
    if (n <= 0 || step < 1 || !param || !grad || !exp_avg || !exp_avg_sq || !norm_partials)
        return (int)hipErrorInvalidValue;
    if (((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16)
        return (int)hipErrorInvalidValue;
    const int64_t nb = norm_blocks(n);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(grad_sqnorm_kernel, dim3((unsigned)nb), dim3(kOptThreads), 0, s, grad, n, norm_partials);
    const int st = xpa_launch_status();
    if (st) return st;
    const double bc1 = 1.0 - pow((double)beta1, (double)step);
    const double bc2 = 1.0 - pow((double)beta2, (double)step);
    const float step_size = (float)((double)lr / bc1);
    const float inv_bc2_sqrt = (float)(1.0 / sqrt(bc2));
    int64_t ab = (n / 4 + kOptThreads - 1) / kOptThreads;
    if (ab < 1) ab = 1;
    if (ab > 2048) ab = 2048;
    hipLaunchKernelGGL(clip_adam_kernel, dim3((unsigned)ab), dim3(kOptThreads), 0, s, param, grad, exp_avg, exp_avg_sq,
                       n, norm_partials, (int)nb, max_norm, beta1, beta2, step_size, inv_bc2_sqrt, eps,
                       total_norm_out, nullptr, 0, nullptr);
    return xpa_launch_status();
}

// K9 with (step_size, 1/sqrt(bc2)) read from a device schedule: sched[2k], sched[2k + 1] for update k = cursor[0]
// (cursor: int32[3] = {update index, block ticket, overflow flag}); the launch advances cursor[0] itself, so a
// captured update (forward + loss + backward + this) replays with the next update's Adam step and learning rate.
// The host fills the schedule once per window of updates (flat.FusedClipAdam.step_sched).
XPA_API int xpa_clip_adam_step_sched(float *param, float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
                                     double *norm_partials, float max_norm, float beta1, float beta2, float eps,
                                     const float *sched, int64_t n_sched, int32_t *cursor, float *total_norm_out,
                                     xpa_stream_t stream) {
    if (n <= 0 || !param || !grad || !exp_avg || !exp_avg_sq || !norm_partials || !sched || !cursor || n_sched <= 0 ||
        n_sched > 0x7fffffff)
        return (int)hipErrorInvalidValue;
    if (((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16)
        return (int)hipErrorInvalidValue;
    const int64_t nb = norm_blocks(n);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(grad_sqnorm_kernel, dim3((unsigned)nb), dim3(kOptThreads), 0, s, grad, n, norm_partials);
    const int st = xpa_launch_status();
    if (st) return st;
    int64_t ab = (n / 4 + kOptThreads - 1) / kOptThreads;
    if (ab < 1) ab = 1;
    if (ab > 2048) ab = 2048;
    hipLaunchKernelGGL(clip_adam_kernel, dim3((unsigned)ab), dim3(kOptThreads), 0, s, param, grad, exp_avg, exp_avg_sq,
                       n, norm_partials, (int)nb, max_norm, beta1, beta2, 0.f, 0.f, eps, total_norm_out, sched,
                       (int)n_sched, cursor);
    return xpa_launch_status();
}

// The host-side schedule entry of update `step` with learning rate lr (the arithmetic of xpa_clip_adam_step).
XPA_API void xpa_adam_sched_entry(float lr, float beta1, float beta2, int64_t step, float *out2) {
    const double bc1 = 1.0 - pow((double)beta1, (double)step);
    const double bc2 = 1.0 - pow((double)beta2, (double)step);
    out2[0] = (float)((double)lr / bc1);
    out2[1] = (float)(1.0 / sqrt(bc2));
}
