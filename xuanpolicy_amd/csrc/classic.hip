// K18 — CartPole-v1 env step on device (BASELINE.json configs[0]).
//
// The reference steps gym's CartPoleEnv one env at a time inside DummyVecEnv_Gym (gym_vec_env.py:201-212;
// dynamics: gym 0.26.2 classic_control/cartpole.py, euler integrator, TimeLimit 500).  Here one thread owns
// one env: the state stays in HBM as f64 (gym keeps Python floats), the observation is its f32 image, and the
// auto-reset draws uniform(-0.05, 0.05) per dim from the counter hash (seed, env, episode, dim) — the CPU
// checker (oracle/synth_env.CartPoleEnv) does the same arithmetic.  The action comes from the env input the
// rollout kernels write (K3 / K14: one-hot [N, 2] for a Categorical head).  Latency-bound: 8 to a few
// thousand envs, 32 B of state + 16 B of observation per env.
#include "xpa_common.h"

namespace {
constexpr double kGravity = 9.8, kMassPole = 0.1, kTotalMass = 1.1, kLength = 0.5, kPoleMassLength = 0.05;
constexpr double kForce = 10.0, kTau = 0.02, kXThreshold = 2.4;
constexpr uint32_t kSaltCartPole = 0xCA27B01Eu;

__device__ __forceinline__ double reset_dim(uint32_t seed, uint32_t env, uint32_t ep, uint32_t d) {
    return (double)xpa_u01(xpa_hash4(seed ^ kSaltCartPole, env, ep, d)) * 0.1 - 0.05;
}

__global__ __launch_bounds__(256) void cartpole_step_kernel(int64_t n_envs, const float *__restrict__ act_in,
                                                            int64_t ld_act, double *__restrict__ state,
                                                            float *__restrict__ obs, int64_t ld_obs,
                                                            float *__restrict__ final_obs, float *__restrict__ rew,
                                                            uint8_t *__restrict__ term, uint8_t *__restrict__ trunc,
                                                            int *__restrict__ ep_step, uint32_t *__restrict__ ep_index,
                                                            float *__restrict__ ep_score,
                                                            float *__restrict__ ep_last_score,
                                                            int *__restrict__ ep_last_len, uint32_t seed,
                                                            int max_episode_steps, double theta_threshold) {
#pragma clang fp contract(off)  // gym's Python arithmetic: every product and sum rounded on its own (no fma)
    const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (n >= n_envs) return;
    double x = state[4 * n], x_dot = state[4 * n + 1], theta = state[4 * n + 2], theta_dot = state[4 * n + 3];
    const int a = act_in[n * ld_act + 1] > 0.5f ? 1 : 0;
    const double force = a == 1 ? kForce : -kForce;
    const double costheta = cos(theta), sintheta = sin(theta);
    const double temp = (force + kPoleMassLength * (theta_dot * theta_dot) * sintheta) / kTotalMass;
    const double thetaacc = (kGravity * sintheta - costheta * temp) /
                            (kLength * (4.0 / 3.0 - kMassPole * (costheta * costheta) / kTotalMass));
    const double xacc = temp - kPoleMassLength * thetaacc * costheta / kTotalMass;
    x = x + kTau * x_dot;
    x_dot = x_dot + kTau * xacc;
    theta = theta + kTau * theta_dot;
    theta_dot = theta_dot + kTau * thetaacc;
    const bool te = x < -kXThreshold || x > kXThreshold || theta < -theta_threshold || theta > theta_threshold;
    const int steps = ep_step[n] + 1;
    const bool tr = steps >= max_episode_steps;  // gym TimeLimit: independent of terminated
    const float score = ep_score[n] + 1.0f;
    final_obs[4 * n] = (float)x;
    final_obs[4 * n + 1] = (float)x_dot;
    final_obs[4 * n + 2] = (float)theta;
    final_obs[4 * n + 3] = (float)theta_dot;
    rew[n] = 1.0f;
    term[n] = te ? 1 : 0;
    trunc[n] = tr ? 1 : 0;
    if (te || tr) {
        const uint32_t ep = ep_index[n] + 1u;
        ep_index[n] = ep;
        ep_last_score[n] = score;
        ep_last_len[n] = steps;
        ep_step[n] = 0;
        ep_score[n] = 0.f;
        x = reset_dim(seed, (uint32_t)n, ep, 0);
        x_dot = reset_dim(seed, (uint32_t)n, ep, 1);
        theta = reset_dim(seed, (uint32_t)n, ep, 2);
        theta_dot = reset_dim(seed, (uint32_t)n, ep, 3);
    } else {
        ep_step[n] = steps;
        ep_score[n] = score;
    }
    state[4 * n] = x;
    state[4 * n + 1] = x_dot;
    state[4 * n + 2] = theta;
    state[4 * n + 3] = theta_dot;
    obs[n * ld_obs] = (float)x;
    obs[n * ld_obs + 1] = (float)x_dot;
    obs[n * ld_obs + 2] = (float)theta;
    obs[n * ld_obs + 3] = (float)theta_dot;
}
}  // namespace

XPA_API int xpa_cartpole_step(int64_t n_envs, const float *act_in, int64_t ld_act, double *state, float *obs,
                              int64_t ld_obs, float *final_obs, float *rew, uint8_t *term, uint8_t *trunc,
                              int32_t *ep_step, uint32_t *ep_index, float *ep_score, float *ep_last_score,
                              int32_t *ep_last_len, uint32_t seed, int32_t max_episode_steps, xpa_stream_t stream) {
    if (n_envs <= 0 || !act_in || ld_act < 2 || !state || !obs || ld_obs < 4 || !final_obs || !rew || !term ||
        !trunc || !ep_step || !ep_index || !ep_score || !ep_last_score || !ep_last_len || max_episode_steps <= 0)
        return (int)hipErrorInvalidValue;
    const double theta_threshold = 12.0 * 2.0 * 3.141592653589793 / 360.0;  // gym: 12 * 2 * math.pi / 360
    hipLaunchKernelGGL(cartpole_step_kernel, dim3((unsigned)((n_envs + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, n_envs, act_in, ld_act, state, obs, ld_obs, final_obs, rew, term, trunc,
                       ep_step, ep_index, ep_score, ep_last_score, ep_last_len, seed, max_episode_steps,
                       theta_threshold);
    return xpa_launch_status();
}
