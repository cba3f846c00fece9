// K18 — CartPole-v1 env step on device (BASELINE.json configs[0]).
//
// The reference steps gym's CartPoleEnv one env at a time inside DummyVecEnv_Gym (gym_vec_env.py:201-212;
// dynamics: gym 0.26.2 classic_control/cartpole.py, euler integrator, TimeLimit 500).  Here one thread owns
// one env: the state stays in HBM as f64 (gym keeps Python floats), the observation is its f32 image, and the
// auto-reset draws uniform(-0.05, 0.05) per dim from the counter hash (seed, env, episode, dim) — the CPU
// checker (oracle/synth_env.CartPoleEnv) does the same arithmetic.  The action comes from the env input the
// rollout kernels write (K3 / K14: one-hot [N, 2] for a Categorical head).  Latency-bound: 8 to a few
// thousand envs, 32 B of state + 16 B of observation per env.
#include "cartpole_body.h"

namespace {
__global__ __launch_bounds__(256) void cartpole_step_kernel(int64_t n_envs, const float *__restrict__ act_in,
                                                            int64_t ld_act, XpaCartPoleEnv e) {
    const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (n >= n_envs) return;
    cartpole::Local s = cartpole::load(e, n);
    bool te, tr;
    float o[4];
    cartpole::step(e, n, act_in[n * ld_act + 1] > 0.5f ? 1 : 0, s, &te, &tr, o);
    cartpole::store(e, n, s);
}
}  // namespace

XPA_API int xpa_cartpole_step(int64_t n_envs, const float *act_in, int64_t ld_act, double *state, float *obs,
                              int64_t ld_obs, float *final_obs, float *rew, uint8_t *term, uint8_t *trunc,
                              int32_t *ep_step, uint32_t *ep_index, float *ep_score, float *ep_last_score,
                              int32_t *ep_last_len, uint32_t seed, int32_t max_episode_steps, xpa_stream_t stream) {
    if (n_envs <= 0 || !act_in || ld_act < 2 || !state || !obs || ld_obs < 4 || !final_obs || !rew || !term ||
        !trunc || !ep_step || !ep_index || !ep_score || !ep_last_score || !ep_last_len || max_episode_steps <= 0)
        return (int)hipErrorInvalidValue;
    const XpaCartPoleEnv e{state,    obs,           ld_obs,          final_obs, rew,
                           term,     trunc,         (int *)ep_step,  ep_index,  ep_score,
                           ep_last_score, (int *)ep_last_len, seed, (int)max_episode_steps,
                           cartpole::kThetaThreshold};
    hipLaunchKernelGGL(cartpole_step_kernel, dim3((unsigned)((n_envs + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, n_envs, act_in, ld_act, e);
    return xpa_launch_status();
}
