/*
 * xuanpolicy_amd — C ABI of the MI355X (gfx950) on-policy PPO-Clip / A2C hot path.
 *
 * Library: xuanpolicy_amd/libxuanpolicy_amd.so (hipcc --offload-arch=gfx950).
 * Conventions (all entry points):
 *   - every pointer is a device pointer owned by the caller (torch tensors on the Python side);
 *     nothing is allocated, freed or synchronised inside, so every call is hipGraph-capturable;
 *   - calls are ordered on `stream` (a hipStream_t; NULL = the legacy default stream);
 *   - the return value is a hipError_t as int: 0 = success, 1 (hipErrorInvalidValue) = bad
 *     arguments (nothing launched), anything else = the launch error;
 *   - [n_envs, horizon] arrays are row-major: element (env n, step t) at n*horizon + t, the layout
 *     of the reference's DummyOnPolicyBuffer (memory_tools.py:12-36, flat index env*T + step at
 *     memory_tools.py:234).
 *
 * The reference (XuanCe 1.0.5 fork, pure Python) has no C ABI; each entry point names the
 * reference function it replaces (paths relative to the reference root).
 */
#ifndef XUANPOLICY_AMD_H
#define XUANPOLICY_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t *xpa_stream_t; /* == hipStream_t */

/* ABI 2 (round 3): n_slots added to xpa_rollout_post_deferred[_norm] / xpa_rollout_bootstrap_fixup; the error
 * word `err` added to xpa_per_sample / xpa_gather_minibatch / xpa_synthatari_step / xpa_maxpool_act_bwd_bias; max_norm of
 * xpa_clip_adam_step[_partials]: < 0 disables clipping, 0 zeroes the gradient (ABI 1 callers passing 0 to mean "no
 * clipping" must pass -1). */
/* ABI 3 (round 4): xpa_rollout_post_deferred_norm takes (slot_src, ld_slot) after ld_final — the rows a kept
 * truncation's bootstrap is formed from when they are not the final observations (A2C: the next, reset, observation;
 * NULL: final_obs as before); XpaSmallRolloutArgs gains slot_reset_obs (the same choice for K32); xpa_rollout_post
 * takes v_boot_mid after v_boot (nullable: the bootstrap values of closures before the rollout's last step, A2C's
 * V(norm(reset_obs)); the last step's closures use v_boot). */
/* ABI 4 (round 6): the batched column-sum finalizes that take a ticket (xpa_colsum_finalize_batch_sq / _sq_loss / _map)
 * need int32 [XPA_COLSUM_TICKET_INTS] there, zero-initialised and left at zero (two ticket levels on separate lines:
 * ~300 blocks counting on one int serialised their atomics). */
#define XPA_ABI_VERSION 4
#define XPA_COLSUM_TICKET_INTS 4096

/* Device-resident rollout cursor read by the per-step kernels, so a captured step replays
 * without host-side arguments changing: ptr = buffer column being written (DummyOnPolicyBuffer.ptr,
 * memory_tools.py:203), step = global env-step counter (RNG key). */
typedef struct {
    int32_t ptr;
    uint32_t step;
    int32_t reserved[2];
} xpa_cursor_t;

enum { XPA_ALGO_PPO = 0, XPA_ALGO_A2C = 1 };
enum { XPA_DIST_GAUSSIAN = 0, XPA_DIST_CATEGORICAL = 1 };

/* Loss scalars written by xpa_policy_loss_finalize, in this order. */
enum {
    XPA_OUT_ACTOR_LOSS = 0, /* -mean(min(clip(r)A, rA))  or  -mean(A logp)                        */
    XPA_OUT_CRITIC_LOSS = 1, /* mean((v - R)^2)                                                    */
    XPA_OUT_ENTROPY = 2,     /* mean(entropy)                                                       */
    XPA_OUT_LOSS = 3,        /* actor - ent_coef*entropy + vf_coef*critic                           */
    XPA_OUT_CLIP_RATIO = 4,  /* frac(r < 1-eps or r > 1+eps)   (PPO only, 0 for A2C)                */
    XPA_OUT_VALUE_MEAN = 5,  /* mean(v)                                                              */
    XPA_OUT_COUNT = 6
};

int xpa_abi_version(void);

/* K1 — GAE / discounted returns over a whole [n_envs, horizon] buffer.
 * Replaces DummyOnPolicyBuffer.finish_path (xuance/common/memory_tools.py:206-229) called for
 * every path the agent closes (xuance/torch/agents/policy_gradient/ppoclip_agent.py:69-101,
 * a2c_agent.py:66-98).  closed[n,t] != 0 marks the last step of a path closed with bootstrap
 * value boot[n,t]; positions after a row's last closure are not written (as in the reference).
 * use_gae = 0 selects the discount_cumsum branch (memory_tools.py:222-225).
 * Reads rew/val/term (f32), closed (u8), boot (f32 [n_envs, horizon]: streamed densely, its values
 * used only where closed); writes adv, ret (f32). */
int xpa_gae_scan(const float *rew, const float *val, const float *term, const uint8_t *closed,
                 const float *boot, int64_t n_envs, int64_t horizon, float gamma, float gae_lambda,
                 int use_gae, float *adv, float *ret, xpa_stream_t stream);
/* The same launch with two HIP events (hipEvent_t, created by the caller with timing enabled) recorded
 * at the kernel's own start and end (hipExtLaunchKernel): the live per-launch duration bench.py's
 * roofline uses.  NULL events = xpa_gae_scan. */
int xpa_gae_scan_timed(const float *rew, const float *val, const float *term, const uint8_t *closed,
                       const float *boot, int64_t n_envs, int64_t horizon, float gamma, float gae_lambda,
                       int use_gae, float *adv, float *ret, void *ev_start, void *ev_stop, xpa_stream_t stream);

/* K1, compact closures: the fused agent's form (non-Atari, at most one mid-buffer truncation per env
 * per rollout — K8's deferred bootstrap slots).  A row closes at its terminals (term != 0), at step
 * slot_t[n] (>= 0: the env's truncation) and at its last step; the bootstraps are
 * vboot[n] (truncation) and vboot[n_envs + n] (last step; 0 when terminal) — the critic values of the
 * deferred pass.  Fuses xpa_rollout_bootstrap_fixup: writes both bootstraps into boot[n, t] and resets
 * slot_t[n] = -1, so the buffer ends in the state of fixup + xpa_gae_scan.  Reads exactly the
 * algorithmic r, v, d (f32) + 12 B per env; no closure-flag or dense boot stream.
 * ev_start / ev_stop as in xpa_gae_scan_timed (NULL: untimed). */
int xpa_gae_scan_compact(const float *rew, const float *val, const float *term, int32_t *slot_t,
                         const float *vboot, int64_t n_envs, int64_t horizon, float gamma, float gae_lambda,
                         int use_gae, float *adv, float *ret, float *boot, void *ev_start, void *ev_stop,
                         xpa_stream_t stream);

/* K1V, value-fused compact scan: xpa_gae_scan_compact with the deferred pass's value head inside it.
 * Replaces the critic's last layer on [truncation slots; last observations] (gaussian.py:73-77 /
 * categorical.py:83-85: v = critic(state)[:, 0], as the agent bootstraps at ppoclip_agent.py:69-75, 95-100)
 * plus the fixup + finish_path GAE (memory_tools.py:206-229).  z_critic [2 n_envs, ld] (row stride ld,
 * 16-B aligned) holds the critic's hidden-layer pre-activations (rows [0, n) the truncation slots, [n, 2n)
 * the last-step observations); V = act(z) . w_critic + b_critic[0] (act 0 identity, 1 LeakyReLU(slope),
 * 2 tanh; hidden = 256), bitwise K14's xpa_value_head.  Then exactly xpa_gae_scan_compact with
 * vboot = V.  horizon % 4 == 0 and >= 36.  ev_start / ev_stop as in xpa_gae_scan_timed. */
int xpa_gae_scan_value(const float *rew, const float *val, const float *term, int32_t *slot_t, int act,
                       const float *z_critic, int64_t ld, float slope, const float *w_critic,
                       const float *b_critic, int64_t n_envs, int64_t horizon, int64_t hidden, float gamma,
                       float gae_lambda, int use_gae, float *adv, float *ret, float *boot, void *ev_start,
                       void *ev_stop, xpa_stream_t stream);

/* Measurement aid (no reference counterpart): an empty one-wave kernel launched with the same
 * dispatch-attached events as xpa_gae_scan_timed — the fixed per-launch cost of that clock (both events NULL:
 * a plain empty launch, for other clocks). */
int xpa_dispatch_floor_timed(void *ev_start, void *ev_stop, xpa_stream_t stream);
/* Measurement aid: K1's algorithmic bytes moved with no scan (3 f32 streams read, 2 written, n elements,
 * 16-B aligned, n % 4 == 0), timed by the same dispatch-attached events: the copy floor K1 is held to. */
int xpa_stream_copy_timed(const float *r, const float *v, const float *d, float *a, float *o, int64_t n,
                          void *ev_start, void *ev_stop, xpa_stream_t stream);

/* K4 — minibatch gather.  Replaces the fancy-index gather of DummyOnPolicyBuffer.sample
 * (memory_tools.py:231-240) for the observation rows (the rest is read through `idx` by the loss
 * kernel), and produces the per-minibatch advantage moments for adv-norm (memory_tools.py:241-242).
 * obs_out[b] = obs[idx[b]] (row_bytes each); adv_partials[g] = (sum, sum of squares) in f64 over
 * rows [g*64, (g+1)*64); xpa_gather_num_partials(batch) rows.  adv/adv_partials may be NULL.
 * n_rows = rows of obs/adv: an index outside [0, n_rows) is never dereferenced (its output row is
 * zeroed, it adds nothing to the moments and, when err != NULL, it is counted in *err). */
int64_t xpa_gather_num_partials(int64_t batch);
int xpa_gather_minibatch(const int64_t *idx, int64_t batch, int64_t n_rows, const void *obs,
                         int64_t obs_row_bytes, void *obs_out, const float *adv, double *adv_partials,
                         int32_t *err, xpa_stream_t stream);

/* K2 — fused policy/value loss forward + backward for one minibatch.
 * Replaces PPOCLIP_Learner.update's loss (xuance/torch/learners/policy_gradient/ppoclip_learner.py:32-44)
 * and A2C_Learner.update's loss (a2c_learner.py:24-31), with DiagGaussianDistribution /
 * CategoricalDistribution log_prob and entropy (xuance/torch/utils/distributions.py:39-101).
 * head: mu [batch, act_dim] (Gaussian, with logstd [act_dim]) or logits [batch, act_dim] (Categorical).
 * v: predicted values [batch].  Per-sample inputs act/old_logp/adv/ret are read at row idx[b]
 * (idx == NULL: row b; an idx outside [0, n_rows) is never dereferenced and the sample contributes
 * nothing); act is [n_rows, act_dim] (Gaussian) or [n_rows] float-coded indices (Categorical).
 * adv_partials (from xpa_gather_minibatch, n_adv_partials rows) != NULL applies per-minibatch
 * normalisation (adv - mean) / (std_pop + 1e-8) (memory_tools.py:241-242); NULL uses adv as given.
 * Writes d loss/d head [batch, act_dim], d loss/d v [batch] and per-block partial sums
 * (xpa_loss_num_partials(batch) rows of xpa_loss_partial_width(act_dim) floats). */
int64_t xpa_loss_num_partials(int64_t batch);
int64_t xpa_loss_partial_width(int64_t act_dim);
int xpa_policy_loss_fwd_bwd(int algo, int dist, int64_t batch, int64_t act_dim, const float *head,
                            const float *logstd, const float *v, const int64_t *idx, int64_t n_rows,
                            const float *act,
                            const float *old_logp, const float *adv, const float *ret,
                            const double *adv_partials, int64_t n_adv_partials, float clip_range,
                            float vf_coef, float ent_coef, float *d_head, float *d_v, float *partials,
                            xpa_stream_t stream);
/* Deterministic reduction of the partials: scalars[XPA_OUT_COUNT] (the info dict of
 * ppoclip_learner.py:53-63 / a2c_learner.py:36-47) and d loss/d logstd [act_dim] (Gaussian). */
int xpa_policy_loss_finalize(int algo, int dist, int64_t batch, int64_t act_dim, const float *partials,
                             int64_t n_partials, float vf_coef, float ent_coef, float *scalars,
                             float *d_logstd, xpa_stream_t stream);
/* The same, also writing sum(d_logstd^2) (0 for Categorical) into *sq_out (nullable): that gradient's
 * share of the clip norm for xpa_clip_adam_step_partials (the norm torch.nn.utils.clip_grad_norm_ takes
 * over all parameters in ppoclip_learner.py:47-48, a2c_learner.py:34). */
int xpa_policy_loss_finalize_sq(int algo, int dist, int64_t batch, int64_t act_dim, const float *partials,
                                int64_t n_partials, float vf_coef, float ent_coef, float *scalars, float *d_logstd,
                                double *sq_out, xpa_stream_t stream);

/* Epoch permutation for minibatch sampling (replaces the np.random.shuffle of an arange(buffer_size),
 * ppoclip_agent.py:76-81): out = a pseudo-random permutation of [0, n) keyed by (seed, counter)
 * (4-round Feistel over 2h >= log2(n) bits with cycle walking), n <= 2^31. */
int xpa_random_permutation(int64_t n, uint32_t seed, uint32_t counter, int64_t *out, xpa_stream_t stream);

/* K5 — RunningMeanStd over observations (xuance/common/statistic_tools.py:63-112) and observation
 * normalisation (xuance/torch/agents/agent.py:104-116).
 * xpa_rms_partials: per-block f64 sums of (x - shift) and (x - shift)^2 over x[n, dim] (row stride
 * ld floats); shift must be the `mean` array later passed to xpa_rms_merge (the running mean).
 * xpa_rms_merge: batch moments from the partials, then update_from_moments into mean/var
 * (f32 [dim]) and *count (f64) — one block.  n = rows the partials cover (n_partials * 256 or fewer
 * for one rank; the global row count when the partials were SUM-reduced across ranks).
 * xpa_obs_normalize: out = clip((x - mean) / (sqrt(var) + 1e-8), -clip_range, clip_range);
 * also copied to col_out + cursor->ptr*dim (row stride col_ld) when col_out != NULL. */
int64_t xpa_rms_num_partials(int64_t n);
int xpa_rms_partials(const float *x, int64_t n, int64_t dim, int64_t ld, const float *shift,
                     double *partials, xpa_stream_t stream);
int xpa_rms_merge(const double *partials, int64_t n_partials, int64_t n, int64_t dim, float *mean,
                  float *var, double *count, xpa_stream_t stream);
/* xpa_rms_partials + xpa_rms_merge in one launch (shift = mean): the last block to finish (an atomic
 * ticket, int32 [1], zero-initialised by the caller and left at zero) merges every block's partials in
 * block order — the same arithmetic and order as xpa_rms_merge.  partials: xpa_rms_num_partials(n) x 2 x
 * dim doubles. */
int xpa_rms_update(const float *x, int64_t n, int64_t dim, int64_t ld, float *mean, float *var, double *count,
                   double *partials, int32_t *ticket, xpa_stream_t stream);
int xpa_obs_normalize(const float *x, int64_t n, int64_t dim, int64_t ldx, const float *mean,
                      const float *var, float clip_range, float *out, int64_t ldo, float *col_out,
                      int64_t col_ld, const xpa_cursor_t *cursor, xpa_stream_t stream);

/* K3 — rollout action sampling + log-prob + store.  Replaces PPOCLIP_Agent._action
 * (ppoclip_agent.py:50-57: stochastic_sample + log_prob + three D2H copies) and the action/value/
 * log-prob part of DummyOnPolicyBuffer.store (memory_tools.py:196-204).
 * Gaussian: a = mu + exp(logstd) * eps, eps ~ N(0,1) from a counter hash of (seed, cursor->step, env, dim).
 * Categorical: inverse-CDF sample of softmax(logits) from one hashed uniform per env.
 * Stores act [n_envs, horizon, act_dim] (float-coded index for Categorical), logp and val
 * [n_envs, horizon] at column cursor->ptr, and the env input into env_in (row stride ld_env):
 * clip(a, -act_clip, act_clip) (Gaussian) or one-hot(a) (Categorical). */
int xpa_rollout_sample(int dist, int64_t n_envs, int64_t act_dim, int64_t horizon, const float *head,
                       const float *logstd, const float *v, const xpa_cursor_t *cursor, uint32_t seed,
                       float act_clip, float *buf_act, float *buf_logp, float *buf_val, float *env_in,
                       int64_t ld_env, xpa_stream_t stream);

/* K7 — SynthBox environment step (the synthetic env plugged in through the reference's NewEnv hook,
 * xuance/environment/__init__.py:76-78, replacing DummyVecEnv_Gym.step_wait, gym_vec_env.py:201-212).
 * pre[n, :] = W s_n + U a_n (a GEMM the caller runs on X = [s | env action] with Wcat = [W | U]).
 * s' = tanh(pre + noise * xi), r = -mean(s'^2), terminated = s'[0] > term_thresh,
 * truncated = episode_step + 1 >= max_episode_steps; done envs auto-reset (reset_obs semantics).
 * Writes final_obs (s'), state (X[:, :obs_dim], row stride ld_state: s' or the reset state),
 * rew, term, trunc, and the per-env episode counters. */
int xpa_synthbox_step(int64_t n_envs, int64_t obs_dim, const float *pre, uint32_t seed,
                      int32_t max_episode_steps, float noise, float term_thresh, float reset_scale,
                      float *state, int64_t ld_state, float *final_obs, float *rew, uint8_t *term,
                      uint8_t *trunc, int32_t *ep_step, uint32_t *ep_index, float *ep_score,
                      float *ep_last_score, int32_t *ep_last_len, xpa_stream_t stream);

/* K18 — CartPole-v1 environment step (BASELINE.json configs[0]; replaces DummyVecEnv_Gym.step_wait over gym's
 * CartPoleEnv, gym_vec_env.py:201-212; dynamics of gym 0.26.2 classic_control/cartpole.py with TimeLimit(500)).
 * One thread per env: f64 state [n_envs, 4], action = act_in[n * ld_act + 1] > 0.5 (the one-hot env input the
 * rollout kernels write), euler step, reward 1, terminated on |x| > 2.4 or |theta| > 12 deg, truncated at
 * max_episode_steps; done envs auto-reset with hashed uniform(-0.05, 0.05) states.  Writes final_obs (f32 image
 * of the stepped state), obs (row stride ld_obs: the state or the reset state), rew, term, trunc, counters. */
int xpa_cartpole_step(int64_t n_envs, const float *act_in, int64_t ld_act, double *state, float *obs,
                      int64_t ld_obs, float *final_obs, float *rew, uint8_t *term, uint8_t *trunc,
                      int32_t *ep_step, uint32_t *ep_index, float *ep_score, float *ep_last_score,
                      int32_t *ep_last_len, uint32_t seed, int32_t max_episode_steps, xpa_stream_t stream);

/* K32 — `steps` whole device env steps of a small-MLP Categorical PPO / A2C agent on CartPole in ONE launch (one
 * workgroup; the step loop of ppoclip_agent.py:43-101 / a2c_agent.py:42-98 with DummyVecEnv_Gym's auto-reset):
 * per step, obs_rms.update (xpa_rms_update's sums and merge, in its order), the normalisation into obs_norm and the
 * buffer column (xpa_obs_normalize), the policy forward — representation Linear(d_in, h0) + act, actor Linear(h0,
 * h1) + act -> Linear(h1, k), critic Linear(h0, h2) + act -> Linear(h2, 1) — K3's Categorical sample + stores
 * (xpa_rollout_sample), K18's CartPole step (xpa_cartpole_step) and K8's deferred-bootstrap post step with the
 * final-observation normalisation (xpa_rollout_post_deferred_norm); the cursor advances by `steps`.  Every stage
 * but the forward is the multi-kernel path's arithmetic bit for bit (the forward's dot products are f32 fma chains
 * in a fixed order).  Replaces ~10 launches per env step of the C1 configuration.  Limits: n_envs <= 256,
 * d_in == 4 (CartPole), h0 in {32, 64}, h1, h2 in {32, 64}, k == 2, xpa_small_rollout_lds_floats(...) <= 16384.
 * use_obsnorm = 0: the statistics are read, not updated (the agent's use_obsnorm False). */
typedef struct XpaSmallRolloutArgs {
    int n_envs, horizon, steps, d_in, h0, h1, h2, k, act_code, use_obsnorm, n_slots, mask_returns, use_rewnorm;
    int max_episode_steps;
    int slot_reset_obs; /* 1: a kept truncation row is the env's next (reset) observation (A2C, a2c_agent.py:88-95) */
    float slope, obs_clip, gamma, rew_range;
    uint32_t seed, env_seed;
    const float *W0, *b0, *W1, *b1, *W2, *b2, *Wa, *ba, *Wc, *bc;
    float *obs_mean, *obs_var;
    double *obs_count;
    float *obs_norm;
    int64_t ld_norm;
    float *buf_obs, *buf_act, *buf_logp, *buf_val, *buf_rew, *buf_term;
    uint8_t *buf_closed;
    float *buf_boot;
    float *act_in;
    int64_t ld_act;
    double *env_state;
    float *env_obs;
    int64_t ld_obs;
    float *final_obs, *env_rew;
    uint8_t *env_term, *env_trunc;
    int32_t *ep_step;
    uint32_t *ep_index;
    float *ep_score, *ep_last_score;
    int32_t *ep_last_len;
    float *returns, *ret_mean, *ret_var;
    double *ret_count;
    float *slot_obs;
    int32_t *slot_t, *overflow;
    float *boot_norm;
    int64_t ld_boot;
    xpa_cursor_t *cursor;
    int64_t *stamps; /* diagnostics (nullable): s_memtime cycles per phase summed over the steps, [9] */
} XpaSmallRolloutArgs;
int64_t xpa_small_rollout_lds_floats(int64_t n_envs, int64_t d_in, int64_t h0, int64_t h1, int64_t h2, int64_t k);
int xpa_small_rollout_cartpole(const XpaSmallRolloutArgs *args, xpa_stream_t stream);

/* K19 — PER-DQN TD target, loss, gradient and priorities (BASELINE.json configs[4]; replaces the tensor algebra
 * of PerDQN_Learner.update, xuance/torch/learners/qlearning_family/perdqn_learner.py:23-30, 48).
 * y = rew + (gamma * (1 - term)) * max_a targetQ[b, a]; p = evalQ[b, act[b]]; dQ[b, :] = one-hot(act[b]) * 2 (p - y) / B
 * (d mse / d evalQ); td_abs[b] = |y - p| (the new priorities for xpa_per_update_priorities);
 * scalars[0] = mean((p - y)^2) (Qloss), scalars[1] = mean(p) (predictQ).  act: float-coded indices; out-of-range
 * ones are clamped and counted into *err (may be NULL).  One block; deterministic. */
int xpa_dqn_td_loss(int64_t batch, int64_t n_actions, const float *evalQ, int64_t ld_eval, const float *targetQ,
                    int64_t ld_tgt, const float *act, const float *rew, const float *term, float gamma, float *dQ,
                    int64_t ld_dq, float *td_abs, float *scalars, int32_t *err, xpa_stream_t stream);

/* K8 — rollout post-step bookkeeping.  Replaces, per step, DummyOnPolicyBuffer.store of
 * rewards/terminals (memory_tools.py:196-204) with reward normalisation (agent.py:118-123), the
 * return tracker and ret_rms update (ppoclip_agent.py:87-92 with the (1-term) mask; a2c_agent.py:84
 * without), and the agent's path closing (ppoclip_agent.py:69-75, 89-101): closed/boot columns for
 * xpa_gae_scan (atari_lifeloss = 1: a terminal without truncation does not close the path,
 * ppoclip_agent.py:93-94).  Advances cursor->ptr (mod horizon) and cursor->step.
 * Workspace: partials = 3 * xpa_rollout_post_num_blocks(n_envs) doubles, ticket = one uint32 that is
 * 0 before the first call (the kernel leaves it at 0). */
int64_t xpa_rollout_post_num_blocks(int64_t n_envs);
int xpa_rollout_post(int64_t n_envs, int64_t horizon, const float *rew, const uint8_t *term,
                     const uint8_t *trunc, const float *v_boot, const float *v_boot_mid, xpa_cursor_t *cursor,
                     float *ret_mean,
                     float *ret_var, double *ret_count, float *returns, float *buf_rew, float *buf_term,
                     uint8_t *buf_closed, float *buf_boot, float gamma, int mask_returns, int use_rewnorm,
                     float rew_range, int atari_lifeloss, double *partials, uint32_t *ticket,
                     xpa_stream_t stream);

/* K9 — fused global-norm gradient clipping + Adam over flat fp32 buffers (all 16-B aligned).
 * Replaces torch.nn.utils.clip_grad_norm_ + torch.optim.Adam.step in PPOCLIP_Learner.update /
 * A2C_Learner.update (ppoclip_learner.py:47-49, a2c_learner.py:34-35) for the Adam(eps=1e-5) the runner
 * builds (xuance/torch/runners/runner_drl.py:71).  max_norm < 0 disables clipping (max_norm = 0 zeroes the gradient,
 * as clip_grad_norm_(params, 0) does).  step is the
 * 1-based Adam step count.  norm_partials: xpa_grad_norm_num_partials(n) doubles of scratch.
 * Writes the pre-clip total norm to *total_norm_out when non-NULL. */
int64_t xpa_grad_norm_num_partials(int64_t n);
int xpa_clip_adam_step(float *param, float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
                       double *norm_partials, float max_norm, float lr, float beta1, float beta2, float eps,
                       int64_t step, float *total_norm_out, xpa_stream_t stream);
/* K9 from squared-norm partials already written by the gradient producers (world size 1: the batched
 * column-sum finalize's per-tile partials + the loss finalize's d logstd share): no norm pass over the
 * flat gradient.  Same clip_grad_norm_ + Adam.step as xpa_clip_adam_step (ppoclip_learner.py:47-49,
 * a2c_learner.py:34-35).  sq_partials: n_sq doubles summing to |grad|^2; the clip + Adam arithmetic is
 * xpa_clip_adam_step's. */
int xpa_clip_adam_step_partials(float *param, float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
                                const double *sq_partials, int64_t n_sq, float max_norm, float lr, float beta1,
                                float beta2, float eps, int64_t step, float *total_norm_out, xpa_stream_t stream);
/* K9 with the learning rate and Adam step read from a device schedule, so that a captured update (forward + loss +
 * backward + this) can be replayed for the next update: sched[2k] = lr_k / (1 - beta1^step_k), sched[2k + 1] =
 * 1 / sqrt(1 - beta2^step_k) (xpa_adam_sched_entry computes an entry with xpa_clip_adam_step's arithmetic), k =
 * cursor[0]; cursor is int32[3] = {update index, block ticket (0 between launches), overflow flag}.  The launch
 * advances cursor[0] by one (its last block to finish reading); k >= n_sched is clamped to n_sched - 1 and sets
 * cursor[2].  The host refills sched and resets cursor once per window of updates (flat.FusedClipAdam). */
int xpa_clip_adam_step_sched(float *param, float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
                             double *norm_partials, float max_norm, float beta1, float beta2, float eps,
                             const float *sched, int64_t n_sched, int32_t *cursor, float *total_norm_out,
                             xpa_stream_t stream);
void xpa_adam_sched_entry(float lr, float beta1, float beta2, int64_t step, float *out2);

/* K30 — one whole PPO-Clip / A2C minibatch update of a small MLP actor-critic in ONE launch (one workgroup, every
 * activation in LDS): representation Linear(d_in, h0) + act, actor Linear(h0, h1) + act -> Linear(h1, k) (Categorical
 * logits), critic Linear(h0, h2) + act -> Linear(h2, 1).  Rows through idx from obs [n_rows, obs_ld] and the flat
 * act / old_logp / adv / ret buffers (memory_tools.py:230-243, with the minibatch adv normalisation when
 * use_advnorm), the forward, K2's categorical loss (the OUT_KEYS scalars into `scalars`), the backward (every
 * gradient into its view of the flat gradient buffer), clip_grad_norm_(max_norm; < 0: none) and Adam over the flat
 * buffers [0, n) with (lr, step) from the device schedule at cursor (xpa_clip_adam_step_sched's convention; the
 * launch advances cursor[0]).  Replaces ~25 launches per update of the C1 configuration (ppoclip_learner.py:24-65).
 * Limits: d_in <= 32, h0, h1, h2 multiples of 32 and <= 256, 2 <= k <= 16, xpa_small_mlp_lds_floats(...) <= 40704;
 * the flat buffers 16-B aligned with n % 4 == 0.  The products run on v_mfma_f32_32x32x2_f32 (exact f32 fma chains). */
typedef struct XpaSmallMlpArgs {
    int batch, d_in, h0, h1, h2, k, act_code, algo, use_advnorm, n_sched;
    float slope, clip_range, vf_coef, ent_coef, max_norm, beta1, beta2, eps;
    const float *obs;
    int64_t obs_ld;
    const int64_t *idx;
    int64_t n_rows;
    const float *actions, *old_logp, *adv, *ret;
    const float *W0, *b0, *W1, *b1, *W2, *b2, *Wa, *ba, *Wc, *bc;
    float *gW0, *gb0, *gW1, *gb1, *gW2, *gb2, *gWa, *gba, *gWc, *gbc;
    float *param, *grad, *exp_avg, *exp_avg_sq;
    int64_t n;
    const float *sched;
    int32_t *cursor;
    float *scalars, *total_norm_out;
    int64_t *stamps;   /* diagnostics (nullable): s_memtime at the kernel's phase boundaries, thread 0 */
    /* split form (n_groups = ceil(batch / 32) in [2, 16]; 0 or 1: one workgroup): workgroup g forms the forward /
     * backward of minibatch rows [32 g, 32 g + 32) and writes its partial gradients into grad_part[g * n ...] (at the
     * flat buffer's offsets; zero-initialised once, 16-B aligned) and its loss sums into loss_part[8 g ...]; a second
     * launch sums them in g order, clips and steps Adam. */
    int n_groups;
    float *grad_part;
    double *loss_part;
} XpaSmallMlpArgs;
int64_t xpa_small_mlp_lds_floats(int64_t batch, int64_t d_in, int64_t h0, int64_t h1, int64_t h2, int64_t k);
int xpa_small_mlp_update(const XpaSmallMlpArgs *args, xpa_stream_t stream);

/* K10 — activation backward fused with bias-gradient column sums for one MLP layer (row-major
 * [rows, cols]).  Replaces the activation backward and the bias-gradient reduction torch autograd runs
 * per mlp_block (xuance/torch/utils/layers.py:8-24) inside loss.backward() (ppoclip_learner.py:46).
 * act: 0 = identity (column sums of dh only; dz unused), 1 = LeakyReLU/ReLU (mask from the activation
 * output h, slope), 2 = tanh (1 - h^2).  dz = dh * act'(h) (dz may alias dh; NULL = do not store);
 * partials: xpa_act_bwd_num_partials(rows) x cols floats; xpa_colsum_finalize sums them in a fixed
 * order into out[cols] (the bias gradient). */
int64_t xpa_act_bwd_num_partials(int64_t rows);
int xpa_act_bwd_colsum(int act, const float *dh, const float *h, int64_t rows, int64_t cols, float slope,
                       float *dz, float *partials, xpa_stream_t stream);
int xpa_colsum_finalize(const float *partials, int64_t n_partials, int64_t cols, float *out,
                        xpa_stream_t stream);

/* K11 — backward of a thin output layer (k <= 32 outputs, weight w [k, hidden], no activation) fused
 * with the activation backward of the hidden layer feeding it (output h [rows, hidden]): the tail
 * of the actor / critic heads (gaussian.py:8-51, categorical.py:16-58).  Given d_head [rows, k]
 * (row stride ldd): dz = (d_head w) * act'(h) [rows, hidden]; per-block partials of
 * dW = d_head^T h (xpa_head_bwd_num_partials(rows) x k x hidden), of the hidden bias gradient (x hidden)
 * and of the output bias gradient (x k; NULL = skip); reduce each with xpa_colsum_finalize. */
int64_t xpa_head_bwd_num_partials(int64_t rows);
int xpa_head_backward(int act, int64_t k, const float *d_head, int64_t ldd, const float *h, const float *w,
                      int64_t rows, int64_t hidden, float slope, float *dz, float *partial_dw,
                      float *partial_db_hidden, float *partial_db_out, xpa_stream_t stream);

/* K12 — fused head: hidden activation + output Linear + loss + backward in one pass per head.
 * Replaces, for a head [Linear(., 256) + act] -> [Linear(256, K)], the tail of the forward
 * (gaussian.py:8-51 / categorical.py:16-58), the loss of PPOCLIP_Learner.update
 * (ppoclip_learner.py:32-44) / A2C_Learner.update (a2c_learner.py:24-31) and autograd's backward down
 * to the hidden pre-activation z [batch, 256] (ppoclip_learner.py:46).  Per-row inputs
 * (act, old_logp, adv, ret) are read at idx[b] (idx NULL: at b) with the same adv normalisation,
 * tie rules and invalid-index behaviour as xpa_policy_loss_fwd_bwd.  Outputs: dz [batch, 256]; per-block
 * partials (xpa_head_fused_num_partials(batch) rows) of dW_out (x K*256), db_hidden (x 256) and db_out
 * (x K) for xpa_colsum_finalize, and one loss-partials row per block in xpa_policy_loss_fwd_bwd's
 * layout (width >= xpa_loss_partial_width(K)): the actor kernel fills the surrogate / entropy / clip /
 * dlogstd columns, the critic kernel the squared-error / value columns, so one
 * xpa_policy_loss_finalize over the shared array yields the loss scalars and d logstd.
 * act: 0 identity, 1 LeakyReLU(slope) / ReLU (slope 0), 2 tanh.  K <= 18; hidden must be 256; z and dz
 * rows have stride ld (>= 256, multiple of 4); z and w 16-B aligned. */
int64_t xpa_head_fused_num_partials(int64_t batch);
int xpa_head_fused_actor(int algo, int dist, int act, int64_t batch, int64_t act_dim, int64_t hidden, int64_t ld,
                         const float *z, const float *w, const float *b, float slope, const float *logstd,
                         const int64_t *idx, int64_t n_rows, const float *act_buf, const float *old_logp,
                         const float *adv, const double *adv_partials, int64_t n_adv_partials, float clip_range,
                         float ent_coef, float *dz, float *partial_dw, float *partial_db_hidden,
                         float *partial_db_out, float *loss_partials, int64_t loss_width, xpa_stream_t stream);
int xpa_head_fused_critic(int act, int64_t batch, int64_t hidden, int64_t ld, const float *z, const float *w, const float *b,
                          float slope, const int64_t *idx, int64_t n_rows, const float *ret, float vf_coef,
                          float *dz, float *partial_dw, float *partial_db_hidden, float *partial_db_out,
                          float *loss_partials, int64_t loss_width, xpa_stream_t stream);

/* Batched xpa_colsum_finalize: out_i[c] = sum over the n_partials[i] rows of partials_i[:, c] for
 * up to 16 segments in one launch (host arrays of n_segs entries; the pointers they hold are device
 * pointers).  Same fixed-order f64 sums as xpa_colsum_finalize. */
int xpa_colsum_finalize_batch(int n_segs, const float *const *partials, const int64_t *n_partials,
                              const int64_t *cols, float *const *outs, xpa_stream_t stream);
/* Column tiles (= blocks) of one batched finalize over these segments (n_partials rows x cols). */
int64_t xpa_colsum_batch_tiles(int n_segs, const int64_t *n_partials, const int64_t *cols);
/* xpa_colsum_finalize_batch that also produces the clip norm of its outputs: sq (nullable; tiles + 2
 * doubles) holds at sq[0] a share written beforehand (e.g. xpa_policy_loss_finalize_sq's d logstd); each
 * tile writes its sum of squared outputs to sq[1 + tile], and the last block to finish (atomic tickets,
 * int32 [XPA_COLSUM_TICKET_INTS], zero-initialised and left at zero) writes the fixed-order total of sq[0 .. tiles] to
 * sq[1 + tiles] — the single partial xpa_clip_adam_step_partials then reads. */
int xpa_colsum_finalize_batch_sq(int n_segs, const float *const *partials, const int64_t *n_partials,
                                 const int64_t *cols, float *const *outs, double *sq, int32_t *ticket,
                                 xpa_stream_t stream);
/* xpa_colsum_finalize_batch_sq with xpa_policy_loss_finalize_sq run by one extra (last) block of the same
 * launch: the loss scalars and d logstd as that call writes them, its d logstd share of the clip norm in
 * sq[0] (so sq[0] need not be written beforehand).  sq and ticket are required. */
int xpa_colsum_finalize_batch_sq_loss(int n_segs, const float *const *partials, const int64_t *n_partials,
                                      const int64_t *cols, float *const *outs, double *sq, int32_t *ticket, int algo,
                                      int dist, int64_t batch, int64_t act_dim, const float *loss_partials,
                                      int64_t n_loss_partials, float vf_coef, float ent_coef, float *scalars,
                                      float *d_logstd, xpa_stream_t stream);

/* K14 — rollout policy head: the last hidden activation and both output layers of the actor-critic
 * (gaussian.py:8-51 / categorical.py:16-58 forward in PPOCLIP_Agent._action, ppoclip_agent.py:50-57)
 * fused with xpa_rollout_sample: z_actor / z_critic [n_envs, 256] are the hidden pre-activations
 * (row stride ld, e.g. the halves of a paired [n, 512] GEMM output); the value and mu / logits are
 * formed in the kernel and the sample / log-prob / value / env input are stored exactly as
 * xpa_rollout_sample does (same RNG stream).  act_dim <= 32.
 * xpa_value_head: v_out[n] = act(z_critic) . w_critic + b_critic alone (the bootstrap value of
 * ppoclip_agent.py:77-81 on the normalised final observations). */
int xpa_rollout_policy_head(int dist, int act, int64_t n_envs, int64_t act_dim, int64_t horizon, int64_t hidden,
                            int64_t ld, const float *z_actor, const float *z_critic, float slope,
                            const float *w_actor, const float *b_actor, const float *w_critic,
                            const float *b_critic, const float *logstd, const xpa_cursor_t *cursor, uint32_t seed,
                            float act_clip, float *buf_act, float *buf_logp, float *buf_val, float *env_in,
                            int64_t ld_env, xpa_stream_t stream);
int xpa_value_head(int act, int64_t n, int64_t hidden, int64_t ld, const float *z_critic, float slope,
                   const float *w_critic, const float *b_critic, float *v_out, xpa_stream_t stream);
/* K14 (Gaussian) with the SynthBox env step of the same env fused after the sample — the agent's
 * `self.envs.step(acts)` right after `self._action(obs)` (ppoclip_agent.py:65-66) in one launch (K7's arithmetic; the
 * env pre-activation [W | U] (s | clip(a)) as a fixed-order fmaf chain from the state row and the sampled
 * actions instead of the env GEMM): one launch in place of K14 + env GEMM + xpa_synthbox_step.  state: the
 * env's [n_envs, ld_state] input rows (s | a), obs_dim <= 64 state columns followed by act_dim action
 * columns (written with the clipped actions, as env_in); wcat_t: [W | U]^T, [obs_dim + act_dim, obs_dim];
 * the env arguments are xpa_synthbox_step's. */
int xpa_rollout_policy_head_synthbox(int act, int64_t n_envs, int64_t act_dim, int64_t horizon, int64_t hidden,
                                     int64_t ld, const float *z_actor, const float *z_critic, float slope,
                                     const float *w_actor, const float *b_actor, const float *w_critic,
                                     const float *b_critic, const float *logstd, const xpa_cursor_t *cursor,
                                     uint32_t seed, float act_clip, float *buf_act, float *buf_logp, float *buf_val,
                                     int64_t obs_dim, const float *wcat_t, uint32_t env_seed,
                                     int32_t max_episode_steps, float noise, float term_thresh, float reset_scale,
                                     float *state, int64_t ld_state, float *final_obs, float *rew, uint8_t *term,
                                     uint8_t *trunc, int32_t *ep_step, uint32_t *ep_index, float *ep_score,
                                     float *ep_last_score, int32_t *ep_last_len, xpa_stream_t stream);

/* K16 — K12 with the hidden layer's GEMM on the fp32 matrix cores (v_mfma_f32_32x32x2_f32): the
 * pre-activations z = x w_hidden^T + b_hidden of each [64 x 256] tile are formed in registers and never
 * written to HBM; the rest is exactly K12 (same outputs, partial layouts and loss-partials columns).
 * x: the hidden layer's input [batch, 256] (row stride ldx); w_hidden [256, 256] row-major (the
 * Linear's weight), b_hidden [256]; dz rows have stride ld_dz. */
int xpa_head_gemm_actor(int algo, int dist, int act, int64_t batch, int64_t act_dim, int64_t hidden, const float *x,
                        int64_t ldx, const float *w_hidden, const float *b_hidden, int64_t ld_dz, const float *w,
                        const float *b, float slope, const float *logstd, const int64_t *idx, int64_t n_rows,
                        const float *act_buf, const float *old_logp, const float *adv, const double *adv_partials,
                        int64_t n_adv_partials, float clip_range, float ent_coef, float *dz, float *partial_dw,
                        float *partial_db_hidden, float *partial_db_out, float *loss_partials, int64_t loss_width,
                        xpa_stream_t stream);
int xpa_head_gemm_critic(int act, int64_t batch, int64_t hidden, const float *x, int64_t ldx, const float *w_hidden,
                         const float *b_hidden, int64_t ld_dz, const float *w, const float *b, float slope,
                         const int64_t *idx, int64_t n_rows, const float *ret, float vf_coef, float *dz,
                         float *partial_dw, float *partial_db_hidden, float *partial_db_out, float *loss_partials,
                         int64_t loss_width, xpa_stream_t stream);

/* K16W — K16 on one 512-thread block per CU with specialised waves: 4 run the hidden GEMM of tile n + 1 on the
 * matrix cores while 2 run the K12 epilogue of tile n and 2 issue the operand DMAs (the epilogue overlaps the GEMM
 * by construction).  Same arguments, outputs, partial rows (xpa_head_fused_num_partials; rows beyond its grid of
 * xpa_head_gemm_ws_grid(batch) <= 256 blocks are written as zeros) and arithmetic as xpa_head_gemm_actor / _critic,
 * bit for bit; act_dim <= 8. */
int64_t xpa_head_gemm_ws_grid(int64_t batch);
int xpa_head_gemm_ws_probe(int mask); /* diagnostics: parts of K16W switched off (tools/k16w_ab.py); 0 = production */
/* test support: fill every CU's LDS with NaN bit patterns, so a following kernel that reads LDS it did not write
 * produces NaN (tests/test_gpu_fused_mlp.py) */
int xpa_lds_poison(xpa_stream_t stream);
int xpa_head_gemm_ws_actor(int algo, int dist, int act, int64_t batch, int64_t act_dim, int64_t hidden, const float *x,
                           int64_t ldx, const float *w_hidden, const float *b_hidden, int64_t ld_dz, const float *w,
                           const float *b, float slope, const float *logstd, const int64_t *idx, int64_t n_rows,
                           const float *act_buf, const float *old_logp, const float *adv, const double *adv_partials,
                           int64_t n_adv_partials, float clip_range, float ent_coef, float *dz, float *partial_dw,
                           float *partial_db_hidden, float *partial_db_out, float *loss_partials, int64_t loss_width,
                           xpa_stream_t stream);
int xpa_head_gemm_ws_critic(int act, int64_t batch, int64_t hidden, const float *x, int64_t ldx,
                            const float *w_hidden, const float *b_hidden, int64_t ld_dz, const float *w, const float *b,
                            float slope, const int64_t *idx, int64_t n_rows, const float *ret, float vf_coef, float *dz,
                            float *partial_dw, float *partial_db_hidden, float *partial_db_out, float *loss_partials,
                            int64_t loss_width, xpa_stream_t stream);

/* K16S — K16 with the hidden GEMM on the bf16 matrix cores by the three-way split of K40 (xpa_s3_gemm): the same
 * arguments, outputs and epilogue as xpa_head_gemm_actor / _critic; the GEMM carries the f32 GEMM's error (not K16's
 * bits) at 6/16 of its matrix-core cycles. */
int xpa_head_gemm_s3_actor(int algo, int dist, int act, int64_t batch, int64_t act_dim, int64_t hidden, const float *x,
                           int64_t ldx, const float *w_hidden, const float *b_hidden, int64_t ld_dz, const float *w,
                           const float *b, float slope, const float *logstd, const int64_t *idx, int64_t n_rows,
                           const float *act_buf, const float *old_logp, const float *adv, const double *adv_partials,
                           int64_t n_adv_partials, float clip_range, float ent_coef, float *dz, float *partial_dw,
                           float *partial_db_hidden, float *partial_db_out, float *loss_partials, int64_t loss_width,
                           xpa_stream_t stream);
int xpa_head_gemm_s3_critic(int act, int64_t batch, int64_t hidden, const float *x, int64_t ldx,
                            const float *w_hidden, const float *b_hidden, int64_t ld_dz, const float *w, const float *b,
                            float slope, const int64_t *idx, int64_t n_rows, const float *ret, float vf_coef, float *dz,
                            float *partial_dw, float *partial_db_hidden, float *partial_db_out, float *loss_partials,
                            int64_t loss_width, xpa_stream_t stream);

/* K16P — K16S with w_hidden replaced by the three bf16 planes of Wh^T (xpa_s3_split_b(w_hidden, 256, 256, 1, 256, out):
 * split once per update) DMA'd as they are; the other arguments, outputs and arithmetic are K16S's. */
int xpa_head_gemm_s3p_actor(int algo, int dist, int act, int64_t batch, int64_t act_dim, int64_t hidden, const float *x,
                            int64_t ldx, const float *w_hidden_split, const float *b_hidden, int64_t ld_dz,
                            const float *w, const float *b, float slope, const float *logstd, const int64_t *idx,
                            int64_t n_rows, const float *act_buf, const float *old_logp, const float *adv,
                            const double *adv_partials, int64_t n_adv_partials, float clip_range, float ent_coef,
                            float *dz, float *partial_dw, float *partial_db_hidden, float *partial_db_out,
                            float *loss_partials, int64_t loss_width, xpa_stream_t stream);
int xpa_head_gemm_s3p_critic(int act, int64_t batch, int64_t hidden, const float *x, int64_t ldx,
                             const float *w_hidden_split, const float *b_hidden, int64_t ld_dz, const float *w,
                             const float *b, float slope, const int64_t *idx, int64_t n_rows, const float *ret,
                             float vf_coef, float *dz, float *partial_dw, float *partial_db_hidden,
                             float *partial_db_out, float *loss_partials, int64_t loss_width, xpa_stream_t stream);
/* K16Q (r04) — K16P's arguments and outputs bit for bit with the waves tiled 32 rows x 128 columns (one A fragment
 * split per wave and chunk instead of two). */
int xpa_head_gemm_s3q_actor(int algo, int dist, int act, int64_t batch, int64_t act_dim, int64_t hidden, const float *x,
                            int64_t ldx, const float *w_hidden_split, const float *b_hidden, int64_t ld_dz,
                            const float *w, const float *b, float slope, const float *logstd, const int64_t *idx,
                            int64_t n_rows, const float *act_buf, const float *old_logp, const float *adv,
                            const double *adv_partials, int64_t n_adv_partials, float clip_range, float ent_coef,
                            float *dz, float *partial_dw, float *partial_db_hidden, float *partial_db_out,
                            float *loss_partials, int64_t loss_width, xpa_stream_t stream);
int xpa_head_gemm_s3q_critic(int act, int64_t batch, int64_t hidden, const float *x, int64_t ldx,
                             const float *w_hidden_split, const float *b_hidden, int64_t ld_dz, const float *w,
                             const float *b, float slope, const int64_t *idx, int64_t n_rows, const float *ret,
                             float vf_coef, float *dz, float *partial_dw, float *partial_db_hidden,
                             float *partial_db_out, float *loss_partials, int64_t loss_width, xpa_stream_t stream);

/* K16X — K16 with the representation's first layer Linear(d_in <= 20, 256) + activation `act` (K13's, bit for bit)
 * in the prologue: each block forms its tile's h rows from the minibatch's gathered observation rows x_rows
 * [batch, d_in] (row stride ld_rows; e.g. xpa_thin_linear_act_fwd_gather with h = NULL), w_in [256, d_in], b_in [256],
 * writes them to h_out (required; row stride ld_h: the backward's copy) and runs K16's k loop on them (A operand read
 * back from L2).  Otherwise exactly K16 (act_dim <= 8).  The learner's critic then runs plain K16 on h_out. */
int xpa_head_gemm_trunk_actor(int algo, int dist, int act, int64_t batch, int64_t act_dim, int64_t hidden,
                              const float *x_rows, int64_t ld_rows, int64_t d_in, const float *w_in, const float *b_in,
                              float slope_in, float *h_out, int64_t ld_h, const float *w_hidden, const float *b_hidden,
                              int64_t ld_dz, const float *w, const float *b, float slope, const float *logstd,
                              const int64_t *idx, int64_t n_rows, const float *act_buf, const float *old_logp,
                              const float *adv, const double *adv_partials, int64_t n_adv_partials, float clip_range,
                              float ent_coef, float *dz, float *partial_dw, float *partial_db_hidden,
                              float *partial_db_out, float *loss_partials, int64_t loss_width, xpa_stream_t stream);
int xpa_head_gemm_trunk_critic(int act, int64_t batch, int64_t hidden, const float *x_rows, int64_t ld_rows,
                               int64_t d_in, const float *w_in, const float *b_in, float slope_in, float *h_out,
                               int64_t ld_h, const float *w_hidden, const float *b_hidden, int64_t ld_dz, const float *w,
                               const float *b, float slope, const int64_t *idx, int64_t n_rows, const float *ret,
                               float vf_coef, float *dz, float *partial_dw, float *partial_db_hidden,
                               float *partial_db_out, float *loss_partials, int64_t loss_width, xpa_stream_t stream);

/* K40 — f32 GEMM on the bf16 matrix cores by a three-way split of each f32 operand into bf16 (hi + mid + lo, exact)
 * and the six products above 2^-24 relative (csrc/sgemm3.hip): the f32 GEMM's accuracy at 2.67x the f32 MFMA rate.
 * Replaces the hidden-layer matmuls of loss.backward() in PPOCLIP_Learner.update (ppoclip_learner.py:40-46) /
 * A2C_Learner.update (a2c_learner.py:33-39) — here dX of the paired hidden layer, dz_pair [B, 512] . Wh_pair [512, 256].
 * xpa_s3_split_b: B [k, n] with element (i, j) at b[i * sk + j * sn] -> out (xpa_s3_split_bytes(k, n) bytes, 16-B
 *   aligned), the three bf16 planes in the GEMM's operand order; k % 16 == 0, n == 256.
 * xpa_s3_gemm: c [m, 256] (row stride ldc) = a [m, k] (f32, row stride lda, 16-B aligned rows) . B, from B's split. */
int64_t xpa_s3_split_bytes(int64_t k, int64_t n);
int xpa_s3_probe(int mask); /* diagnostics: parts of K40 / K41 switched off (tools/s3_ab.py --probe); 0 = production */
int xpa_s3_split_b(const float *b, int64_t k, int64_t n, int64_t sk, int64_t sn, void *out, xpa_stream_t stream);
/* n_mat <= 4 splits (n = 256 each) in one launch: the arrays hold each matrix's pointer, k, strides and output */
int xpa_s3_split_batch(int n_mat, const float *const *b, const int64_t *k, const int64_t *sk, const int64_t *sn,
                       void *const *out, xpa_stream_t stream);
int xpa_s3_gemm(const float *a, int64_t lda, const void *b_split, float *c, int64_t ldc, int64_t m, int64_t k, int64_t n,
                xpa_stream_t stream);
/* K40G (r05): n <= 32 problems c[p] [m, 256] (row stride ldc) = a[p] [m, k] (row stride lda, 16-B aligned) . B[p]
 * (xpa_s3_split_b planes) of one shape in ONE launch (grid (m / 256) x n): the column blocks and k parts of a GEMM wider
 * than 256 columns (C3's fc layer).  Host arrays of device pointers; each problem's output is xpa_s3_gemm's bit for
 * bit. */
int xpa_s3_gemm_group(int n, const float *const *a, const void *const *b_split, float *const *c, int64_t lda,
                      int64_t ldc, int64_t m, int64_t k, xpa_stream_t stream);
/* K40G with the previous block's activation backward (r05, C3's fc data gradient into conv3): c[p] = (a[p] . B[p]) x
 * act'(y[p]) (act 0 identity / 1 LeakyReLU(slope) from the output y / 2 tanh; y[p] at c[p]'s offsets, row stride
 * ldc), equal to xpa_act_bwd_bias's dz bit for bit, and per (problem, 256-row block) the column sums of c[p] per
 * channel (column mod channels; channels 32 or 64, every c[p] starting at a multiple of channels columns) in
 * bias_partial [xpa_s3_gemm_group_act_num_partials(n, m)][channels] for xpa_colsum_finalize.  K22 folded in. */
int64_t xpa_s3_gemm_group_act_num_partials(int n, int64_t m);
int xpa_s3_gemm_group_act(int n, const float *const *a, const void *const *b_split, float *const *c,
                          const float *const *y, int64_t lda, int64_t ldc, int64_t m, int64_t k, int act, float slope,
                          int64_t channels, float *bias_partial, xpa_stream_t stream);
/* K41 — the weight gradient dW = a^T b over the batch on the same split (a [rows, m] = dz, row stride lda; b [rows, 256]
 * = the layer input, row stride ldb; m % 128 == 0), split-K: out [slices, m, 256] holds one partial per slice of
 * ceil(rows / slices) rows (rounded up to 32), summed by the caller — the learner's fixed-order f64 finalize, as for
 * the batched f32 GEMM it replaces.  xpa_s3_wgrad_num_slices: the slice count that fills the chip (0: bad shape). */
int64_t xpa_s3_wgrad_num_slices(int64_t rows, int64_t m);
/* K42 — xpa_s3_gemm's g = dz . B kept in registers and the first representation layer's backward (K13's,
 * xpa_thin_linear_act_bwd) done on it: dz1 = g * act'(h) (h [rows, 256] = the layer's output, act as K13), per-block
 * partials of db1 [G, 256] and dW1 [G, 256 * d_in] (x [rows, d_in] = the layer's input rows, d_in <= 32);
 * G = xpa_s3_gemm_trunk_bwd_num_partials(rows).  g itself is never written. */
int64_t xpa_s3_gemm_trunk_bwd_num_partials(int64_t rows);
int xpa_s3_gemm_trunk_bwd(const float *dz, int64_t ldz, const void *b_split, int64_t k, const float *h, int64_t ldh,
                          const float *x, int64_t ldx, int64_t rows, int64_t d_in, int act, float slope,
                          float *partial_dw, float *partial_db, xpa_stream_t stream);
int xpa_s3_wgrad(const float *a, int64_t lda, const float *b, int64_t ldb, int64_t rows, int64_t m, int64_t n,
                 int64_t slices, float *out, xpa_stream_t stream);
/* K42S (r04): xpa_s3_gemm_trunk_bwd with act' taken from h's sign bits (h_sign: 32 bytes per row, byte b bit j =
 * h[row, 32 j + b] > 0, as xpa_head_gemm_s3r_actor writes them) instead of h; act 0 (identity) or 1 (LeakyReLU /
 * ReLU).  The same outputs bit for bit; 32 B instead of 1 KiB read per row. */
int xpa_s3_gemm_trunk_bwd_sign(const float *dz, int64_t ldz, const void *b_split, int64_t k, const unsigned *h_sign,
                               const float *x, int64_t ldx, int64_t rows, int64_t d_in, int act, float slope,
                               float *partial_dw, float *partial_db, xpa_stream_t stream);
/* r05 — the critic's factored backward (LeakyReLU / ReLU hidden layer, one output unit: dz_c[r, c] = dv[r] wc[c]
 * (slope + (1 - slope) m[r, c]), m = [h_c > 0]), replacing the critic's half of the paired hidden layer's dX and dW
 * inside loss.backward() of PPOCLIP_Learner.update / A2C_Learner.update (ppoclip_learner.py:40-46, a2c_learner.py:33-39)
 * by masked GEMMs whose mask operand is exact in bf16 (three split products instead of six) and never storing dz_c.
 * xpa_head_gemm_s3q_critic_mask: xpa_head_gemm_s3q_critic that also writes the hidden activations' sign bits
 *   (mask [batch][8] u32, bit c & 31 of word c >> 5 = h[row, c] > 0) and d loss / d v per row (dv [batch]); dz may be
 *   NULL (not stored).
 * xpa_s3_split_batch_scaled: xpa_s3_split_batch with matrix i's rows k >= rs_from[i] scaled by rs_a[i] *
 *   rs_w[i][k - rs_from[i]] before the split (rs_w[i] NULL: none), and with cs_out, cs_out[j] = cs_slope * sum_c
 *   rs_w[c] B[rs_from + c][j] for the first scaled matrix.
 * xpa_s3_gemm_trunk_bwd_crit: K42S with the critic's half of g = dz_pair . Wh_pair as dv[r] (m . V + cs), V = (1 -
 *   slope) diag(wc) Wh_c and cs = slope wc . Wh_c (b_split = the scaled split of [Wh_a; Wh_c], k_a + k_c rows).
 * xpa_s3_wgrad_pair: the paired layer's weight-gradient slices, out_a [sa, 256, 256] of dz_a^T h and out_c
 *   [sc, 256, 256] of wc[c] ((1 - slope) m^T Y + slope colsum(Y)), Y = dv (.) h; slice counts and rows per slice from
 *   xpa_s3_wgrad_pair_slices. */
int xpa_head_gemm_s3q_critic_mask(int act, int64_t batch, int64_t hidden, const float *x, int64_t ldx,
                                  const float *w_hidden_split, const float *b_hidden, int64_t ld_dz, const float *w,
                                  const float *b, float slope, const int64_t *idx, int64_t n_rows, const float *ret,
                                  float vf_coef, float *dz, float *partial_dw, float *partial_db_hidden,
                                  float *partial_db_out, float *loss_partials, int64_t loss_width, xpa_stream_t stream,
                                  unsigned *mask, float *dv);
int xpa_s3_split_batch_scaled(int n_mat, const float *const *b, const int64_t *k, const int64_t *sk, const int64_t *sn,
                              void *const *out, const float *const *rs_w, const float *rs_a, const int64_t *rs_from,
                              float *cs_out, float cs_slope, xpa_stream_t stream);
int xpa_s3_gemm_trunk_bwd_crit(const float *dz_a, int64_t ldz, const void *b_split, int64_t k_a, int64_t k_c,
                               const unsigned *crit_mask, const float *crit_dv, const float *crit_cs,
                               const unsigned *h_sign, const float *x, int64_t ldx, int64_t rows, int64_t d_in, int act,
                               float slope, float *partial_dw, float *partial_db, xpa_stream_t stream);
int xpa_s3_wgrad_pair_slices(int64_t rows, int64_t *sa, int64_t *sc, int64_t *per_a, int64_t *per_c);
int xpa_s3_wgrad_pair_tune(int sa_target); /* the actor's share of 128 slices (default 68) */
int xpa_s3_wgrad_pair(const float *dz_a, int64_t lda, const float *h, int64_t ldb, int64_t rows,
                      const unsigned *crit_mask, const float *crit_dv, const float *crit_wc, float crit_slope,
                      int64_t sa, int64_t per_a, int64_t sc, int64_t per_c, float *out_a, float *out_c,
                      xpa_stream_t stream);
/* r05 — a wide representation layer (C4: Linear(376, 256) + LeakyReLU, mlp_block of layers.py:8-24 inside
 * ppoclip_learner.py:31-33's policy(obs) and its loss.backward()) on the split GEMMs instead of the f32 library GEMMs:
 * xpa_gather_minibatch_pitched: K4 into rows of pitch out_row_bytes (the pitch's tail untouched: a zero pad stays zero).
 * xpa_s3_split_batch_padded: xpa_s3_split_batch where matrix i holds kv[i] <= k[i] rows, rows kv .. k - 1 split as 0.
 * xpa_s3_gemm_bias_act (K40F): C = act(A . B + bias), act 0 identity / 1 LeakyReLU / 2 tanh, with sign_out (act 0 / 1,
 *   nullable) the output's sign bits (the h_sign layout of xpa_s3_gemm_trunk_bwd_sign).
 * xpa_s3_gemm_trunk_bwd_dz (K42W) / xpa_s3_gemm_trunk_bwd_crit_dz: K42S / K42C whose epilogue stores dz1 = g act'(h)
 *   [rows, 256] (ld_out) and the db1 partials [G, 256] instead of the thin layer's dW (that comes from xpa_s3_wgrad on
 *   the padded rows and dz1, i.e. dW^T slices [S, k_pad, 256]).
 * xpa_colsum_finalize_batch_map: xpa_colsum_finalize_batch(_sq(_loss)) with per-segment output maps tmap [n][3] =
 *   (inner, valid, ld): inner 0 = identity, else partial column r inner + i -> out[i ld + r] for r < valid (dropped
 *   otherwise) — K41V's dW^T slices finalized straight into W [256][376]; loss_partials NULL: no loss block. */
/* r05: xpa_rollout_post_deferred_norm with the NEXT step's obs_rms.update folded in (ppoclip_agent.py:62-63: the
 * reference updates obs_rms with each observation before acting on it): rms_x [n_envs, obs_dim] (row stride rms_ld) =
 * the observation the env step just produced; rms_part f64 [2 * xpa_rollout_post_num_blocks(n_envs), obs_dim];
 * obs_mean / obs_var / obs_count updated in place by the last block after every block normalised with the old
 * statistics.  obs_dim <= 64.  The next step then normalises without an rms launch of its own. */
int xpa_rollout_post_deferred_norm_rms(
    int64_t n_envs, int64_t horizon, const float *rew, const uint8_t *term, const uint8_t *trunc, const float *final_obs,
    int64_t ld_final, const float *slot_src, int64_t ld_slot, int64_t obs_dim, float *obs_mean, float *obs_var,
    double *obs_count, float obs_clip, float *boot_norm, int64_t ld_norm, float *slot_obs, int32_t *slot_t,
    int64_t n_slots, int32_t *overflow, xpa_cursor_t *cursor, float *ret_mean, float *ret_var, double *ret_count,
    float *returns, float *buf_rew, float *buf_term, uint8_t *buf_closed, float *buf_boot, float gamma,
    int mask_returns, int use_rewnorm, float rew_range, int atari_lifeloss, double *partials, uint32_t *ticket,
    const float *rms_x, int64_t rms_ld, double *rms_part, xpa_stream_t stream);
/* r05, the row-index forms of K40F / K41V (C4's wide trunk straight from the rollout buffer, no gathered copy): A's
 * row r is row idx[r] of a; k (K40F) / m (K41V) may exceed a's row width (a zero-padded B, or output rows the caller
 * drops) when the buffer has readable, finite slack after its last row.  K41V: rows per slice <= 1536. */
int xpa_s3_gemm_bias_act_rows(const float *a, int64_t lda, const int64_t *ridx, const void *b_split, float *c,
                              int64_t ldc, int64_t m, int64_t k, const float *bias, int act, float slope,
                              unsigned *sign_out, xpa_stream_t stream);
int xpa_s3_wgrad_rows(const float *a, int64_t lda, const int64_t *aidx, const float *b, int64_t ldb, int64_t rows,
                      int64_t m, int64_t n, int64_t slices, float *out, xpa_stream_t stream);
/* r06 — K41V over rows narrower than its 128-row output tiles (C3's first fc layer: dW^T = flat^T g, flat [B, 3136]):
 * m <= lda + 127; the last tile reads past each row, and after the last row into slack the caller keeps readable and
 * finite; those output rows are garbage for the caller's finalize map to drop.  Replaces the fc weight gradient of
 * loss.backward() through AC_CNN_Atari's first Linear (xuance/torch/representations/cnn.py:45-93). */
int xpa_s3_wgrad_padded(const float *a, int64_t lda, const float *b, int64_t ldb, int64_t rows, int64_t m, int64_t n,
                        int64_t slices, float *out, xpa_stream_t stream);
/* K40R (r05): the rollout's paired hidden layer z [m, 512] = x [m, 256] . [B0 | B1] + bias on the split (B0 / B1 =
 * Wh_actor^T / Wh_critic^T split by xpa_s3_split_b, k = 256): 64-row x 128-column blocks for the rollout's few rows
 * (ppoclip_agent.py:63 self.action(obs) -> the policy's hidden layers); each output equals xpa_s3_gemm's + bias. */
int xpa_s3_gemm_rows_pair(const float *a, int64_t lda, const void *b0_split, const void *b1_split, const float *bias,
                          float *c, int64_t ldc, int64_t m, xpa_stream_t stream);
int xpa_gather_minibatch_pitched(const int64_t *idx, int64_t batch, int64_t n_rows, const void *obs,
                                 int64_t obs_row_bytes, void *obs_out, int64_t out_row_bytes, const float *adv,
                                 double *adv_partials, int32_t *err, xpa_stream_t stream);
int xpa_s3_split_batch_padded(int n_mat, const float *const *b, const int64_t *k, const int64_t *kv, const int64_t *sk,
                              const int64_t *sn, void *const *out, xpa_stream_t stream);
int xpa_s3_gemm_bias_act(const float *a, int64_t lda, const void *b_split, float *c, int64_t ldc, int64_t m, int64_t k,
                         const float *bias, int act, float slope, unsigned *sign_out, xpa_stream_t stream);
int xpa_s3_gemm_trunk_bwd_dz(const float *dz, int64_t ldz, const void *b_split, int64_t k, const unsigned *h_sign,
                             int64_t rows, int act, float slope, float *dz_out, int64_t ld_out, float *partial_db,
                             xpa_stream_t stream);
int xpa_s3_gemm_trunk_bwd_crit_dz(const float *dz_a, int64_t ldz, const void *b_split, int64_t k_a, int64_t k_c,
                                  const unsigned *crit_mask, const float *crit_dv, const float *crit_cs,
                                  const unsigned *h_sign, int64_t rows, int act, float slope, float *dz_out,
                                  int64_t ld_out, float *partial_db, xpa_stream_t stream);
int xpa_colsum_finalize_batch_map(int n_segs, const float *const *partials, const int64_t *n_partials,
                                  const int64_t *cols, float *const *outs, const int64_t *tmap, double *sq,
                                  int32_t *ticket, int algo, int dist, int64_t batch, int64_t act_dim,
                                  const float *loss_partials, int64_t n_loss_partials, float vf_coef, float ent_coef,
                                  float *scalars, float *d_logstd, xpa_stream_t stream);
/* K16R (r04): xpa_head_gemm_s3p_actor / _critic (w_hidden = the split buffer of Wh^T) with the heads' input h formed
 * inside from the gathered minibatch rows (the representation's one thin layer: x_rows [batch, d_in <= 20], w_in
 * [256, d_in], b_in, the heads' activation at slope_in) — xpa_thin_linear_act_fwd's h bit for bit, so the update
 * reads no h for the heads (ppoclip_learner.py:31-33 policy(obs) forward, layers.py:8-24 mlp_block).  The actor
 * writes h (h_out, for the weight gradient) and, when h_sign is given, its sign bits (xpa_s3_gemm_trunk_bwd_sign).
 * act_dim <= 8. */
int xpa_head_gemm_s3r_actor(int algo, int dist, int act, int64_t batch, int64_t act_dim, int64_t hidden,
                            const float *x_rows, int64_t ld_rows, int64_t d_in, const float *w_in, const float *b_in,
                            float slope_in, float *h_out, int64_t ld_h, unsigned *h_sign, const void *w_hidden,
                            const float *b_hidden, int64_t ld_dz, const float *w, const float *b, float slope,
                            const float *logstd, const int64_t *idx, int64_t n_rows, const float *act_buf,
                            const float *old_logp, const float *adv, const double *adv_partials,
                            int64_t n_adv_partials, float clip_range, float ent_coef, float *dz, float *partial_dw,
                            float *partial_db_hidden, float *partial_db_out, float *loss_partials, int64_t loss_width,
                            xpa_stream_t stream);
int xpa_head_gemm_s3r_critic(int act, int64_t batch, int64_t hidden, const float *x_rows, int64_t ld_rows,
                             int64_t d_in, const float *w_in, const float *b_in, float slope_in, const void *w_hidden,
                             const float *b_hidden, int64_t ld_dz, const float *w, const float *b, float slope,
                             const int64_t *idx, int64_t n_rows, const float *ret, float vf_coef, float *dz,
                             float *partial_dw, float *partial_db_hidden, float *partial_db_out, float *loss_partials,
                             int64_t loss_width, xpa_stream_t stream);

/* K6 — prioritized replay (PerOffPolicyBuffer, memory_tools.py:369-492; Sum/MinSegmentTree,
 * segtree_tool.py:4-86) with f64 trees on device: one [n_envs, 2*capacity] array per tree (node 1 =
 * root, leaf i at capacity + i; neutral 0 / +inf), capacity = next power of two >= n_size.
 * xpa_per_store: leaf ptr of every env = max_priority[e] ** alpha, ancestors updated (store, :437-439).
 * xpa_per_update_priorities: for each env e, entries k of idx / priorities [n_envs, batch_per_env]:
 *   leaf = (p == 0 ? 1e-8 : p) ** alpha (a repeated index keeps its last entry, as the sequential
 *   reference loop does), max_priority[e] = max(max_priority[e], p); ancestors rebuilt level by
 *   level.  An index outside [0, size) is skipped and counted in *err (the reference asserts).
 *   scratch: int32 [n_envs, capacity] filled with -1 once; left at -1.
 * xpa_per_sample: per env, batch_per_env stratified draws mass = u*len + k*len with len =
 *   sum(0, size - 1) / batch_per_env (leaves [0, size-2]: the reference's exclusive end), the
 *   prefix-sum descent, and the IS weights (p_sample * size^-beta) / (p_min * size^-beta).  u from
 *   `uniforms` (f64 [n_envs*batch_per_env], e.g. the reference's recorded random.random() draws) or, if
 *   NULL, a counter hash of (seed, counter, env, k).  steps = index (wrap_uint8 != 0: index & 255, the
 *   reference's astype(np.uint8)), flat_index (optional) = env * n_size + step for
 *   xpa_gather_minibatch.  size >= 2 (the reference recurses forever at size 1).  A descent that lands past the
 *   stored leaves (mass rounded to >= the stored total) is clamped to step size - 1 and counted in *err (if not
 *   NULL): the reference would fail its update_priorities assert on it. */
int xpa_per_store(double *sum_tree, double *min_tree, const double *max_priority, int64_t n_envs,
                  int64_t capacity, int64_t ptr, double alpha, xpa_stream_t stream);
int xpa_per_update_priorities(double *sum_tree, double *min_tree, double *max_priority, int *scratch,
                              int64_t n_envs, int64_t capacity, int64_t size, const int64_t *idx,
                              const float *priorities, int64_t batch_per_env, double alpha, int *err,
                              xpa_stream_t stream);
int xpa_per_sample(const double *sum_tree, const double *min_tree, int64_t n_envs, int64_t capacity, int64_t size,
                   int64_t batch_per_env, int64_t n_size, const double *uniforms, uint32_t seed, uint32_t counter,
                   double beta, int wrap_uint8, int64_t *steps, int64_t *flat_index, double *weights, int32_t *err,
                   xpa_stream_t stream);

/* Column store of raw observation rows into the rollout buffer at the device cursor:
 * dst[(i * horizon + cursor->ptr) * row_bytes ...] = src[i * row_bytes ...] for i < n (the uint8 Atari
 * frames of DummyOnPolicyBuffer_Atari.store, memory_tools.py:196-204, 526-560).  row_bytes % 16 == 0,
 * 16-B aligned pointers. */
int xpa_store_column(const void *src, int64_t n, int64_t row_bytes, void *dst, int64_t horizon,
                     const xpa_cursor_t *cursor, xpa_stream_t stream);

/* K15 — SynthAtari env step (the Atari-shaped synthetic env of SURVEY.md §8(d); spec + CPU checker
 * oracle/synth_env.py SynthAtariEnv), replacing DummyVecEnv_Atari / Atari_Env stepping for the benchmark
 * (gym_vec_env.py:201-212, 234-238; gym_env.py:186-241).  stack / final_obs: uint8 [n_envs, 84, 84, 4]
 * (channel 3 newest); the action is the one-hot row of act_in (row stride ld_act) written by the
 * sampler.  Writes the stepped stack to final_obs, reward sign, terminated (life lost or game over),
 * truncated (game over or step limit); on game over the env resets (stack = 4 copies of the new
 * episode's first frame).  Per-env int32 state: ep_step, ep_index, lives, paddle; f32 scores.
 * An act_in row with no entry > 0.5 steps action 0 and counts in *err (if not NULL).
 * xpa_synthatari_reset: stack = the first frame of episode ep_index[n], 4 times. */
int xpa_synthatari_step(int64_t n_envs, int64_t n_actions, const float *act_in, int64_t ld_act, uint32_t seed,
                        int32_t max_episode_steps, uint8_t *stack, uint8_t *final_obs, float *rew, uint8_t *term,
                        uint8_t *trunc, int32_t *ep_step, int32_t *ep_index, int32_t *lives, int32_t *paddle,
                        float *ep_score, float *ep_last_score, int32_t *ep_last_len, int32_t *err,
                        xpa_stream_t stream);
int xpa_synthatari_reset(int64_t n_envs, uint32_t seed, uint8_t *stack, const int32_t *ep_index,
                         xpa_stream_t stream);

/* K8 with deferred bootstrap values: instead of v_boot, a mid-buffer truncation of env n (a path closed
 * with a bootstrap, ppoclip_agent.py:95-100) stores its normalised final-observation row boot_obs[n]
 * (row stride ld_boot, obs_dim floats) in the env's first free slot k < n_slots: slot_obs[k n_envs + n]
 * ([n_slots n_envs, obs_dim]) and slot_t[k n_envs + n] = t (slot_t [n_slots, n_envs] starts at -1).  A
 * truncation finding every slot taken counts in *overflow (and reuses the last slot).  The caller sizes n_slots
 * so that this cannot happen: an env whose only truncation source is a time limit of L steps truncates at most
 * ceil((horizon - 1) / L) times before the last step of a rollout.  After the last step,
 * values = V([slot_obs; boot_obs]) ([(n_slots + 1) n_envs]: the truncation slots, then the last step's final
 * observations, ppoclip_agent.py:69-75) and xpa_rollout_bootstrap_fixup writes buf_boot at every recorded
 * truncation and at the last column (0 where terminal), resetting slot_t to -1. */
int xpa_rollout_post_deferred(int64_t n_envs, int64_t horizon, const float *rew, const uint8_t *term,
                              const uint8_t *trunc, const float *boot_obs, int64_t ld_boot, int64_t obs_dim,
                              float *slot_obs, int32_t *slot_t, int64_t n_slots, int32_t *overflow,
                              xpa_cursor_t *cursor, float *ret_mean, float *ret_var, double *ret_count,
                              float *returns, float *buf_rew, float *buf_term, uint8_t *buf_closed, float *buf_boot,
                              float gamma, int mask_returns, int use_rewnorm, float rew_range, int atari_lifeloss,
                              double *partials, uint32_t *ticket, xpa_stream_t stream);
/* xpa_rollout_post_deferred with the normalisation of the final observations folded in: final_obs holds
 * the RAW observations; a kept truncation row is normalised with obs_mean / obs_var (clip obs_clip,
 * xpa_obs_normalize's arithmetic) into slot_obs, and at the rollout's last step every env's normalised
 * final observation is written into boot_norm [n_envs, ld_norm] (the input of the deferred critic pass).
 * slot_src [n_envs, ld_slot] (nullable, RAW): the rows kept truncations are formed from instead of final_obs — the
 * env's next (reset) observations for A2C, whose critic call sees obs[i] = reset_obs (a2c_agent.py:88-95); the
 * last step's boot_norm rows are final_obs either way (the full-buffer closures, a2c_agent.py:67-72). */
int xpa_rollout_post_deferred_norm(int64_t n_envs, int64_t horizon, const float *rew, const uint8_t *term,
                                   const uint8_t *trunc, const float *final_obs, int64_t ld_final,
                                   const float *slot_src, int64_t ld_slot, int64_t obs_dim,
                                   const float *obs_mean, const float *obs_var, float obs_clip, float *boot_norm,
                                   int64_t ld_norm, float *slot_obs, int32_t *slot_t, int64_t n_slots,
                                   int32_t *overflow, xpa_cursor_t *cursor, float *ret_mean, float *ret_var,
                                   double *ret_count, float *returns, float *buf_rew, float *buf_term,
                                   uint8_t *buf_closed, float *buf_boot, float gamma, int mask_returns, int use_rewnorm,
                                   float rew_range, int atari_lifeloss, double *partials, uint32_t *ticket,
                                   xpa_stream_t stream);
int xpa_rollout_bootstrap_fixup(int64_t n_envs, int64_t horizon, const float *values, int32_t *slot_t,
                                int64_t n_slots, const float *buf_term, float *buf_boot, xpa_stream_t stream);

/* K13 — first representation layer Linear(d_in, 256) + activation for a small d_in (<= 64): Basic_MLP's
 * first mlp_block (xuance/torch/representations/mlp.py:21-51, utils/layers.py:8-24) as HBM-streaming
 * kernels.  Forward: h = act(x W^T + b), x [rows, d_in] (row stride ldx), w [256, d_in], h [rows, 256]
 * (row stride ldh).  Backward (the layer is the first of the network, so no dX): from g = d loss/d h
 * and h, per-block partials of dW (xpa_thin_bwd_num_partials(rows) rows of 256*d_in, laid out as w) and
 * of db (rows of 256), each reduced by xpa_colsum_finalize.  act: 0 identity, 1 LeakyReLU(slope) /
 * ReLU, 2 tanh. */
int64_t xpa_thin_bwd_num_partials(int64_t rows);
int xpa_thin_linear_act_fwd(int act, const float *x, int64_t ldx, int64_t rows, int64_t d_in, int64_t d_out,
                            const float *w, const float *b, float slope, float *h, int64_t ldh, xpa_stream_t stream);
/* K13 with K4's minibatch gather folded in (the update's fast path, ppoclip_agent.py:76-85 / memory_tools.py:231-242):
 * the rows are x[idx[r]] of the full flattened rollout buffer x [n_rows, d_in] (an index outside [0, n_rows) gives a
 * zero row), so the gathered minibatch never materialises; with adv_partials (f64 [xpa_gather_num_partials(rows), 2])
 * the forward also writes xpa_gather_minibatch's per-minibatch advantage moments of adv[idx] bit for bit, and with
 * x_out ([rows, d_in] contiguous) the gathered rows themselves (what the backward then reads contiguously).  The
 * _bwd_gather form reads the rows through idx instead.  Otherwise as xpa_thin_linear_act_fwd / _bwd. */
int xpa_thin_linear_act_fwd_gather(int act, const float *x, int64_t ldx, int64_t n_rows, const int64_t *idx,
                                   int64_t rows, int64_t d_in, int64_t d_out, const float *w, const float *b,
                                   float slope, float *h, int64_t ldh, const float *adv, double *adv_partials,
                                   float *x_out, xpa_stream_t stream);
/* Diagnostics: bit 1 makes xpa_thin_linear_act_fwd_gather_sign store h with plain stores (default non-temporal). */
int xpa_thin_probe(int mask);
/* Diagnostics: 1 makes the head kernels store dz with plain (not non-temporal) stores. */
int xpa_head_store_probe(int plain);
/* r06 A/B: the K16 heads' second-slot blocks (blockIdx >= 256) start n x ~0.85 us late, so their k loop overlaps the
 * first blocks' epilogue; 0 (the default) = off.  Returns a hipError. */
int xpa_head_stagger(int n);
/* The gather form writing h and its sign bits as well (r04; h_sign: 32 bytes per row, byte b bit j = h[row, 32 j + b]
 * > 0, the layout xpa_s3_gemm_trunk_bwd_sign reads); act 0 / 1. */
int xpa_thin_linear_act_fwd_gather_sign(int act, const float *x, int64_t ldx, int64_t n_rows, const int64_t *idx,
                                        int64_t rows, int64_t d_in, int64_t d_out, const float *w, const float *b,
                                        float slope, float *h, int64_t ldh, const float *adv, double *adv_partials,
                                        float *x_out, unsigned *h_sign, xpa_stream_t stream);
int xpa_thin_linear_act_bwd_gather(int act, const float *g, int64_t ldg, const float *h, int64_t ldh, int64_t rows,
                                   const float *x, int64_t ldx, int64_t n_rows, const int64_t *idx, int64_t d_in,
                                   int64_t d_out, float slope, float *partial_dw, float *partial_db,
                                   xpa_stream_t stream);
/* The rollout's forward with the observation normalisation fused in: x holds RAW observations;
 * xn = clip((x - mean) / (sqrt(var) + 1e-8), +-clip) (xpa_obs_normalize's arithmetic) is written to xn
 * [rows, ldn] and, when col != NULL, into the rollout buffer column cursor->ptr of col (row stride col_ld
 * floats, as xpa_obs_normalize's col_out), and h = act(xn W^T + b) as xpa_thin_linear_act_fwd. */
int xpa_thin_linear_act_fwd_norm(int act, const float *x, int64_t ldx, int64_t rows, int64_t d_in, int64_t d_out,
                                 const float *w, const float *b, float slope, float *h, int64_t ldh,
                                 const float *mean, const float *var, float clip, float *xn, int64_t ldn,
                                 float *col, int64_t col_ld, const xpa_cursor_t *cursor, xpa_stream_t stream);
int xpa_thin_linear_act_bwd(int act, const float *g, int64_t ldg, const float *h, int64_t ldh, int64_t rows,
                            const float *x, int64_t ldx, int64_t d_in, int64_t d_out, float slope, float *partial_dw,
                            float *partial_db, xpa_stream_t stream);

/* C3 / C5 convolutional trunk (AC_CNN_Atari xuance/torch/representations/cnn.py:45-93, Basic_CNN :5-40): the
 * elementwise passes around the MIOpen convolutions, every tensor NHWC ([rows = B*H*W, C] row-major).
 * K20: dst[i] = float32(src[i] / 255.0) with the reference's arithmetic (NumPy float64 division, then the
 * float32 cast; cnn.py:89-92), bit for bit; n bytes in, n floats out (16-B aligned buffers take the vector path). */
int xpa_frames_to_f32(const uint8_t *src, int64_t n, float *dst, xpa_stream_t stream);
/* r05: the conv kernels' arithmetic — bit 0: K25B (conv1 forward), bit 1: K26B (conv1 weight gradient) on the bf16
 * matrix cores with the frames exact and the f32 operand split three ways; bit 2: K27B (xpa_conv_dgrad_s2k) with both
 * operands split three ways (six products, f32-GEMM accuracy).  A cleared bit selects the fp32-MFMA form (K25 / K26 /
 * K27); so does an operand of 2^31 bytes or more (the bf16 forms read through one buffer record).  Bit 3: K27B at 3
 * blocks per CU (an A/B probe; measured slower).  mask < 0 only reads.  Returns the previous mask (default 7). */
int xpa_conv1_form(int mask);
/* r05: K28's arithmetic (xpa_conv_fwd / xpa_conv_dgrad) — bit 0: K28B, the implicit GEMM on the bf16 matrix cores with
 * both f32 operands split three ways (six products, f32-GEMM accuracy), taken where the GEMM's input channels are a
 * multiple of 16; bit 1: K28B with 3 row tiles per wave (A/B, forward only); 0 = the fp32-MFMA K28 (the default: K28B
 * measured no faster inside the C3 update).  mask < 0 only reads.  Returns the previous mask. */
int xpa_conv_igemm_form(int mask);
/* K25 — the first conv block straight from the uint8 frames (C3 AC_CNN_Atari / C5 Basic_CNN: cnn_block
 * xuance/torch/utils/layers.py:36-57 on observations / 255.0, cnn.py:89-92): y = act(conv2d(x / 255, w, stride, pad)
 * + bias) with x uint8 NHWC [batch, height, width, 4] (4-B aligned), w [32, 4, 8, 8] (torch's Conv2d layout), y f32
 * NHWC [batch, OH, OW, 32], OH = (height + 2 pad - 8) / stride + 1 (zero padding).  Computed as sum x (w / 255) on
 * fp32 MFMA (exact f32 fma chains; the 1/255 rounds once on the weight instead of once on the frame value).  act as xpa_bias_act.  channels must be 4,
 * kernel 8 and out_channels 32 (else hipErrorInvalidValue).  r05 default (K25B, xpa_conv1_form bit 0): the same sum
 * on the bf16 matrix cores — the bytes are exact in bf16 and w / 255 is cut into its exact three-way bf16 split, so
 * each term is x (w / 255) rounded once as on fp32 MFMA; only the order of the f32 sum over taps differs. */
int xpa_conv1_u8_fwd(int act, const uint8_t *x, int64_t batch, int64_t height, int64_t width, int64_t channels,
                     int64_t kernel, int64_t stride, int64_t pad, const float *w, const float *bias,
                     int64_t out_channels, float slope, float *y, xpa_stream_t stream);
/* K27 — the data gradient of a stride-s (1 or 2), 2s x 2s conv with 32 input / 64 output channels (the Nature CNN's
 * second conv: 4 x 4 stride 2 pad 1, 32 -> 64; torch's convolution_backward input gradient inside loss.backward(),
 * a2c_learner.py:31-33): dx NHWC [batch, in_h, in_w, 32] = conv_transpose(dy NHWC [batch, out_h, out_w, 64] (16-B
 * aligned), w [64, 32, 2s, 2s]), every element written (no accumulation into dx).  fp32 MFMA, one implicit GEMM per
 * stride residue class (K = 4 taps x 64 channels).  out_h / out_w must be the forward's output size. */
int xpa_conv_dgrad_s2k(const float *dy, int64_t batch, int64_t out_h, int64_t out_w, int64_t out_channels,
                       const float *w, int64_t in_channels, int64_t kernel, int64_t stride, int64_t pad, int64_t in_h,
                       int64_t in_w, float *dx, xpa_stream_t stream);
/* K26 — K25's weight gradient from the uint8 frames (the first conv's dW in loss.backward()): per-block partials
 * [xpa_conv1_u8_wgrad_num_partials(), 32 * 4 * 8 * 8] in the weight layout [n][c][ky][kx] of
 * sum_rows dz[row, n] x[row's tap] / 255 (dz NHWC [batch, OH, OW, 32] f32: the gradient at the conv's output after
 * the activation backward; x as xpa_conv1_u8_fwd), reduced by xpa_colsum_finalize into the weight gradient. */
int64_t xpa_conv1_u8_wgrad_num_partials(void);
int xpa_conv1_u8_wgrad(const float *dz, const uint8_t *x, int64_t batch, int64_t height, int64_t width,
                       int64_t channels, int64_t kernel, int64_t stride, int64_t pad, int64_t out_channels,
                       float *partial, xpa_stream_t stream);
/* K26 with the conv block's activation backward + bias gradient folded in (act >= 0: K22 on the first conv's output
 * never runs): dz here is d loss / d y at the block's OUTPUT y (NHWC f32, the forward's K25 output), the kernel
 * forms dh act'(y) itself (act as xpa_bias_act) and also writes per-block bias partials
 * [xpa_conv1_u8_wgrad_num_partials(), 32] for xpa_colsum_finalize.  act = -1: exactly xpa_conv1_u8_wgrad. */
int xpa_conv1_u8_wgrad_act(int act, const float *dz, const float *y, float slope, const uint8_t *x, int64_t batch,
                           int64_t height, int64_t width, int64_t channels, int64_t kernel, int64_t stride,
                           int64_t pad, int64_t out_channels, float *partial, float *bias_partial,
                           xpa_stream_t stream);
/* K21: y = act(y + bias) in place over [rows, cols] (bias [cols] or NULL): the conv / Linear bias and the
 * activation of cnn_block / mlp_block (xuance/torch/utils/layers.py:8-57).  cols % 4 == 0 and cols / 4 must
 * divide 256; act 0 identity, 1 LeakyReLU(slope) / ReLU, 2 tanh. */
int xpa_bias_act(int act, float *y, int64_t rows, int64_t cols, const float *bias, float slope, xpa_stream_t stream);
/* K22: dz = dh * act'(h) (dz may alias dh; NULL: not written) and per-block column sums of dz, the bias gradient
 * (xpa_act_bwd_bias_num_partials(rows, cols) rows of cols, reduced by xpa_colsum_finalize): the backward of
 * K21 over a conv / fc layer's output.  Same cols constraint as K21; 16-B aligned. */
int64_t xpa_act_bwd_bias_num_partials(int64_t rows, int64_t cols);
int xpa_act_bwd_bias(int act, const float *dh, const float *h, int64_t rows, int64_t cols, float slope, float *dz,
                     float *partials, xpa_stream_t stream);
/* K23: out[b, c] = max over the hw positions of x [batch, hw, channels] (NHWC), argmax[b, c] its position — Basic_CNN's
 * AdaptiveMaxPool2d((1, 1)) (cnn.py:5-40) with torch's rule: the first maximum wins, a NaN always replaces. */
int xpa_global_maxpool(const float *x, int64_t batch, int64_t hw, int64_t channels, float *out, int32_t *argmax,
                       xpa_stream_t stream);
/* K24: the backward of K23 and of the activation before it, with the conv bias gradient: dz[b, p, c] =
 * (p == argmax[b, c] ? dout[b, c] : 0) * act'(h[b, p, c]) over [batch * hw, channels], and the column-sum partials
 * of dz as xpa_act_bwd_bias (xpa_act_bwd_bias_num_partials(batch * hw, channels) rows).  An argmax outside
 * [0, hw) routes nothing and counts in *err (if not NULL). */
int xpa_maxpool_act_bwd_bias(int act, const float *dout, const int32_t *argmax, const float *h, int64_t batch,
                             int64_t hw, int64_t channels, float slope, float *dz, float *partials, int32_t *err,
                             xpa_stream_t stream);

/* K28 / K29 — generic NHWC convolutions of the CNN trunks as implicit GEMMs on the fp32 matrix cores (exact f32
 * fma chains), replacing MIOpen on the explicit CNN path (conv blocks of AC_CNN_Atari / Basic_CNN,
 * xuance/torch/utils/layers.py:27-57, xuance/torch/representations/cnn.py:5-93, and their backward in
 * loss.backward(), a2c_learner.py:31-33 / perdqn_learner.py:37-40).  Tensors NHWC f32; w in torch's layout
 * [out_c][in_c][kernel][kernel]; in_c a multiple of 4, <= 64; out_c <= 64; xpa_conv_igemm_ok(in_c, out_c, kernel)
 * tells whether the weight image fits the 160 KiB LDS (the forward and, with the channel counts swapped, the data
 * gradient).  act: 0 identity, 1 LeakyReLU(slope) / ReLU (slope 0), 2 tanh.
 * The operands must each be under 2 GiB (32-bit buffer offsets).
 * xpa_conv_fwd: y = act(conv(x, w) + bias) [batch, OH, OW, out_c] (bias nullable).
 * xpa_conv_dgrad: dx [batch, in_h, in_w, in_c] = the data gradient of the conv from dy [batch, out_h, out_w, out_c]
 *   (stride 1 or 2); with act_prev >= 0, dx = that * act'(y_prev) (the previous block's activation backward, act' from
 *   its OUTPUT y_prev) and, when bias_partial != NULL, its column sums per block
 *   ([xpa_conv_dgrad_num_partials(batch, in_h, in_w)][in_c], xpa_colsum_finalize -> the previous block's bias grad).
 * xpa_conv_wgrad: per-block partials [xpa_conv_wgrad_num_partials()][out_c][in_c][kernel][kernel] of
 *   dW = sum over output pixels of dz x (xpa_colsum_finalize -> the weight gradient, weight layout); dz = g, or with
 *   act >= 0, g * act'(y) (y = the block's forward output) and then bias_partial [num_partials][out_c] too. */
int xpa_conv_igemm_ok(int64_t in_channels, int64_t out_channels, int64_t kernel);
int xpa_conv_fwd(int act, const float *x, int64_t batch, int64_t in_h, int64_t in_w, int64_t in_c, const float *w,
                 const float *bias, int64_t out_c, int64_t kernel, int64_t stride, int64_t pad, float slope, float *y,
                 xpa_stream_t stream);
int64_t xpa_conv_dgrad_num_partials(int64_t batch, int64_t in_h, int64_t in_w);
int xpa_conv_dgrad(const float *dy, int64_t batch, int64_t out_h, int64_t out_w, int64_t out_c, const float *w,
                   int64_t in_c, int64_t kernel, int64_t stride, int64_t pad, int64_t in_h, int64_t in_w, int act_prev,
                   const float *y_prev, float slope, float *dx, float *bias_partial, xpa_stream_t stream);
int64_t xpa_conv_wgrad_num_partials(void);
int xpa_conv_wgrad(int act, const float *g, const float *y, float slope, const float *x, int64_t batch, int64_t in_h,
                   int64_t in_w, int64_t in_c, int64_t out_c, int64_t kernel, int64_t stride, int64_t pad,
                   float *partial, float *bias_partial, xpa_stream_t stream);
/* Diagnostics: on != 0 makes xpa_conv_wgrad take its streaming form (operands straight from global memory) even where
 * the LDS-slab form applies (both give the same sums up to f32 association; process-global, not thread-safe). */
void xpa_conv_wgrad_force_stream(int on);

/* r06, K14F — one device env step's last launch: xpa_rollout_policy_head_synthbox (policy heads, sample, store, SynthBox
 * env step) and K8's deferred + normalised post step (xpa_rollout_post_deferred_norm; with obs_count non-NULL also the
 * next step's obs_rms.update, xpa_rollout_post_deferred_norm_rms) in ONE launch: the tail of ppoclip_agent.py:65-75
 * (envs.step, reward normalisation, memory.store, the path closing of finish_path's callers) and the obs_rms.update of
 * ppoclip_agent.py:62-63 for the next observation.  slot_from_next: kept truncation rows are the env's next observation
 * (A2C's reset_obs bootstrap, a2c_agent.py:88-95) instead of its final one.  part / tickets: the workspace sized by
 * xpa_rollout_step_workspace (f64 partials, returned in doubles; *n_tickets int32 tickets zeroed once, left zero by every
 * launch).  The partial sums are taken in a fixed order (any block arrival order gives the same bits). */
int64_t xpa_rollout_step_workspace(int64_t n_envs, int64_t obs_dim, int rms, int64_t *n_tickets);
/* r06, K40V: v [m] = act(a [m, k] . B + bias) . w_out + b_out[0] (act 0 identity / 1 LeakyReLU (slope) / 2 tanh; B the
 * 256-column planes of xpa_s3_split_b; a 16-B aligned, lda % 4 == 0, k % 16 == 0): the critic from its last hidden layer's
 * input to the value in one launch — the rollout's deferred bootstrap rows (critic(x), ppoclip_agent.py:95-101), whose
 * values then go to the compact GAE scan (xpa_gae_scan_compact). */
int xpa_s3_gemm_value(const float *a, int64_t lda, const void *b_split, float *v, int64_t m, int64_t k,
                      const float *bias, int act, float slope, const float *w_out, const float *b_out,
                      xpa_stream_t stream);
/* K40T (r06): the rollout's trunk and paired hidden layer in one launch — xpa_thin_linear_act_fwd_norm (d_in <= 18,
 * d_out 256: obs normalisation + Basic_MLP's first layer, mlp.py:21-51; normalised rows to xn and the buffer column)
 * followed by xpa_s3_gemm_rows_pair on its h, with h formed in LDS and never stored (ppoclip_agent.py:63
 * self.action(obs) -> representation + the policy's hidden layers).  z equals the two-launch form's bit for bit. */
int xpa_s3_gemm_rows_pair_trunk(int act, const float *x, int64_t ldx, int64_t d_in, const float *w, const float *b,
                                float slope, const float *mean, const float *var, float clip, float *xn, int64_t ldn,
                                float *col, int64_t col_ld, const xpa_cursor_t *cursor, const void *b0_split,
                                const void *b1_split, const float *bias, float *c, int64_t ldc, int64_t m,
                                xpa_stream_t stream);
/* Diagnostics: bits 1 / 2 / 4 end K14F's tail after the block partials / the group tickets / the group sums (results
 * then invalid: timing only; tools/k14f_probe.py); 0 = production. */
int xpa_k14f_probe(int bits);
int xpa_rollout_step_synthbox(
    int act, int64_t n_envs, int64_t act_dim, int64_t horizon, int64_t hidden, int64_t ld, const float *z_actor,
    const float *z_critic, float slope, const float *w_actor, const float *b_actor, const float *w_critic,
    const float *b_critic, const float *logstd, xpa_cursor_t *cursor, uint32_t seed, float act_clip, float *buf_act,
    float *buf_logp, float *buf_val, int64_t obs_dim, const float *wcat_t, uint32_t env_seed, int32_t max_episode_steps,
    float noise, float term_thresh, float reset_scale, float *state, int64_t ld_state, float *final_obs, float *rew,
    uint8_t *term, uint8_t *trunc, int32_t *ep_step, uint32_t *ep_index, float *ep_score, float *ep_last_score,
    int32_t *ep_last_len, float *slot_obs, int32_t *slot_t, int64_t n_slots, int32_t *overflow, int slot_from_next,
    float *obs_mean, float *obs_var, double *obs_count, float obs_clip, float *boot_norm, int64_t ld_norm,
    float *ret_mean, float *ret_var, double *ret_count, float *returns, float *buf_rew, float *buf_term,
    uint8_t *buf_closed, float *buf_boot, float gamma, int mask_returns, int use_rewnorm, float rew_range,
    int atari_lifeloss, double *part, int32_t *tickets, xpa_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* XUANPOLICY_AMD_H */
