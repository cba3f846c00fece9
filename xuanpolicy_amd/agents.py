"""PPO-Clip and A2C agents: the reference's on-policy training loop, device-resident on one GPU.

Mirrors (reference paths):
  Agent base            xuance/torch/agents/agent.py:7-141 (obs/reward normalisation, logging, save/load)
  PPOCLIP_Agent.train   xuance/torch/agents/policy_gradient/ppoclip_agent.py:59-111
  A2C_Agent.train       xuance/torch/agents/policy_gradient/a2c_agent.py:57-107
  REGISTRY              xuance/torch/agents/__init__.py:68-111 ("PPO_Clip", "A2C")
Same constructor (config, envs, policy, optimizer, scheduler, device) and config keys
(n_steps, n_epoch, n_minibatch, gamma, gae_lambda, use_gae, use_advnorm, use_obsnorm, use_rewnorm,
obsnorm_range, rewnorm_range, vf_coef, ent_coef, clip_range, clip_grad_norm / clip_grad, ...).

One env step of the hot loop (device env, no host sync):
   K5  RunningMeanStd.update(obs) + normalise -> policy input and buffer column
   --  policy heads forward (PyTorch-ROCm GEMMs, no autograd)
   K3  sample action, log-prob, store act/logp/value
   K7  env step (GEMM + xpa_synthbox_step, auto-reset)
   K5c normalise the final obs with the same statistics -> critic forward (truncation bootstrap)
   K8  reward norm, return tracker, ret_rms, terminals, path closures; cursor += 1
When the buffer is full: K1 GAE over [n_envs, n_steps]; then n_epoch x n_minibatch updates of
K4 gather -> heads forward -> K2 loss fwd+bwd -> autograd backward -> [all-reduce] -> clip -> Adam.
Host-side envs (numpy VecEnvs) are supported through the same kernels with per-step H2D/D2H copies.

Semantic notes: action sampling uses the counter-hash RNG on device, not torch's
CPU generator; the truncation bootstrap value V(norm(final obs)) is computed for every env each step
(the reference recomputes a full batch once per truncated env, ppoclip_agent.py:99-100); ret_rms merges
all finished envs of a step in one Chan update (mathematically equal to the reference's sequential
single-value updates).
"""
import ctypes
import json
import os
import time

import numpy as np
import torch

from . import _lib, ops
from .buffer import DummyOnPolicyBuffer, DummyOnPolicyBuffer_Atari
from .fused_mlp import Rows
from .learners import A2C_Learner, PerDQN_Learner, PPOCLIP_Learner
from .policies import policy_discrete, policy_heads, space_shape

FLOAT_MAX = 3.0e38


def _cfg(config, name, default):
    return getattr(config, name, default)


# r05: fold the next step's obs_rms.update into K8 on the device-env path (xpa_rollout_post_deferred_norm_rms).
# Measured neutral at C2 (profiles/r05/r05fold: rollout 5.70 / 5.68 ms on vs 5.68 / 5.69 off — the merge chain moves
# into K8, 6.5 + 7.7 -> 15.0 us), so it is an opt-in (bench.py --fold-rms on); off keeps the reference's update order
# exactly, also around test() calls (which update obs_rms with the test observations, ppoclip_agent.py:125)
FOLD_RMS = False
# r06: K8's post step (and, with per-rank obs statistics, the next step's obs_rms.update) inside the env-fused K14 launch
# (K14F, ops.rollout_policy_head_synthbox(post=)): a C2 env step in three launches instead of five
FUSE_POST = True
# r06 (opt-in, XPA_VALUE_GEMM=1 / bench --gae-form k40v): the deferred bootstrap rows' critic on K40V (split GEMM +
# value-head epilogue) feeding the compact GAE scan.  The scan is faster (5.3 vs 6.0 us) but K40V's launch, 64 blocks
# each streaming all of B, costs 25.6 us against the library GEMM's 15.1 for the value form: 30.9 vs 21.1 us per
# iteration, so the value-fused scan (K1V) stays the default
VALUE_GEMM = os.environ.get("XPA_VALUE_GEMM", "0") == "1"


def rms_rollout_sync(start, end, all_reduce_sum):
    """sync_obs_rms = "rollout" (r06): the rank's rows of a rollout recovered from its running statistics — end = start
    (+) B, Chan's merge being associative over the per-step merges (statistic_tools.py:86-112) — as (n, sum, sum of squares)
    in f64, SUM-reduced over the ranks, and merged into start: the statistics one RunningMeanStd over every rank's rows
    would hold, up to the f32 rounding of the stored mean / var.  start / end = (mean f32 [D], var f32 [D], count f64 [1]);
    returns (mean f32, var f32, count f64)."""
    m0, v0, c0 = start[0].double(), start[1].double(), start[2].double()
    m1, v1, c1 = end[0].double(), end[1].double(), end[2].double()
    n = c1 - c0
    s1 = m1 * c1 - m0 * c0                                       # the rows' sum
    mb = s1 / n
    m2 = v1 * c1 - v0 * c0 - (mb - m0) ** 2 * c0 * n / c1       # the rows' squared deviations about their own mean
    red = torch.cat([n, s1, m2 + s1 * mb])                      # (n, sum, sum of squares)
    all_reduce_sum(red)
    D = m0.shape[0]
    N, S1, Q = red[:1], red[1:1 + D], red[1 + D:]
    mB = S1 / N
    m2B = torch.clamp(Q - S1 * mB, min=0.0)
    tot = c0 + N
    delta = mB - m0
    mean = m0 + delta * N / tot
    var = (v0 * c0 + m2B + delta * delta * c0 * N / tot) / tot
    return mean.float(), var.float(), tot

class _OnPolicyAgent:
    algo = "ppo"

    def __init__(self, config, envs, policy, optimizer, scheduler=None, device=None):
        self.config = config
        self.envs = envs
        self.policy = policy
        self.render = _cfg(config, "render", False)
        self.n_envs = envs.num_envs
        self.n_steps = config.n_steps
        self.n_minibatch = config.n_minibatch
        self.n_epoch = config.n_epoch
        self.gamma = config.gamma
        self.gae_lam = config.gae_lambda
        self.atari = _cfg(config, "env_name", "") == "Atari"
        self.observation_space = envs.observation_space
        self.action_space = envs.action_space
        self.device = next(policy.parameters()).device
        self.discrete = policy_discrete(policy)
        self.dist = "categorical" if self.discrete else "gaussian"
        self.auxiliary_info_shape = {"old_logp": ()} if self.algo == "ppo" else {}
        Buffer = DummyOnPolicyBuffer_Atari if self.atari else DummyOnPolicyBuffer
        self.buffer_size = self.n_envs * self.n_steps
        self.batch_size = self.buffer_size // self.n_minibatch
        self.memory = Buffer(self.observation_space, self.action_space, self.auxiliary_info_shape, self.n_envs,
                             self.n_steps, _cfg(config, "use_gae", True), _cfg(config, "use_advnorm", True),
                             self.gamma, self.gae_lam, device=self.device)
        self.learner = self._make_learner(config, policy, optimizer, scheduler)
        # A2C bootstraps a mid-rollout truncation with V(norm(reset_obs)): a2c_agent.py:88-95 writes obs[i] =
        # reset_obs into next_obs before its critic call (PPO calls the critic first, ppoclip_agent.py:95-101, and
        # both use the final observations for the full-buffer closures).  False: the final observation for A2C too.
        self.boot_from_reset = self.algo == "a2c" and bool(_cfg(config, "a2c_reset_bootstrap", True))
        self.use_obsnorm = bool(_cfg(config, "use_obsnorm", False))
        self.use_rewnorm = bool(_cfg(config, "use_rewnorm", False))
        self.obsnorm_range = float(_cfg(config, "obsnorm_range", 5))
        self.rewnorm_range = float(_cfg(config, "rewnorm_range", 5))
        dev, N, T = self.device, self.n_envs, self.n_steps
        self.obs_shape = space_shape(self.observation_space)
        D = int(np.prod(self.obs_shape)) if len(self.obs_shape) else 1
        self.obs_dim = D
        f32 = dict(dtype=torch.float32, device=dev)
        # RunningMeanStd state (statistic_tools.py:35-60): mean 0, var 1, count 1e-4
        self.obs_mean = torch.zeros((D,), **f32)
        self.obs_var = torch.ones((D,), **f32)
        self.obs_count = torch.full((1,), 1e-4, dtype=torch.float64, device=dev)
        self.ret_mean = torch.zeros((1,), **f32)
        self.ret_var = torch.ones((1,), **f32)
        self.ret_count = torch.full((1,), 1e-4, dtype=torch.float64, device=dev)
        self.returns = torch.zeros((N,), **f32)
        self.cursor = ops.new_cursor(dev)
        self.post_ws = ops.post_workspace(N, dev)
        # Raw observations (uint8 Atari frames without obs normalisation, DummyOnPolicyBuffer_Atari): stored
        # and fed to the policy as they are (AC_CNN_Atari scales by 1/255 on device).
        self.raw_obs = self.memory.observations.dtype == torch.uint8 and not self.use_obsnorm
        self.obs_norm = None if self.raw_obs else torch.empty((N, D), **f32)
        self.boot_obs = None if self.raw_obs else torch.empty((N, D), **f32)
        self.rms_part = (torch.empty((2 * ops.rms_num_partials(N), D), dtype=torch.float64, device=dev)
                         if self.use_obsnorm else None)
        self._rms_ticket = torch.zeros((1,), dtype=torch.int32, device=dev)   # xpa_rms_update's arrival count
        self._policy_in = self.obs_norm
        self.logp_scratch = None if self.algo == "ppo" else torch.zeros((N, T), **f32)
        self.obs_mb = None
        self.adv_part = None
        self.seed = int(_cfg(config, "seed", 1))
        self._perm_counter = 0
        self._perm_buf = None
        self.device_env = hasattr(envs, "step_device")
        self.fuse_env_step = True   # device SynthBox env stepped inside K14 when possible (_env_fused)
        self.fuse_value_gae = True  # deferred bootstraps' value head inside the GAE scan (xpa_gae_scan_value)
        # r06 (K40V): with fuse_value_gae, the deferred bootstraps' critic to the value on the split GEMM (the value head in
        # its epilogue) and the compact GAE scan on exactly SURVEY.md §8(d)'s bytes, where it applies
        self.value_gemm = VALUE_GEMM
        self.fuse_gather = True     # minibatch gather + adv moments inside the update's K13 (fused_mlp.Rows)
        # r05: the next step's obs_rms.update folded into K8 (xpa_rollout_post_deferred_norm_rms) on the device-env
        # path; _rms_pending: the current observation's statistics are not merged yet (the first step, or after
        # anything but a folded step produced env.obs), so that step runs the standalone update first.  An env reset
        # (envs.reset bumps envs.resets) re-arms it.  test() does not: its obs_rms.update merges other rows, and the
        # folded merge of env.obs already happened (the Chan merge is order-independent up to rounding)
        self.fold_rms = FOLD_RMS
        self.fuse_post = FUSE_POST
        self._k14f_ws = None
        self._rms_pending = True
        self._rms_resets = getattr(envs, "resets", 0)
        self._rms_fold_part = None
        # K32: whole device env steps (RMS, normalise, forward, sample, env, post) in one launch (_small_rollout)
        self.fused_rollout = bool(_cfg(config, "fused_rollout", True))
        self._k32 = self._k32_key = None
        self.current_step = 0
        self.current_episode = np.zeros((N,), np.int32)
        self.iterations = 0
        self.last_info = None
        self.infos = []          # host copies, one dict per buffer-full phase
        self.log_hook = None     # optional callable(info: dict, step: int) (tensorboard/wandb adapter)
        self.timers = {"rollout": 0.0, "update": 0.0}
        self.phase_events = None
        self.update_log = None   # a list: every update's device loss scalars are appended (tests / diagnostics)
        self._t = 0
        self._host_obs = None
        self.use_graph = bool(_cfg(config, "cuda_graph", True)) and self.device.type == "cuda"
        # Data-parallel normalisation variants; default = per-shard statistics with one
        # gradient all-reduce per minibatch.
        #   sync_obs_rms:   SUM the per-step RMS partials across ranks (identical obs statistics everywhere)
        #   global_advnorm: AVG each minibatch's advantage moments across ranks (global adv-norm)
        self.world = 1
        import torch.distributed as tdist
        if tdist.is_available() and tdist.is_initialized():
            self.world = tdist.get_world_size()
        #   sync_obs_rms = "rollout" (r06): per-rank statistics inside a rollout (graph-captured, folded into K14F), merged
        #                   across ranks once per rollout, before the update (rms_rollout_sync)
        sync_mode = _cfg(config, "sync_obs_rms", False)
        dp_rms = self.world > 1 and self.use_obsnorm
        self.sync_obs_rms_rollout = dp_rms and isinstance(sync_mode, str) and sync_mode.lower() == "rollout"
        self.sync_obs_rms = dp_rms and bool(sync_mode) and not self.sync_obs_rms_rollout
        self._rms_c0 = None
        self.global_advnorm = bool(_cfg(config, "global_advnorm", False)) and self.world > 1
        if self.sync_obs_rms:
            self.use_graph = False  # the per-step collective runs outside a captured graph
        # Deferred truncation bootstraps: the critic runs once per iteration on [truncation slots;
        # last-step obs] instead of on every env at every step.  Only the device envs qualify: their one truncation
        # source is the time limit, so an env truncates at most ceil((T - 1) / max_episode_steps) times before the
        # rollout's last step, and K8 keeps that many slots per env (1 when max_episode_steps >= n_steps, the C1 / C2
        # / C4 case); a host VecEnv may truncate for other reasons (per-step bootstraps).
        max_ep = int(getattr(envs, "max_episode_steps", getattr(envs, "max_episode_length", 0)) or 0)
        self.defer_boot = (bool(_cfg(config, "defer_bootstrap", True)) and not self.raw_obs
                           and hasattr(envs, "step_device") and max_ep > 0)
        if self.defer_boot:
            S = max(1, -(-(T - 1) // max_ep))
            self.n_slots = S
            # [truncation slots (slot-major, S x N rows); last-step observations] as one buffer: the deferred critic
            # pass reads it whole (no concatenation launch)
            pair = torch.zeros(((S + 1) * N, D), **f32)
            self.slot_obs, self.boot_obs = pair[:S * N], pair[S * N:]
            self._boot_pair = pair
            self.slot_t = torch.full((S * N,), -1, dtype=torch.int32, device=dev)
            self.slot_overflow = torch.zeros((1,), dtype=torch.int32, device=dev)
            self._overflow_host = self._overflow_event = None
        # Raw-frame device envs whose truncations are always terminal (SynthAtari): K8 gets no per-step bootstrap
        # values (every mid-rollout close is terminal, boot 0) and the last step's are formed after the rollout —
        # one critic forward per iteration instead of one per env step (a2c_agent.py:66-72, 86-98).
        self.raw_defer = (self.raw_obs and self.device_env and bool(_cfg(config, "defer_bootstrap", True))
                          and bool(getattr(envs, "truncation_implies_terminal", False)))
        self._zero_vboot = torch.zeros((N,), **f32) if self.raw_defer else None
        # A2C over raw-frame device envs without that contract: a truncation at step t < T - 1 bootstraps with
        # V(reset frames) = V(obs of step t + 1), which is exactly the value the rollout stores in column t + 1 (the
        # same frames through the same critic forward, weights unchanged inside a rollout), so it is read from there
        # after the rollout (_raw_mid_from_next) instead of a second critic forward over every env at every step
        self.raw_mid_next = (self.raw_obs and self.device_env and self.boot_from_reset and not self.raw_defer
                             and bool(_cfg(config, "defer_bootstrap", True)))
        self._graph = None
        self._graph_pool = None
        # device env steps per replayed graph (train() falls back to single-step replays at chunk boundaries it
        # cannot meet); 1 = per-step graphs
        self.graph_chunk = int(_cfg(config, "graph_chunk", min(self.n_steps, 128)))
        self._chunk_graph = self._chunk_key = None
        # Model / log directories and the logger (agent.py:33-70).  model_dir_save is seed_<seed>_<time>
        # under model_dir, model_dir_load is model_dir itself (what load_model searches); both are created
        # when first written, not at construction (tests and benches build many agents).
        time_string = time.asctime().replace(" ", "").replace(":", "_")
        seed_tag = "seed_%d_" % self.seed
        model_dir = _cfg(config, "model_dir", "./models/")
        self.log_dir = _cfg(config, "log_dir", "./logs/")
        self.model_dir_save = os.path.join(os.getcwd(), model_dir, seed_tag + time_string)
        self.model_dir_load = model_dir
        self.writer = _make_writer(_cfg(config, "logger", "none"), os.path.join(os.getcwd(), self.log_dir,
                                                                               seed_tag + time_string))
        self.use_wandb = False
        # The reference's runner hands over the policy and a torch Adam; the hot path re-homes the parameters
        # into flat buffers (learner.enable_fast_path) so the fused kernels own the update.
        if bool(_cfg(config, "fast_path", True)) and self.device.type == "cuda":
            if bool(_cfg(config, "tunableop", True)):
                from .runner import enable_tuned_gemms
                enable_tuned_gemms()
            self.learner.enable_fast_path(fused_optimizer=bool(_cfg(config, "fused_adam", True)))
            # small minibatches: one hipGraph per minibatch slot (learners._graphed_mlp_update); the agent loop's
            # inputs are persistent buffers, which the graphs need (the drop-in learner.update path keeps it off)
            self.learner.graph_updates = bool(_cfg(config, "graph_update", True))

    def _make_learner(self, config, policy, optimizer, scheduler):
        raise NotImplementedError

    # ---- normalisation (agent.py:104-123) -----------------------------------------------------------
    def _obs_clip(self):
        return self.obsnorm_range if self.use_obsnorm else FLOAT_MAX

    def _normalize_into(self, x, out, to_buffer):
        mem = self.memory
        if to_buffer:
            T, D = self.n_steps, self.obs_dim
            ops.obs_normalize(x, self.obs_mean, self.obs_var, self._obs_clip(), out, col_out=mem.observations,
                              col_ld=T * D, cursor=self.cursor)
        else:
            ops.obs_normalize(x, self.obs_mean, self.obs_var, self._obs_clip(), out)

    # ---- one env step ---------------------------------------------------------------------------------
    def _rollout_mlp(self):
        """The learner's FusedActorCritic when it can drive the rollout forward (K14), else None."""
        fm_get = getattr(self.learner, "_fused_mlp", None)
        fm = fm_get() if fm_get is not None else None
        return fm if fm is not None and fm.rollout_ok else None

    def _env_fused(self, fm):
        """True when the device env's step runs inside the rollout's K14 launch (ops.rollout_policy_head_synthbox);
        fuse_env_step = False keeps the separate env GEMM + K7 launches."""
        ok = getattr(self.envs, "fusable_with_policy_step", None)
        return bool(fm is not None and self.fuse_env_step and ok is not None and ok(self.dist))

    def _sample_into_buffer(self, raw_x=None, fuse_env=False, post=None):
        """raw_x: the raw observations, normalised inside the fused trunk (see _rollout_step_device).
        fuse_env: also step the device env inside K14 (the caller then skips env.step_device()).
        post (with fuse_env): K8's post step in the same launch (K14F, _k14f_post; the caller then skips _post)."""
        mem = self.memory
        logp_buf = mem.auxiliary_infos["old_logp"] if self.algo == "ppo" else self.logp_scratch
        env_in = self.envs.act_in if self.device_env else self._act_scratch()
        fm = self._rollout_mlp()
        env = self.envs if fuse_env else None
        if raw_x is not None:
            T, D = self.n_steps, self.obs_dim
            fm.rollout_act(raw_x, self.dist, self.cursor, self.seed, mem.actions, logp_buf, mem.values, env_in,
                           act_clip=1.0, norm=(self.obs_mean, self.obs_var, self._obs_clip(), self.obs_norm,
                                               mem.observations, T * D, self.cursor), env=env, post=post)
            return
        if fm is not None:
            fm.rollout_act(self._policy_in, self.dist, self.cursor, self.seed, mem.actions, logp_buf, mem.values,
                           env_in, act_clip=1.0, env=env, post=post)
            return
        if post is not None:
            raise RuntimeError("K14F needs the fused rollout forward")
        head, logstd, v = self._heads(self._policy_in)
        ops.rollout_sample(self.dist, head.contiguous(), logstd, v.contiguous(), self.cursor, self.seed,
                           mem.actions, logp_buf, mem.values, env_in, act_clip=1.0)

    def _rollout_cnn(self):
        """The learner's explicit CNN forward (fused_cnn.FusedCNNActorCritic) for raw-frame policies, else None."""
        get = getattr(self.learner, "_fused_cnn", None)
        return get() if (get is not None and self.raw_obs) else None

    @torch.no_grad()
    def _heads(self, x):
        fc = self._rollout_cnn() if x.dtype == torch.uint8 else None
        if fc is not None:
            return fc.heads(x)
        return policy_heads(self.policy, x)

    def _act_scratch(self):
        if getattr(self, "_env_in", None) is None:
            A = self.action_space.n if self.discrete else int(np.prod(self.action_space.shape))
            self._env_in = torch.zeros((self.n_envs, A), dtype=torch.float32, device=self.device)
        return self._env_in

    def _post(self, rew, term, trunc, final_obs):
        mem = self.memory
        # A2C over a device env stepped per step (replayed graphs: the host does not know which column is the last):
        # both bootstrap values, K8 takes V(next obs) for closures before the last step (boot_from_reset)
        mid = self.boot_from_reset and self.device_env
        if self.raw_obs:
            v_boot = self._zero_vboot if self.raw_defer else self._heads(final_obs)[2]
            v_mid = (self._heads(self.envs.obs)[2] if (mid and not self.raw_defer and not self.raw_mid_next)
                     else None)
            self._post_kernel(rew, term, trunc, v_boot, v_mid)
            return
        if self.defer_boot:
            # final-obs normalisation folded into K8: kept truncation rows and, at the last step, every env's
            # normalised final observation (boot_obs) — no separate normalise launch per step; with fold_rms also the
            # next step's obs_rms.update (its statistics then merged once this step's normalisations are done)
            mem = self.memory
            rms = None
            if self._rms_fold_ok():
                if self._rms_fold_part is None:
                    self._rms_fold_part = torch.empty((2 * int(ops.lib().xpa_rollout_post_num_blocks(self.n_envs)),
                                                       self.obs_dim), dtype=torch.float64, device=self.device)
                rms = (self.envs.obs, self.obs_count, self._rms_fold_part)
            ops.rollout_post(rew, term, trunc, None, self.cursor, self.ret_mean, self.ret_var, self.ret_count,
                             self.returns, mem.rewards, mem.terminals, mem.closed, mem.boot, self.gamma,
                             mask_returns=(self.algo == "ppo"), use_rewnorm=self.use_rewnorm,
                             rew_range=self.rewnorm_range, atari_lifeloss=self.atari,
                             deferred=(final_obs, self.slot_obs, self.slot_t, self.slot_overflow, self.obs_mean,
                                       self.obs_var, self._obs_clip(), self.boot_obs)
                             + ((self.envs.obs,) if self.boot_from_reset else ()),
                             workspace=self.post_ws, rms=rms)
            return
        self._normalize_into(final_obs, self.boot_obs, False)
        v_boot = self._boot_values(self.boot_obs)
        v_mid = None
        if mid:
            if getattr(self, "_mid_obs", None) is None:
                self._mid_obs = torch.empty_like(self.boot_obs)
            self._normalize_into(self.envs.obs, self._mid_obs, False)
            v_mid = self._boot_values(self._mid_obs)
        self._post_kernel(rew, term, trunc, v_boot, v_mid)

    def _boot_values(self, x):
        fm = self._rollout_mlp()
        if fm is not None:
            return fm.rollout_value(x)
        with torch.no_grad():
            return policy_heads(self.policy, x)[2]

    def _post_kernel(self, rew, term, trunc, v_boot, v_mid=None):
        mem = self.memory
        ops.rollout_post(rew, term, trunc, v_boot.contiguous(), self.cursor, self.ret_mean, self.ret_var,
                         self.ret_count, self.returns, mem.rewards, mem.terminals, mem.closed, mem.boot, self.gamma,
                         mask_returns=(self.algo == "ppo"), use_rewnorm=self.use_rewnorm,
                         rew_range=self.rewnorm_range, atari_lifeloss=self.atari, workspace=self.post_ws,
                         v_boot_mid=v_mid.contiguous() if v_mid is not None else None)

    def _rms_fold_ok(self):
        """The next step's obs_rms.update rides in the step's last launch — K14F (_k14f_on) or, with FOLD_RMS, K8 —
        (device env, per-rank statistics, deferred bootstraps, D <= 64)."""
        return ((self.fold_rms or self._k14f_on()) and self.device_env and self.use_obsnorm and not self.sync_obs_rms
                and self.defer_boot and not self.raw_obs and self.obs_dim <= 64 and self.envs.obs.dim() == 2
                and self.envs.obs.stride(1) == 1)

    def _k14f_on(self, fuse=None):
        """K8's post step runs inside the env-fused K14 launch (K14F): fused env step, deferred bootstraps."""
        if fuse is None:
            fuse = self._env_fused(self._rollout_mlp())
        return bool(fuse and self.fuse_post and self.defer_boot and not self.raw_obs)

    def _k14f_post(self, fuse):
        """K14F's post-step arguments (ops.rollout_policy_head_synthbox(post=)) — the deferred, normalised K8 call of
        _post, with the next step's obs_rms.update where _rms_fold_ok — or None where K14F does not apply."""
        if not self._k14f_on(fuse):
            return None
        rms = self._rms_fold_ok()
        if self._k14f_ws is None or self._k14f_ws[0] != rms:   # graph-capture safe: allocated on the first (eager) step
            self._k14f_ws = (rms, ops.rollout_step_workspace(self.n_envs, self.obs_dim, rms, self.device))
        mem = self.memory
        return dict(slot_obs=self.slot_obs, slot_t=self.slot_t, overflow=self.slot_overflow,
                    slot_from_next=self.boot_from_reset, obs_mean=self.obs_mean, obs_var=self.obs_var,
                    obs_count=self.obs_count if rms else None, obs_clip=self._obs_clip(), boot_norm=self.boot_obs,
                    ret_mean=self.ret_mean, ret_var=self.ret_var, ret_count=self.ret_count, returns=self.returns,
                    buf_rew=mem.rewards, buf_term=mem.terminals, buf_closed=mem.closed, buf_boot=mem.boot,
                    gamma=self.gamma, mask_returns=(self.algo == "ppo"), use_rewnorm=self.use_rewnorm,
                    rew_range=self.rewnorm_range, atari_lifeloss=self.atari, workspace=self._k14f_ws[1])

    def _rms_update(self, x):
        if self.sync_obs_rms:
            import torch.distributed as tdist
            ops.rms_update(x, self.obs_mean, self.obs_var, self.obs_count, partials=self.rms_part,
                           reduce_partials=lambda t: tdist.all_reduce(t, op=tdist.ReduceOp.SUM), world=self.world)
        else:
            ops.rms_update(x, self.obs_mean, self.obs_var, self.obs_count, partials=self.rms_part,
                           ticket=self._rms_ticket)

    def _sync_rms_rollout(self):
        """sync_obs_rms = "rollout": every rank's rollout rows merged into the common start statistics (rms_rollout_sync,
        one all-reduce of 2 D + 1 doubles per rollout), so every rank leaves the rollout with the same obs_rms."""
        import torch.distributed as tdist
        m, v, c = rms_rollout_sync(self._rms_c0, (self.obs_mean, self.obs_var, self.obs_count),
                                   lambda t: tdist.all_reduce(t, op=tdist.ReduceOp.SUM))
        self.obs_mean.copy_(m)
        self.obs_var.copy_(v)
        self.obs_count.copy_(c)
        self._rms_c0 = None

    def _small_rollout(self):
        """K32's argument block (xpa_small_rollout_cartpole) when whole device env steps run as one launch: a CartPole
        device env with deferred bootstraps, no per-step collective, and the small_policy_layers policy shape; else
        None.  Rebuilt when the parameters are re-homed (the block holds their pointers)."""
        if not self.fused_rollout or not self.device_env or self.device.type != "cuda":
            return None
        key = tuple(p.data_ptr() for p in self.policy.parameters()) + (self.memory.observations.data_ptr(),
                                                                      self.memory.actions.data_ptr())
        if self._k32_key != key:
            self._k32_key, self._k32 = key, self._build_small_rollout()
        return self._k32

    def _build_small_rollout(self):
        env = self.envs
        get = getattr(self.learner, "small_policy_layers", None)
        layers = get() if get is not None else None
        if (layers is None or getattr(env, "kind", None) != "cartpole" or not self.defer_boot or self.raw_obs
                or self.sync_obs_rms or self.algo not in ("ppo", "a2c") or self.obs_dim != 4):
            return None
        (l0, l1, la, l2, lc), code, slope = layers
        N, T, D = self.n_envs, self.n_steps, self.obs_dim
        h0, h1, h2, k = l0.out_features, l1.out_features, l2.out_features, la.out_features
        if h0 not in (32, 64) or h1 not in (32, 64) or h2 not in (32, 64) or k != 2 or l0.in_features != D:
            return None
        lf = int(ops.lib().xpa_small_rollout_lds_floats(N, D, h0, h1, h2, k))
        if not 0 < lf <= 16384:
            return None
        mem = self.memory
        bufs = (mem.observations, mem.actions, mem.values, mem.rewards, mem.terminals, mem.boot)
        if any(b.dtype != torch.float32 or not b.is_contiguous() for b in bufs) or not mem.closed.is_contiguous():
            return None
        a = _lib.XpaSmallRolloutArgs()
        a.n_envs, a.horizon, a.steps, a.d_in, a.h0, a.h1, a.h2, a.k = N, T, 1, D, h0, h1, h2, k
        a.act_code, a.use_obsnorm, a.n_slots = int(code), int(self.use_obsnorm), int(self.n_slots)
        a.mask_returns, a.use_rewnorm, a.max_episode_steps = int(self.algo == "ppo"), int(self.use_rewnorm), \
            int(env.max_episode_steps)
        a.slot_reset_obs = int(self.boot_from_reset)
        a.slope, a.obs_clip, a.gamma, a.rew_range = float(slope), float(self._obs_clip()), float(self.gamma), \
            float(self.rewnorm_range)
        a.seed, a.env_seed = int(self.seed) & 0xFFFFFFFF, int(env.noise_seed) & 0xFFFFFFFF
        p = ops._p
        a.W0, a.b0, a.W1, a.b1, a.W2, a.b2 = (p(l0.weight), p(l0.bias), p(l1.weight), p(l1.bias), p(l2.weight),
                                              p(l2.bias))
        a.Wa, a.ba, a.Wc, a.bc = p(la.weight), p(la.bias), p(lc.weight), p(lc.bias)
        a.obs_mean, a.obs_var, a.obs_count = p(self.obs_mean), p(self.obs_var), p(self.obs_count)
        a.obs_norm, a.ld_norm = p(self.obs_norm), self.obs_norm.stride(0)
        logp_buf = mem.auxiliary_infos["old_logp"] if self.algo == "ppo" else self.logp_scratch
        a.buf_obs, a.buf_act, a.buf_logp, a.buf_val = p(mem.observations), p(mem.actions), p(logp_buf), p(mem.values)
        a.buf_rew, a.buf_term, a.buf_closed, a.buf_boot = p(mem.rewards), p(mem.terminals), p(mem.closed), p(mem.boot)
        a.act_in, a.ld_act = p(env.act_in), env.act_in.stride(0)
        a.env_state, a.env_obs, a.ld_obs = p(env.state), p(env.obs), env.obs.stride(0)
        a.final_obs, a.env_rew, a.env_term, a.env_trunc = p(env.final_obs), p(env.rew), p(env.term), p(env.trunc)
        a.ep_step, a.ep_index, a.ep_score = p(env.ep_step), p(env.ep_index), p(env.ep_score)
        a.ep_last_score, a.ep_last_len = p(env.ep_last_score), p(env.ep_last_len)
        a.returns, a.ret_mean, a.ret_var, a.ret_count = p(self.returns), p(self.ret_mean), p(self.ret_var), \
            p(self.ret_count)
        a.slot_obs, a.slot_t, a.overflow = p(self.slot_obs), p(self.slot_t), p(self.slot_overflow)
        a.boot_norm, a.ld_boot = p(self.boot_obs), self.boot_obs.stride(0)
        a.cursor = p(self.cursor)
        return a

    def _small_rollout_launch(self, a, steps):
        a.steps = int(steps)
        _lib.check(ops.lib().xpa_small_rollout_cartpole(ctypes.byref(a), ops._stream(self.device)),
                   "xpa_small_rollout_cartpole")

    def _rollout_step_device(self):
        env = self.envs
        k32 = self._small_rollout()
        if k32 is not None:
            self._small_rollout_launch(k32, 1)
            return
        x = env.obs
        if self.raw_obs:
            ops.store_column(x, self.memory.observations, self.cursor)
            self._policy_in = x
        else:
            if getattr(env, "resets", 0) != self._rms_resets:
                self._rms_resets, self._rms_pending = getattr(env, "resets", 0), True
            if self.use_obsnorm and (self._rms_pending or not self._rms_fold_ok()):
                self._rms_update(x)
                self._rms_pending = False
            fm = self._rollout_mlp()
            if fm is not None and fm.thin0 and x.stride(1) == 1:
                fuse = self._env_fused(fm)
                post = self._k14f_post(fuse)
                # normalisation fused into the trunk's first layer
                self._sample_into_buffer(raw_x=x, fuse_env=fuse, post=post)
                if not fuse:
                    env.step_device()
                if post is None:
                    self._post(env.rew, env.term, env.trunc, env.final_obs)
                return
            self._normalize_into(x, self.obs_norm, True)
        fuse = self._env_fused(self._rollout_mlp())
        post = self._k14f_post(fuse)
        self._sample_into_buffer(fuse_env=fuse, post=post)
        if not fuse:
            env.step_device()
        if post is None:
            self._post(env.rew, env.term, env.trunc, env.final_obs)

    def _rollout_step_graph(self):
        """The device env step captured once into a hipGraph and replayed: every per-step argument
        (buffer column, RNG step) lives in the device cursor, so the same graph serves all steps."""
        if self._small_rollout() is not None:   # one launch per step: nothing to capture
            self._rollout_step_device()
            return
        key = tuple(p.data_ptr() for p in self.policy.parameters())
        if self._graph is not None and key != self._graph_key:
            self._graph = None  # parameters were re-homed (e.g. flat buffers attached): re-capture
        if self._graph is None:
            self._graph_key = key
            side = torch.cuda.Stream(self.device)
            side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(side):
                self._rollout_step_device()        # a real step (also warms up BLAS handles)
            torch.cuda.current_stream(self.device).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=self._graph_pool):
                self._rollout_step_device()        # recorded, not executed
            self._graph = g
            return
        self._graph.replay()

    def _rollout_chunk_graph(self, k):
        """k consecutive device env steps captured into ONE hipGraph (k x 5 kernels) and replayed as a unit: a
        per-step replay leaves the GPU idle ~8 us between graphs while the host launches the next (r02 trace:
        127 such gaps = 1.0 ms of a 72 ms iteration).  Same replay invariance as _rollout_step_graph."""
        k32 = self._small_rollout()
        if k32 is not None:   # the k steps as one K32 launch
            self._small_rollout_launch(k32, k)
            return k
        key = (k,) + tuple(p.data_ptr() for p in self.policy.parameters())
        if self._chunk_graph is not None and key != self._chunk_key:
            self._chunk_graph = None
        if self._chunk_graph is None:
            if self._graph is None:
                self._rollout_step_graph()   # a real first step + the single-step graph (warm-up, BLAS handles)
                return 1
            self._chunk_key = key
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=self._graph_pool):
                for _ in range(k):
                    self._rollout_step_device()   # recorded, not executed
            self._chunk_graph = g
        self._chunk_graph.replay()
        return k

    def _rollout_step_host(self):
        """One step of ppoclip_agent.py:59-111 / a2c_agent.py:57-107 over a host VecEnv (numpy in / out, reset_obs
        in infos; gym_vec_env.py:148-231): the same kernels with per-step H2D / D2H copies, and the loop's host
        semantics kept as they are (checked step for step against oracle.cpu_ref.VecAgentRef,
        tests/test_gpu_hostenv.py):
          * a train() call starts from envs.buf_obs (ppoclip_agent.py:60): a row whose env ended on the previous
            call's last step still holds its final observation there;
          * without obs-norm the reference stores `obs` after envs.step, and on a call's first step that is
            envs.buf_obs itself: the column holds what that array holds after the step (DummyVecEnv writes it in
            place, SubprocVecEnv rebinds it — the object kept here is read either way);
          * done envs continue from infos[i]["reset_obs"]; with env_name "Atari" a life loss (terminal, not
            truncated) keeps the path and the observation (ppoclip_agent.py:93-94);
          * A2C's mid-rollout truncation bootstraps are V(norm(reset_obs)) (a2c_agent.py:88-95, boot_from_reset)."""
        env, dev = self.envs, self.device
        dt = np.uint8 if self.raw_obs else np.float32
        shape = (self.n_envs,) + (tuple(self.obs_shape) if self.raw_obs else (-1,))
        alias = None
        if self._host_obs is None:
            self._host_obs = np.array(env.buf_obs, dt, copy=True).reshape(shape)
            if not self.use_obsnorm:
                alias = env.buf_obs
        x = torch.as_tensor(self._host_obs, device=dev)
        if self.raw_obs:
            ops.store_column(x.contiguous(), self.memory.observations, self.cursor)
            self._policy_in = x
        else:
            if self.use_obsnorm:
                self._rms_update(x)
            self._normalize_into(x, self.obs_norm, True)
        self._sample_into_buffer()
        t = self._t
        acts = (self.memory.actions[:, t]).cpu().numpy()
        if self.discrete:
            acts = acts.astype(np.int64)
        next_obs, rews, terms, truncs, infos = env.step(acts)
        if alias is not None:   # the stored column is what the vec env's buf_obs holds now
            col = self.memory.observations[:, t]
            col.copy_(torch.as_tensor(np.asarray(alias, dt).reshape(col.shape), device=dev))
        next_obs = np.asarray(next_obs, dt).reshape(shape)
        obs = next_obs.copy()
        for i in range(self.n_envs):
            if terms[i] or truncs[i]:
                if self.atari and not truncs[i]:
                    continue
                obs[i] = np.asarray(infos[i]["reset_obs"], dt).reshape(obs[i].shape)
                self.current_episode[i] += 1
        # K8 reads the bootstrap rows where a path closes: the final observations, except A2C's mid-rollout
        # truncations (reset_obs); the last step's closures use the final observations for every algorithm
        boot_src = obs if (self.boot_from_reset and t < self.n_steps - 1) else next_obs
        self._post(torch.as_tensor(np.asarray(rews, np.float32), device=dev),
                   torch.as_tensor(np.asarray(terms, np.uint8), device=dev),
                   torch.as_tensor(np.asarray(truncs, np.uint8), device=dev), torch.as_tensor(boot_src, device=dev))
        self._host_obs = obs

    # ---- buffer-full phase ------------------------------------------------------------------------------
    def epoch_permutation(self, n, counter=None):
        """The minibatch permutation of the next epoch (ppoclip_agent.py:76-81): a device Feistel
        permutation keyed by (config.seed, epoch counter) — one launch instead of a sort."""
        if counter is not None:   # an explicit epoch (tests, replays): a fresh tensor, no live buffer touched
            return ops.random_permutation(n, self.seed, counter,
                                          out=torch.empty(n, dtype=torch.int64, device=self.device))
        counter = self._perm_counter
        self._perm_counter += 1
        if self._perm_buf is None or self._perm_buf.shape[0] != n:
            self._perm_buf = torch.empty(n, dtype=torch.int64, device=self.device)
        return ops.random_permutation(n, self.seed, counter, out=self._perm_buf)

    def _deferred_bootstraps(self, hidden_only=False):
        """V([truncation slots; last-step final obs]) in one critic pass ([2N] values), or with hidden_only the
        critic's hidden pre-activations ([2N, 256], for the value-fused scan xpa_gae_scan_value; None when the
        policy has no fused critic)."""
        x = self._boot_pair
        fm = self._rollout_mlp()
        if hidden_only:
            return fm.rollout_value_hidden(x)
        if fm is not None:
            v = fm.rollout_value(x)
        else:
            with torch.no_grad():
                v = policy_heads(self.policy, x)[2].contiguous()
        return v.reshape(-1)

    def _raw_last_bootstraps(self):
        """raw_defer: V(final frames of the last step) for the last column's bootstraps (0 where terminal), written
        by xpa_rollout_bootstrap_fixup; a mid-rollout non-terminal close (which would have needed its own value)
        contradicts the env's truncation_implies_terminal contract and raises."""
        mem = self.memory
        T = self.n_steps
        bad = bool(((mem.closed[:, :T - 1] != 0) & (mem.terminals[:, :T - 1] == 0)).any())
        if bad:
            raise RuntimeError("a non-terminal truncation inside the rollout: the env breaks truncation_implies_"
                               "terminal; set config.defer_bootstrap = False")
        N = self.n_envs
        if getattr(self, "_raw_vb", None) is None:
            self._raw_vb = torch.zeros((2 * N,), dtype=torch.float32, device=self.device)
            self._raw_slots = torch.full((N,), -1, dtype=torch.int32, device=self.device)
        self._raw_vb[N:].copy_(self._heads(self.envs.final_obs)[2])
        ops.bootstrap_fixup(self._raw_vb, self._raw_slots, mem.terminals, mem.boot)

    def _raw_mid_from_next(self):
        """raw_mid_next: the bootstrap of every non-terminal close before the last step is V(reset frames) =
        values[:, t + 1] (a2c_agent.py:88-95: obs[i] = reset_obs, then the critic on next_obs); K8 wrote V(final
        frames) there, which only the last column keeps."""
        mem = self.memory
        T = self.n_steps
        if T < 2:
            return
        mid = (mem.closed[:, :T - 1] != 0) & (mem.terminals[:, :T - 1] == 0)
        b = mem.boot[:, :T - 1]
        b.copy_(torch.where(mid, mem.values[:, 1:T], b))

    def _check_overflow(self):
        # More truncations per env than slots cannot happen for the device envs (their one truncation source is the
        # time limit, and __init__ sizes n_slots from it), so this guard of the env contract is checked without a
        # host sync: copied to pinned memory here and read one iteration later.
        if self._overflow_host is None:
            self._overflow_host = torch.zeros((1,), dtype=torch.int32, pin_memory=True)
            self._overflow_event = torch.cuda.Event()
        elif self._overflow_event.query() and int(self._overflow_host[0]):
            raise RuntimeError("an env truncated more often than its time limit allows within one rollout (device env "
                               "contract broken); set config.defer_bootstrap = False")
        self._overflow_host.copy_(self.slot_overflow, non_blocking=True)
        self._overflow_event.record()

    def _update_phase(self):
        mem = self.memory
        mem.size = self.n_steps
        if self.raw_defer:
            self._raw_last_bootstraps()
        elif self.raw_mid_next:
            self._raw_mid_from_next()
        zc = vk = None
        one_slot = self.defer_boot and self.n_slots == 1   # the fused scans take one deferred truncation per env
        if (one_slot and not self.atari and not mem._pending and self.fuse_value_gae and self.value_gemm
                and self._rollout_mlp() is not None):
            if getattr(self, "_vboot", None) is None:
                self._vboot = torch.empty(self._boot_pair.shape[0], dtype=torch.float32, device=self.device)
            vk = self._rollout_mlp().rollout_value_split(self._boot_pair, out=self._vboot)
        if (vk is None and one_slot and not self.atari and not mem._pending and self.fuse_value_gae
                and ops.gae_value_ok(self.n_steps) and self._rollout_mlp() is not None):
            zc = self._deferred_bootstraps(hidden_only=True)
        if vk is not None:
            # K40V's values, then one launch: the fixup's bootstrap writes fused into the compact-closure GAE scan
            ops.gae_scan_compact(mem.rewards, mem.values, mem.terminals, self.slot_t, vk, mem.gamma, mem.gae_lam,
                                 mem.use_gae, adv=mem._advantages, ret=mem._returns, boot=mem.boot)
            mem._dirty = False
            self.gae_form = "compact"
        elif zc is not None:
            # one launch: the critic's output layer, the fixup's bootstrap writes and the compact GAE scan
            fm = self._rollout_mlp()
            lin_co = fm.critic[-1][0]
            _, code, slope = fm.critic[-2]
            ops.gae_scan_value(mem.rewards, mem.values, mem.terminals, self.slot_t, zc, (code, slope), lin_co.weight,
                               lin_co.bias, mem.gamma, mem.gae_lam, mem.use_gae, adv=mem._advantages,
                               ret=mem._returns, boot=mem.boot)
            mem._dirty = False
            self.gae_form = "value"
        elif self.defer_boot:
            vboot = self._deferred_bootstraps()
            if one_slot and not self.atari and not mem._pending:
                # one launch: the fixup's bootstrap writes fused into the compact-closure GAE scan
                ops.gae_scan_compact(mem.rewards, mem.values, mem.terminals, self.slot_t, vboot, mem.gamma,
                                     mem.gae_lam, mem.use_gae, adv=mem._advantages, ret=mem._returns, boot=mem.boot)
                mem._dirty = False
                self.gae_form = "compact"
            else:
                ops.bootstrap_fixup(vboot, self.slot_t, mem.terminals, mem.boot)
                mem.compute_advantages()
        else:
            mem.compute_advantages()
        NT, B = self.buffer_size, self.batch_size
        obs_flat = mem.observations.reshape((NT,) + tuple(mem.observations.shape[2:]))
        act_flat = mem.actions.reshape(-1)
        adv_flat = mem.advantages.reshape(-1)
        ret_flat = mem.returns.reshape(-1)
        logp_flat = mem.auxiliary_infos["old_logp"].reshape(-1) if self.algo == "ppo" else None
        use_advnorm = mem.use_advnorm
        scalars = None
        fm = self._rollout_mlp() if not self.global_advnorm else None
        rows_path = fm is not None and self.fuse_gather and fm.rows_ok(obs_flat)
        # graphed small-batch updates (C1): the epoch's minibatches go to the learner as one list, which replays them
        # as one captured graph once every slot is captured (learners.update_epoch)
        epoch_batches = (not rows_path and not self.global_advnorm and getattr(self.learner, "graph_updates", False)
                         and hasattr(self.learner, "update_epoch"))
        # K30: the whole small-MLP update (gather + forward + loss + backward + clip + Adam) in one launch per
        # minibatch, an epoch of them one captured graph (learners.small_epoch)
        small = (not rows_path and not self.global_advnorm and hasattr(self.learner, "small_update_ok")
                 and self.learner.small_update_ok(obs_flat, B))
        for _ in range(self.n_epoch):
            perm = self.epoch_permutation(NT)
            if small:
                batches = [(perm[s:s + B], act_flat, adv_flat, ret_flat, logp_flat) for s in range(0, NT, B)]
                outs = self.learner.small_epoch(obs_flat, batches, use_advnorm, keep_all=self.update_log is not None)
                scalars = outs[-1]
                if self.update_log is not None:
                    self.update_log.extend(outs)
                continue
            batches = []
            for start in range(0, NT, B):
                idx = perm[start:start + B]
                b = idx.shape[0]
                if rows_path:
                    # K4 folded into K13: the update reads the minibatch rows (and forms the adv moments) through idx
                    parts = self.__dict__.setdefault("_adv_parts", {})
                    g = ops.gather_num_partials(b)
                    if g not in parts:   # one per minibatch size (a ragged last minibatch keeps its own)
                        parts[g] = torch.empty((g, 2), dtype=torch.float64, device=self.device)
                    self.adv_part = parts[g]
                    part = self.adv_part if use_advnorm else None
                    scalars = self.learner.update_fused(Rows(obs_flat, idx), idx, act_flat, adv_flat, ret_flat,
                                                        logp_flat, part)
                    if self.update_log is not None:
                        self.update_log.append(scalars.clone())
                    continue
                # one (obs_mb, adv_part) pair per minibatch size: a ragged last minibatch keeps its own buffers, so
                # the pointers the learner's slot graphs are keyed by stay stable across epochs
                mbs = self.__dict__.setdefault("_mb_bufs", {})
                bufs = mbs.get((b, obs_flat.dtype, tuple(obs_flat.shape[1:])))
                if bufs is None:
                    bufs = (torch.empty((b,) + tuple(obs_flat.shape[1:]), dtype=obs_flat.dtype, device=self.device),
                            torch.empty((ops.gather_num_partials(b), 2), dtype=torch.float64, device=self.device))
                    mbs[(b, obs_flat.dtype, tuple(obs_flat.shape[1:]))] = bufs
                self.obs_mb, self.adv_part = bufs
                def gather(idx=idx, obs_out=self.obs_mb, part=self.adv_part):
                    return ops.gather_minibatch(idx, obs_flat, adv=adv_flat if use_advnorm else None,
                                                obs_out=obs_out, adv_partials=part if use_advnorm else None)
                if epoch_batches:
                    batches.append((self.obs_mb, idx, act_flat, adv_flat, ret_flat, logp_flat,
                                    self.adv_part if use_advnorm else None, gather))
                    continue
                if not self.global_advnorm:
                    # the gather rides in the learner's slot graph when the update is graphed (writes obs_mb / adv_part)
                    scalars = self.learner.update_fused(self.obs_mb, idx, act_flat, adv_flat, ret_flat, logp_flat,
                                                        self.adv_part if use_advnorm else None, pre=gather)
                    if self.update_log is not None:
                        self.update_log.append(scalars.clone())
                    continue
                obs_mb, part = gather()
                if part is not None:
                    import torch.distributed as tdist
                    tdist.all_reduce(part, op=tdist.ReduceOp.SUM)   # (sum, sumsq) over all ranks' minibatches,
                    part.div_(self.world)                           # averaged: mean / var of the global minibatch
                scalars = self.learner.update_fused(obs_mb, idx, act_flat, adv_flat, ret_flat, logp_flat, part)
                if self.update_log is not None:
                    self.update_log.append(scalars.clone())
            if batches:
                outs = self.learner.update_epoch(batches, keep_all=self.update_log is not None)
                scalars = outs[-1]
                if self.update_log is not None:
                    self.update_log.extend(outs)
        self.last_info = scalars
        self.iterations += 1
        if self.defer_boot:
            # after the whole update is enqueued: a D2H copy here no longer holds the host back before the critic
            # pass + GAE (issued right after the rollout graph, it made the GPU idle 30-100 us before K1V)
            self._check_overflow()

    def log_infos(self, info, x_index):
        """agent.py:81-94: every entry to the logger (tensorboard when importable, else JSON lines in
        log_dir) and to log_hook."""
        if self.log_hook is not None:
            self.log_hook(info, x_index)
        if self.writer is not None:
            self.writer.write(info, x_index)

    def _host_info(self):
        info = self.learner._info(self.last_info)
        info["iteration"] = self.iterations
        info["step"] = self.current_step
        return info

    # ---- public API (ppoclip_agent.py:59-111) -------------------------------------------------------------
    def train(self, train_steps, log=True):
        if not self.device_env:
            step_fn = self._rollout_step_host
            self._host_obs = None   # every call starts from envs.buf_obs (ppoclip_agent.py:60)
        else:
            step_fn = self._rollout_step_graph if self.use_graph else self._rollout_step_device
        chunk = self.graph_chunk if (self.device_env and self.use_graph) else 1
        left = train_steps
        while left > 0:
            t0 = time.perf_counter()
            if self._t == 0:
                if self.sync_obs_rms_rollout:   # the common statistics every rank starts this rollout from
                    self._rms_c0 = (self.obs_mean.clone(), self.obs_var.clone(), self.obs_count.clone())
                fc = self._rollout_cnn()
                if fc is not None:
                    fc.refresh()   # outside any captured graph: the replays read the refreshed weight copy
                fm = self._rollout_mlp()
                if fm is not None:
                    fm.rollout_refresh()   # K40R's weight planes for this rollout (same: outside the graphs)
            if chunk > 1 and left >= chunk and self._t % chunk == 0 and self.n_steps - self._t >= chunk:
                k = self._rollout_chunk_graph(chunk)
            else:
                step_fn()
                k = 1
            left -= k
            self._t += k
            self.memory.ptr = self._t % self.n_steps
            self.memory.size = min(self.memory.size + k, self.n_steps)
            self.current_step += self.n_envs * k
            t1 = time.perf_counter()
            self.timers["rollout"] += t1 - t0
            if self._t == self.n_steps:
                if self.sync_obs_rms_rollout and self._rms_c0 is not None:
                    self._sync_rms_rollout()
                if self.phase_events is not None:   # measurement hook (bench.py): rollout | update split
                    self.phase_events.append(("rollout_end", torch.cuda.Event(enable_timing=True)))
                    self.phase_events[-1][1].record()
                self._update_phase()
                if self.phase_events is not None:
                    self.phase_events.append(("update_end", torch.cuda.Event(enable_timing=True)))
                    self.phase_events[-1][1].record()
                self._t = 0
                self.memory.ptr, self.memory.size = 0, 0
                if log:
                    info = self._host_info()
                    self.infos.append(info)
                    self.log_infos(info, self.current_step)
                self.timers["update"] += time.perf_counter() - t1

    def save_model(self, model_name):
        """agent.py:74-76: the policy's state_dict to model_dir_save/model_name."""
        os.makedirs(self.model_dir_save, exist_ok=True)
        self.learner.save_model(self.model_dir_save + "/" + model_name)

    def load_model(self, path, seed=1):
        """agent.py:78-79 -> learner.py:27-48 (newest file of the seed_<seed> directory under path)."""
        self.learner.load_model(path, seed)

    # ---- test (ppoclip_agent.py:113-165, a2c_agent.py:109-160) ----------------------------------------
    @torch.no_grad()
    def _test_action(self, x):
        head, logstd, _ = policy_heads(self.policy, x)
        if self.discrete:
            a = torch.distributions.Categorical(logits=head).sample()
        else:
            a = head + logstd.exp() * torch.randn_like(head)   # stochastic_sample of Normal(mu, exp(logstd))
        return a.cpu().numpy()

    def _test_obs(self, obs):
        """The reference updates obs_rms in test() too (ppoclip_agent.py:125) and normalises with it."""
        x = obs if isinstance(obs, torch.Tensor) else torch.as_tensor(np.asarray(obs))
        if self.raw_obs:
            return x.to(self.device)
        x = x.to(device=self.device, dtype=torch.float32).reshape(x.shape[0], -1).contiguous()
        if self.use_obsnorm:
            ops.rms_update(x, self.obs_mean, self.obs_var, self.obs_count)
        out = torch.empty_like(x)
        ops.obs_normalize(x, self.obs_mean, self.obs_var, self._obs_clip(), out)
        return out

    def test(self, env_fn, test_episode):
        """Run the current policy (stochastic actions) on env_fn()'s envs until test_episode episodes have
        ended; returns their scores (infos[i]['episode_score'])."""
        test_envs = env_fn()
        num_envs = test_envs.num_envs
        current_episode, scores, best_score = 0, [], -np.inf
        obs, _ = test_envs.reset()
        obs = obs.cpu().numpy() if isinstance(obs, torch.Tensor) else np.asarray(obs)
        verbose = bool(_cfg(self.config, "test_mode", False))
        while current_episode < test_episode:
            acts = self._test_action(self._test_obs(obs))
            if self.discrete:
                acts = acts.astype(np.int64)
            next_obs, rewards, terminals, truncations, infos = test_envs.step(acts)
            obs = np.array(next_obs, copy=True)
            for i in range(num_envs):
                if terminals[i] or truncations[i]:
                    if self.atari and not truncations[i]:   # life loss: the game goes on
                        continue
                    obs[i] = infos[i]["reset_obs"]
                    scores.append(infos[i]["episode_score"])
                    current_episode += 1
                    best_score = max(best_score, infos[i]["episode_score"])
                    if verbose:
                        print("Episode: %d, Score: %.2f" % (current_episode, infos[i]["episode_score"]))
        if verbose:
            print("Best Score: %.2f" % best_score)
        self.log_infos({"Test-Episode-Rewards/Mean-Score": float(np.mean(scores)),
                        "Test-Episode-Rewards/Std-Score": float(np.std(scores))}, self.current_step)
        test_envs.close()
        return scores

    def finish(self):
        if self.writer is not None:
            self.writer.close()


class PPOCLIP_Agent(_OnPolicyAgent):
    algo = "ppo"

    def _make_learner(self, config, policy, optimizer, scheduler):
        return PPOCLIP_Learner(policy, optimizer, scheduler, _cfg(config, "device", None), _cfg(config, "model_dir", "./"),
                               vf_coef=config.vf_coef, ent_coef=config.ent_coef, clip_range=config.clip_range,
                               clip_grad_norm=config.clip_grad_norm, use_grad_clip=_cfg(config, "use_grad_clip", True))


class A2C_Agent(_OnPolicyAgent):
    algo = "a2c"

    def _make_learner(self, config, policy, optimizer, scheduler):
        return A2C_Learner(policy, optimizer, scheduler, _cfg(config, "device", None), _cfg(config, "model_dir", "./"),
                           config.vf_coef, config.ent_coef, config.clip_grad)


class PerDQN_Agent:
    """perdqn_agent.py:4-95 (BASELINE.json configs[4]): e-greedy DQN with prioritized replay, device-resident.

    Same constructor and train(train_steps) loop as the reference: each step stores (obs, act, rew, term, next)
    in the PER buffer (K6 store: the new leaf at max priority), and every training_frequency steps after
    start_training samples a batch (K6 sample: stratified prefix-sum descent + IS weights; K4 gathers the uint8
    frames), runs PerDQN_Learner.update (Q forwards / backward on PyTorch-ROCm, K19 TD / loss / gradient /
    priorities) and writes the |TD| priorities back (K6 update) without leaving the GPU.  PER_beta and the
    e-greedy rate follow perdqn_agent.py:74-95.  With a device env (step_device / act_in, e.g. the SynthAtari
    vec env with 18 actions) the loop never copies frames to the host; the coin flip of the e-greedy choice is
    the reference's np.random draw (one host draw per step, no sync)."""

    def __init__(self, config, envs, policy, optimizer, scheduler=None, device=None):
        from .per import PerOffPolicyBuffer
        self.config = config
        self.envs = envs
        self.policy = policy
        self.device = torch.device(device if device is not None else _cfg(config, "device", "cuda:0"))
        self.n_envs = envs.num_envs
        self.gamma = config.gamma
        self.train_frequency = config.training_frequency
        self.start_training = config.start_training
        self.start_greedy, self.end_greedy = config.start_greedy, config.end_greedy
        self.egreedy = config.start_greedy
        self.decay_step_greedy = _cfg(config, "decay_step_greedy", 1)
        self.observation_space, self.action_space = envs.observation_space, envs.action_space
        self.PER_beta0 = self.PER_beta = config.PER_beta0
        self.atari = _cfg(config, "env_name", "") == "Atari"
        obs_dtype = torch.uint8 if self.atari else torch.float32
        self.memory = PerOffPolicyBuffer(self.observation_space, self.action_space, {}, self.n_envs, config.n_size,
                                         config.batch_size, config.PER_alpha, device=self.device,
                                         seed=_cfg(config, "seed", 1), obs_dtype=obs_dtype)
        self.learner = PerDQN_Learner(policy, optimizer, scheduler, self.device, _cfg(config, "model_dir", "./"),
                                      config.gamma, config.sync_frequency)
        self.device_env = hasattr(envs, "step_device")
        self.current_step = 0
        self.current_episode = np.zeros(self.n_envs, np.int32)
        self.infos = []
        # perdqn_agent.py:57-66: train() starts from `obs = self.envs.buf_obs` and stores `obs` after envs.step, so the
        # first store of every train() call holds whatever that array holds after the step: the step's frames for a
        # vec env that writes buf_obs in place (DummyVecEnv, gym_vec_env.py:228), the pre-step ones for one that
        # rebinds it (SubprocVecEnv, gym_vec_env.py:101).  A host vec env is handled by keeping that object and
        # storing its contents; the device envs model the in-place DummyVecEnv (their final_obs).  Reproduced by
        # default (a drop-in stores what the reference stores); False stores the pre-step frames.
        self.alias_first_obs = bool(_cfg(config, "alias_first_obs", True))
        # optional callable() -> uniforms [n_envs, batch / n_envs] for the next PER sample (e.g. the reference's
        # recorded random.random() draws, memory_tools.py:415); None: the buffer's counter-hash uniforms
        self.uniform_source = None

    def _action(self, obs, egreedy=0.0):
        """perdqn_agent.py:47-54: argmax of the eval Q row, or (with probability egreedy, one draw for all envs)
        uniform random actions from np.random, as the reference draws them."""
        q = self.learner.q_values(obs)
        argmax_action = q.argmax(dim=-1)
        random_action = np.random.choice(self.action_space.n, self.n_envs)
        if np.random.rand() < egreedy:
            return torch.as_tensor(random_action, device=self.device)
        return argmax_action

    def _env_step(self, acts):
        """(next observation to store, rew, term, trunc); the observation the policy sees next is env.obs (device
        env: the kernel already continued done envs from their reset state) or self._host_obs."""
        env = self.envs
        if self.device_env:
            env.act_in.zero_()
            env.act_in.scatter_(1, acts.long().reshape(-1, 1), 1.0)
            env.step_device()
            return env.final_obs, env.rew, env.term, env.trunc
        nxt, rew, term, trunc, infos = env.step(acts.cpu().numpy())
        self._host_obs = np.array(nxt, copy=True)
        for i in range(self.n_envs):   # perdqn_agent.py:76-83: continue from reset_obs (not on an Atari life loss)
            if (term[i] or trunc[i]) and not (self.atari and not trunc[i]):
                self._host_obs[i] = infos[i]["reset_obs"]
        return nxt, rew, term, trunc

    def train(self, train_steps, sync_info=False):
        """perdqn_agent.py:56-95.  A host vec env: every call starts from envs.buf_obs (perdqn_agent.py:57), whose rows
        of envs that ended on the previous call's last step still hold their final frames."""
        env = self.envs
        buf0 = None
        if not self.device_env:
            buf0 = env.buf_obs
            self._host_obs = np.array(buf0, copy=True)
        for k in range(train_steps):
            obs = env.obs.clone() if self.device_env else self._host_obs
            acts = self._action(obs, self.egreedy)
            nxt, rew, term, trunc = self._env_step(acts)
            first = obs
            if k == 0 and self.alias_first_obs:
                first = nxt if self.device_env else np.array(buf0, copy=True)
            self.memory.store(first, acts, rew, term, nxt)
            if self.current_step > self.start_training and self.current_step % self.train_frequency == 0:
                u = self.uniform_source() if self.uniform_source is not None else None
                o, a, r, d, n, w, idxes = self.memory.sample(self.PER_beta, uniforms=u)
                td_abs, info = self.learner.update(o, a, r, n, d, sync_info=sync_info)
                self.memory.update_priorities(idxes, td_abs, check=False)
                info["epsilon-greedy"] = self.egreedy
                self.infos.append(info)
            self.PER_beta += (1 - self.PER_beta0) / train_steps
            self.egreedy = self.egreedy - (self.start_greedy - self.end_greedy) / train_steps
            self.current_step += self.n_envs
            if self.egreedy > self.end_greedy:
                self.egreedy = self.egreedy - (self.start_greedy - self.end_greedy) / self.decay_step_greedy


    def check_errors(self):
        """The device loop's error words since the last call (one host sync): PER sample draws clamped past the
        stored leaves, gathered indices outside the replay buffer, env steps without an action, actions outside
        [0, n) in the TD kernel, max-pool argmax outside the window.  All 0 unless something upstream is corrupt."""
        out = dict(zip(("per_sample", "gather"), self.memory.check_errors()))
        for name, t in (("env", getattr(self.envs, "err", None)), ("td_action", self.learner._err)):
            out[name] = int(t.item()) if t is not None else 0
            if t is not None:
                t.zero_()
        fq = self.learner._fused_q()
        e = getattr(fq.eval_trunk, "err", None) if fq is not None else None
        out["maxpool"] = int(e.item()) if e is not None else 0
        if e is not None:
            e.zero_()
        return out


REGISTRY = {"PPO_Clip": PPOCLIP_Agent, "A2C": A2C_Agent, "PerDQN": PerDQN_Agent}
Agent = _OnPolicyAgent


def get_total_iters(agent_name, args):
    """agent.py:144-145: the LinearLR horizon the runner and the examples use."""
    return args.running_steps


class _JsonlWriter:
    """Scalar sink for log_infos when no tensorboard / wandb is importable: one JSON object per line."""

    def __init__(self, log_dir):
        self.path = os.path.join(log_dir, "scalars.jsonl")
        self._f = None

    def write(self, info, step):
        if self._f is None:
            os.makedirs(os.path.dirname(self.path), exist_ok=True)
            self._f = open(self.path, "a")
        rec = {"step": int(step)}
        for k, v in info.items():
            if isinstance(v, dict):
                rec.update({"%s/%s" % (k, kk): float(vv) for kk, vv in v.items()})
            elif isinstance(v, (int, float, np.floating, np.integer)):
                rec[k] = float(v)
        self._f.write(json.dumps(rec) + "\n")

    def close(self):
        if self._f is not None:
            self._f.close()
            self._f = None


class _TensorboardWriter:
    def __init__(self, writer):
        self.w = writer

    def write(self, info, step):
        for k, v in info.items():
            if isinstance(v, dict):
                self.w.add_scalars(k, v, step)
            else:
                self.w.add_scalar(k, v, step)

    def close(self):
        self.w.close()


def _make_writer(logger, log_dir):
    """config.logger: 'tensorboard' / 'wandb' (the reference's choices) or 'none'.  tensorboard and wandb
    are optional: without them the scalars go to log_dir/scalars.jsonl."""
    if logger in (None, "none", "None", False):
        return None
    if logger == "tensorboard":
        try:
            from torch.utils.tensorboard import SummaryWriter
            os.makedirs(log_dir, exist_ok=True)
            return _TensorboardWriter(SummaryWriter(log_dir))
        except ImportError:
            pass
    return _JsonlWriter(log_dir)
