"""Device-resident synthetic vector environments for the on-policy benchmark (BASELINE.json configs).

SynthBoxVecEnv(n_envs, D, A) is the SynthBox(D, A) env of SURVEY.md §8(d), plugged in where the
reference builds envs (xuance/environment/__init__.py:76-78 NewEnv hook; DummyVecEnv_Gym contract of
xuance/environment/gym/gym_vec_env.py:148-231).  The state lives in HBM and a step is one GEMM
(X @ Wcat^T, hipBLASLt) plus the xpa_synthbox_step kernel, with auto-reset on done.

Dynamics (spec shared with the CPU checker oracle/synth_env.py; all randomness from a counter hash):
    x = W s + U clip(a, -1, 1) + NOISE * xi      (Discrete: U[:, a] via a one-hot row)
    s' = tanh(x), r = -mean(s'^2), terminated = s'[0] > TERM_THRESH, truncated at max_episode_steps
    reset s0 = RESET_SCALE * (2u - 1)
The host-facing step(actions) -> (obs, rew, term, trunc, infos) exists for the VecEnv contract and
tests; the agent's hot loop uses step_device() and never leaves the GPU.
"""
import numpy as np
import torch

from . import _lib, ops

W_GAIN, U_GAIN, NOISE, TERM_THRESH, RESET_SCALE = 1.25, 0.6, 0.35, 0.92, 0.1
SALT_W, SALT_U, SALT_RESET = 0x57A7E000, 0x0AC7E000, 0x5EED0000


def _mix32(x):
    x = np.asarray(x, dtype=np.uint32).copy()
    with np.errstate(over="ignore"):
        x ^= x >> np.uint32(16)
        x *= np.uint32(0x85EBCA6B)
        x ^= x >> np.uint32(13)
        x *= np.uint32(0xC2B2AE35)
        x ^= x >> np.uint32(16)
    return x


def _hash4(seed, k0, k1, k2):
    h = _mix32(_mix32(np.uint32(seed & 0xFFFFFFFF)) ^ np.asarray(k0, np.uint32))
    h = _mix32(h ^ np.asarray(k1, np.uint32))
    return _mix32(h ^ np.asarray(k2, np.uint32))


def _u01(h):
    return (np.asarray(h, np.uint32) >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def synthbox_matrices(seed, D, A, discrete=False):
    i = np.arange(D, dtype=np.uint32)[:, None]
    W = (2.0 * _u01(_hash4(seed, SALT_W, i, np.arange(D, dtype=np.uint32)[None, :])) - 1.0) * np.sqrt(3.0 / D) * W_GAIN
    gain, fan = (1.0, 1) if discrete else (U_GAIN, A)
    U = (2.0 * _u01(_hash4(seed, SALT_U, i, np.arange(A, dtype=np.uint32)[None, :])) - 1.0) * np.sqrt(3.0 / fan) * gain
    return W.astype(np.float32), U.astype(np.float32)


def synthbox_reset_states(seed, env_ids, episodes, D):
    e = np.asarray(env_ids, np.uint32)[:, None]
    ep = np.asarray(episodes, np.uint32)[:, None]
    d = np.arange(D, dtype=np.uint32)[None, :]
    return ((2.0 * _u01(_hash4(seed ^ SALT_RESET, e, ep, d)) - 1.0) * RESET_SCALE).astype(np.float32)


class _Box:
    def __init__(self, shape):
        self.shape = tuple(shape)
        self.low = -np.ones(shape, np.float32)
        self.high = np.ones(shape, np.float32)
        self.dtype = np.float32


class _Discrete:
    def __init__(self, n):
        self.n, self.shape, self.dtype = int(n), (), np.int64


class SynthBoxVecEnv:
    """n_envs SynthBox(D, A) environments resident on one GPU."""

    def __init__(self, n_envs, obs_dim, act_dim, seed=1, discrete=False, max_episode_steps=1000, device=None,
                 shard=0):
        self.num_envs, self.D, self.A = int(n_envs), int(obs_dim), int(act_dim)
        self.seed, self.discrete, self.max_episode_steps = int(seed), bool(discrete), int(max_episode_steps)
        self.max_episode_length = self.max_episode_steps
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        # Data-parallel shards share the dynamics (W, U from `seed`) but draw noise/reset states from a
        # per-shard stream; shard 0 is bit-identical to the CPU checker.
        self.shard = int(shard)
        self.noise_seed = (self.seed ^ ((0x9E3779B9 * self.shard) & 0xFFFFFFFF)) & 0xFFFFFFFF
        self.observation_space = _Box((self.D,))
        self.action_space = _Discrete(self.A) if discrete else _Box((self.A,))
        W, U = synthbox_matrices(self.seed, self.D, self.A, self.discrete)
        dev, N, D, A = self.device, self.num_envs, self.D, self.A
        self.Wcat_t = torch.as_tensor(np.concatenate([W, U], axis=1).T.copy(), device=dev)  # [D + A, D]
        self.X = torch.zeros((N, D + A), dtype=torch.float32, device=dev)                   # [state | action]
        self.pre = torch.empty((N, D), dtype=torch.float32, device=dev)
        self.final_obs = torch.empty((N, D), dtype=torch.float32, device=dev)
        self.rew = torch.zeros((N,), dtype=torch.float32, device=dev)
        self.term = torch.zeros((N,), dtype=torch.uint8, device=dev)
        self.trunc = torch.zeros((N,), dtype=torch.uint8, device=dev)
        self.ep_step = torch.zeros((N,), dtype=torch.int32, device=dev)
        self.ep_index = torch.zeros((N,), dtype=torch.int32, device=dev)  # read as uint32 by the kernel
        self.ep_score = torch.zeros((N,), dtype=torch.float32, device=dev)
        self.ep_last_score = torch.zeros((N,), dtype=torch.float32, device=dev)
        self.ep_last_len = torch.zeros((N,), dtype=torch.int32, device=dev)
        self.reset()

    @property
    def obs(self):
        """Current observation [N, D] (a strided view of X)."""
        return self.X[:, :self.D]

    @property
    def act_in(self):
        """Env action input [N, A] (a strided view of X): clipped action or one-hot."""
        return self.X[:, self.D:]

    @property
    def buf_obs(self):
        return self.obs

    def reset(self):
        self.resets = getattr(self, "resets", 0) + 1   # agents re-arm a folded obs-RMS merge (K8R)
        ids = np.arange(self.num_envs)
        s0 = synthbox_reset_states(self.noise_seed, ids, np.zeros(self.num_envs), self.D)
        self.X.zero_()
        self.X[:, :self.D] = torch.as_tensor(s0, device=self.device)
        for t in (self.ep_step, self.ep_index, self.ep_score, self.ep_last_score, self.ep_last_len, self.rew,
                  self.term, self.trunc):
            t.zero_()
        return self.obs.clone(), [{} for _ in range(self.num_envs)]

    def fusable_with_policy_step(self, dist):
        """True when the rollout's K14 can run this env's step in the same launch
        (ops.rollout_policy_head_synthbox): continuous actions and at most 64 state dims."""
        return dist == "gaussian" and not self.discrete and self.D <= 64

    def step_device(self):
        """One env step for all envs from the action already written into act_in."""
        torch.mm(self.X, self.Wcat_t, out=self.pre)
        rc = ops.lib().xpa_synthbox_step(self.num_envs, self.D, ops._p(self.pre), self.noise_seed,
                                         self.max_episode_steps, NOISE, TERM_THRESH, RESET_SCALE, ops._p(self.X),
                                         self.X.stride(0), ops._p(self.final_obs), ops._p(self.rew),
                                         ops._p(self.term), ops._p(self.trunc), ops._p(self.ep_step),
                                         ops._p(self.ep_index), ops._p(self.ep_score), ops._p(self.ep_last_score),
                                         ops._p(self.ep_last_len), ops._stream(self.device))
        _lib.check(rc, "xpa_synthbox_step")

    def step(self, actions):
        """VecEnv contract (gym_vec_env.py:201-212): returns host copies of (obs, rew, term, trunc, infos)
        with infos[i]['reset_obs'] for done envs."""
        a = torch.as_tensor(np.asarray(actions) if not isinstance(actions, torch.Tensor) else actions,
                            device=self.device)
        if self.discrete:
            self.act_in.zero_()
            self.act_in.scatter_(1, a.long().reshape(-1, 1), 1.0)
        else:
            self.act_in.copy_(torch.clamp(a.float().reshape(self.num_envs, self.A), -1.0, 1.0))
        self.step_device()
        obs = self.final_obs.cpu().numpy()
        rew = self.rew.cpu().numpy()
        term = self.term.cpu().numpy().astype(bool)
        trunc = self.trunc.cpu().numpy().astype(bool)
        nxt = self.obs.cpu().numpy()
        lens, scores = self.ep_step.cpu().numpy(), self.ep_score.cpu().numpy()
        last_len, last_score = self.ep_last_len.cpu().numpy(), self.ep_last_score.cpu().numpy()
        infos = []
        for i in range(self.num_envs):
            done = term[i] or trunc[i]
            info = {"episode_step": int(last_len[i] if done else lens[i]),
                    "episode_score": float(last_score[i] if done else scores[i])}
            if done:
                info["reset_obs"] = nxt[i].copy()
            infos.append(info)
        return obs, rew, term, trunc, infos

    def close(self):
        pass


class _ImageBox:
    def __init__(self, shape):
        self.shape = tuple(shape)
        self.low = np.zeros(shape, np.uint8)
        self.high = np.full(shape, 255, np.uint8)
        self.dtype = np.uint8


class SynthAtariVecEnv:
    """n_envs SynthAtari envs (uint8 4x84x84 frame stacks, Discrete(n_actions), reward sign, lives) resident
    on one GPU — the C3 / C5 shapes of BASELINE.json.  Spec and CPU checker: oracle/synth_env.py
    (SynthAtariEnv); kernel: csrc/atari.hip (K15).  Same interface as SynthBoxVecEnv: obs, act_in,
    final_obs, rew/term/trunc, step_device(), host step() with the DummyVecEnv_Atari contract."""

    HW, STACK = 84, 4

    def __init__(self, n_envs, n_actions=6, seed=1, max_episode_steps=27000, device=None, shard=0):
        self.num_envs, self.n_actions = int(n_envs), int(n_actions)
        self.seed, self.max_episode_steps = int(seed), int(max_episode_steps)
        self.max_episode_length = self.max_episode_steps
        # the reference's Atari flag rules (gym_env.py:193-209): a game over or the step limit sets terminated AND
        # truncated, so a truncation never needs a bootstrap value (finish_path(0)) — the agent then evaluates the
        # critic only on the last step's observations, once per rollout
        self.truncation_implies_terminal = True
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.shard = int(shard)
        self.noise_seed = (self.seed ^ ((0x9E3779B9 * self.shard) & 0xFFFFFFFF)) & 0xFFFFFFFF
        shape = (self.HW, self.HW, self.STACK)
        self.observation_space = _ImageBox(shape)
        self.action_space = _Discrete(self.n_actions)
        dev, N = self.device, self.num_envs
        self.stack = torch.zeros((N,) + shape, dtype=torch.uint8, device=dev)
        self.final_obs = torch.zeros((N,) + shape, dtype=torch.uint8, device=dev)
        self._act = torch.zeros((N, self.n_actions), dtype=torch.float32, device=dev)
        self.rew = torch.zeros((N,), dtype=torch.float32, device=dev)
        self.term = torch.zeros((N,), dtype=torch.uint8, device=dev)
        self.trunc = torch.zeros((N,), dtype=torch.uint8, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        self.ep_step, self.ep_index = torch.zeros((N,), **i32), torch.zeros((N,), **i32)
        self.lives, self.paddle = torch.zeros((N,), **i32), torch.zeros((N,), **i32)
        self.ep_last_len = torch.zeros((N,), **i32)
        self.ep_score = torch.zeros((N,), dtype=torch.float32, device=dev)
        self.ep_last_score = torch.zeros((N,), dtype=torch.float32, device=dev)
        self.err = torch.zeros((1,), dtype=torch.int32, device=dev)   # steps taken with no action set (K15)
        self.reset()

    @property
    def obs(self):
        return self.stack

    @property
    def act_in(self):
        return self._act

    @property
    def buf_obs(self):
        return self.stack

    def reset(self):
        self.resets = getattr(self, "resets", 0) + 1   # agents re-arm a folded obs-RMS merge (K8R)
        for t in (self.ep_step, self.ep_index, self.ep_score, self.ep_last_score, self.ep_last_len, self.rew,
                  self.term, self.trunc, self._act):
            t.zero_()
        self.lives.fill_(5)
        self.paddle.fill_(38)
        _lib.check(ops.lib().xpa_synthatari_reset(self.num_envs, self.noise_seed, ops._p(self.stack),
                                                  ops._p(self.ep_index), ops._stream(self.device)),
                   "xpa_synthatari_reset")
        return self.stack.clone(), [{} for _ in range(self.num_envs)]

    def step_device(self):
        rc = ops.lib().xpa_synthatari_step(self.num_envs, self.n_actions, ops._p(self._act), self._act.stride(0),
                                           self.noise_seed, self.max_episode_steps, ops._p(self.stack),
                                           ops._p(self.final_obs), ops._p(self.rew), ops._p(self.term),
                                           ops._p(self.trunc), ops._p(self.ep_step), ops._p(self.ep_index),
                                           ops._p(self.lives), ops._p(self.paddle), ops._p(self.ep_score),
                                           ops._p(self.ep_last_score), ops._p(self.ep_last_len),
                                           ops._p(self.err), ops._stream(self.device))
        _lib.check(rc, "xpa_synthatari_step")

    def step(self, actions):
        """DummyVecEnv_Atari contract (gym_vec_env.py:201-212): host copies of (obs, rew, term, trunc, infos);
        infos[i]['reset_obs'] after a game over."""
        a = torch.as_tensor(np.asarray(actions) if not isinstance(actions, torch.Tensor) else actions,
                            device=self.device).long().reshape(-1, 1)
        self._act.zero_()
        self._act.scatter_(1, a, 1.0)
        self.step_device()
        obs = self.final_obs.cpu().numpy()
        rew = self.rew.cpu().numpy()
        term = self.term.cpu().numpy().astype(bool)
        trunc = self.trunc.cpu().numpy().astype(bool)
        nxt = self.stack.cpu().numpy()
        lens, scores = self.ep_step.cpu().numpy(), self.ep_score.cpu().numpy()
        last_len, last_score = self.ep_last_len.cpu().numpy(), self.ep_last_score.cpu().numpy()
        infos = []
        for i in range(self.num_envs):
            info = {"episode_step": int(last_len[i] if trunc[i] else lens[i]),
                    "episode_score": float(last_score[i] if trunc[i] else scores[i])}
            if trunc[i]:
                info["reset_obs"] = nxt[i].copy()
            infos.append(info)
        return obs, rew, term, trunc, infos

    def close(self):
        pass


# ---- CartPole-v1 (BASELINE.json configs[0]) -------------------------------------------------------------------
SALT_CARTPOLE = 0xCA27B01E


def cartpole_reset_states(seed, env_ids, episodes):
    """uniform(-0.05, 0.05) per dim from the counter hash (f32-exact uniform, then f64), as K18 draws them."""
    e = np.asarray(env_ids, np.uint32)[:, None]
    ep = np.asarray(episodes, np.uint32)[:, None]
    d = np.arange(4, dtype=np.uint32)[None, :]
    return _u01(_hash4(seed ^ SALT_CARTPOLE, e, ep, d)).astype(np.float64) * 0.1 - 0.05


class CartPoleVecEnv:
    """n_envs CartPole-v1 envs resident on one GPU (K18 xpa_cartpole_step, csrc/classic.hip): gym 0.26.2's
    dynamics with TimeLimit(500), f64 state, f32 observations, Discrete(2) actions read from the one-hot env
    input the rollout kernels write.  Same interface as SynthBoxVecEnv (obs, act_in, final_obs, rew / term /
    trunc, step_device(), host step() with DummyVecEnv_Gym's contract).  CPU checker:
    oracle/synth_env.CartPoleEnv."""
    kind = "cartpole"   # agents._small_rollout: K32 steps this env inside the fused rollout step

    def __init__(self, n_envs, seed=1, max_episode_steps=500, device=None, shard=0):
        self.num_envs, self.seed, self.max_episode_steps = int(n_envs), int(seed), int(max_episode_steps)
        self.max_episode_length = self.max_episode_steps
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.shard = int(shard)
        self.noise_seed = (self.seed ^ ((0x9E3779B9 * self.shard) & 0xFFFFFFFF)) & 0xFFFFFFFF
        self.observation_space = _Box((4,))
        self.observation_space.low = np.full(4, -np.inf, np.float32)
        self.observation_space.high = np.full(4, np.inf, np.float32)
        self.action_space = _Discrete(2)
        dev, N = self.device, self.num_envs
        self.state = torch.zeros((N, 4), dtype=torch.float64, device=dev)
        self._obs = torch.zeros((N, 4), dtype=torch.float32, device=dev)
        self._act = torch.zeros((N, 2), dtype=torch.float32, device=dev)
        self.final_obs = torch.zeros((N, 4), dtype=torch.float32, device=dev)
        self.rew = torch.zeros((N,), dtype=torch.float32, device=dev)
        self.term = torch.zeros((N,), dtype=torch.uint8, device=dev)
        self.trunc = torch.zeros((N,), dtype=torch.uint8, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        self.ep_step, self.ep_index, self.ep_last_len = (torch.zeros((N,), **i32) for _ in range(3))
        self.ep_score = torch.zeros((N,), dtype=torch.float32, device=dev)
        self.ep_last_score = torch.zeros((N,), dtype=torch.float32, device=dev)
        self.reset()

    @property
    def obs(self):
        return self._obs

    @property
    def act_in(self):
        """Env action input [N, 2]: the one-hot of the sampled action (K3 / K14 write it)."""
        return self._act

    @property
    def buf_obs(self):
        return self._obs

    def reset(self):
        self.resets = getattr(self, "resets", 0) + 1   # agents re-arm a folded obs-RMS merge (K8R)
        s0 = cartpole_reset_states(self.noise_seed, np.arange(self.num_envs), np.zeros(self.num_envs))
        self.state.copy_(torch.as_tensor(s0, device=self.device))
        self._obs.copy_(self.state.float())
        for t in (self.ep_step, self.ep_index, self.ep_score, self.ep_last_score, self.ep_last_len, self.rew,
                  self.term, self.trunc):
            t.zero_()
        return self._obs.clone(), [{} for _ in range(self.num_envs)]

    def fusable_with_policy_step(self, dist):
        return False

    def step_device(self):
        rc = ops.lib().xpa_cartpole_step(self.num_envs, ops._p(self._act), self._act.stride(0), ops._p(self.state),
                                         ops._p(self._obs), self._obs.stride(0), ops._p(self.final_obs),
                                         ops._p(self.rew), ops._p(self.term), ops._p(self.trunc),
                                         ops._p(self.ep_step), ops._p(self.ep_index), ops._p(self.ep_score),
                                         ops._p(self.ep_last_score), ops._p(self.ep_last_len), self.noise_seed,
                                         self.max_episode_steps, ops._stream(self.device))
        _lib.check(rc, "xpa_cartpole_step")

    def step(self, actions):
        """VecEnv contract (gym_vec_env.py:201-212): host copies of (obs, rew, term, trunc, infos)."""
        a = torch.as_tensor(np.asarray(actions) if not isinstance(actions, torch.Tensor) else actions,
                            device=self.device).long().reshape(-1, 1)
        self._act.zero_()
        self._act.scatter_(1, a, 1.0)
        self.step_device()
        obs = self.final_obs.cpu().numpy()
        rew = self.rew.cpu().numpy()
        term = self.term.cpu().numpy().astype(bool)
        trunc = self.trunc.cpu().numpy().astype(bool)
        nxt = self._obs.cpu().numpy()
        lens, scores = self.ep_step.cpu().numpy(), self.ep_score.cpu().numpy()
        last_len, last_score = self.ep_last_len.cpu().numpy(), self.ep_last_score.cpu().numpy()
        infos = []
        for i in range(self.num_envs):
            done = term[i] or trunc[i]
            info = {"episode_step": int(last_len[i] if done else lens[i]),
                    "episode_score": float(last_score[i] if done else scores[i])}
            if done:
                info["reset_obs"] = nxt[i].copy()
            infos.append(info)
        return obs, rew, term, trunc, infos

    def close(self):
        pass
