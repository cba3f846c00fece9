"""ORACLE / TEST INFRASTRUCTURE — CPU restatement of the reference's on-policy PPO-Clip / A2C path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.  It is
the checker for the HIP path and the CPU baseline timed beside it; nothing in xuanpolicy_amd/ imports
it.  Pinned against golden vectors captured from the reference itself (tests/golden/*.npz, produced
by tests/golden/make_golden.py, which imports /root/reference in the build container).

Each piece cites the reference code it restates (paths relative to /root/reference):
  BufferRef            xuance/common/memory_tools.py:143-245 (DummyOnPolicyBuffer)
  gae_rows             memory_tools.py:206-229 applied at the agent's closure points
                       (xuance/torch/agents/policy_gradient/ppoclip_agent.py:69-101)
  RunningMeanStdRef    xuance/common/statistic_tools.py:35-112
  loss_grads_ref       xuance/torch/learners/policy_gradient/ppoclip_learner.py:32-44,
                       a2c_learner.py:24-31, xuance/torch/utils/distributions.py:39-101
  ActorCriticRef       xuance/torch/policies/gaussian.py:8-77, categorical.py:16-85,
                       xuance/torch/representations/mlp.py:21-51, xuance/torch/utils/layers.py:8-24
  LearnerRef           ppoclip_learner.py:24-65, a2c_learner.py:19-50
  AgentLoopRef         ppoclip_agent.py:59-111, a2c_agent.py:57-107, xuance/torch/agents/agent.py:104-123
  build_qnetwork_ref   xuance/torch/policies/deterministic.py:6-25 (BasicQhead), 148-182 (BasicQnetwork),
                       xuance/torch/representations/cnn.py:5-40 (Basic_CNN)
  dqn_td_ref           xuance/torch/learners/qlearning_family/perdqn_learner.py:23-30 (closed form)
  PerDQNLearnerRef     perdqn_learner.py:17-48
"""
import ctypes
import math
import os
import time

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _lib():
    """liboracle_gae.so (built by oracle/Makefile); None if not built."""
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "_build", "liboracle_gae.so")
        if not os.path.exists(path):
            return None
        lib = ctypes.CDLL(path)
        f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
        u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
        lib.oracle_finish_path.argtypes = [f32p, f32p, f32p, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                           ctypes.c_double, ctypes.c_double, ctypes.c_int, f32p, f32p]
        lib.oracle_gae_rows.argtypes = [f32p, f32p, f32p, u8p, f32p, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                        ctypes.c_double, ctypes.c_int, f32p, f32p]
        _LIB = lib
    return _LIB


def build_oracle():
    """Compile oracle/gae_ref.c (called by __graft_entry__.build())."""
    import subprocess
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _lib()


# ----------------------------------------------------------------------------------------------
# GAE
# ----------------------------------------------------------------------------------------------
def finish_path_py(rew, val, term, start, end, bootstrap, gamma, lam, use_gae, adv, ret):
    """Pure-Python restatement of memory_tools.py:206-229 for one row (small cases only)."""
    n = end - start
    if n <= 0:
        return
    if use_gae:
        last = 0.0
        for k in range(n - 1, -1, -1):
            t = start + k
            vnext = bootstrap if k == n - 1 else float(val[t + 1])
            nd = 1.0 - float(term[t])
            delta = float(rew[t]) + nd * gamma * vnext - float(val[t])
            last = delta + nd * gamma * lam * last
            adv[t] = last
            ret[t] = last + float(val[t])
    else:
        run = bootstrap
        for k in range(n - 1, -1, -1):
            t = start + k
            vnext = bootstrap if k == n - 1 else float(val[t + 1])
            run = float(rew[t]) + gamma * run
            ret[t] = run
            adv[t] = float(rew[t]) + gamma * vnext - float(val[t])


def finish_path_np(rew, val, term, start, end, bootstrap, gamma, lam, use_gae, adv, ret):
    """memory_tools.py:206-229 restated with its own data flow (np.append of the bootstrap, a reversed Python loop over
    NumPy scalars): the CPU baseline's GAE, so the baseline pays what the reference pays for it (the C restatement in
    gae_ref.c is ~8x faster; tools/cpu_calibrate.py)."""
    path = np.arange(start, end).astype(np.int32)
    vs = np.append(np.array(val[path]), [bootstrap], axis=0)
    if use_gae:
        rewards = np.array(rew[path])
        advantages = np.zeros_like(rewards)
        dones = np.array(term[path])
        last = 0
        for t in reversed(range(len(path))):
            delta = rewards[t] + (1 - dones[t]) * gamma * vs[t + 1] - vs[t]
            advantages[t] = last = delta + (1 - dones[t]) * gamma * lam * last
        returns = advantages + vs[:-1]
    else:
        rewards = np.append(np.array(rew[path]), [bootstrap], axis=0)
        returns = np.zeros_like(rewards)
        run = 0.0
        for t in reversed(range(len(rewards))):
            run = rewards[t] + gamma * run
            returns[t] = run
        returns = returns[:-1]
        advantages = rewards[:-1] + gamma * vs[1:] - vs[:-1]
    ret[path] = returns
    adv[path] = advantages


def gae_rows(rew, val, term, closed, boot, gamma, lam, use_gae=True, adv=None, ret=None):
    """GAE over a full [N, T] buffer cut into paths by closure flags (see gae_ref.c)."""
    rew = np.ascontiguousarray(rew, np.float32)
    val = np.ascontiguousarray(val, np.float32)
    term = np.ascontiguousarray(term, np.float32)
    closed = np.ascontiguousarray(closed, np.uint8)
    boot = np.ascontiguousarray(boot, np.float32)
    N, T = rew.shape
    adv = np.zeros((N, T), np.float32) if adv is None else adv
    ret = np.zeros((N, T), np.float32) if ret is None else ret
    lib = _lib()
    if lib is not None:
        lib.oracle_gae_rows(rew, val, term, closed, boot, N, T, float(gamma), float(lam), int(use_gae), adv, ret)
        return adv, ret
    for n in range(N):
        start = 0
        for t in range(T):
            if closed[n, t]:
                finish_path_py(rew[n], val[n], term[n], start, t + 1, float(boot[n, t]), gamma, lam, use_gae,
                               adv[n], ret[n])
                start = t + 1
    return adv, ret


# ----------------------------------------------------------------------------------------------
# Buffer
# ----------------------------------------------------------------------------------------------
class BufferRef:
    """Restatement of DummyOnPolicyBuffer (memory_tools.py:143-245).  Storage is numpy float32
    [n_envs, n_size, ...] like create_memory (memory_tools.py:12-36); obs dtype uint8 for Atari
    (memory_tools.py:526-560).  Records closures so tests can hand them to the GPU kernel."""

    def __init__(self, obs_shape, act_shape, aux_shape, n_envs, n_size, use_gae=True, use_advnorm=True,
                 gamma=0.99, gae_lam=0.95, obs_dtype=np.float32, gae_impl="c"):
        self.obs_shape, self.act_shape, self.aux_shape = tuple(obs_shape), tuple(act_shape), dict(aux_shape or {})
        self.n_envs, self.n_size = n_envs, n_size
        self.buffer_size = n_envs * n_size
        self.use_gae, self.use_advnorm = use_gae, use_advnorm
        self.gamma, self.gae_lam = gamma, gae_lam
        self.obs_dtype = obs_dtype
        self.gae_impl = gae_impl   # "c": gae_ref.c (checker); "np": the reference's own data flow (CPU baseline)
        self.start_ids = np.zeros(n_envs, np.int64)
        self.clear()

    def clear(self):
        self.ptr, self.size = 0, 0
        N, T = self.n_envs, self.n_size
        self.observations = np.zeros((N, T) + self.obs_shape, self.obs_dtype)
        self.actions = np.zeros((N, T) + self.act_shape, np.float32)
        self.rewards = np.zeros((N, T), np.float32)
        self.returns = np.zeros((N, T), np.float32)
        self.values = np.zeros((N, T), np.float32)
        self.terminals = np.zeros((N, T), np.float32)
        self.advantages = np.zeros((N, T), np.float32)
        self.auxiliary_infos = {k: np.zeros((N, T) + tuple(v), np.float32) for k, v in self.aux_shape.items()}
        self.closed = np.zeros((N, T), np.uint8)
        self.boot = np.zeros((N, T), np.float32)

    @property
    def full(self):
        return self.size >= self.n_size

    def store(self, obs, acts, rews, value, terminals, aux_info=None):
        p = self.ptr
        self.observations[:, p] = obs
        self.actions[:, p] = acts
        self.rewards[:, p] = rews
        self.values[:, p] = value
        self.terminals[:, p] = terminals
        if aux_info:
            for k, v in aux_info.items():
                self.auxiliary_infos[k][:, p] = v
        self.ptr = (self.ptr + 1) % self.n_size
        self.size = min(self.size + 1, self.n_size)

    def finish_path(self, val, i):
        end = self.n_size if self.full else self.ptr
        start = int(self.start_ids[i])
        if end > start:
            self.closed[i, end - 1] = 1
            self.boot[i, end - 1] = val
            lib = _lib() if self.gae_impl == "c" else None
            if self.gae_impl == "np":
                finish_path_np(self.rewards[i], self.values[i], self.terminals[i], start, end, float(val),
                               self.gamma, self.gae_lam, self.use_gae, self.advantages[i], self.returns[i])
            elif lib is not None:
                lib.oracle_finish_path(self.rewards[i], self.values[i], self.terminals[i], start, end, float(val),
                                       float(self.gamma), float(self.gae_lam), int(self.use_gae),
                                       self.advantages[i], self.returns[i])
            else:
                finish_path_py(self.rewards[i], self.values[i], self.terminals[i], start, end, float(val),
                               self.gamma, self.gae_lam, self.use_gae, self.advantages[i], self.returns[i])
        self.start_ids[i] = self.ptr

    def sample(self, indexes):
        assert self.full, "Not enough transitions for on-policy buffer to random sample"
        env, step = divmod(np.asarray(indexes), self.n_size)
        obs = self.observations[env, step]
        act = self.actions[env, step]
        ret = self.returns[env, step]
        val = self.values[env, step]
        adv = self.advantages[env, step]
        if self.use_advnorm:
            adv = (adv - np.mean(adv)) / (np.std(adv) + 1e-8)
        aux = {k: v[env, step] for k, v in self.auxiliary_infos.items()}
        return obs, act, ret, val, adv, aux


# ----------------------------------------------------------------------------------------------
# RunningMeanStd
# ----------------------------------------------------------------------------------------------
class RunningMeanStdRef:
    """statistic_tools.py:35-112 (non-MPI branch): Chan parallel-variance merge, count init 1e-4."""

    def __init__(self, shape, epsilon=1e-4):
        self.mean = np.zeros(shape, np.float32)
        self.var = np.ones(shape, np.float32)
        self.count = epsilon

    @property
    def std(self):
        return np.sqrt(self.var)

    def update(self, x):
        x = np.asarray(x)
        self.update_from_moments(np.mean(x, axis=0), np.square(np.std(x, axis=0)), x.shape[0])

    def update_from_moments(self, batch_mean, batch_var, batch_count):
        delta = batch_mean - self.mean
        tot = self.count + batch_count
        new_mean = self.mean + delta * batch_count / tot
        m2 = self.var * self.count + batch_var * batch_count + np.square(delta) * self.count * batch_count / tot
        self.mean = new_mean
        self.var = m2 / tot
        self.count = tot


def process_observation(obs, rms, obs_range=5.0, eps=1e-8):
    """agent.py:104-116."""
    return np.clip((obs - rms.mean) / (rms.std + eps), -obs_range, obs_range)


def process_reward(rew, ret_rms, rew_range=5.0):
    """agent.py:118-123."""
    std = np.clip(ret_rms.std, 0.1, 100)
    return np.clip(rew / std, -rew_range, rew_range)


# ----------------------------------------------------------------------------------------------
# Loss + closed-form gradients (float64 numpy)
# ----------------------------------------------------------------------------------------------
LOG_SQRT_2PI = math.log(math.sqrt(2.0 * math.pi))


def loss_grads_ref(algo, dist, head, logstd, v, act, adv, ret, old_logp=None, clip_range=0.2, vf_coef=0.25,
                   ent_coef=0.0):
    """Loss scalars and d loss / d{head, logstd, v} for one minibatch.

    algo: "ppo" (ppoclip_learner.py:36-44) or "a2c" (a2c_learner.py:24-31).
    dist: "gaussian" (head = mu [B, A], logstd [A]) or "categorical" (head = logits [B, K]).
    Gradients follow torch autograd's tie rules: clamp passes gradient on min <= x <= max,
    minimum() splits a tie half/half.
    Returns (info dict, d_head [B, A], d_logstd [A] or None, d_v [B]).
    """
    head = np.asarray(head, np.float64)
    v = np.asarray(v, np.float64)
    adv = np.asarray(adv, np.float64)
    ret = np.asarray(ret, np.float64)
    B = head.shape[0]
    if dist == "gaussian":
        logstd = np.asarray(logstd, np.float64)
        x = np.asarray(act, np.float64)
        scale = np.exp(logstd)
        var = scale * scale
        diff = x - head
        lp = -(diff * diff) / (2 * var) - np.log(scale) - LOG_SQRT_2PI
        logp = lp.sum(-1)
        ent_b = np.full(B, np.sum(0.5 + 0.5 * math.log(2 * math.pi) + np.log(scale)))
        dlogp_dhead = diff / var
        dlogp_dlogstd = diff * diff / var - 1.0
    else:
        z = head
        zmax = z.max(-1, keepdims=True)
        lse = zmax + np.log(np.exp(z - zmax).sum(-1, keepdims=True))
        logits_n = z - lse
        p = np.exp(logits_n)
        a = np.asarray(act).astype(np.int64).reshape(-1)
        logp = logits_n[np.arange(B), a]
        ent_b = -(p * logits_n).sum(-1)
        onehot = np.zeros_like(z)
        onehot[np.arange(B), a] = 1.0
        dlogp_dhead = onehot - p
        dH_dz = -p * (logits_n + ent_b[:, None])
    if algo == "ppo":
        ratio = np.exp(logp - np.asarray(old_logp, np.float64))
        lo, hi = 1.0 - clip_range, 1.0 + clip_range
        clamped = np.clip(ratio, lo, hi)
        s1 = clamped * adv
        s2 = adv * ratio
        m = np.minimum(s1, s2)
        a_loss = -m.mean()
        inr = (ratio >= lo) & (ratio <= hi)
        g1 = np.where(inr, adv, 0.0)
        w1 = np.where(s1 < s2, 1.0, np.where(s1 == s2, 0.5, 0.0))
        w2 = np.where(s2 < s1, 1.0, np.where(s1 == s2, 0.5, 0.0))
        dm_dratio = w1 * g1 + w2 * adv
        dlogp = -(1.0 / B) * dm_dratio * ratio
        clip_ratio = float(((ratio < lo).sum() + (ratio > hi).sum()) / B)
    else:
        a_loss = -(adv * logp).mean()
        dlogp = -adv / B
        clip_ratio = None
    c_loss = np.mean((v - ret) ** 2)
    e_loss = ent_b.mean()
    loss = a_loss - ent_coef * e_loss + vf_coef * c_loss
    d_v = vf_coef * 2.0 * (v - ret) / B
    if dist == "gaussian":
        d_head = dlogp[:, None] * dlogp_dhead
        d_logstd = (dlogp[:, None] * dlogp_dlogstd).sum(0) - ent_coef
    else:
        d_head = dlogp[:, None] * dlogp_dhead - (ent_coef / B) * dH_dz
        d_logstd = None
    info = {"actor-loss": a_loss, "critic-loss": c_loss, "entropy": e_loss, "loss": loss,
            "predict_value": v.mean()}
    if clip_ratio is not None:
        info["clip_ratio"] = clip_ratio
    return info, d_head, d_logstd, d_v


# ----------------------------------------------------------------------------------------------
# torch-CPU policy / learner / agent loop (CPU baseline)
# ----------------------------------------------------------------------------------------------
def _torch():
    import torch
    return torch


def build_actor_critic_ref(obs_dim, act_dim, rep_hidden, actor_hidden, critic_hidden, discrete=False,
                           activation="LeakyReLU"):
    """Actor-critic with the reference's module layout and state_dict keys:
    representation.model.*, actor.mu.* + actor.logstd (Gaussian) / actor.model.* (Categorical),
    critic.model.* — gaussian.py:8-77, categorical.py:16-85, mlp.py:21-51, layers.py:8-24."""
    torch = _torch()
    nn = torch.nn
    act_cls = getattr(nn, activation)

    def mlp(sizes_in, hidden, out_dim, init_last=True):
        layers, d = [], sizes_in
        for h in hidden:
            lin = nn.Linear(d, h)
            nn.init.orthogonal_(lin.weight)
            nn.init.constant_(lin.bias, 0)
            layers += [lin, act_cls()]
            d = h
        if out_dim is not None:
            lin = nn.Linear(d, out_dim)
            if init_last:
                nn.init.orthogonal_(lin.weight)
                nn.init.constant_(lin.bias, 0)
            layers.append(lin)
        return nn.Sequential(*layers), d

    class Rep(nn.Module):
        def __init__(self):
            super().__init__()
            self.model, self.out_dim = mlp(obs_dim, rep_hidden, None)

        def forward(self, x):
            return {"state": self.model(x)}

    class Actor(nn.Module):
        def __init__(self, d):
            super().__init__()
            net, _ = mlp(d, actor_hidden, act_dim)
            if discrete:
                self.model = net
            else:
                self.mu = net
                self.logstd = nn.Parameter(-torch.ones((act_dim,)))

    class Critic(nn.Module):
        def __init__(self, d):
            super().__init__()
            # Gaussian critic's last layer keeps default init (gaussian.py:47); categorical's is orthogonal.
            self.model, _ = mlp(d, critic_hidden, 1, init_last=discrete)

        def forward(self, x):
            return self.model(x)[:, 0]

    class AC(nn.Module):
        def __init__(self):
            super().__init__()
            self.representation = Rep()
            self.actor = Actor(self.representation.out_dim)
            self.critic = Critic(self.representation.out_dim)
            self.discrete = discrete

        def heads(self, obs):
            s = self.representation(obs)["state"]
            if discrete:
                return self.actor.model(s), None, self.critic(s)
            return self.actor.mu(s), self.actor.logstd, self.critic(s)

        def dist(self, head, logstd):
            if discrete:
                return torch.distributions.Categorical(logits=head)
            return torch.distributions.Normal(head, logstd.exp())

    return AC()


def build_atari_ac_ref(n_actions, filters=(32, 64, 64), kernels=(8, 4, 3), strides=(4, 2, 1), fc=(512,),
                       in_shape=(84, 84, 4)):
    """Categorical actor-critic on AC_CNN_Atari with the reference's layout (cnn.py:45-93: conv blocks with padding
    (k - s) // 2 + ReLU, Flatten in (C, H, W) order, fc blocks; categorical.py:61-85 with empty actor / critic hidden
    lists) and its input arithmetic: observations / 255.0 in NumPy float64, transposed to NCHW, cast to float32."""
    torch = _torch()
    nn = torch.nn
    C, H, W = in_shape[2], in_shape[0], in_shape[1]
    layers, c, h, w = [], C, H, W
    for f, k, s in zip(filters, kernels, strides):
        p = (k - s) // 2
        conv = nn.Conv2d(c, f, k, s, padding=p)
        nn.init.orthogonal_(conv.weight, gain=np.sqrt(2))
        nn.init.constant_(conv.bias, 0)
        layers += [conv, nn.ReLU()]
        c, h, w = f, (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    layers.append(nn.Flatten())
    d = c * h * w
    for hdim in fc:
        lin = nn.Linear(d, hdim)
        nn.init.orthogonal_(lin.weight, gain=np.sqrt(2))
        nn.init.constant_(lin.bias, 0)
        layers += [lin, nn.ReLU()]
        d = hdim

    class Rep(nn.Module):
        def __init__(self):
            super().__init__()
            self.model = nn.Sequential(*layers)

        def forward(self, obs):   # float32 as the reference; the parameters' dtype when the oracle runs in f64
            x = np.asarray(obs) / 255.0
            dt = next(self.parameters()).dtype
            return {"state": self.model(torch.as_tensor(np.transpose(x, (0, 3, 1, 2)), dtype=dt))}

    class AC(nn.Module):
        discrete = True

        def __init__(self):
            super().__init__()
            self.representation = Rep()
            self.actor = nn.Module()
            self.actor.model = nn.Sequential(nn.Linear(d, n_actions))
            self.critic_head = nn.Sequential(nn.Linear(d, 1))
            for lin in (self.actor.model[0], self.critic_head[0]):
                nn.init.orthogonal_(lin.weight)
                nn.init.constant_(lin.bias, 0)

        def heads(self, obs):
            s = self.representation(obs)["state"]
            return self.actor.model(s), None, self.critic_head(s)[:, 0]

        def dist(self, head, logstd):
            return torch.distributions.Categorical(logits=head)

    return AC()


class LearnerRef:
    """ppoclip_learner.py:24-65 / a2c_learner.py:19-50 on torch CPU (autograd, Adam, LinearLR)."""

    def __init__(self, policy, optimizer, scheduler, algo="ppo", vf_coef=0.25, ent_coef=0.0, clip_range=0.2,
                 clip_grad_norm=0.5, use_grad_clip=True):
        self.policy, self.optimizer, self.scheduler = policy, optimizer, scheduler
        self.algo, self.vf_coef, self.ent_coef = algo, vf_coef, ent_coef
        self.clip_range, self.clip_grad_norm, self.use_grad_clip = clip_range, clip_grad_norm, use_grad_clip
        self.iterations = 0

    def _kink_hooks_arm(self):
        """Forward hooks recording every (Linear -> LeakyReLU / ReLU) pair's input, pre-activation and activation (the
        activation with retain_grad) for _kink_rows."""
        torch = _torch()
        nn = torch.nn
        self._kink_rec, self._kink_handles = [], []
        for m in self.policy.modules():
            if not isinstance(m, nn.Sequential):
                continue
            mods = list(m)
            for a, b in zip(mods, mods[1:]):
                if isinstance(a, nn.Linear) and isinstance(b, (nn.LeakyReLU, nn.ReLU)):
                    slope = float(b.negative_slope) if isinstance(b, nn.LeakyReLU) else 0.0
                    rec = {"lin": a, "slope": slope}
                    self._kink_rec.append(rec)

                    def lin_hook(mod, inp, out, rec=rec):
                        rec["a"], rec["z"] = inp[0], out

                    def act_hook(mod, inp, out, rec=rec):
                        if out.requires_grad:
                            out.retain_grad()
                        rec["h"] = out
                    self._kink_handles += [a.register_forward_hook(lin_hook), b.register_forward_hook(act_hook)]

    def _kink_hooks_clear(self):
        for hd in getattr(self, "_kink_handles", []):
            hd.remove()
        self._kink_handles, self._kink_rec = [], []

    def _kink_rows(self, cap=16):
        """The (row, unit) pre-activations within 4e-6 of sum |a w| (the split GEMM's f32 error bound) of zero, the
        closest first: [(z, h, row, unit, slope)]."""
        torch = _torch()
        cands = []
        for rec in getattr(self, "_kink_rec", []):
            if "z" not in rec or rec["z"].dim() != 2:
                continue
            z, a, W = rec["z"].detach(), rec["a"].detach(), rec["lin"].weight.detach()
            bound = 4e-6 * (a.abs() @ W.abs().t())
            r = z.abs() / (bound + 1e-30)
            idx = ((r <= 1.0) & (bound > 1e-20)).nonzero()   # (an all-zero input row: z is exact on every side)
            for i, u in idx.tolist():
                cands.append((float(r[i, u]), rec["z"], rec["h"], i, u, rec["slope"]))
        cands.sort(key=lambda c: c[0])
        return [c[1:] for c in cands[:cap]]

    def update(self, obs, act, ret, adv, old_logp=None, capture_grads=False):
        """capture_grads: keep every parameter's gradient before clipping in self.last_grads (lock-step replays)."""
        torch = _torch()
        self.iterations += 1
        if capture_grads:
            self._kink_hooks_arm()
        if not (isinstance(obs, np.ndarray) and obs.dtype == np.uint8):   # raw frames: the policy scales them
            # f32 observations; an f64 replay (precision envelopes) takes them exactly in its parameters' dtype
            obs = torch.as_tensor(obs, dtype=torch.float32).to(next(self.policy.parameters()).dtype)
        act = torch.as_tensor(act)
        head, logstd, v = self.policy.heads(obs)
        ret = torch.as_tensor(ret).to(v.dtype)   # (the parameters' dtype: f32, or f64 for precision envelopes)
        adv = torch.as_tensor(adv).to(v.dtype)
        d = self.policy.dist(head, logstd)
        if self.policy.discrete:
            logp, ent = d.log_prob(act), d.entropy()
        else:
            logp, ent = d.log_prob(act).sum(-1), d.entropy().sum(-1)
        if self.algo == "ppo":
            ratio = (logp - torch.as_tensor(old_logp)).exp().float()
            s1 = ratio.clamp(1.0 - self.clip_range, 1.0 + self.clip_range) * adv
            s2 = adv * ratio
            a_loss = -torch.minimum(s1, s2).mean()
        else:
            a_loss = -(adv * logp).mean()
        c_loss = torch.nn.functional.mse_loss(v, ret)
        e_loss = ent.mean()
        loss = a_loss - self.ent_coef * e_loss + self.vf_coef * c_loss
        self.optimizer.zero_grad()
        boundary = []
        kinks = self._kink_rows() if capture_grads else []
        if capture_grads and self.algo == "ppo":
            # rows whose ratio sits within f32 rounding of a clip bound (the window below): which branch of min() /
            # clamp() they take is not decided by the math, so a correct f32 implementation may include or drop their
            # unclipped gradient  d(-A ratio / B) / d theta.  Kept per row (at most 16) for the lock-step checks.
            lo, hi = 1 - self.clip_range, 1 + self.clip_range
            r64 = ratio.detach().double()
            near = (((r64 - lo).abs() < 2e-4 * lo) | ((r64 - hi).abs() < 2e-4 * hi)).nonzero().flatten()[:16]
            params = list(self.policy.parameters())
            for i in near.tolist():
                g = torch.autograd.grad(-(adv[i] * ratio[i]) / ratio.shape[0], params, retain_graph=True,
                                        allow_unused=True)
                boundary.append([torch.zeros_like(p) if x is None else x.detach().clone() for p, x in zip(params, g)])
        loss.backward(retain_graph=bool(kinks))
        if capture_grads:
            self.last_grads = [p.grad.detach().clone() for p in self.policy.parameters()]
            # (row, unit) pre-activations within the f32 GEMM's rounding of a (Leaky)ReLU kink: the side the device's
            # z lands on is not decided by the math either; flipping it changes that row's gradient by
            # (s_other - s) dL/dh(row, unit) grad_theta z(row, unit).  Kept per candidate (at most 16) beside the
            # clip-bound rows.
            params = list(self.policy.parameters())
            for z, h, i, u, slope in kinks:
                if h.grad is None:
                    continue
                s_cur = 1.0 if float(z[i, u].detach()) > 0 else slope
                g = torch.autograd.grad(z[i, u], params, retain_graph=True, allow_unused=True)
                f = ((slope if s_cur == 1.0 else 1.0) - s_cur) * float(h.grad[i, u])
                boundary.append([torch.zeros_like(p) if x is None else f * x.detach() for p, x in zip(params, g)])
            self._kink_hooks_clear()
            self.boundary_grads = boundary
        if self.algo == "a2c" or self.use_grad_clip:
            torch.nn.utils.clip_grad_norm_(self.policy.parameters(), self.clip_grad_norm)
        self.optimizer.step()
        if self.scheduler is not None:
            self.scheduler.step()
        info = {"actor-loss": a_loss.item(), "critic-loss": c_loss.item(), "entropy": e_loss.item(),
                "learning_rate": self.optimizer.param_groups[0]["lr"], "predict_value": v.mean().item()}
        if self.algo == "ppo":
            lo, hi = 1 - self.clip_range, 1 + self.clip_range
            info["clip_ratio"] = float(((ratio < lo).sum() + (ratio > hi).sum()) / ratio.shape[0])
            # rows whose ratio sits within the device's f32 rounding of a clip bound: their side of it is not decided by
            # the math.  The window is the ratio's relative error after a few f32 updates: log pi of a 17-dim Gaussian
            # sums 17 terms of magnitude ~10 (C4's head; an exp of a difference carries it as a relative error)
            r = ratio.detach().double()
            win = 2e-4
            info["clip_boundary_rows"] = int(((r - lo).abs() < win * lo).sum() + ((r - hi).abs() < win * hi).sum())
        return info


class AgentLoopRef:
    """CPU baseline: the reference's on-policy loop (ppoclip_agent.py:59-111 / a2c_agent.py:57-107)
    over a DummyVecEnv-style list of per-env SynthBoxEnv objects (gym_vec_env.py:201-212).

    Phase timers (act, env, store, gae, sample, update) mirror BASELINE.md's breakdown."""

    def __init__(self, envs, policy, learner, n_steps, n_epoch, n_minibatch, gamma=0.99, gae_lambda=0.95,
                 algo="ppo", use_gae=True, use_advnorm=True, use_obsnorm=True, use_rewnorm=True,
                 obsnorm_range=5.0, rewnorm_range=5.0, vectorized_env=None, gae_impl="np"):
        self.envs = envs                          # list of per-env objects (Dummy) or None
        self.venv = vectorized_env                # SynthBoxVec (numpy-vectorised variant) or None
        self.n_envs = len(envs) if envs is not None else vectorized_env.num_envs
        self.policy, self.learner = policy, learner
        self.n_steps, self.n_epoch, self.n_minibatch = n_steps, n_epoch, n_minibatch
        self.gamma, self.algo = gamma, algo
        self.use_obsnorm, self.use_rewnorm = use_obsnorm, use_rewnorm
        self.obsnorm_range, self.rewnorm_range = obsnorm_range, rewnorm_range
        first = envs[0] if envs is not None else None
        D = first.D if first is not None else vectorized_env.D
        A = first.A if first is not None else vectorized_env.A
        self.discrete = first.discrete if first is not None else vectorized_env.discrete
        act_shape = () if self.discrete else (A,)
        aux = {"old_logp": ()} if algo == "ppo" else {}
        self.memory = BufferRef((D,), act_shape, aux, self.n_envs, n_steps, use_gae, use_advnorm, gamma, gae_lambda,
                                gae_impl=gae_impl)
        self.obs_rms = RunningMeanStdRef((D,))
        self.ret_rms = RunningMeanStdRef(())
        self.returns = np.zeros(self.n_envs, np.float32)
        self.buffer_size = self.n_envs * n_steps
        self.batch_size = self.buffer_size // n_minibatch
        self.timers = {k: 0.0 for k in ("act", "env", "store", "gae", "sample", "update")}
        self.n_updates = 0
        self.update_times = []   # seconds per (sample + learner.update), for the baseline's spread
        if envs is not None:
            self.obs = np.stack([e.reset()[0] for e in envs]).astype(np.float32)
        else:
            self.obs = vectorized_env.reset()

    def _proc_obs(self, obs):
        return process_observation(obs, self.obs_rms, self.obsnorm_range) if self.use_obsnorm else obs

    def _proc_rew(self, rew):
        return process_reward(rew, self.ret_rms, self.rewnorm_range) if self.use_rewnorm else rew

    def _action(self, obs):
        torch = _torch()
        with torch.no_grad():
            head, logstd, v = self.policy.heads(torch.as_tensor(obs, dtype=torch.float32))
            d = self.policy.dist(head, logstd)
            a = d.sample()
            lp = d.log_prob(a) if self.discrete else d.log_prob(a).sum(-1)
        return a.numpy(), v.numpy(), lp.numpy()

    def _env_step(self, acts):
        if self.venv is not None:
            final, r, term, trunc, nxt = self.venv.step(acts)
            return final, r, term, trunc, [{"reset_obs": nxt[i]} for i in range(self.n_envs)]
        obs = np.zeros_like(self.obs)
        rews = np.zeros(self.n_envs, np.float32)
        terms = np.zeros(self.n_envs, bool)
        truncs = np.zeros(self.n_envs, bool)
        infos = []
        for e, env in enumerate(self.envs):
            o, rews[e], terms[e], truncs[e], info = env.step(acts[e])
            if terms[e] or truncs[e]:
                info["reset_obs"], _ = env.reset()
            obs[e] = o
            infos.append(info)
        return obs, rews, terms, truncs, infos

    def run_steps(self, n_env_steps, max_updates=None, on_update=None):
        """Run `n_env_steps` loop iterations (each steps all envs once).  `max_updates` bounds the
        number of learner updates per buffer-full phase (for a bounded CPU-baseline sample)."""
        obs = self.obs
        tm = self.timers
        for _ in range(n_env_steps):
            t0 = time.perf_counter()
            self.obs_rms.update(obs)
            obs = self._proc_obs(obs)
            acts, vals, logps = self._action(obs)
            t1 = time.perf_counter()
            next_obs, rews, terms, truncs, infos = self._env_step(acts)
            t2 = time.perf_counter()
            aux = {"old_logp": logps} if self.algo == "ppo" else None
            self.memory.store(obs, acts, self._proc_rew(rews), vals, terms, aux)
            tm["act"] += t1 - t0
            tm["env"] += t2 - t1
            tm["store"] += time.perf_counter() - t2
            if self.memory.full:
                t3 = time.perf_counter()
                _, bvals, _ = self._action(self._proc_obs(next_obs))
                t4 = time.perf_counter()
                for i in range(self.n_envs):
                    self.memory.finish_path(0.0 if terms[i] else bvals[i], i)
                t5 = time.perf_counter()
                tm["act"] += t4 - t3
                tm["gae"] += t5 - t4
                idx = np.arange(self.buffer_size)
                done_updates = 0
                for _ in range(self.n_epoch):
                    np.random.shuffle(idx)
                    for start in range(0, self.buffer_size, self.batch_size):
                        if max_updates is not None and done_updates >= max_updates:
                            break
                        ts = time.perf_counter()
                        ob, ac, rt, vl, ad, ax = self.memory.sample(idx[start:start + self.batch_size])
                        tu = time.perf_counter()
                        info = self.learner.update(ob, ac, rt, ad, ax.get("old_logp"))
                        te = time.perf_counter()
                        tm["sample"] += tu - ts
                        tm["update"] += te - tu
                        self.update_times.append(te - ts)
                        done_updates += 1
                        self.n_updates += 1
                        if on_update is not None:
                            on_update(info)
                self.memory.clear()
            if self.algo == "ppo":
                self.returns = (1 - terms) * self.gamma * self.returns + rews
            else:
                self.returns = self.gamma * self.returns + rews
            obs = next_obs
            for i in range(self.n_envs):
                if terms[i] or truncs[i]:
                    self.ret_rms.update(self.returns[i:i + 1])
                    self.returns[i] = 0.0
                    if self.algo == "a2c":   # a2c_agent.py:88-95: reset_obs replaces the row before the critic call
                        obs[i] = infos[i]["reset_obs"]
                    if terms[i]:
                        self.memory.finish_path(0.0, i)
                    else:
                        _, bv, _ = self._action(self._proc_obs(next_obs))
                        self.memory.finish_path(bv[i], i)
                    obs[i] = infos[i]["reset_obs"]
        self.obs = obs


class VecAgentRef:
    """The reference's on-policy train() loop over a host VecEnv, step for step: ppoclip_agent.py:59-111 (algo "ppo")
    and a2c_agent.py:57-107 (algo "a2c") with agent.py:104-123's observation / reward processing — the loop a user of
    the reference runs over DummyVecEnv_Gym / SubprocVecEnv_Gym (envs: buf_obs + step(acts) -> (obs, rew, term, trunc,
    infos with reset_obs), e.g. synth_env.DummyVecEnvRef).

    Two hooks replace what a replay cannot reproduce: action_source(obs) -> the actions to take (the device agent's
    recorded draws; the reference samples torch's CPU generator), and on_full(self) runs where the reference runs
    its n_epoch x n_minibatch updates (after the full-buffer finish_path calls, before memory.clear(); the tests
    snapshot the buffer there and replay the updates with the device permutations).  The policy computes values and
    the log-probabilities of the given actions (`heads(obs)` / `dist(head, logstd)`, f64 in the tests).

    The loop's quirks are kept, since a drop-in must reproduce them:
      * every train() call restarts from envs.buf_obs (ppoclip_agent.py:60): rows of envs that ended on the previous
        call's last step still hold their final observation there;
      * without obs-norm, `obs` is envs.buf_obs itself on a call's first step, and the store runs after envs.step,
        so a vec env that writes buf_obs in place (DummyVecEnv) has that column hold the post-step observations;
      * A2C replaces obs[i] (= next_obs[i]) by reset_obs BEFORE the critic call of a mid-rollout truncation, so the
        bootstrap is V(norm(reset_obs)) (a2c_agent.py:88-95); PPO calls the critic first: V(norm(final obs))
        (ppoclip_agent.py:95-101); the full-buffer closures use V(norm(next_obs)) before either (:69-75);
      * Atari (env_name "Atari"): a terminal without truncation (a life loss) keeps the path open and the obs
        (ppoclip_agent.py:93-94); ret_rms / the return tracker still see it;
      * returns: PPO masks with (1 - terminal) (ppoclip_agent.py:87), A2C does not (a2c_agent.py:82)."""

    def __init__(self, envs, policy, algo, n_steps, action_source, on_full=None, gamma=0.99, gae_lambda=0.95,
                 use_gae=True, use_advnorm=True, use_obsnorm=True, use_rewnorm=True, obsnorm_range=5.0,
                 rewnorm_range=5.0, atari=False, discrete=False):
        self.envs, self.policy, self.algo = envs, policy, algo
        self.action_source, self.on_full = action_source, on_full
        self.n_envs, self.n_steps = envs.num_envs, n_steps
        self.gamma, self.atari, self.discrete = gamma, atari, discrete
        self.use_obsnorm, self.use_rewnorm = use_obsnorm, use_rewnorm
        self.obsnorm_range, self.rewnorm_range = obsnorm_range, rewnorm_range
        obs_shape = tuple(envs.observation_space.shape)
        act_shape = () if discrete else tuple(envs.action_space.shape)
        aux = {"old_logp": ()} if algo == "ppo" else {}
        self.memory = BufferRef(obs_shape, act_shape, aux, self.n_envs, n_steps, use_gae, use_advnorm, gamma, gae_lambda,
                                obs_dtype=np.uint8 if atari else np.float32)
        self.obs_rms = RunningMeanStdRef(obs_shape)
        self.ret_rms = RunningMeanStdRef(())
        self.returns = np.zeros((self.n_envs,), np.float32)
        self.current_step = 0

    def _proc_obs(self, obs):
        return process_observation(obs, self.obs_rms, self.obsnorm_range) if self.use_obsnorm else obs

    def _proc_rew(self, rew):
        return process_reward(rew, self.ret_rms, self.rewnorm_range) if self.use_rewnorm else rew

    def _eval(self, obs, acts=None):
        """(values, log-probs of acts or None) — the critic / distribution part of _action (ppoclip_agent.py:50-57)."""
        torch = _torch()
        dt = next(self.policy.parameters()).dtype
        x = obs if (isinstance(obs, np.ndarray) and obs.dtype == np.uint8) else torch.as_tensor(np.asarray(obs), dtype=dt)
        with torch.no_grad():
            head, logstd, v = self.policy.heads(x)
            lp = None
            if acts is not None:
                d = self.policy.dist(head, logstd)
                a = torch.as_tensor(np.asarray(acts))
                lp = d.log_prob(a.long()) if self.discrete else d.log_prob(a.to(dt)).sum(-1)
                lp = lp.numpy()
        return v.numpy(), lp

    def train(self, train_steps):
        obs = self.envs.buf_obs
        for _ in range(train_steps):
            if self.use_obsnorm:   # RunningMeanStd.update only matters with obs-norm (its statistics are unused else)
                self.obs_rms.update(obs)
            obs = self._proc_obs(obs)
            acts = self.action_source(obs)
            value, logps = self._eval(obs, acts)
            next_obs, rewards, terminals, truncs, infos = self.envs.step(acts)
            aux = {"old_logp": logps} if self.algo == "ppo" else None
            self.memory.store(obs, acts, self._proc_rew(rewards), value, terminals, aux)
            if self.memory.full:
                vals, _ = self._eval(self._proc_obs(next_obs))
                for i in range(self.n_envs):
                    self.memory.finish_path(0.0 if terminals[i] else vals[i], i)
                if self.on_full is not None:
                    self.on_full(self)
                self.memory.clear()
            if self.algo == "ppo":
                self.returns = (1 - terminals) * self.gamma * self.returns + rewards
            else:
                self.returns = self.gamma * self.returns + rewards
            obs = next_obs
            for i in range(self.n_envs):
                if terminals[i] or truncs[i]:
                    self.ret_rms.update(self.returns[i:i + 1])
                    self.returns[i] = 0.0
                    if self.atari and not truncs[i]:
                        continue
                    if self.algo == "a2c":
                        obs[i] = infos[i]["reset_obs"]
                    if terminals[i]:
                        self.memory.finish_path(0.0, i)
                    else:
                        vals, _ = self._eval(self._proc_obs(next_obs))
                        self.memory.finish_path(vals[i], i)
                    obs[i] = infos[i]["reset_obs"]
            self.current_step += self.n_envs


# ---------------------------------------------------------------------------------------------------------------
# PER-DQN (BASELINE.json configs[4]).
def build_qnetwork_ref(n_actions, filters, kernels, strides, q_hidden, in_shape=(84, 84, 4)):
    """BasicQnetwork over Basic_CNN with the reference's module layout / state_dict keys
    (representation.model.*, target_representation.model.*, eval_Qhead.model.*, target_Qhead.model.*)."""
    import copy
    torch = _torch()
    nn = torch.nn

    class BasicCNNRef(nn.Module):   # cnn.py:5-40: conv blocks (padding (k - s) // 2) + ReLU, global max pool
        def __init__(self):
            super().__init__()
            layers, (C, H, W) = [], (in_shape[2], in_shape[0], in_shape[1])
            for k, st, f in zip(kernels, strides, filters):
                pad = int((k - st) // 2)
                layers += [nn.Conv2d(C, f, k, st, padding=pad), nn.ReLU()]
                C = f
            layers += [nn.AdaptiveMaxPool2d((1, 1)), nn.Flatten()]
            self.model = nn.Sequential(*layers)

        def forward(self, obs):   # obs / 255.0 on the host (f64), NHWC -> NCHW, float32 (parameters' dtype in f64 runs)
            dt = next(self.parameters()).dtype
            x = torch.as_tensor(np.transpose(np.asarray(obs) / 255.0, (0, 3, 1, 2)), dtype=dt)
            return {"state": self.model(x)}

    class QheadRef(nn.Module):    # deterministic.py:6-25
        def __init__(self):
            super().__init__()
            layers, d = [], filters[-1]
            for h in q_hidden:
                layers += [nn.Linear(d, h), nn.ReLU()]
                d = h
            layers += [nn.Linear(d, n_actions)]
            self.model = nn.Sequential(*layers)

        def forward(self, x):
            return self.model(x)

    class QnetRef(nn.Module):     # deterministic.py:148-182
        def __init__(self):
            super().__init__()
            self.representation = BasicCNNRef()
            self.target_representation = copy.deepcopy(self.representation)
            self.eval_Qhead = QheadRef()
            self.target_Qhead = copy.deepcopy(self.eval_Qhead)

        def forward(self, obs):
            q = self.eval_Qhead(self.representation(obs)["state"])
            return None, q.argmax(dim=-1), q

        def target(self, obs):
            q = self.target_Qhead(self.target_representation(obs)["state"])
            return None, q.argmax(dim=-1).detach(), q.detach()

        def copy_target(self):
            for ep, tp in zip(self.representation.parameters(), self.target_representation.parameters()):
                tp.data.copy_(ep)
            for ep, tp in zip(self.eval_Qhead.parameters(), self.target_Qhead.parameters()):
                tp.data.copy_(ep)

    return QnetRef()


def dqn_td_ref(evalQ, targetQ, act, rew, term, gamma):
    """perdqn_learner.py:23-30 in closed form (f32 numpy, torch's operation order):
    y = rew + (gamma * (1 - term)) * max_a' targetQ,  p = evalQ[act],  loss = mean((p - y)^2),
    d loss / d evalQ = 2 (p - y) / B at (b, act_b), |TD| = |y - p|."""
    evalQ, targetQ = np.asarray(evalQ, np.float32), np.asarray(targetQ, np.float32)
    a = np.asarray(act).astype(np.int64)
    B = evalQ.shape[0]
    y = np.asarray(rew, np.float32) + (np.float32(gamma) * (np.float32(1) - np.asarray(term, np.float32))) * \
        targetQ.max(-1)
    p = evalQ[np.arange(B), a]
    d = (p - y).astype(np.float32)
    dq = np.zeros_like(evalQ)
    dq[np.arange(B), a] = np.float32(2.0) * d / np.float32(B)
    return float(np.mean(d.astype(np.float64) ** 2)), np.abs(y - p).astype(np.float32), dq, float(p.mean())


class PerDQNLearnerRef:
    """perdqn_learner.py:17-48 on torch CPU: TD target from the target network, MSE, Adam, LinearLR, hard target
    copy every sync_frequency updates; returns (|TD error|, info)."""

    def __init__(self, policy, optimizer, scheduler, gamma=0.99, sync_frequency=100):
        self.policy, self.optimizer, self.scheduler = policy, optimizer, scheduler
        self.gamma, self.sync_frequency, self.iterations = gamma, sync_frequency, 0

    def update(self, obs, act, rew, nxt, term):
        torch = _torch()
        self.iterations += 1
        act, rew, term = torch.as_tensor(act), torch.as_tensor(rew), torch.as_tensor(term)
        _, _, evalQ = self.policy(obs)
        rew, term = rew.to(evalQ.dtype), term.to(evalQ.dtype)
        _, _, targetQ = self.policy.target(nxt)
        targetQ = rew + self.gamma * (1 - term) * targetQ.max(dim=-1).values
        predictQ = (evalQ * torch.nn.functional.one_hot(act.long(), evalQ.shape[1])).sum(dim=-1)
        td = targetQ - predictQ
        loss = torch.nn.functional.mse_loss(predictQ, targetQ)
        self.optimizer.zero_grad()
        loss.backward()
        self.optimizer.step()
        if self.scheduler is not None:
            self.scheduler.step()
        if self.iterations % self.sync_frequency == 0:
            self.policy.copy_target()
        info = {"Qloss": loss.item(), "learning_rate": self.optimizer.param_groups[0]["lr"],
                "predictQ": predictQ.mean().item()}
        return np.abs(td.detach().numpy()), info
