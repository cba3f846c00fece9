"""Device-resident drop-in for the reference's on-policy buffer.

Mirrors xuance/common/memory_tools.py:143-245 (DummyOnPolicyBuffer) and :526-560
(DummyOnPolicyBuffer_Atari): same constructor, methods (store / finish_path / sample / clear / full)
and attributes (ptr, size, start_ids, n_envs, n_size, buffer_size, observations, actions, rewards,
returns, values, terminals, advantages, auxiliary_infos).  The arrays are torch tensors in HBM laid
out [n_envs, n_size, ...] row-major exactly like create_memory (memory_tools.py:12-36), so the flat
sample index env*T + step (memory_tools.py:234) is the row index of the flattened buffer.

Differences by design (documented in DESIGN.md):
  * finish_path(val, i) records the closure (closed/boot columns) instead of running a Python loop;
    GAE for every recorded path runs in one HIP launch (xpa_gae_scan) the first time advantages are
    needed (sample(), compute_advantages(), or reading .returns/.advantages through the properties).
    The values are the same the reference would have computed at closure time: a path's inputs are
    never modified after it is stored.
  * clear() zeroes in place (no reallocation), so captured hipGraphs keep valid pointers.
  * sample() returns device tensors (the learners accept them directly).
"""
import numpy as np
import torch

from . import ops
from .policies import space_shape


def _dev(device):
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device(device)


OBS_SLACK = 128   # elements of zeroed slack after the observation buffer (see DummyOnPolicyBuffer.__init__)

class DummyOnPolicyBuffer:
    obs_dtype = torch.float32

    def __init__(self, observation_space, action_space, auxiliary_shape, n_envs, n_size, use_gae=True,
                 use_advnorm=True, gamma=0.99, gae_lam=0.95, device=None):
        self.observation_space, self.action_space = observation_space, action_space
        self.auxiliary_shape = dict(auxiliary_shape or {})
        self.n_envs, self.n_size = int(n_envs), int(n_size)
        self.buffer_size = self.n_envs * self.n_size
        self.use_gae, self.use_advnorm = use_gae, use_advnorm
        self.gamma, self.gae_lam = gamma, gae_lam
        self.device = _dev(device)
        self.obs_shape = space_shape(observation_space)
        self.act_shape = space_shape(action_space)
        self.start_ids = np.zeros(self.n_envs, np.int64)
        N, T, dev = self.n_envs, self.n_size, self.device
        f32 = dict(dtype=torch.float32, device=dev)
        # r05: OBS_SLACK zeroed elements after the last row (same allocation): the update's split GEMMs may read a row
        # tile past a row's end (C4's 376-wide trunk read through the minibatch index, fused_mlp._wide_forward)
        n_obs = N * T * int(np.prod(self.obs_shape, dtype=np.int64))
        self.observations = torch.zeros(n_obs + OBS_SLACK, dtype=self.obs_dtype, device=dev)[:n_obs].view(
            (N, T) + self.obs_shape)
        self.actions = torch.zeros((N, T) + self.act_shape, **f32)
        self.rewards = torch.zeros((N, T), **f32)
        self._returns = torch.zeros((N, T), **f32)
        self.values = torch.zeros((N, T), **f32)
        self.terminals = torch.zeros((N, T), **f32)
        self._advantages = torch.zeros((N, T), **f32)
        self.auxiliary_infos = {k: torch.zeros((N, T) + tuple(v), **f32) for k, v in self.auxiliary_shape.items()}
        # closure record consumed by xpa_gae_scan
        self.closed = torch.zeros((N, T), dtype=torch.uint8, device=dev)
        self.boot = torch.zeros((N, T), **f32)
        self._pending = []          # host-side closures from finish_path(val, i)
        self._dirty = False
        self.ptr, self.size = 0, 0

    # ---- reference API ---------------------------------------------------------------------------
    @property
    def full(self):
        return self.size >= self.n_size

    def clear(self):
        self.ptr, self.size = 0, 0
        for t in (self.observations, self.actions, self.rewards, self._returns, self.values, self.terminals,
                  self._advantages, self.closed, self.boot):
            t.zero_()
        for t in self.auxiliary_infos.values():
            t.zero_()
        self._pending.clear()
        self._dirty = False

    def _put(self, dst, data):
        if data is None:
            return
        if isinstance(data, torch.Tensor):
            dst[:, self.ptr] = data.to(device=dst.device, dtype=dst.dtype)
        else:
            dst[:, self.ptr] = torch.as_tensor(np.asarray(data), dtype=dst.dtype).to(dst.device, non_blocking=True)

    def store(self, obs, acts, rews, value, terminals, aux_info=None):
        """memory_tools.py:196-204."""
        self._put(self.observations, obs)
        self._put(self.actions, acts)
        self._put(self.rewards, rews)
        self._put(self.values, value)
        self._put(self.terminals, terminals)
        if aux_info:
            for k, v in aux_info.items():
                self._put(self.auxiliary_infos[k], v)
        self.ptr = (self.ptr + 1) % self.n_size
        self.size = min(self.size + 1, self.n_size)

    def finish_path(self, val, i):
        """memory_tools.py:206-229: records the closure of env i's open path at the current end."""
        end = self.n_size if self.full else self.ptr
        if end > self.start_ids[i]:
            self._pending.append((int(i), end - 1, float(val)))
            self._dirty = True
        self.start_ids[i] = self.ptr

    def finish_paths(self, vals, env_mask=None):
        """Vectorised finish_path for all envs (or env_mask) at once; vals a device or host [n_envs] array."""
        end = self.n_size if self.full else self.ptr
        idx = np.arange(self.n_envs) if env_mask is None else np.nonzero(np.asarray(env_mask))[0]
        idx = idx[end > self.start_ids[idx]]
        if len(idx):
            self._flush()
            vals_t = torch.as_tensor(vals, dtype=torch.float32, device=self.device).reshape(-1)
            ii = torch.as_tensor(idx, device=self.device)
            self.closed[ii, end - 1] = 1
            self.boot[ii, end - 1] = vals_t[ii] if vals_t.numel() == self.n_envs else vals_t
            self._dirty = True
        self.start_ids[idx] = self.ptr

    def _flush(self):
        if self._pending:
            p = np.asarray(self._pending, dtype=np.float64)
            ii = torch.as_tensor(p[:, 0].astype(np.int64), device=self.device)
            tt = torch.as_tensor(p[:, 1].astype(np.int64), device=self.device)
            self.closed[ii, tt] = 1
            self.boot[ii, tt] = torch.as_tensor(p[:, 2].astype(np.float32), device=self.device)
            self._pending.clear()

    def compute_advantages(self):
        """One xpa_gae_scan over the whole buffer for every recorded closure."""
        self._flush()
        ops.gae_scan(self.rewards, self.values, self.terminals, self.closed, self.boot, self.gamma, self.gae_lam,
                     self.use_gae, adv=self._advantages, ret=self._returns)
        self._dirty = False

    @property
    def returns(self):
        if self._dirty:
            self.compute_advantages()
        return self._returns

    @property
    def advantages(self):
        if self._dirty:
            self.compute_advantages()
        return self._advantages

    def sample(self, indexes):
        """memory_tools.py:231-245; returns device tensors."""
        assert self.full, "Not enough transitions for on-policy buffer to random sample"
        if self._dirty:
            self.compute_advantages()
        idx = torch.as_tensor(np.asarray(indexes) if not isinstance(indexes, torch.Tensor) else indexes,
                              dtype=torch.int64, device=self.device)
        flat = lambda t: t.reshape((self.buffer_size,) + tuple(t.shape[2:]))  # noqa: E731
        obs, part = ops.gather_minibatch(idx, flat(self.observations), adv=flat(self._advantages))
        act = flat(self.actions)[idx]
        ret = flat(self._returns)[idx]
        val = flat(self.values)[idx]
        adv = flat(self._advantages)[idx]
        if self.use_advnorm:
            s = part.sum(0)
            n = idx.numel()
            mean = s[0] / n
            std = torch.sqrt(torch.clamp(s[1] / n - mean * mean, min=0.0))
            adv = ((adv.double() - mean) / (std.float().double() + 1e-8)).float()
        aux = {k: flat(v)[idx] for k, v in self.auxiliary_infos.items()}
        return obs, act, ret, val, adv, aux


class DummyOnPolicyBuffer_Atari(DummyOnPolicyBuffer):
    """memory_tools.py:526-560: uint8 observations."""
    obs_dtype = torch.uint8
