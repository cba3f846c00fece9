"""Prioritized replay buffer on device — drop-in for the reference's PerOffPolicyBuffer.

Mirrors (reference paths):
  PerOffPolicyBuffer          xuance/common/memory_tools.py:369-492 (same constructor arguments,
                              store / sample(beta) / update_priorities / clear, attributes n_envs,
                              n_size, batch_size, size, ptr, observations, next_observations,
                              actions, rewards, terminals)
  Sum/MinSegmentTree          xuance/common/segtree_tool.py:4-86 (as f64 arrays in HBM, K6)
The trees, priorities and every transition array live in HBM; sample() returns device tensors
(gathered by K4 through the sampled flat indices) and update_priorities() accepts device tensors, so
a GPU learner never round-trips through the host.  Semantics follow the reference with its pinned
NumPy 1.21 arithmetic (f64 trees); documented deltas:
  * wrap_uint8 (default False): the reference casts the chosen steps to uint8
    (memory_tools.py:465), which wraps indices >= 256 for n_size > 256; True reproduces that for
    parity, False returns the intended int64 indices.
  * obs_dtype: the reference stores observations as float32 (create_memory default); Atari-shaped
    uint8 frames may be kept as uint8 (4x less HBM: 1 M x 4x84x84 = 28 GB instead of 113 GB per array),
    gathered as uint8.
  * sample() draws its uniforms from a counter hash of (seed, call, env, k) unless `uniforms` is given
    (the reference calls random.random(), memory_tools.py:415).
  * clear() also resets the trees to empty (the reference empties the tree lists, after which store()
    fails); like the reference it keeps ptr and size.
"""
import numpy as np
import torch

from . import _lib, ops


def _shape(space):
    if space is None:
        return ()
    return tuple(space.shape) if getattr(space, "shape", None) is not None else ()


def _next_pow2(n):
    c = 1
    while c < n:
        c *= 2
    return c


class PerOffPolicyBuffer:
    def __init__(self, observation_space, action_space, auxiliary_shape, n_envs, n_size, batch_size, alpha=0.6,
                 device="cuda", seed=1, wrap_uint8=False, obs_dtype=torch.float32):
        self.observation_space, self.action_space, self.auxiliary_shape = observation_space, action_space, auxiliary_shape
        self.n_envs, self.n_size, self.batch_size = int(n_envs), int(n_size), int(batch_size)
        if self.batch_size % self.n_envs:
            raise ValueError("batch_size must be a multiple of n_envs (the reference splits it evenly)")
        self._alpha = float(alpha)
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("PerOffPolicyBuffer lives on a ROCm device; xuanpolicy_amd has no CPU path")
        self.seed, self.wrap_uint8, self.obs_dtype = int(seed), bool(wrap_uint8), obs_dtype
        self.size, self.ptr = 0, 0
        self.capacity = _next_pow2(self.n_size)
        self._alloc()
        self._calls = 0

    def _alloc(self):
        N, S, dev = self.n_envs, self.n_size, self.device
        obs_shape, act_shape = _shape(self.observation_space), _shape(self.action_space)
        self.observations = torch.zeros((N, S) + obs_shape, dtype=self.obs_dtype, device=dev)
        self.next_observations = torch.zeros((N, S) + obs_shape, dtype=self.obs_dtype, device=dev)
        self.actions = torch.zeros((N, S) + act_shape, dtype=torch.float32, device=dev)
        self.rewards = torch.zeros((N, S), dtype=torch.float32, device=dev)
        self.terminals = torch.zeros((N, S), dtype=torch.float32, device=dev)
        cap = self.capacity
        self.sum_tree = torch.zeros((N, 2 * cap), dtype=torch.float64, device=dev)
        self.min_tree = torch.full((N, 2 * cap), float("inf"), dtype=torch.float64, device=dev)
        self._max_priority = torch.ones(N, dtype=torch.float64, device=dev)
        self._scratch = torch.full((N, cap), -1, dtype=torch.int32, device=dev)
        self._err = torch.zeros(1, dtype=torch.int32, device=dev)
        # error words of the sample descent (draws clamped to the last stored step) and of the row gathers (an index
        # outside the buffer): counted on device, read by check_errors() (one sync, at the caller's choice)
        self._sample_err = torch.zeros(1, dtype=torch.int32, device=dev)
        self._gather_err = torch.zeros(1, dtype=torch.int32, device=dev)

    # ---- memory_tools.py:429-443 ----------------------------------------------------------------
    def _put(self, dst, data):
        t = torch.as_tensor(np.asarray(data) if not isinstance(data, torch.Tensor) else data)
        dst[:, self.ptr] = t.to(device=self.device, dtype=dst.dtype).reshape(dst[:, self.ptr].shape)

    def store(self, obs, acts, rews, terminals, next_obs):
        self._put(self.observations, obs)
        self._put(self.actions, acts)
        self._put(self.rewards, rews)
        self._put(self.terminals, terminals)
        self._put(self.next_observations, next_obs)
        _lib.check(ops.lib().xpa_per_store(ops._p(self.sum_tree), ops._p(self.min_tree), ops._p(self._max_priority),
                                           self.n_envs, self.capacity, self.ptr, self._alpha, ops._stream(self.device)),
                   "xpa_per_store")
        self.ptr = (self.ptr + 1) % self.n_size
        self.size = min(self.size + 1, self.n_size)

    # ---- memory_tools.py:446-480 ----------------------------------------------------------------
    def sample_indices(self, beta, uniforms=None):
        """(steps [n_envs, b] int64 (or uint8-wrapped values), flat [n_envs*b] int64, weights [n_envs, b] f64)."""
        assert beta > 0
        if self.size < 2:
            raise ValueError("PerOffPolicyBuffer.sample needs size >= 2 (the reference recurses forever at 1)")
        b = self.batch_size // self.n_envs
        steps = torch.empty((self.n_envs, b), dtype=torch.int64, device=self.device)
        flat = torch.empty(self.n_envs * b, dtype=torch.int64, device=self.device)
        weights = torch.empty((self.n_envs, b), dtype=torch.float64, device=self.device)
        if uniforms is not None:
            uniforms = torch.as_tensor(uniforms, dtype=torch.float64).to(self.device).reshape(-1).contiguous()
            if uniforms.numel() != self.n_envs * b:
                raise ValueError("uniforms must have n_envs * batch_size / n_envs entries")
        self._calls += 1
        _lib.check(ops.lib().xpa_per_sample(ops._p(self.sum_tree), ops._p(self.min_tree), self.n_envs, self.capacity,
                                            self.size, b, self.n_size, ops._p(uniforms), self.seed & 0xFFFFFFFF,
                                            self._calls & 0xFFFFFFFF, float(beta), int(self.wrap_uint8), ops._p(steps),
                                            ops._p(flat), ops._p(weights), ops._p(self._sample_err),
                                            ops._stream(self.device)), "xpa_per_sample")
        return steps, flat, weights

    def _gather(self, arr, flat):
        rows = arr.reshape((self.n_envs * self.n_size,) + tuple(arr.shape[2:]))
        out, _ = ops.gather_minibatch(flat, rows, err=self._gather_err)
        return out

    def sample(self, beta, uniforms=None):
        steps, flat, weights = self.sample_indices(beta, uniforms)
        return (self._gather(self.observations, flat), self._gather(self.actions, flat),
                self._gather(self.rewards, flat), self._gather(self.terminals, flat),
                self._gather(self.next_observations, flat), weights, steps)

    # ---- memory_tools.py:482-492 ----------------------------------------------------------------
    def update_priorities(self, idxes, priorities, check=True):
        """idxes [n_envs, b] (as sample() returned them), priorities [n_envs * b] (|TD error|).
        check=True raises like the reference's assert when an index is outside [0, size) (one sync)."""
        b = self.batch_size // self.n_envs
        idx = torch.as_tensor(np.asarray(idxes) if not isinstance(idxes, torch.Tensor) else idxes)
        idx = idx.to(device=self.device, dtype=torch.int64).reshape(-1).contiguous()
        pr = torch.as_tensor(np.asarray(priorities) if not isinstance(priorities, torch.Tensor) else priorities)
        pr = pr.to(device=self.device, dtype=torch.float32).reshape(-1).contiguous()
        if idx.numel() != self.n_envs * b or pr.numel() != self.n_envs * b:
            raise ValueError("idxes / priorities must have n_envs * batch_size / n_envs entries")
        if check:
            self._err.zero_()
        _lib.check(ops.lib().xpa_per_update_priorities(ops._p(self.sum_tree), ops._p(self.min_tree),
                                                       ops._p(self._max_priority), ops._p(self._scratch), self.n_envs,
                                                       self.capacity, max(self.size, 1), ops._p(idx), ops._p(pr), b,
                                                       self._alpha, ops._p(self._err), ops._stream(self.device)),
                   "xpa_per_update_priorities")
        if check and int(self._err.item()):
            raise AssertionError("update_priorities: index outside [0, size)")

    def check_errors(self):
        """(sample draws clamped past the stored leaves, gathered indices outside the buffer) since the last call;
        one host sync.  Both are 0 unless the trees or indices are corrupt."""
        out = (int(self._sample_err.item()), int(self._gather_err.item()))
        self._sample_err.zero_()
        self._gather_err.zero_()
        return out

    def clear(self):
        self._alloc()

    # reference-style accessors for the trees (tests / inspection)
    @property
    def max_priority(self):
        return self._max_priority
