"""CPU restatement of the reference's prioritized replay (test infrastructure only — imported by
tests/ and bench.py's cpu_baseline leg, never by the product path).

Follows (reference paths):
  SegmentTree / SumSegmentTree / MinSegmentTree   xuance/common/segtree_tool.py:4-86
  PerOffPolicyBuffer                              xuance/common/memory_tools.py:369-492
Pinned by tests/golden/per.npz (captured from the reference by tests/golden/make_golden.py).

Arithmetic: trees hold Python / NumPy scalar objects combined with operator.add / min, exactly as
the reference does, so the result type follows NumPy's promotion rules:
  * pinned=False — the NumPy running here (2.x, NEP 50): np.float32 priority ** alpha stays float32,
    float32 + float32 nodes stay float32.  Reproduces the fixtures bitwise.
  * pinned=True  — the reference's pinned NumPy 1.21 (setup.py:48): value-based casting makes
    np.float32 ** float a float64, so every leaf and node is f64.  This is what xuanpolicy_amd's K6
    kernels implement (f64 trees).
Sampling takes the uniforms explicitly (the reference draws them with random.random(),
memory_tools.py:415); the fixtures record them.
"""
import operator

import numpy as np


class SegmentTreeRef:
    def __init__(self, capacity, op, neutral):
        assert capacity > 0 and capacity & (capacity - 1) == 0
        self.capacity = capacity
        self.value = [neutral for _ in range(2 * capacity)]
        self.op = op

    def _reduce(self, start, end, node, lo, hi):
        # segtree_tool.py:11-24 (inclusive end)
        if start == lo and end == hi:
            return self.value[node]
        mid = (lo + hi) // 2
        if end <= mid:
            return self._reduce(start, end, 2 * node, lo, mid)
        if mid + 1 <= start:
            return self._reduce(start, end, 2 * node + 1, mid + 1, hi)
        return self.op(self._reduce(start, mid, 2 * node, lo, mid), self._reduce(mid + 1, end, 2 * node + 1, mid + 1, hi))

    def reduce(self, start=0, end=None):
        # segtree_tool.py:26-32: `end` is exclusive (end -= 1 before the inclusive helper)
        if end is None:
            end = self.capacity
        if end < 0:
            end += self.capacity
        end -= 1
        if end < start:
            raise ValueError("empty range (the reference recurses forever here)")
        return self._reduce(start, end, 1, 0, self.capacity - 1)

    def __setitem__(self, idx, val):
        idx = int(idx) + self.capacity
        self.value[idx] = val
        idx //= 2
        while idx >= 1:
            self.value[idx] = self.op(self.value[2 * idx], self.value[2 * idx + 1])
            idx //= 2

    def __getitem__(self, idx):
        return self.value[self.capacity + int(idx)]

    def array(self):
        return np.asarray([float(v) for v in self.value], np.float64)


class SumTreeRef(SegmentTreeRef):
    def __init__(self, capacity):
        super().__init__(capacity, operator.add, 0.0)

    def sum(self, start=0, end=None):
        return self.reduce(start, end)

    def find_prefixsum_idx(self, prefixsum):
        # segtree_tool.py:62-71
        assert 0 <= prefixsum <= self.sum() + 1e-5
        idx = 1
        while idx < self.capacity:
            if self.value[2 * idx] > prefixsum:
                idx = 2 * idx
            else:
                prefixsum -= self.value[2 * idx]
                idx = 2 * idx + 1
        return idx - self.capacity


class MinTreeRef(SegmentTreeRef):
    def __init__(self, capacity):
        super().__init__(capacity, min, float("inf"))

    def min(self, start=0, end=None):
        return self.reduce(start, end)


def next_pow2(n):
    c = 1
    while c < n:
        c *= 2
    return c


class PerBufferRef:
    """memory_tools.py:369-492 (trees, priorities, index choices and IS weights; the transition arrays
    are plain [n_envs, n_size, ...] numpy arrays as create_memory makes them)."""

    def __init__(self, n_envs, n_size, batch_size, alpha=0.6, obs_shape=(), pinned=True, wrap_uint8=True):
        self.n_envs, self.n_size, self.batch_size, self.alpha = n_envs, n_size, batch_size, alpha
        self.pinned, self.wrap_uint8 = pinned, wrap_uint8
        cap = next_pow2(n_size)
        self.capacity = cap
        self.it_sum = [SumTreeRef(cap) for _ in range(n_envs)]
        self.it_min = [MinTreeRef(cap) for _ in range(n_envs)]
        self.max_priority = np.ones(n_envs)
        self.size, self.ptr = 0, 0
        self.obs_shape = tuple(obs_shape)
        self.observations = np.zeros((n_envs, n_size) + self.obs_shape, np.float32)
        self.next_observations = np.zeros((n_envs, n_size) + self.obs_shape, np.float32)
        self.actions = np.zeros((n_envs, n_size), np.float32)
        self.rewards = np.zeros((n_envs, n_size), np.float32)
        self.terminals = np.zeros((n_envs, n_size), np.float32)

    def store(self, obs, acts, rews, terminals, next_obs):
        # memory_tools.py:429-443
        p = self.ptr
        self.observations[:, p] = obs
        self.actions[:, p] = acts
        self.rewards[:, p] = rews
        self.terminals[:, p] = terminals
        self.next_observations[:, p] = next_obs
        for i in range(self.n_envs):
            v = self.max_priority[i] ** self.alpha
            self.it_sum[i][p] = v
            self.it_min[i][p] = v
        self.ptr = (self.ptr + 1) % self.n_size
        self.size = min(self.size + 1, self.n_size)

    def sample_indices(self, beta, uniforms):
        """memory_tools.py:411-465: per env, batch/n_envs stratified prefix-sum descents over the
        mass sum(0, size - 1) (= leaves [0, size-2], the exclusive-end quirk), IS weights, and the
        uint8 cast of the chosen steps (wrap_uint8=True, the reference) or plain int64 indices."""
        b = self.batch_size // self.n_envs
        assert beta > 0
        uniforms = np.asarray(uniforms, np.float64).reshape(self.n_envs, b)
        steps = np.zeros((self.n_envs, b), np.float64)
        weights = np.zeros((self.n_envs, b))
        for i in range(self.n_envs):
            p_total = self.it_sum[i].sum(0, self.size - 1)
            every = p_total / b
            idxes = [int(self.it_sum[i].find_prefixsum_idx(uniforms[i, k] * every + k * every)) for k in range(b)]
            p_min = self.it_min[i].min() / self.it_sum[i].sum()
            max_weight = p_min * self.size ** (-beta)
            ws = []
            for idx in idxes:
                p_sample = self.it_sum[i][idx] / self.it_sum[i].sum()
                weight = p_sample * self.size ** (-beta)
                ws.append(weight / max_weight)
            steps[i] = idxes
            weights[i] = np.array(ws)
        steps = steps.astype(np.uint8) if self.wrap_uint8 else steps.astype(np.int64)
        return steps, weights

    def sample(self, beta, uniforms):
        steps, weights = self.sample_indices(beta, uniforms)
        b = self.batch_size // self.n_envs
        env = np.arange(self.n_envs).repeat(b)
        st = steps.reshape(-1).astype(np.int64)
        return (self.observations[env, st], self.actions[env, st], self.rewards[env, st], self.terminals[env, st],
                self.next_observations[env, st], weights, steps)

    def update_priorities(self, idxes, priorities):
        # memory_tools.py:482-492 (sequential: a repeated index keeps the last value)
        b = self.batch_size // self.n_envs
        priorities = np.asarray(priorities).reshape(self.n_envs, b)
        idxes = np.asarray(idxes).astype(np.int64).reshape(self.n_envs, b)
        for i in range(self.n_envs):
            for idx, priority in zip(idxes[i], priorities[i]):
                if self.pinned:
                    priority = float(priority)      # NumPy 1.21 value-based casting: f64 arithmetic
                if priority == 0:
                    priority += 1e-8
                assert 0 <= idx < self.size
                v = priority ** self.alpha
                self.it_sum[i][idx] = v
                self.it_min[i][idx] = v
                self.max_priority[i] = max(self.max_priority[i], priority)

    def trees(self):
        return (np.stack([t.array() for t in self.it_sum]), np.stack([t.array() for t in self.it_min]))
