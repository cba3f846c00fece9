"""GPU: K6 prioritized replay (xuanpolicy_amd.per.PerOffPolicyBuffer through the C ABI) against the
oracle (oracle/per_ref.py, pinned f64 semantics) and the reference's own fixtures (tests/golden/per.npz)."""
import numpy as np
import pytest
import torch

from oracle.per_ref import PerBufferRef

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


class _Box:
    def __init__(self, shape):
        self.shape = shape


class _Disc:
    shape = ()


def _trees(buf):
    return buf.sum_tree.cpu().numpy(), buf.min_tree.cpu().numpy()


def _close_tree(got, exp, rtol):
    fin = np.isfinite(exp)
    assert np.array_equal(np.isfinite(got), fin)
    np.testing.assert_allclose(got[fin], exp[fin], rtol=rtol, atol=1e-300)


@pytest.mark.parametrize("tag", ["small", "wrap"])
def test_per_buffer_replays_reference_fixture(golden, tag):
    from xuanpolicy_amd.per import PerOffPolicyBuffer
    g = golden("per.npz")
    n_envs, n_size, batch, cap = (int(v) for v in g[tag + "/config"])
    alpha, beta = (float(v) for v in g[tag + "/alpha_beta"])
    buf = PerOffPolicyBuffer(_Box((3,)), _Disc(), {}, n_envs, n_size, batch, alpha, device=DEV, wrap_uint8=True)
    ref = PerBufferRef(n_envs, n_size, batch, alpha, obs_shape=(3,), pinned=True)
    assert buf.capacity == cap
    obs, act, rew, term, nxt = (g[tag + "/" + k] for k in ("obs", "act", "rew", "term", "next"))
    t, r = 0, 0
    while tag + "/r%d/n_store" % r in g:
        pr = tag + "/r%d/" % r
        for _ in range(int(g[pr + "n_store"])):
            buf.store(obs[t], act[t], rew[t], term[t], nxt[t])
            ref.store(obs[t], act[t], rew[t], term[t], nxt[t])
            t += 1
        s, m = _trees(buf)
        rs, rm = ref.trees()
        _close_tree(s, rs, 1e-13)
        _close_tree(m, rm, 1e-13)
        _close_tree(s, g[pr + "tree_sum_after_store"], 1e-6)
        ob, ac, rw, te, nx, w, steps = buf.sample(beta, uniforms=g[pr + "uniforms"])
        assert np.array_equal(steps.cpu().numpy(), g[pr + "step_choices"].astype(np.int64))
        np.testing.assert_allclose(w.cpu().numpy(), g[pr + "weights"], rtol=1e-6)
        _, _, _, _, _, rw_ref, rsteps = ref.sample(beta, g[pr + "uniforms"])
        np.testing.assert_allclose(w.cpu().numpy(), rw_ref, rtol=1e-12)
        for k, v in (("obs", ob), ("act", ac), ("rew", rw), ("term", te), ("next", nx)):
            assert np.array_equal(v.cpu().numpy(), g[pr + k].astype(np.float32)), k
        buf.update_priorities(steps, g[pr + "priorities"])
        ref.update_priorities(rsteps.astype(np.int64), g[pr + "priorities"])
        s, m = _trees(buf)
        rs, rm = ref.trees()
        _close_tree(s, rs, 1e-13)
        _close_tree(m, rm, 1e-13)
        _close_tree(s, g[pr + "tree_sum_after_update"], 1e-6)
        np.testing.assert_allclose(buf.max_priority.cpu().numpy(), ref.max_priority, rtol=0)
        assert (buf.size, buf.ptr) == tuple(g[pr + "size_ptr"])
        r += 1
    assert r >= 2


def test_per_buffer_matches_oracle_random_rounds():
    """n_size > 256 with intended int64 indices, repeated indices, zero priorities, ring wrap-around."""
    from xuanpolicy_amd.per import PerOffPolicyBuffer
    rng = np.random.default_rng(0)
    n_envs, n_size, batch, alpha, beta = 4, 3000, 1024, 0.6, 0.4
    buf = PerOffPolicyBuffer(_Box((2,)), _Disc(), {}, n_envs, n_size, batch, alpha, device=DEV)
    ref = PerBufferRef(n_envs, n_size, batch, alpha, obs_shape=(2,), pinned=True, wrap_uint8=False)
    b = batch // n_envs
    for rnd, n_store in enumerate([1500, 1200, 900]):
        for _ in range(n_store):
            o = rng.normal(size=(n_envs, 2)).astype(np.float32)
            a = rng.integers(0, 5, n_envs).astype(np.float32)
            z = np.zeros(n_envs, np.float32)
            buf.store(o, a, z, z, o)
            ref.store(o, a, z, z, o)
        u = rng.random(n_envs * b)
        _, _, _, _, _, w, steps = buf.sample(beta, uniforms=u)
        _, _, _, _, _, rw, rsteps = ref.sample(beta, u)
        assert np.array_equal(steps.cpu().numpy(), rsteps)
        np.testing.assert_allclose(w.cpu().numpy(), rw, rtol=1e-12)
        prio = (rng.random(batch) * 3).astype(np.float32)
        prio[::5] = 0
        idx = rsteps.copy()
        idx[:, ::7] = idx[:, :1]               # repeated indices: the last entry must win
        buf.update_priorities(torch.as_tensor(idx, device=DEV), torch.as_tensor(prio, device=DEV))
        ref.update_priorities(idx, prio)
        s, m = _trees(buf)
        rs, rm = ref.trees()
        _close_tree(s, rs, 1e-12)
        _close_tree(m, rm, 1e-12)
        np.testing.assert_allclose(buf.max_priority.cpu().numpy(), ref.max_priority, rtol=0)
    with pytest.raises(AssertionError):
        bad = np.zeros((n_envs, b), np.int64)
        bad[1, 3] = n_size + 5
        buf.update_priorities(bad, np.ones(batch, np.float32))


def test_per_full_size_tree_properties():
    """C5 sizes (8 envs x 131 072 slots = 1 M transitions, batch 2048): after bulk leaves + K6 updates,
    every internal node equals the op of its children, sampled indices follow the priorities."""
    from xuanpolicy_amd.per import PerOffPolicyBuffer
    n_envs, n_size, batch = 8, 131072, 2048
    buf = PerOffPolicyBuffer(_Box((1,)), _Disc(), {}, n_envs, n_size, batch, 0.6, device=DEV)
    cap = buf.capacity
    g = torch.Generator(device=DEV).manual_seed(0)
    leaves = torch.rand((n_envs, cap), generator=g, device=DEV, dtype=torch.float64) + 0.05
    buf.sum_tree[:, cap:] = leaves
    buf.min_tree[:, cap:] = leaves
    lvl = cap
    while lvl > 1:   # bulk build (test set-up only)
        half = lvl // 2
        buf.sum_tree[:, half:lvl] = buf.sum_tree[:, lvl:2 * lvl:2] + buf.sum_tree[:, lvl + 1:2 * lvl:2]
        buf.min_tree[:, half:lvl] = torch.minimum(buf.min_tree[:, lvl:2 * lvl:2], buf.min_tree[:, lvl + 1:2 * lvl:2])
        lvl = half
    buf.size = n_size
    for it in range(3):
        steps, flat, w = buf.sample_indices(0.5)
        st = steps.cpu().numpy()
        assert st.min() >= 0 and st.max() < n_size - 1 + 1
        assert np.isfinite(w.cpu().numpy()).all() and (w.cpu().numpy() >= 1 - 1e-12).all()
        assert np.array_equal(flat.cpu().numpy(), (np.arange(n_envs)[:, None] * n_size + st).reshape(-1))
        pr = torch.rand(batch, generator=g, device=DEV) * 4
        buf.update_priorities(steps, pr)
    s, m = buf.sum_tree, buf.min_tree
    kids_s = s[:, 2:2 * cap:2] + s[:, 3:2 * cap:2]
    kids_m = torch.minimum(m[:, 2:2 * cap:2], m[:, 3:2 * cap:2])
    assert torch.equal(s[:, 1:cap], kids_s) and torch.equal(m[:, 1:cap], kids_m)
    # stratified sampling follows the priorities: high-priority region drawn more often
    buf.sum_tree[:, cap:] = 1.0
    buf.sum_tree[:, cap:cap + 1024] = 100.0
    buf.min_tree[:, cap:] = 1.0
    lvl = cap
    while lvl > 1:
        half = lvl // 2
        buf.sum_tree[:, half:lvl] = buf.sum_tree[:, lvl:2 * lvl:2] + buf.sum_tree[:, lvl + 1:2 * lvl:2]
        buf.min_tree[:, half:lvl] = torch.minimum(buf.min_tree[:, lvl:2 * lvl:2], buf.min_tree[:, lvl + 1:2 * lvl:2])
        lvl = half
    steps, _, _ = buf.sample_indices(0.5)
    frac = (steps < 1024).double().mean().item()
    exp = 1024 * 100.0 / (1024 * 100.0 + (n_size - 1 - 1024))
    assert abs(frac - exp) < 0.01, (frac, exp)
