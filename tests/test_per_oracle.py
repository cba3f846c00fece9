"""K6 oracle (oracle/per_ref.py) pinned to the reference's PerOffPolicyBuffer / segment trees
(tests/golden/per.npz, G6): bitwise under this container's NumPy promotion (pinned=False), and
within f32 rounding of the leaves under the reference's pinned NumPy 1.21 f64 semantics
(pinned=True, what the HIP kernels implement)."""
import numpy as np
import pytest

from oracle.per_ref import PerBufferRef


def _replay(g, tag, pinned, check):
    n_envs, n_size, batch, cap = (int(v) for v in g[tag + "/config"])
    alpha, beta = (float(v) for v in g[tag + "/alpha_beta"])
    ref = PerBufferRef(n_envs, n_size, batch, alpha, obs_shape=(3,), pinned=pinned)
    assert ref.capacity == cap
    obs, act, rew, term, nxt = (g[tag + "/" + k] for k in ("obs", "act", "rew", "term", "next"))
    t = 0
    r = 0
    while tag + "/r%d/n_store" % r in g:
        pr = tag + "/r%d/" % r
        for _ in range(int(g[pr + "n_store"])):
            ref.store(obs[t], act[t], rew[t], term[t], nxt[t])
            t += 1
        check(pr + "tree_sum_after_store", ref.trees()[0])
        check(pr + "tree_min_after_store", ref.trees()[1])
        ob, ac, rw, te, nx, w, steps = ref.sample(beta, g[pr + "uniforms"])
        check(pr + "step_choices", steps, exact=True)
        check(pr + "weights", w)
        for k, v in (("obs", ob), ("act", ac), ("rew", rw), ("term", te), ("next", nx)):
            check(pr + k, v, exact=True)
        ref.update_priorities(steps.astype(np.int64), g[pr + "priorities"])
        check(pr + "tree_sum_after_update", ref.trees()[0])
        check(pr + "tree_min_after_update", ref.trees()[1])
        check(pr + "max_priority", ref.max_priority)
        assert (ref.size, ref.ptr) == tuple(g[pr + "size_ptr"])
        r += 1
    return r


@pytest.mark.parametrize("tag", ["small", "wrap"])
def test_per_oracle_bitwise_vs_reference(golden, tag):
    g = golden("per.npz")

    def check(key, got, exact=False):
        exp = g[key]
        got = np.asarray(got)
        assert got.shape == exp.shape, key
        assert np.array_equal(got.astype(exp.dtype), exp), key
    assert _replay(g, tag, pinned=False, check=check) >= 2


@pytest.mark.parametrize("tag", ["small", "wrap"])
def test_per_oracle_pinned_f64_vs_reference(golden, tag):
    g = golden("per.npz")

    def check(key, got, exact=False):
        exp = g[key]
        got = np.asarray(got)
        if exact:
            assert np.array_equal(got.astype(exp.dtype), exp), key
        else:   # NumPy 2 keeps updated leaves and their f32+f32 parents in float32 (<= 1e-6 rel)
            fin = np.isfinite(exp)
            assert np.array_equal(np.isfinite(got), fin), key
            np.testing.assert_allclose(got[fin], exp[fin], rtol=1e-6, atol=1e-12, err_msg=key)
    _replay(g, tag, pinned=True, check=check)


def test_per_wrap_fixture_documents_uint8_cast(golden):
    """n_size = 300 > 256: the reference's chosen steps wrap modulo 256 (memory_tools.py:465)."""
    g = golden("per.npz")
    ref = PerBufferRef(1, 300, 16, 0.5, obs_shape=(3,), wrap_uint8=False)
    obs, act, rew, term, nxt = (g["wrap/" + k] for k in ("obs", "act", "rew", "term", "next"))
    for t in range(int(g["wrap/r0/n_store"])):
        ref.store(obs[t], act[t], rew[t], term[t], nxt[t])
    steps, _ = ref.sample_indices(0.7, g["wrap/r0/uniforms"])
    assert steps.max() >= 256
    assert np.array_equal((steps % 256).astype(np.uint8), g["wrap/r0/step_choices"])
