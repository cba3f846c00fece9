"""G11 (CPU): the oracle's host-loop restatement against the reference's own train() over its own host VecEnvs.

tests/golden/make_golden.py (capture_vecloop, run in the build container where /root/reference imports) recorded
PPOCLIP_Agent.train / A2C_Agent.train (ppoclip_agent.py:59-111, a2c_agent.py:57-107) over DummyVecEnv_Gym,
DummyVecEnv_Atari and SubprocVecEnv_Gym (gym_vec_env.py:40-231) of SynthBox / SynthAtari envs, in several train()
calls.  Here oracle.cpu_ref.VecAgentRef over oracle.synth_env.DummyVecEnvRef (rebind=True for the Subproc contract)
replays the recorded actions with the reference's f32 weights (its post-update weights loaded at every full-buffer
point, so the fixture pins the loop itself; the learner is pinned by G3-G5) and must reproduce every stored column,
closure, bootstrap, advantage / return, the RunningMeanStd states and the return tracker.  These are the oracle
pieces tests/test_gpu_hostenv.py holds the device agent to."""
import os

import numpy as np
import pytest
import torch

from oracle import cpu_ref
from oracle.synth_env import DummyVecEnvRef, SynthAtariEnv, SynthBoxEnv, _Box, _Discrete

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["ppo_gauss_norm", "ppo_gauss_raw", "a2c_cat_norm", "ppo_gauss_raw_subproc", "atari_a2c"]
ATARI_NET = dict(filters=[8, 8], kernels=[8, 4], strides=[4, 2], fc=[16])   # make_golden.VEC_ATARI_NET


def _load(name):
    return dict(np.load(os.path.join(HERE, "vecloop_%s.npz" % name)))


def _setup(name, g):
    N, T, D, A, max_ep, obsnorm, discrete, seed = (int(v) for v in g["config"][:8])
    atari = name.startswith("atari")
    if atari:
        envs = DummyVecEnvRef([SynthAtariEnv(i, seed=seed, n_actions=A, max_episode_steps=max_ep) for i in range(N)],
                              _Box(0, 255, (84, 84, 4)), _Discrete(A), atari=True)
        pol = cpu_ref.build_atari_ac_ref(A, ATARI_NET["filters"], ATARI_NET["kernels"], ATARI_NET["strides"],
                                         ATARI_NET["fc"])
    else:
        envs = DummyVecEnvRef([SynthBoxEnv(D, A, seed=seed, env_index=i, discrete=bool(discrete),
                                           max_episode_steps=max_ep) for i in range(N)],
                              rebind=name.endswith("subproc"))
        pol = cpu_ref.build_actor_critic_ref(D, A, [64], [64], [64], discrete=bool(discrete))
    return envs, pol, atari, bool(obsnorm), bool(discrete), N, T


def _load_sd(pol, g, prefix, k=None):
    # by state_dict order (the CNN oracle names its critic head critic_head.*, the reference critic.model.*)
    src = [key for key in g if key.startswith(prefix)]
    keys = list(pol.state_dict().keys())
    assert len(src) == len(keys)
    pol.load_state_dict({dst: torch.as_tensor(g[key] if k is None else g[key][k]) for dst, key in zip(keys, src)})


def _close(a, b, what, rtol=0.0, atol=0.0):
    np.testing.assert_allclose(np.asarray(a, np.float64), np.asarray(b, np.float64), rtol=rtol, atol=atol, err_msg=what)


@pytest.mark.parametrize("name", CASES)
def test_oracle_host_loop_reproduces_reference_train(name):
    g = _load(name)
    envs, pol, atari, obsnorm, discrete, N, T = _setup(name, g)
    _load_sd(pol, g, "sd0/")
    pol.float()
    envs.reset()
    acts = g["env_actions"]
    feed = {"k": 0}

    def action_source(_obs):
        a = acts[feed["k"]]
        feed["k"] += 1
        return a
    seen = {"k": 0}
    # tolerances: the oracle runs the reference's arithmetic in the same f32 / f64 types, so values agree to the last
    # few ulps (torch CPU kernels may pick other reduction orders across builds); the buffer's discrete columns exactly
    tol = dict(rtol=2e-6, atol=2e-6)

    def on_full(ref):
        k = seen["k"]
        mem = ref.memory
        msg = "%s iteration %d " % (name, k)
        if atari:
            np.testing.assert_array_equal(mem.observations.reshape(N, T, -1).astype(np.int64).sum(-1),
                                          g["it/frame_sum"][k], err_msg=msg + "frames")
        else:
            _close(mem.observations, g["it/obs"][k], msg + "obs", **tol)
        np.testing.assert_array_equal(mem.actions, g["it/act"][k], err_msg=msg + "actions")
        np.testing.assert_array_equal(mem.terminals, g["it/term"][k], err_msg=msg + "terminals")
        np.testing.assert_array_equal(mem.closed, g["closed"][k], err_msg=msg + "closures")
        _close(mem.rewards, g["it/rew"][k], msg + "rewards", **tol)
        _close(mem.values, g["it/val"][k], msg + "values", **tol)
        _close(mem.boot, g["boot"][k], msg + "bootstraps", **tol)
        if "old_logp" in mem.auxiliary_infos:
            _close(mem.auxiliary_infos["old_logp"], g["it/logp"][k], msg + "old_logp", **tol)
        _close(mem.advantages, g["it/adv"][k], msg + "advantages", rtol=1e-5, atol=1e-5)
        _close(mem.returns, g["it/ret"][k], msg + "returns", rtol=1e-5, atol=1e-5)
        _check_rms(ref, g, "it/", k, msg)
        _load_sd(pol, g, "it/sd/", k)   # the reference's weights after this iteration's updates
        pol.float()
        seen["k"] += 1

    ref = cpu_ref.VecAgentRef(envs, pol, "ppo" if name.startswith("ppo") else "a2c", T, action_source, on_full=on_full,
                              use_obsnorm=obsnorm, use_rewnorm=obsnorm, atari=atari, discrete=discrete)
    for k in g["calls"]:
        ref.train(int(k))
    assert seen["k"] == g["it/act"].shape[0] and feed["k"] == acts.shape[0]
    _check_rms(ref, g, "end/", None, name + " end ")
    # the case must exercise what it is there for
    term, closed = g["it/term"], g["closed"]
    if atari:
        assert int(((term != 0) & (closed == 0)).sum()) > 0, "life losses that keep the path open"
    else:
        assert int(((closed[:, :, :T - 1] != 0) & (term[:, :, :T - 1] == 0)).sum()) >= N, "mid-rollout truncations"


def _check_rms(ref, g, p, k, msg):
    def v(key):
        return g[p + key] if k is None else g[p + key][k]
    if ref.use_obsnorm:
        _close(ref.obs_rms.mean, v("obs_mean"), msg + "obs_rms.mean", rtol=1e-12, atol=1e-12)
        _close(ref.obs_rms.var, v("obs_var"), msg + "obs_rms.var", rtol=1e-12, atol=1e-12)
        _close(ref.obs_rms.count, v("obs_count"), msg + "obs_rms.count")
    _close(ref.ret_rms.mean, v("ret_mean"), msg + "ret_rms.mean", rtol=1e-6, atol=1e-7)
    _close(ref.ret_rms.var, v("ret_var"), msg + "ret_rms.var", rtol=1e-6, atol=1e-7)
    _close(ref.ret_rms.count, v("ret_count"), msg + "ret_rms.count")
    _close(ref.returns, v("returns"), msg + "returns tracker", rtol=1e-6, atol=1e-6)


def test_subproc_contract_differs_from_dummy_only_by_the_alias():
    """Same envs, actions and weights: the reference's SubprocVecEnv_Gym run stores the PRE-step observations on each
    train() call's first step (buf_obs is rebound), DummyVecEnv_Gym's the post-step ones (written in place).  (The
    second iteration differs throughout: its weights were trained on different first columns.)"""
    a, b = _load("ppo_gauss_raw"), _load("ppo_gauss_raw_subproc")
    T = int(a["config"][1])
    np.testing.assert_array_equal(a["env_actions"][:T], b["env_actions"][:T])
    first_cols = [0, 5, 10]   # calls (5, 5, 6) in iteration 0
    diff = np.abs(a["it/obs"][0] - b["it/obs"][0]).max(axis=(0, 2))
    assert all(diff[c] > 0 for c in first_cols)
    assert np.all(diff[[c for c in range(16) if c not in first_cols]] == 0)
