"""GPU: C1 (BASELINE.json configs[0]) — PPO-Clip on CartPole-v1, 8 envs x 128 steps, [64] nets.

  * K18 (xpa_cartpole_step) against the oracle's restatement of gym 0.26.2's CartPoleEnv + TimeLimit
    (oracle/synth_env.CartPoleEnv): every step's observation, reward, terminated / truncated flag and auto-reset
    state, through the VecEnv contract (gym_vec_env.py:201-212).  Parity against gym itself is unpinned (gym is
    not installed and the reference holds no recorded CartPole trajectories).
  * one PPO iteration on device (K3 sampling into the buffer, K8, deferred bootstraps, K1 GAE, K4 / K2 / K9
    updates) replayed through the CPU oracle learner (tests/_oracle_replay.py)."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref
from tests._oracle_replay import replay_last_step_iteration

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cpu_ref.build_oracle()


def test_cartpole_env_matches_oracle():
    from oracle.synth_env import CartPoleEnv
    from xuanpolicy_amd.envs import CartPoleVecEnv
    N, steps, max_ep = 37, 700, 60
    env = CartPoleVecEnv(N, seed=5, max_episode_steps=max_ep, device=DEV)
    ref = [CartPoleEnv(i, seed=5, max_episode_steps=max_ep) for i in range(N)]
    np.testing.assert_array_equal(env.obs.cpu().numpy(), np.stack([r.reset()[0] for r in ref]))
    rng = np.random.default_rng(1)
    n_term = n_trunc = 0
    for t in range(steps):
        a = rng.integers(0, 2, N)
        obs, rew, term, trunc, infos = env.step(a)
        for i, r in enumerate(ref):
            o, rw, te, tr, info = r.step(a[i])
            np.testing.assert_allclose(obs[i], o, rtol=1e-6, atol=1e-7)
            assert rw == rew[i] == 1.0 and te == term[i] and tr == trunc[i], (t, i)
            assert info["episode_step"] == infos[i]["episode_step"]
            if te or tr:
                np.testing.assert_array_equal(infos[i]["reset_obs"], r.reset()[0])   # hashed reset: exact
                assert info["episode_score"] == infos[i]["episode_score"]
            n_term += int(te)
            n_trunc += int(tr)
        # keep the checker on the device's f64 state (sin / cos may differ in the last ulp between libm and ocml)
        st = env.state.cpu().numpy()
        for i, r in enumerate(ref):
            np.testing.assert_allclose(r.state, st[i], rtol=1e-12, atol=1e-14)
            r.state = st[i].copy()
    assert n_term > 0 and n_trunc > 0


def test_ppo_cartpole_iteration_matches_oracle():
    from xuanpolicy_amd.runner import build_cartpole_ppo
    N, T, H = 8, 128, 64
    n_epoch, n_mb = 4, 4
    agent = build_cartpole_ppo(n_envs=N, n_steps=T, hidden=H, seed=3, device=DEV, n_epoch=n_epoch, n_minibatch=n_mb,
                               max_episode_steps=T + 9)
    assert agent.device_env and agent.defer_boot and agent.config.gamma == 0.98
    agent.train(T, log=False)
    agent.train(T - 1, log=False)
    replay_last_step_iteration(agent, 4, 2, [H], True, "ppo", agent.config.ent_coef, n_epoch, n_mb)


def test_graphed_updates_match_eager():
    """learners._graphed_mlp_update: the per-slot hipGraph replays give the eager update's parameters (two iterations,
    8 epochs x 8 slots: warm-up, capture + replay, and replays)."""
    from xuanpolicy_amd.runner import build_cartpole_ppo
    out = []
    for graphed in (False, True):
        agent = build_cartpole_ppo(n_envs=8, n_steps=128, hidden=64, seed=4, device=DEV, graph_update=graphed)
        for _ in range(2):
            agent.train(128, log=False)
        torch.cuda.synchronize()
        graphs = getattr(agent.learner, "_slot_graphs", {})
        n_graphs = sum(isinstance(v, tuple) for v in graphs.values())
        assert (n_graphs == 8) if graphed else (n_graphs == 0), n_graphs
        assert not getattr(agent.learner, "_graph_failed", False)
        out.append([p.detach().cpu().numpy().copy() for p in agent.policy.parameters()])
    for a, b in zip(*out):
        np.testing.assert_allclose(b, a, rtol=1e-6, atol=1e-7)
