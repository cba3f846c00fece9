"""GPU: the agent over a HOST VecEnv (north_star's DummyVecEnv/SubprocVecEnv producer) against the reference loop.

`_OnPolicyAgent._rollout_step_host` (xuanpolicy_amd/agents.py) drives a numpy VecEnv with the reference's step
contract (gym_vec_env.py:148-231, restated as oracle.synth_env.DummyVecEnvRef) through the device kernels, with
per-step H2D / D2H copies.  oracle.cpu_ref.VecAgentRef runs the reference's train() loop step for step
(ppoclip_agent.py:59-111, a2c_agent.py:57-107, agent.py:104-123) on an identical env fed the actions the device
drew, with an f64 copy of the device policy.  Checked, per iteration:

  * the whole rollout buffer: stored (normalised) observations, actions, normalised rewards, values, old
    log-probs, terminals, path closures and their bootstrap values, advantages / returns of the reference's own
    finish_path calls; the obs / return RunningMeanStd state;
  * the loop's quirks: train() restarting from envs.buf_obs (stale final rows of envs that ended on the previous
    call's last step), the first-store alias of buf_obs without obs-norm, reset_obs continuation, A2C's
    V(norm(reset_obs)) truncation bootstrap, and with env_name "Atari" a life loss (terminal, not truncated) that
    keeps the path and the frames (ppoclip_agent.py:93-94);
  * the last iteration through tests/_oracle_replay: GAE of the device buffer at 1e-5 (north_star), every update's
    loss scalars at 1e-4 with the device permutations, the final weights.
"""
import numpy as np
import pytest
import torch

from oracle import cpu_ref
from oracle.synth_env import DummyVecEnvRef, SynthAtariEnv, SynthBoxEnv, _Box, _Discrete
from tests._oracle_replay import _load_by_order, replay_last_step_iteration
from tests.test_gpu_kernels import _gae_close as _gae_close_kernels


def _gae_close(got, ref, msg):
    try:
        _gae_close_kernels(got, ref)
    except AssertionError as e:
        raise AssertionError(msg + ": " + str(e)) from None

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cpu_ref.build_oracle()


def _snapshot(mem):
    out = {k: np.array(getattr(mem, k), copy=True) for k in ("observations", "actions", "rewards", "values", "terminals",
                                                              "closed", "boot", "advantages", "returns")}
    out["old_logp"] = np.array(mem.auxiliary_infos["old_logp"], copy=True) if "old_logp" in mem.auxiliary_infos else None
    return out


def _check_rollout(agent, ref, snap, it):
    """The device buffer of one iteration against the reference loop's buffer at its full-buffer point."""
    mem = agent.memory
    msg = "iteration %d " % it
    obs = mem.observations.cpu().numpy()
    if obs.dtype == np.uint8:
        np.testing.assert_array_equal(obs, snap["observations"], err_msg=msg + "frames")
    else:
        np.testing.assert_allclose(obs, snap["observations"], rtol=1e-5, atol=1e-5, err_msg=msg + "obs")
    np.testing.assert_array_equal(mem.actions.cpu().numpy(), snap["actions"], err_msg=msg + "actions")
    np.testing.assert_array_equal(mem.terminals.cpu().numpy(), snap["terminals"], err_msg=msg + "terminals")
    np.testing.assert_array_equal(mem.closed.cpu().numpy(), snap["closed"], err_msg=msg + "closures")
    np.testing.assert_allclose(mem.rewards.cpu().numpy(), snap["rewards"], rtol=1e-5, atol=1e-6, err_msg=msg + "rew")
    np.testing.assert_allclose(mem.values.cpu().numpy(), snap["values"], rtol=1e-4, atol=1e-4, err_msg=msg + "values")
    np.testing.assert_allclose(mem.boot.cpu().numpy(), snap["boot"], rtol=1e-4, atol=1e-4, err_msg=msg + "bootstraps")
    if snap["old_logp"] is not None:
        np.testing.assert_allclose(mem.auxiliary_infos["old_logp"].cpu().numpy(), snap["old_logp"], rtol=1e-4, atol=2e-4,
                                   err_msg=msg + "old_logp")
    # (1) the device's GAE of its own columns: the oracle's finish_path arithmetic at north_star's 1e-5
    cols = [getattr(mem, k).cpu().numpy() for k in ("rewards", "values", "terminals", "closed", "boot")]
    adv_d, ret_d = mem.advantages.cpu().numpy(), mem.returns.cpu().numpy()
    adv_o, ret_o = cpu_ref.gae_rows(*cols, mem.gamma, mem.gae_lam)
    _gae_close(adv_d, adv_o, msg + "adv (device columns)")
    _gae_close(ret_d, ret_o, msg + "ret (device columns)")
    # (2) against the reference loop's own finish_path results: the columns differ by the f32-vs-f64 rounding held
    # above (values / bootstraps 1e-4, rewards 1e-5), and a discounted sum of such differences is bounded by the
    # measured column differences propagated through the scan: |d adv| <= (|d r| + (1 + gamma) |d v| + gamma |d boot|)
    # / (1 - gamma lambda) — an envelope measured on the case, not a blanket tolerance
    g, lam = float(mem.gamma), float(mem.gae_lam)
    dr = np.abs(cols[0] - snap["rewards"]).max()
    dv = np.abs(cols[1] - snap["values"]).max()
    db = np.abs(cols[4] - snap["boot"]).max()
    env_adv = (dr + (1 + g) * dv + g * db) / (1 - g * lam) + 1e-6
    np.testing.assert_allclose(adv_d, snap["advantages"], rtol=0, atol=env_adv, err_msg=msg + "adv (reference loop)")
    np.testing.assert_allclose(ret_d, snap["returns"], rtol=0, atol=env_adv + dv, err_msg=msg + "ret (reference loop)")
    assert env_adv < 2e-3, (msg, "envelope", env_adv)
    if agent.use_obsnorm:
        np.testing.assert_allclose(agent.obs_mean.cpu().numpy(), ref.obs_rms.mean, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(agent.obs_var.cpu().numpy(), ref.obs_rms.var, rtol=1e-5, atol=1e-6)
        assert abs(float(agent.obs_count) - ref.obs_rms.count) < 1e-6
    np.testing.assert_allclose(float(agent.ret_mean), float(ref.ret_rms.mean), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(float(agent.ret_var), float(ref.ret_rms.var), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(agent.returns.cpu().numpy(), ref.returns, rtol=1e-5, atol=1e-5)


def _run(agent, host, ref_env, pol, algo, discrete, A, ent, n_epoch, n_mb, atari, first_calls):
    """Two iterations: the first split into train() calls of `first_calls` steps, the second's last step through
    the update replay; the reference loop makes the same calls."""
    N, T = agent.n_envs, agent.n_steps
    cfg = agent.config
    feed = {"k": 0}

    def action_source(_obs):
        a = host.actions[feed["k"]]
        feed["k"] += 1
        return a
    snaps = []
    ref = cpu_ref.VecAgentRef(ref_env, pol, algo, T, action_source, on_full=lambda r: snaps.append(_snapshot(r.memory)),
                              gamma=cfg.gamma, gae_lambda=cfg.gae_lambda, use_obsnorm=agent.use_obsnorm,
                              use_rewnorm=agent.use_rewnorm, obsnorm_range=cfg.obsnorm_range,
                              rewnorm_range=cfg.rewnorm_range, atari=atari, discrete=discrete)
    _load_by_order(pol, agent)
    pol.double()
    assert sum(first_calls) == T
    for k in first_calls:
        agent.train(k, log=False)
        ref.train(k)
    torch.cuda.synchronize()
    assert len(snaps) == 1
    _check_rollout(agent, ref, snaps[0], 0)
    # iteration 2 from the device's updated weights; its last step runs inside the update replay
    _load_by_order(pol, agent)
    pol.double()
    agent.train(T - 1, log=False)
    ref.train(T - 1)
    # without obs-norm the first store of each train() call (columns 0 and T - 1 here) aliases the post-step buf_obs
    alias = (0, T - 1) if not agent.use_obsnorm and not getattr(host, "rebind", False) else ()
    replay_last_step_iteration(agent, None, A, None, discrete, algo, ent, n_epoch, n_mb,
                               pol=_fresh_like(pol), alias_cols=alias)
    ref.train(1)
    assert len(snaps) == 2 and feed["k"] == 2 * T
    _check_rollout(agent, ref, snaps[1], 1)
    return snaps


def _fresh_like(pol):
    import copy
    return copy.deepcopy(pol)


def _synthbox_agent(agent_name, discrete, A, obsnorm, N, T, max_ep, seed=5, rebind=False):
    import xuanpolicy_amd.runner as R
    D = 17
    method = "ppo" if agent_name == "PPO_Clip" else "a2c"

    def envs():
        e = DummyVecEnvRef([SynthBoxEnv(D, A, seed=seed, env_index=i, discrete=discrete, max_episode_steps=max_ep)
                            for i in range(N)], rebind=rebind)
        e.reset()
        return e
    cfg = R.get_arguments(method, "synthbox", "SynthBox-v0")
    cfg.agent, cfg.parallels, cfg.n_steps, cfg.n_epoch, cfg.n_minibatch = agent_name, N, T, 2, 4
    cfg.obs_dim, cfg.act_dim, cfg.discrete, cfg.seed = D, A, discrete, seed
    cfg.policy = "Categorical_AC" if discrete else "Gaussian_AC"
    cfg.representation_hidden_size = cfg.actor_hidden_size = cfg.critic_hidden_size = [64]
    cfg.use_obsnorm = cfg.use_rewnorm = obsnorm
    cfg.ent_coef = 0.01
    torch.manual_seed(seed)
    host = envs()
    agent = R.build_agent(cfg, DEV, envs=host)
    return agent, host, envs(), D


@pytest.mark.parametrize("agent_name,discrete,A,obsnorm,rebind", [
    ("PPO_Clip", False, 6, True, False),     # the mujoco.yaml flags: obs / reward normalisation
    ("A2C", True, 4, True, False),           # V(norm(reset_obs)) truncation bootstraps
    ("PPO_Clip", False, 6, False, False),    # no obs-norm: the first-store alias of buf_obs on every train() call
    ("PPO_Clip", False, 6, False, True),     # SubprocVecEnv_Gym's contract: buf_obs rebound, so no alias; f64
                                             # rewards; reset_obs of shape (1, D) (gym_vec_env.py:89-121)
    ("A2C", True, 4, True, True),
])
def test_host_vecenv_agent_matches_reference_loop(agent_name, discrete, A, obsnorm, rebind):
    """The oracle loop (VecAgentRef over DummyVecEnvRef, rebind=False / True) is pinned against the reference's own
    train() over DummyVecEnv_Gym / SubprocVecEnv_Gym by G11 (tests/test_vecloop_golden_cpu.py)."""
    N, T, max_ep = 16, 16, 5
    agent, host, ref_env, D = _synthbox_agent(agent_name, discrete, A, obsnorm, N, T, max_ep, rebind=rebind)
    assert not agent.device_env and not agent.defer_boot
    algo = "ppo" if agent_name == "PPO_Clip" else "a2c"
    assert agent.boot_from_reset == (algo == "a2c")
    pol = cpu_ref.build_actor_critic_ref(D, A, [64], [64], [64], discrete=discrete,
                                         activation=getattr(agent.config, "activation", "LeakyReLU"))
    # train() calls of 5 + 5 + 6 steps: every call boundary falls on a step where envs ended (max_episode_steps 5)
    snaps = _run(agent, host, ref_env, pol, algo, discrete, A, 0.01, 2, 4, False, (5, 5, 6))
    for s in snaps:   # the cases must exercise mid-rollout truncations and their bootstraps
        mid = (s["closed"][:, :T - 1] != 0) & (s["terminals"][:, :T - 1] == 0)
        assert mid.sum() >= N and np.abs(s["boot"][:, :T - 1][mid]).min() > 0


def test_host_vecenv_a2c_bootstrap_is_reset_obs_value():
    """A2C's truncation bootstrap differs from PPO's: with the flag off (a2c_reset_bootstrap False) the device agent
    bootstraps from the final observation and the buffer no longer matches the reference loop's."""
    N, T = 16, 16
    agent, host, ref_env, D = _synthbox_agent("A2C", True, 4, True, N, T, 5)
    agent.boot_from_reset = False
    pol = cpu_ref.build_actor_critic_ref(D, 4, [64], [64], [64], discrete=True,
                                         activation=getattr(agent.config, "activation", "LeakyReLU"))
    _load_by_order(pol, agent)
    pol.double()
    snaps = []
    feed = {"k": 0}

    def src(_o):
        feed["k"] += 1
        return host.actions[feed["k"] - 1]
    cfg = agent.config
    ref = cpu_ref.VecAgentRef(ref_env, pol, "a2c", T, src, on_full=lambda r: snaps.append(_snapshot(r.memory)),
                              gamma=cfg.gamma, gae_lambda=cfg.gae_lambda, discrete=True)
    agent.train(T, log=False)
    ref.train(T)
    boot = agent.memory.boot.cpu().numpy()
    mid = (snaps[0]["closed"][:, :T - 1] != 0) & (snaps[0]["terminals"][:, :T - 1] == 0)
    assert mid.sum() > 0 and np.abs(boot[:, :T - 1][mid] - snaps[0]["boot"][:, :T - 1][mid]).max() > 1e-3


def test_host_vecenv_atari_a2c_matches_reference_loop():
    """env_name "Atari" over a host DummyVecEnv_Atari of SynthAtari envs (uint8 frame stacks, life losses = terminal
    without truncation, game overs = terminal + truncated): raw frames stored, the small AC_CNN_Atari on the explicit
    CNN path, no obs-norm (so every train() call's first column is the post-step buf_obs, as G8 records)."""
    import xuanpolicy_amd.runner as R
    N, T, K, max_ep, seed = 8, 32, 6, 40, 3
    net = dict(filters=[8, 8], kernels=[8, 4], strides=[4, 2], fc=[32])

    def envs():
        e = DummyVecEnvRef([SynthAtariEnv(i, seed=seed, n_actions=K, max_episode_steps=max_ep) for i in range(N)],
                           _Box(0, 255, (84, 84, 4)), _Discrete(K), atari=True)
        e.reset()
        return e
    cfg = R.get_arguments("a2c", "atari", "SynthAtari-v0")
    cfg.parallels, cfg.n_steps, cfg.n_epoch, cfg.n_minibatch, cfg.seed = N, T, 2, 4, seed
    cfg.filters, cfg.kernels, cfg.strides, cfg.fc_hidden_sizes = net["filters"], net["kernels"], net["strides"], net["fc"]
    torch.manual_seed(seed)
    host = envs()
    agent = R.build_agent(cfg, DEV, envs=host)
    assert agent.raw_obs and agent.atari and not agent.device_env
    pol = cpu_ref.build_atari_ac_ref(K, net["filters"], net["kernels"], net["strides"], net["fc"])
    snaps = _run(agent, host, envs(), pol, "a2c", True, K, cfg.ent_coef, 2, 4, True, (17, 15))
    lifeloss = sum(int(((s["terminals"] != 0) & (s["closed"] == 0)).sum()) for s in snaps)
    assert lifeloss > 0, "the case must exercise life losses that keep the path open"
