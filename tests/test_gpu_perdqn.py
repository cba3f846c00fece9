"""GPU: C5 (BASELINE.json configs[4]) — PER-DQN on device.

  * K19 (xpa_dqn_td_loss) against the oracle's closed form (oracle/cpu_ref.dqn_td_ref, perdqn_learner.py:23-30);
  * G9: the reference's PerDQN_Learner.update (4 updates, target copies every 2) replayed through the device
    PerDQN_Learner (BasicQnetwork over Basic_CNN on MIOpen / hipBLASLt + K19): |TD|, info, parameters;
  * the device PerDQN_Agent loop (K15 SynthAtari env with 18 actions, K6 store / sample / priority update,
    K4 uint8 frame gathers) runs and keeps its trees consistent."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _close(got, ref, rtol, atol, msg=""):
    """assert_allclose with an elementwise atol array."""
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    bad = ~(np.abs(got - ref) <= np.asarray(atol) + rtol * np.abs(ref))
    assert not bad.any(), "%s: got %s ref %s atol %s" % (msg, got[bad], ref[bad], np.broadcast_to(atol, got.shape)[bad])


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("B,A", [(2048, 18), (3, 2), (1500, 7)])
def test_dqn_td_kernel_matches_oracle(B, A):
    from xuanpolicy_amd import ops
    rng = np.random.default_rng(B + A)
    eq = rng.normal(0, 1, (B, A)).astype(np.float32)
    tq = rng.normal(0, 1, (B, A)).astype(np.float32)
    tq[::5, 0] = tq[::5].max(1)        # ties in the max
    act = rng.integers(0, A, B).astype(np.float32)
    rew = rng.normal(0, 1, B).astype(np.float32)
    term = (rng.random(B) < 0.3).astype(np.float32)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    dq, td, sc = ops.dqn_td_loss(torch.as_tensor(eq, device=DEV), torch.as_tensor(tq, device=DEV),
                                 torch.as_tensor(act, device=DEV), torch.as_tensor(rew, device=DEV),
                                 torch.as_tensor(term, device=DEV), 0.99, err=err)
    loss, rtd, rdq, pq = cpu_ref.dqn_td_ref(eq, tq, act, rew, term, 0.99)
    np.testing.assert_array_equal(td.cpu().numpy(), rtd)            # f32 element ops in the same order: exact
    np.testing.assert_allclose(dq.cpu().numpy(), rdq, rtol=1e-6, atol=0)
    s = sc.cpu().numpy()
    assert abs(s[0] - loss) <= 1e-6 * max(1.0, loss) and abs(s[1] - pq) <= 1e-6 * max(1.0, abs(pq))
    assert int(err) == 0
    bad = torch.as_tensor(act, device=DEV).clone()
    bad[0], bad[1] = -1.0, float(A)                                 # out of range: clamped and counted
    ops.dqn_td_loss(torch.as_tensor(eq, device=DEV), torch.as_tensor(tq, device=DEV), bad,
                    torch.as_tensor(rew, device=DEV), torch.as_tensor(term, device=DEV), 0.99, err=err)
    assert int(err) == 2


def _perdqn_batch(seed, k, B, A):
    rng = np.random.default_rng(seed * 1000 + k)
    obs = rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)
    nxt = rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)
    act = rng.integers(0, A, B).astype(np.float32)
    rew = rng.normal(0, 1, B).astype(np.float32)
    term = (rng.random(B) < 0.2).astype(np.float32)
    return obs, act, rew, nxt, term


@pytest.mark.parametrize("fixture", ["perdqn.npz", "perdqn_prod.npz"])
def test_perdqn_learner_replays_reference(golden, fixture, conv_path):
    """G9 / G9P: the reference's PerDQN_Learner updates replayed.  perdqn_prod.npz is the production Basic_CNN
    ([32, 64, 64] / [8, 4, 3] / [4, 2, 1] + q 512) at the C5 batch of 2048: K25 conv1 from the uint8 frames, K23 / K24
    max pool, K26 / K27 in the backward, K19."""
    from xuanpolicy_amd.learners import PerDQN_Learner
    from xuanpolicy_amd.policies import BasicQnetwork, Basic_CNN
    g = golden(fixture)
    # G9P: per-update envelopes of the exact f64 replay's distance from the f32 reference (make_envelopes.py); the
    # tolerances are max(base, 3 x envelope), so update 0 is held to the base tolerances
    env = golden(fixture.replace(".npz", "_env.npz")) if fixture != "perdqn.npz" else None
    B, A, n_up, seed, sync = (int(x) for x in g["config"])
    net = [int(x) for x in g["net"]]
    nl = (len(net) - 1) // 3

    class Disc:
        n, shape = A, ()
    rep = Basic_CNN((84, 84, 4), net[nl:2 * nl], net[2 * nl:3 * nl], net[:nl], None, None, torch.nn.ReLU, DEV)
    pol = BasicQnetwork(Disc(), rep, net[3 * nl:], None, None, torch.nn.ReLU, DEV)
    pol.load_state_dict({k[4:]: torch.as_tensor(v) for k, v in g.items() if k.startswith("sd0/")})
    opt = torch.optim.Adam(pol.parameters(), 1e-3, eps=1e-5)
    sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.5, total_iters=10)
    lrn = PerDQN_Learner(pol, opt, sch, DEV, "./", float(g["gamma"]), sync)
    fq = lrn._fused_q()
    assert fq is not None
    if net[:2] == [32, 64]:
        assert fq.eval_trunk.u8_conv1 and fq.eval_trunk._dgrad_ok(fq.eval_trunk.convs[1][0])
    for k in range(n_up):
        obs, act, rew, nxt, term = _perdqn_batch(seed, k, B, A)
        td, info = lrn.update(torch.as_tensor(obs, device=DEV), act, rew, torch.as_tensor(nxt, device=DEV), term)
        assert td.device.type == "cuda" and td.dtype == torch.float32
        td_tol = max(1e-5, 3 * float(env["td"][k])) if env is not None else 1e-5
        info_tol = np.maximum(1e-6, 3 * env["info"][k]) if env is not None else 1e-6
        np.testing.assert_allclose(td.cpu().numpy(), g["td_abs"][k], rtol=1e-4, atol=td_tol, err_msg="update %d" % k)
        _close([info["Qloss"], info["learning_rate"], info["predictQ"]], g["infos"][k], 1e-4, info_tol,
               "update %d" % k)
        for key, v in pol.state_dict().items():
            if "sd%d/%s" % (k + 1, key) in g:
                tol = max(1e-5, 3 * float(env["sd/" + key])) if env is not None else 1e-5
                np.testing.assert_allclose(v.cpu().numpy(), g["sd%d/%s" % (k + 1, key)], rtol=1e-3, atol=tol,
                                           err_msg=key)
    assert all(("sd%d/%s" % (n_up, key)) in g for key in pol.state_dict())


@pytest.mark.parametrize("filters", [[8, 8], [32, 64]])
def test_perdqn_agent_loop_on_device(filters, conv_path):
    """[8, 8]: the r02 intermittent-fault configuration (4 / 8-channel convs), which since r03 runs K28 / K29 for every
    conv — the small-channel MIOpen route it faulted on is refused (fused_cnn._library_conv_guard, tested below);
    [32, 64]: the production first two convs (K25 / K26 / K27; conv2's weight gradient on K29 or MIOpen per
    conv_path).  Every device error word stays 0."""
    from xuanpolicy_amd.runner import build_perdqn
    agent = build_perdqn(n_envs=4, n_size=256, batch_size=64, device=DEV, start_training=64, sync_frequency=20,
                         filters=filters, kernels=[8, 4], strides=[4, 2], q_hidden_size=[32], max_episode_steps=40)
    assert agent.device_env and agent.memory.observations.dtype == torch.uint8
    assert agent.envs.action_space.n == 18
    agent.train(80, sync_info=True)
    torch.cuda.synchronize()
    assert agent.check_errors() == {"per_sample": 0, "gather": 0, "env": 0, "td_action": 0, "maxpool": 0}
    assert agent.memory.size == 80 and len(agent.infos) > 0
    for info in agent.infos:
        assert np.isfinite([info["Qloss"], info["predictQ"]]).all()
    assert agent.learner.iterations == len(agent.infos)
    # the sum tree's root equals the sum of its leaves (p_i^alpha of every stored transition), every env
    cap = agent.memory.capacity
    st = agent.memory.sum_tree.cpu().numpy()
    np.testing.assert_allclose(st[:, 1], st[:, cap:].sum(1), rtol=1e-12)
    assert (st[:, cap:cap + 80] > 0).all() and (st[:, cap + 80:] == 0).all()
    assert 0.4 < agent.PER_beta <= 1.0 and agent.egreedy < agent.start_greedy


def test_perdqn_agent_train_replays_reference(golden, conv_path):
    """G10: the reference's PerDQN_Agent.train (perdqn_agent.py:56-95) replayed through the device agent — SynthAtari
    device envs (18 actions), the production Basic_CNN + q 512, PER buffer with K6 store / sample / priority update, K4
    frame gathers, PerDQN_Learner (K25 / K23 / K19 / K24 / K26 / K27 + MIOpen / hipBLASLt), target copies every 5
    updates.  np.random is set to the recorded MT19937 state, so the e-greedy coins and random actions are the
    reference's; each PER sample takes the recorded random.random() uniforms.  Checked: every env action, every
    update's sampled steps, |TD| priorities and info dict, the beta / epsilon schedules, the final sum / min trees,
    max priorities and weights (eval and target)."""
    from xuanpolicy_amd.runner import build_perdqn
    g = golden("perdqn_agent.npz")
    N, n_size, batch, A, steps, seed, max_ep, start, sync, decay = (int(x) for x in g["config"])
    eps0, eps1, beta0, alpha, gamma, lr, lr_end = (float(x) for x in g["hyper"])
    net = [int(x) for x in g["net"]]
    nl = (len(net) - 1) // 3
    agent = build_perdqn(n_envs=N, n_size=n_size, batch_size=batch, seed=seed, device=DEV, start_training=start,
                         sync_frequency=sync, decay_step_greedy=decay, PER_alpha=alpha, PER_beta0=beta0,
                         start_greedy=eps0, end_greedy=eps1, training_frequency=1, gamma=gamma, learning_rate=lr,
                         max_episode_steps=max_ep, filters=net[:nl], kernels=net[nl:2 * nl], strides=net[2 * nl:3 * nl],
                         q_hidden_size=net[3 * nl:])
    assert agent.device_env and agent.envs.action_space.n == A and agent.alias_first_obs
    agent.policy.load_state_dict({k[4:]: torch.as_tensor(v) for k, v in g.items() if k.startswith("sd0/")})
    opt = agent.learner.optimizer
    agent.learner.scheduler = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=lr_end,
                                                                total_iters=100)
    fq = agent.learner._fused_q()
    assert fq is not None and fq.eval_trunk.u8_conv1
    # recorded draws: the MT19937 state before train(), the PER uniforms of every sample
    np.random.set_state(("MT19937", g["np_state_keys"], int(g["np_state_pos"][0]), int(g["np_state_pos"][1]),
                         float(g["np_state_gauss"])))
    uni = iter(g["upd_uniforms"])
    agent.uniform_source = lambda: next(uni)
    acts, samples, betas = [], [], []
    real_step, real_sample = agent._env_step, agent.memory.sample

    def env_step(a):
        acts.append(a.cpu().numpy().astype(np.int64))
        return real_step(a)

    def sample(beta, uniforms=None):
        betas.append(beta)
        out = real_sample(beta, uniforms=uniforms)
        samples.append(out[-1].cpu().numpy())
        return out
    agent._env_step, agent.memory.sample = env_step, sample
    tds = []
    real_prio = agent.memory.update_priorities

    def prio(idx, td, check=True):
        tds.append(td.cpu().numpy().copy())
        return real_prio(idx, td, check=True)
    agent.memory.update_priorities = prio
    agent.train(steps, sync_info=True)
    torch.cuda.synchronize()
    assert agent.check_errors() == {"per_sample": 0, "gather": 0, "env": 0, "td_action": 0, "maxpool": 0}
    np.testing.assert_array_equal(np.stack(acts), g["env_actions"])
    n_up = g["upd_td"].shape[0]
    assert len(samples) == n_up and len(agent.infos) == n_up
    np.testing.assert_array_equal(np.asarray(betas), g["upd_beta"])
    for k in range(n_up):
        np.testing.assert_array_equal(samples[k], g["upd_steps"][k], err_msg="sampled steps, update %d" % k)
        np.testing.assert_allclose(tds[k], g["upd_td"][k], rtol=1e-4, atol=1e-5, err_msg="|TD|, update %d" % k)
        info = agent.infos[k]
        np.testing.assert_allclose([info["Qloss"], info["learning_rate"], info["predictQ"]], g["upd_info"][k],
                                   rtol=1e-4, atol=1e-6, err_msg="info, update %d" % k)
    np.testing.assert_allclose([agent.PER_beta, agent.egreedy], g["final_beta_eps"], rtol=1e-12)
    mem = agent.memory
    assert [mem.size, mem.ptr] == list(g["size_ptr"])
    # leaves are |TD|^alpha of priorities matched at rtol 1e-4 / atol 1e-5 above
    np.testing.assert_allclose(mem.sum_tree.cpu().numpy(), g["tree_sum"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(mem.min_tree.cpu().numpy(), g["tree_min"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(mem.max_priority.cpu().numpy(), g["max_priority"], rtol=1e-4)
    for key, v in agent.policy.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), g["sd1/" + key], rtol=1e-3, atol=5e-5, err_msg=key)


def test_small_channel_library_conv_is_refused():
    """use_igemm off on a net with 8-channel convs: the explicit CNN path raises instead of calling MIOpen's NHWC kernels
    for those shapes (the r02 fault suspect)."""
    from xuanpolicy_amd import fused_cnn
    from xuanpolicy_amd.runner import build_perdqn
    agent = build_perdqn(n_envs=2, n_size=64, batch_size=16, device=DEV, start_training=16, filters=[8, 8],
                         kernels=[8, 4], strides=[4, 2], q_hidden_size=[32], max_episode_steps=40)
    fq = agent.learner._fused_q()
    assert fq is not None
    old = fused_cnn._Trunk.use_igemm
    fused_cnn._Trunk.use_igemm = False
    try:
        with pytest.raises(RuntimeError, match="small-channel MIOpen route"):
            agent.learner.q_values(agent.envs.obs)
    finally:
        fused_cnn._Trunk.use_igemm = old
