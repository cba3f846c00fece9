"""Pin the CPU oracle (oracle/) against golden vectors captured from the reference itself
(tests/golden/make_golden.py).  CPU only."""
import os

import numpy as np
import pytest
import torch

from oracle import cpu_ref

GAE_TAGS = ["plain_gae", "plain_nogae", "atari_gae", "atari_nogae"]


@pytest.fixture(scope="module", autouse=True)
def _built():
    cpu_ref.build_oracle()


@pytest.mark.parametrize("tag", GAE_TAGS)
def test_gae_rows_matches_reference(golden, tag):
    g = golden("gae.npz")
    use_gae = tag.endswith("_gae")
    adv, ret = cpu_ref.gae_rows(g[tag + "/rew"], g[tag + "/val"], g[tag + "/term"], g[tag + "/closed"],
                                g[tag + "/boot"], 0.99, 0.95, use_gae)
    np.testing.assert_allclose(adv, g[tag + "/adv"], rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(ret, g[tag + "/ret"], rtol=1e-5, atol=2e-6)
    # every position is covered by a closed path at buffer-full
    assert g[tag + "/closed"][:, -1].all()


def test_gae_python_loop_equals_c(golden):
    g = golden("gae.npz")
    tag = "atari_gae"
    N = 8
    a_c, r_c = cpu_ref.gae_rows(*(g[tag + k][:N] for k in ("/rew", "/val", "/term", "/closed", "/boot")), 0.99, 0.95)
    a_p = np.zeros_like(a_c)
    r_p = np.zeros_like(r_c)
    for n in range(N):
        start = 0
        for t in range(a_c.shape[1]):
            if g[tag + "/closed"][n, t]:
                cpu_ref.finish_path_py(g[tag + "/rew"][n], g[tag + "/val"][n], g[tag + "/term"][n], start, t + 1,
                                       float(g[tag + "/boot"][n, t]), 0.99, 0.95, True, a_p[n], r_p[n])
                start = t + 1
    np.testing.assert_array_equal(a_c, a_p)
    np.testing.assert_array_equal(r_c, r_p)


def test_sample_matches_reference(golden):
    g = golden("gae.npz")
    tag = "plain_gae"
    N, T = g[tag + "/rew"].shape
    buf = cpu_ref.BufferRef((3,), (2,), {"old_logp": ()}, N, T)
    buf.observations[:] = g[tag + "/obs"]
    buf.actions[:] = g[tag + "/act"]
    buf.auxiliary_infos["old_logp"][:] = g[tag + "/logp"]
    buf.values[:] = g[tag + "/val"]
    buf.returns[:] = g[tag + "/ret"]
    buf.advantages[:] = g[tag + "/adv"]
    buf.size = T
    for k in range(2):
        o, a, r, v, ad, ax = buf.sample(g["sample%d/idx" % k])
        np.testing.assert_array_equal(o, g["sample%d/obs" % k])
        np.testing.assert_array_equal(a, g["sample%d/act" % k])
        np.testing.assert_array_equal(r, g["sample%d/ret" % k])
        np.testing.assert_allclose(ad, g["sample%d/adv" % k], rtol=1e-6, atol=1e-6)
        np.testing.assert_array_equal(ax["old_logp"], g["sample%d/logp" % k])


LOSS_CASES = ["ppo_gaussian_6", "ppo_gaussian_17", "ppo_categorical_2", "ppo_categorical_6", "a2c_gaussian_6",
              "a2c_categorical_6"]


@pytest.mark.parametrize("tag", LOSS_CASES)
def test_closed_form_loss_grads_match_reference(golden, tag):
    g = golden("loss.npz")
    algo, dist, _ = tag.split("_")
    info, dh, dls, dv = cpu_ref.loss_grads_ref(algo, dist, g[tag + "/head"], g.get(tag + "/logstd0"), g[tag + "/v"],
                                               g[tag + "/act"], g[tag + "/adv"], g[tag + "/ret"],
                                               g.get(tag + "/old_logp"), 0.2, 0.25, 0.01)
    for k in ("actor-loss", "critic-loss", "entropy", "predict_value"):
        assert abs(info[k] - float(g[tag + "/info/" + k])) < 1e-5, k
    if algo == "ppo":
        assert abs(info["clip_ratio"] - float(g[tag + "/info/clip_ratio"])) < 1e-7
    np.testing.assert_allclose(dh, g[tag + "/dhead"], rtol=1e-4, atol=1e-8)
    np.testing.assert_allclose(dv, g[tag + "/dv"], rtol=1e-4, atol=1e-9)
    if dist == "gaussian":
        np.testing.assert_allclose(dls, g[tag + "/dlogstd"], rtol=1e-4, atol=1e-7)


def _load_sd(policy, g, prefix):
    sd = {k[len(prefix):]: torch.as_tensor(v) for k, v in g.items() if k.startswith(prefix)}
    policy.load_state_dict(sd)


@pytest.mark.parametrize("tag", LOSS_CASES)
def test_torch_cpu_learner_matches_reference(golden, tag):
    g = golden("loss.npz")
    algo, dist, A = tag.split("_")
    A = int(A)
    D = g[tag + "/obs"].shape[1]
    torch.manual_seed(0)
    pol = cpu_ref.build_actor_critic_ref(D, A, [64], [64], [64], discrete=(dist == "categorical"))
    _load_sd(pol, g, tag + "/sd0/")
    opt = torch.optim.Adam(pol.parameters(), 4e-4, eps=1e-5)
    sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.0, total_iters=1000)
    lrn = cpu_ref.LearnerRef(pol, opt, sch, algo, 0.25, 0.01, 0.2, 0.5, True)
    info = lrn.update(g[tag + "/obs"], g[tag + "/act"], g[tag + "/ret"], g[tag + "/adv"], g.get(tag + "/old_logp"))
    for k in ("actor-loss", "critic-loss", "entropy", "predict_value", "learning_rate"):
        assert abs(info[k] - float(g[tag + "/info/" + k])) < 1e-6, k
    for k, v in pol.state_dict().items():
        np.testing.assert_allclose(v.numpy(), g[tag + "/sd1/" + k], rtol=1e-5, atol=1e-7, err_msg=k)


def test_rms_matches_reference(golden):
    g = golden("rms.npz")
    rms = cpu_ref.RunningMeanStdRef((5,))
    for k in range(g["obs/x"].shape[0]):
        rms.update(g["obs/x"][k])
        np.testing.assert_allclose(rms.mean, g["obs/mean"][k], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(rms.var, g["obs/var"][k], rtol=1e-6, atol=1e-7)
        assert abs(rms.count - g["obs/count"][k]) < 1e-9
    r = cpu_ref.RunningMeanStdRef(())
    for k, x in enumerate(g["ret/x"]):
        r.update(np.asarray([x], np.float32))
        assert abs(float(r.mean) - g["ret/mean"][k]) < 1e-5 * max(1, abs(g["ret/mean"][k]))
        assert abs(float(r.var) - g["ret/var"][k]) < 1e-5 * max(1, abs(g["ret/var"][k]))


@pytest.mark.parametrize("name", ["agent_ppo_gauss.npz", "agent_a2c_cat.npz"])
def test_agent_replay_oracle(golden, name):
    """Replay the reference's recorded rollouts through BufferRef + LearnerRef: GAE, sampling
    (recorded permutations), every update's info, and the final parameters."""
    g = golden(name)
    N, T, D, A, n_epoch, n_mb, discrete, _, _ = (int(x) for x in g["config"])
    algo = "ppo" if "ppo" in name else "a2c"
    torch.manual_seed(0)
    pol = cpu_ref.build_actor_critic_ref(D, A, [64], [64], [64], discrete=bool(discrete))
    _load_sd(pol, g, "sd0/")
    opt = torch.optim.Adam(pol.parameters(), 4e-4, eps=1e-5)
    sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.0, total_iters=10000)
    lrn = cpu_ref.LearnerRef(pol, opt, sch, algo, 0.25, 0.01, 0.2, 0.5, True)
    iters = g["obs"].shape[0]
    B = N * T // n_mb
    u = 0
    for it in range(iters):
        adv, ret = cpu_ref.gae_rows(g["rew"][it], g["val"][it], g["term"][it], g["closed"][it], g["boot"][it], 0.99, 0.95)
        np.testing.assert_allclose(adv, g["adv"][it], rtol=1e-5, atol=2e-6)
        np.testing.assert_allclose(ret, g["ret"][it], rtol=1e-5, atol=2e-6)
        buf = cpu_ref.BufferRef((D,), () if discrete else (A,), {"old_logp": ()}, N, T)
        buf.observations[:], buf.actions[:], buf.values[:] = g["obs"][it], g["act"][it], g["val"][it]
        buf.returns[:], buf.advantages[:] = g["ret"][it], g["adv"][it]
        buf.auxiliary_infos["old_logp"][:] = g["logp"][it]
        buf.size = T
        for e in range(n_epoch):
            perm = g["perms"][it * n_epoch + e]
            for s in range(0, N * T, B):
                o, a, r, v, ad, ax = buf.sample(perm[s:s + B])
                info = lrn.update(o, a, r, ad, ax["old_logp"] if algo == "ppo" else None)
                ref = g["infos"][u]
                got = [info["actor-loss"], info["critic-loss"], info["entropy"], info["learning_rate"],
                       info["predict_value"]]
                np.testing.assert_allclose(got, ref[:5], rtol=1e-4, atol=1e-5)
                u += 1
    for k, v in pol.state_dict().items():
        np.testing.assert_allclose(v.numpy(), g["sd1/" + k], rtol=1e-4, atol=1e-5, err_msg=k)


@pytest.mark.parametrize("fixture", ["atari_a2c.npz", "atari_a2c_prod.npz"])
def test_atari_fixture_frames_and_gae_from_oracle(golden, fixture):
    """G8 pinned on CPU: stepping the oracle SynthAtari env with the recorded actions through the reference's
    DummyVecEnv / A2C_Agent observation flow (gym_vec_env.py:201-212, a2c_agent.py:80-92) reproduces the
    rewards, life-loss terminals and per-step frame sums the reference stored, and the oracle GAE over the
    recorded Atari closures (life losses keep the path open) reproduces its advantages and returns."""
    from oracle.synth_env import SynthAtariEnv
    g = golden(fixture)
    N, T, K, _, _, max_ep, seed = (int(x) for x in g["config"])
    envs = [SynthAtariEnv(i, seed=seed, n_actions=K, max_episode_steps=max_ep) for i in range(N)]
    obs = np.stack([e.reset()[0] for e in envs])
    k = 0
    for it in range(g["act"].shape[0]):
        for t in range(T):
            nxt, raw = obs.copy(), obs.copy()
            for i, e in enumerate(envs):
                o, r, te, tr, info = e.step(g["env_actions"][k][i])
                assert r == g["rew"][it][i, t] and te == bool(g["term"][it][i, t])
                if te or tr:
                    info["reset_obs"] = e.reset()[0]
                raw[i] = o
                nxt[i] = info["reset_obs"] if tr else o
            # the first step of train() stores the vec env's live buf_obs AFTER envs.step wrote into it
            # (a2c_agent.py:59-66: obs aliases envs.buf_obs until the first obs = next_obs; no obsnorm copy)
            stored = raw if (it, t) == (0, 0) else obs
            assert np.array_equal(stored.reshape(N, -1).astype(np.int64).sum(-1), g["frame_sum"][it][:, t])
            k += 1
            obs = nxt
        adv, ret = cpu_ref.gae_rows(g["rew"][it], g["val"][it], g["term"][it], g["closed"][it], g["boot"][it],
                                    0.99, 0.95)
        np.testing.assert_allclose(adv, g["adv"][it], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(ret, g["ret"][it], rtol=1e-5, atol=1e-5)
    assert int(g["term"].sum()) > 0 and int(g["closed"].sum()) > 0


def _perdqn_batch(seed, k, B, A):
    """tests/golden/make_golden.py perdqn_batch: the k-th update's inputs (numpy PCG64 is stable)."""
    rng = np.random.default_rng(seed * 1000 + k)
    obs = rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)
    nxt = rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)
    act = rng.integers(0, A, B).astype(np.float32)
    rew = rng.normal(0, 1, B).astype(np.float32)
    term = (rng.random(B) < 0.2).astype(np.float32)
    return obs, act, rew, nxt, term


@pytest.mark.parametrize("fixture", ["perdqn.npz", "perdqn_prod.npz"])
def test_perdqn_learner_ref_matches_reference(golden, fixture):
    """G9 pins the oracle's PER-DQN learner (perdqn_learner.py:17-48 over BasicQnetwork / Basic_CNN): |TD|, the
    info dict and the parameters after each of 4 updates (target copies every 2), and the closed-form TD / loss
    gradient (dqn_td_ref) against the autograd learner."""
    g = golden(fixture)
    B, A, n_up, seed, sync = (int(x) for x in g["config"])
    net = [int(x) for x in g["net"]]
    nl = (len(net) - 1) // 3
    pol = cpu_ref.build_qnetwork_ref(A, net[:nl], net[nl:2 * nl], net[2 * nl:3 * nl], net[3 * nl:])
    pol.load_state_dict({k[4:]: torch.as_tensor(v) for k, v in g.items() if k.startswith("sd0/")})
    opt = torch.optim.Adam(pol.parameters(), 1e-3, eps=1e-5)
    sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.5, total_iters=10)
    lrn = cpu_ref.PerDQNLearnerRef(pol, opt, sch, float(g["gamma"]), sync)
    for k in range(n_up):
        obs, act, rew, nxt, term = _perdqn_batch(seed, k, B, A)
        assert [int(obs.astype(np.int64).sum()), int(nxt.astype(np.int64).sum())] == list(g["input_sums"][k])
        with torch.no_grad():
            eq = pol(obs)[2].numpy()
            tq = pol.target(nxt)[2].numpy()
        loss, td, dq, pq = cpu_ref.dqn_td_ref(eq, tq, act, rew, term, float(g["gamma"]))
        td_l, info = lrn.update(obs, act, rew, nxt, term)
        np.testing.assert_allclose(td, td_l, rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(td_l, g["td_abs"][k], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose([info["Qloss"], info["learning_rate"], info["predictQ"]], g["infos"][k],
                                   rtol=1e-5, atol=1e-7)
        assert abs(loss - info["Qloss"]) <= 1e-5 * max(1.0, loss)
        for key, v in pol.state_dict().items():
            if "sd%d/%s" % (k + 1, key) in g:   # perdqn_prod.npz keeps only the last update's weights
                np.testing.assert_allclose(v.numpy(), g["sd%d/%s" % (k + 1, key)], rtol=1e-5, atol=1e-6, err_msg=key)


def test_fixture_init_regenerates_recorded_start():
    """G8P's starting weights are regenerated (tests/golden/fixture_init.py), not stored: the regenerated tensors
    match the checksums recorded when the reference trained from them, and the generator is the PCG64 stream."""
    import numpy as np
    from tests.golden.fixture_init import checksum, uniform_state
    g = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "atari_a2c_prod.npz"), allow_pickle=False))
    shapes = [(k[len("sd0sum/"):], None) for k in g if k.startswith("sd0sum/")]
    assert len(shapes) == 12    # 3 conv + 1 fc (weight, bias) + actor / critic output layers
    from xuanpolicy_amd.policies import AC_CNN_Atari, Categorical_AC_Policy

    class _Disc:
        n, shape = 6, ()
    torch.manual_seed(0)
    rep = AC_CNN_Atari((84, 84, 4), [8, 4, 3], [4, 2, 1], [32, 64, 64], None, torch.nn.init.orthogonal_,
                       torch.nn.ReLU, "cpu", [512])
    pol = Categorical_AC_Policy(_Disc(), rep, [], [], None, torch.nn.init.orthogonal_, torch.nn.ReLU, "cpu")
    vals = uniform_state([(k, v.shape) for k, v in pol.state_dict().items()], int(g["init_seed"]))
    assert set(vals) == {k for k, _ in shapes}
    for k, v in vals.items():
        np.testing.assert_array_equal(checksum(v), g["sd0sum/" + k], err_msg=k)


def test_perdqn_agent_fixture_schedules():
    """G10 (PerDQN_Agent.train) on CPU: the recorded epsilon / beta schedules follow perdqn_agent.py:74-95 step by step,
    every update's uniforms lie in [0, 1), and the recorded trees are consistent (root = sum of leaves)."""
    import numpy as np
    g = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "perdqn_agent.npz"), allow_pickle=False))
    N, n_size, batch, A, steps, seed, max_ep, start, sync, decay = (int(x) for x in g["config"])
    eps0, eps1, beta0 = (float(x) for x in g["hyper"][:3])
    eps, beta = eps0, beta0
    for k in range(steps):
        assert g["sched_eps"][k] == eps and g["sched_beta"][k] == beta
        beta += (1 - beta0) / steps
        eps = eps - (eps0 - eps1) / steps
        if eps > eps1:
            eps = eps - (eps0 - eps1) / decay
    assert list(g["final_beta_eps"]) == [beta, eps]
    u = g["upd_uniforms"]
    assert u.shape == (g["upd_td"].shape[0], N, batch // N) and (u >= 0).all() and (u < 1).all()
    cap = g["tree_sum"].shape[1] // 2
    np.testing.assert_allclose(g["tree_sum"][:, 1], g["tree_sum"][:, cap:].sum(1), rtol=1e-12)
    assert (g["env_actions"] >= 0).all() and (g["env_actions"] < A).all()
