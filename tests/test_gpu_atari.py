"""GPU: the Atari-shaped path (C3) — K15 SynthAtari env vs its CPU checker (bitwise frames, rewards,
flags, resets), the raw uint8 column store, and A2C iterations with AC_CNN_Atari on device."""
import os

import numpy as np
import pytest
import torch

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


def test_synthatari_matches_oracle():
    from oracle.synth_env import SynthAtariEnv
    from xuanpolicy_amd.envs import SynthAtariVecEnv
    N, K, steps = 5, 6, 400
    env = SynthAtariVecEnv(N, K, seed=3, max_episode_steps=150, device=DEV)
    ref = [SynthAtariEnv(i, seed=3, n_actions=K, max_episode_steps=150) for i in range(N)]
    assert np.array_equal(env.obs.cpu().numpy(), np.stack([r.reset()[0] for r in ref]))
    rng = np.random.default_rng(0)
    n_over = n_life = 0
    for t in range(steps):
        a = rng.integers(0, K, N)
        obs, rew, term, trunc, infos = env.step(a)
        for i, r in enumerate(ref):
            o, rw, te, tr, info = r.step(a[i])
            assert np.array_equal(obs[i], o), (t, i)
            assert rew[i] == rw and term[i] == te and trunc[i] == tr, (t, i)
            assert infos[i]["episode_step"] == info["episode_step"]
            if tr:
                assert np.array_equal(infos[i]["reset_obs"], info["reset_obs"])
            n_over += int(tr)
            n_life += int(te and not tr)
        assert np.array_equal(env.obs.cpu().numpy(), np.stack([r.stack for r in ref]))
    assert n_over > 0 and n_life > 0


def test_store_column_raw_frames():
    from xuanpolicy_amd import ops
    N, T = 33, 7
    x = torch.randint(0, 256, (N, 84, 84, 4), device=DEV, dtype=torch.int32).to(torch.uint8)
    buf = torch.zeros((N, T, 84, 84, 4), dtype=torch.uint8, device=DEV)
    cur = torch.tensor([5, 0, 0, 0], dtype=torch.int32, device=DEV)
    ops.store_column(x, buf, cur)
    assert torch.equal(buf[:, 5], x) and int(buf[:, :5].sum()) == 0 and int(buf[:, 6:].sum()) == 0


@pytest.mark.parametrize("graph", [True, False])
def test_a2c_atari_iterations(graph):
    """Two A2C iterations at a small C3 shape through the device rollout (uint8 frames stored raw,
    CNN forward/backward on MIOpen/hipBLASLt, K2 categorical loss, K1 GAE with life-loss closures)."""
    from xuanpolicy_amd.runner import build_atari_a2c
    agent = build_atari_a2c(n_envs=64, n_steps=32, device=DEV, n_epoch=2, n_minibatch=4, cuda_graph=graph,
                            max_episode_steps=40)
    assert agent.raw_obs and agent.memory.observations.dtype == torch.uint8
    agent.train(64)
    assert len(agent.infos) == 2
    for info in agent.infos:
        assert np.isfinite([info["actor-loss"], info["critic-loss"], info["entropy"]]).all()
        assert 0 < info["entropy"] <= np.log(6) + 1e-5
    mem = agent.memory
    # the buffer holds the frames the env produced (channel 3 of column t+1 = newest frame of step t)
    assert mem.observations.shape == (64, 32, 84, 84, 4)
    assert bool((mem.observations[:, :, 78:82] == 200).any())          # paddle rows present
    assert int(mem.closed.sum()) > 0                                   # game overs closed paths
    assert torch.isfinite(mem.advantages).all() and torch.isfinite(mem.returns).all()


def _load_sd0(pol, g):
    """The fixture's starting weights: stored (sd0/) or regenerated from init_seed (tests/golden/fixture_init.py),
    pinned by the recorded checksums."""
    if "init_seed" not in g:
        pol.load_state_dict({k[4:]: torch.as_tensor(v) for k, v in g.items() if k.startswith("sd0/")})
        return
    from tests.golden.fixture_init import checksum, uniform_state
    sd = pol.state_dict()
    vals = uniform_state([(k, v.shape) for k, v in sd.items()], int(g["init_seed"]))
    for k, v in vals.items():
        np.testing.assert_array_equal(checksum(v), g["sd0sum/" + k], err_msg=k)
    pol.load_state_dict({k: torch.as_tensor(v) for k, v in vals.items()})


def _check_sd1(pol, g, rtol, atol, env=None, efac=3):
    """Final weights against the fixture: whole tensors, or (tensors above fixture_init.BIG) every 16th row + every
    row's sum.  env (tests/golden/make_envelopes.py): per tensor, how far the exact f64 replay lands from the f32
    reference; the tolerance is max(atol, 3 x that)."""
    env = env or {}
    for key, v in pol.state_dict().items():
        a = v.detach().cpu().numpy()
        if "sd1/" + key in g:
            tol = max(atol, efac * float(env.get("sd/" + key, 0)))
            np.testing.assert_allclose(a, g["sd1/" + key], rtol=rtol, atol=tol, err_msg=key)
            continue
        tol = max(atol, efac * float(env.get("sd/" + key + "::rows16", 0)))
        np.testing.assert_allclose(a[::16], g["sd1/" + key + "::rows16"], rtol=rtol, atol=tol, err_msg=key)
        rs = a.reshape(a.shape[0], -1).astype(np.float64).sum(1)
        tol = max(atol * a[0].size ** 0.5, efac * float(env.get("sd/" + key + "::rowsum", 0)))
        np.testing.assert_allclose(rs, g["sd1/" + key + "::rowsum"], rtol=rtol, atol=tol, err_msg=key + " row sums")


def _gae_close(got, ref):
    """north_star's 1e-5 (absolute, plus 1e-5 relative), widened by 2^-20 of the row's largest |value| (the scan's f32
    rounding is relative to the row's largest partial sum; tests/test_gpu_kernels.py::_gae_close)."""
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    row = np.abs(ref).max(axis=-1, keepdims=True)
    tol = 1e-5 + 1e-5 * np.abs(ref) + 2.0 ** -20 * row
    bad = np.abs(got - ref) > tol
    assert not bad.any(), ("GAE mismatch", int(bad.sum()), float(np.abs(got - ref)[bad].max()))


def _replay_atari(g, env, conv_path, efac=3, rtol=1e-4, base_atol=1e-5):
    """Replay a G8 / G12 fixture (make_golden.capture_atari) through the device buffer and the learner the agent uses:
    A2C_Learner (algo 0) or PPOCLIP_Learner (algo 1, old_logp from the buffer's aux column, clip_ratio checked).
    Loss scalars: rtol 1e-4 + max(base_atol, efac x the fixture's f64 envelope) — update 0 (identical starting weights)
    at the base tolerance; GAE at 1e-5 (_gae_close)."""
    from oracle.synth_env import SynthAtariEnv
    from xuanpolicy_amd.buffer import DummyOnPolicyBuffer_Atari
    from xuanpolicy_amd.learners import A2C_Learner, PPOCLIP_Learner
    from xuanpolicy_amd.policies import AC_CNN_Atari, Categorical_AC_Policy
    ppo = int(g["algo"]) == 1 if "algo" in g else False
    N, T, K, n_epoch, n_mb, max_ep, seed = (int(x) for x in g["config"])
    net = [int(x) for x in g["net"]]
    nl = (len(net) - 1) // 3
    filters, kernels, strides, fc = net[:nl], net[nl:2 * nl], net[2 * nl:3 * nl], net[3 * nl:]

    class _Box:
        shape = (84, 84, 4)

    class _Disc:
        n, shape = K, ()
    rep = AC_CNN_Atari((84, 84, 4), kernels, strides, filters, None, torch.nn.init.orthogonal_, torch.nn.ReLU, DEV,
                       fc)
    pol = Categorical_AC_Policy(_Disc(), rep, [], [], None, torch.nn.init.orthogonal_, torch.nn.ReLU, DEV)
    _load_sd0(pol, g)
    if ppo:
        lr, vf, ent, clip, gn = (float(x) for x in g["hyper"])
    else:
        lr, vf, ent, clip, gn = 7e-4, 0.25, 0.01, 0.0, 0.2
    opt = torch.optim.Adam(pol.parameters(), lr, eps=1e-5)
    sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.0, total_iters=10000)
    lrn = (PPOCLIP_Learner(pol, opt, sch, DEV, "./", vf, ent, clip, gn, True) if ppo else
           A2C_Learner(pol, opt, sch, DEV, "./", vf, ent, gn))
    fcn = lrn._fused_cnn()
    assert fcn is not None, "the explicit CNN path (fused_cnn) must run"
    if filters[:2] == [32, 64]:   # the production first convs: K25 / K26 / K27
        assert fcn.trunk_.u8_conv1 and fcn.trunk_._dgrad_ok(fcn.trunk_.convs[1][0])
    buf = DummyOnPolicyBuffer_Atari(_Box(), _Disc(), {"old_logp": ()} if ppo else {}, N, T, True, True, 0.99, 0.95,
                                    device=DEV)
    assert buf.observations.dtype == torch.uint8
    envs = [SynthAtariEnv(i, seed=seed, n_actions=K, max_episode_steps=max_ep) for i in range(N)]
    obs = np.stack([e.reset()[0] for e in envs])
    B = N * T // n_mb
    u = k = 0
    keys = ["actor-loss", "critic-loss", "entropy", "learning_rate", "predict_value"] + (["clip_ratio"] if ppo else [])
    for it in range(g["act"].shape[0]):
        for t in range(T):
            acts = g["env_actions"][k]
            k += 1
            nxt, raw = obs.copy(), obs.copy()
            for i, e in enumerate(envs):    # DummyVecEnv_Gym.step_wait (gym_vec_env.py:201-212)
                o, r, te, tr, info = e.step(acts[i])
                assert r == g["rew"][it][i, t] and te == bool(g["term"][it][i, t])
                if te or tr:
                    info["reset_obs"] = e.reset()[0]
                raw[i] = o
                # a2c_agent.py:88-92 / ppoclip_agent.py:89-101: a game over (truncation) continues from reset_obs, a
                # life loss keeps the stack and the path
                nxt[i] = info["reset_obs"] if tr else o
            # the reference stores after envs.step, and on train()'s first step `obs` still aliases the vec env's
            # buf_obs, which the step overwrote (a2c_agent.py:59-66, ppoclip_agent.py:60-68): that column holds the
            # post-step frames
            stored = raw if (it, t) == (0, 0) else obs
            assert np.array_equal(stored.reshape(N, -1).astype(np.int64).sum(-1), g["frame_sum"][it][:, t])
            aux = {"old_logp": g["old_logp"][it][:, t]} if ppo else None
            buf.store(stored, g["act"][it][:, t], g["rew"][it][:, t], g["val"][it][:, t], g["term"][it][:, t], aux)
            for i in np.nonzero(g["closed"][it][:, t])[0]:
                buf.finish_path(float(g["boot"][it][i, t]), i)
            obs = nxt
        _gae_close(buf.advantages.cpu().numpy(), g["adv"][it])
        _gae_close(buf.returns.cpu().numpy(), g["ret"][it])
        for e in range(n_epoch):
            perm = g["perms"][it * n_epoch + e]
            for s in range(0, N * T, B):
                o, a, r, v, ad, ax = buf.sample(perm[s:s + B])
                assert o.dtype == torch.uint8
                info = lrn.update(o, a, r, v, ad, ax["old_logp"]) if ppo else lrn.update(o, a, r, ad)
                got = [float(info[kk]) for kk in keys]
                ev = env["info"][u] if env is not None else np.zeros(len(keys))
                atol = np.maximum(base_atol, efac * ev)
                if u == 0:
                    atol = np.full(len(keys), base_atol)   # identical starting weights: north_star's tolerance
                if ppo:   # clip fraction: a count / B, exact at update 0 (ratios 1 within f32), then the envelope
                    atol[-1] = 0.0 if u == 0 else max(efac * ev[-1], 2.0 / B)
                if env is not None and os.environ.get("XPA_REPORT_ENVELOPE"):
                    dev = np.abs(np.asarray(got, np.float64) - g["infos"][u])
                    print("ENVELOPE u=%d dev/env=%s" % (u, np.round(dev / np.maximum(ev, 1e-12), 2)))
                _close(got, g["infos"][u], rtol, atol, "update %d" % u)
                u += 1
        buf.clear()
    assert u == len(g["infos"])
    _check_sd1(pol, g, rtol=1e-3, atol=5e-5, env=env, efac=efac)


@pytest.mark.parametrize("fixture", ["atari_a2c.npz", "atari_a2c_prod.npz"])
def test_a2c_atari_replays_reference_agent(golden, fixture, conv_path):
    """G8: the reference's two recorded A2C_Agent iterations on Atari-shaped frames (a2c_agent.py:57-107,
    env_name "Atari": DummyOnPolicyBuffer_Atari memory_tools.py:526-560, AC_CNN_Atari cnn.py:45-93 +
    Categorical_AC_Policy, life losses keep the path open) replayed through the device buffer (uint8 frames,
    K1 GAE with the Atari closures, K4 sample + adv-norm) and A2C_Learner (CNN on K25-K29 or MIOpen per conv_path,
    K2 categorical loss, K9 clip + Adam): GAE, every update's info dict, the final parameters.  The frames are
    regenerated by stepping the oracle SynthAtari env with the recorded actions through the reference's
    DummyVecEnv / agent observation flow and checked against the recorded per-step frame sums.
    atari_a2c_prod.npz (G8P) is the production net (filters [32, 64, 64], kernels [8, 4, 3], strides [4, 2, 1], fc
    512; 8 envs x 64 steps, minibatches of 256) replayed update by update.  A few Adam steps of an f32 net are
    chaotic in the last bits (tests/golden/make_envelopes.py): the prod fixture carries, per update and per tensor, how
    far the exact f64 replay lands from the reference, and the tolerances are max(base, 3 x that envelope) — update 0
    (identical starting weights) is held to the base tolerances (1e-4 relative + 1e-5)."""
    g = golden(fixture)
    env = golden(fixture.replace(".npz", "_env.npz")) if "init_seed" in g else None
    _replay_atari(g, env, conv_path)


@pytest.mark.parametrize("fixture", ["atari_ppo.npz", "atari_ppo_prod.npz"])
def test_ppo_atari_replays_reference_agent(golden, fixture, conv_path):
    """G12 / G12P: examples/ppo/ppo_atari.py's agent — the reference's PPOCLIP_Agent with env_name
    "Atari" (ppoclip_agent.py:24-25: DummyOnPolicyBuffer_Atari; :93-94: a life loss keeps the path open) over
    DummyVecEnv_Atari of SynthAtari, ppo/atari.yaml's coefficients (lr 2.5e-4, clip 0.2, grad norm 0.5, vf 0.25,
    ent 0.01; 4 epochs x 4 minibatches), two recorded iterations, small and production AC_CNN_Atari — replayed
    through the device buffer (old_logp column), FusedCNNActorCritic and K2 in PPO mode (ratio / clip / old_logp,
    clip fraction): GAE at 1e-5, update 0's loss scalars at 1e-4 relative + 1e-5, later updates within 3x the
    fixture's measured f64 envelope (make_envelopes.py), the final weights likewise."""
    g = golden(fixture)
    env = golden(fixture.replace(".npz", "_env.npz"))
    _replay_atari(g, env, conv_path)


def test_atari_deferred_last_bootstrap_matches_per_step():
    """raw_defer (SynthAtari: truncation implies terminal) — one critic forward on the last step's frames after the
    rollout — leaves the buffer exactly as the per-step bootstrap forward does (a2c_agent.py:66-72, 86-98)."""
    from xuanpolicy_amd.runner import build_atari_a2c
    bufs = []
    for defer in (True, False):
        agent = build_atari_a2c(n_envs=48, n_steps=32, device=DEV, n_epoch=1, n_minibatch=4, max_episode_steps=20,
                                defer_bootstrap=defer, seed=5)
        assert agent.raw_defer == defer
        agent.train(32)
        torch.cuda.synchronize()
        m = agent.memory
        bufs.append([t.clone() for t in (m.boot, m.closed, m.terminals, m.advantages, m.returns)])
    assert int(bufs[0][1].sum()) > 48        # game overs inside the rollout as well as the last column
    for a, b in zip(*bufs):
        assert torch.equal(a, b)


def test_a2c_raw_mid_bootstrap_from_next_values_matches_per_step():
    """A2C over raw frames whose truncations are NOT terminal (gym's TimeLimit contract instead of the Atari flag rule):
    a close at step t < T - 1 bootstraps with V(reset frames) (a2c_agent.py:88-95).  raw_mid_next reads it from the
    rollout's own value column t + 1 after the rollout; the per-step form (defer_bootstrap=False) runs a second critic
    forward over every env at every step.  The buffers must be identical."""
    from xuanpolicy_amd.envs import SynthAtariVecEnv
    from xuanpolicy_amd.runner import build_agent, get_arguments

    class TruncOnlyAtari(SynthAtariVecEnv):
        def __init__(self, *a, **kw):
            super().__init__(*a, **kw)
            self.truncation_implies_terminal = False

        def step_device(self):
            super().step_device()
            self.term.mul_((self.trunc == 0).to(torch.uint8))   # game overs / the step limit: truncated only

    bufs = []
    for defer in (True, False):
        cfg = get_arguments("a2c", "atari", "SynthAtari-v0")
        cfg.parallels, cfg.n_steps, cfg.seed, cfg.n_epoch, cfg.n_minibatch = 48, 32, 5, 1, 4
        cfg.max_episode_steps, cfg.defer_bootstrap = 9, defer
        torch.manual_seed(5)
        envs = TruncOnlyAtari(48, 6, seed=5, max_episode_steps=9, device=DEV)
        agent = build_agent(cfg, DEV, envs=envs)
        assert not agent.raw_defer and agent.raw_mid_next == defer
        agent.train(32)
        torch.cuda.synchronize()
        m = agent.memory
        bufs.append([t.clone() for t in (m.values, m.boot, m.closed, m.terminals, m.advantages, m.returns)])
    closed, term = bufs[0][2][:, :-1] != 0, bufs[0][3][:, :-1] != 0
    assert int((closed & ~term).sum()) > 48     # non-terminal closes inside the rollout
    for a, b in zip(*bufs):
        assert torch.equal(a, b)
