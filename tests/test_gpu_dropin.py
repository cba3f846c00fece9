"""GPU drop-in parity: the reference's interfaces (DummyOnPolicyBuffer, PPOCLIP_Learner, A2C_Learner,
PPOCLIP_Agent) served by xuanpolicy_amd must reproduce the reference's numbers on the same data."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref, synth_env

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cpu_ref.build_oracle()


class _Box:
    def __init__(self, shape):
        self.shape = tuple(shape)


class _Disc:
    def __init__(self, n):
        self.n, self.shape = n, ()


def _policy(D, A, discrete, hidden=64):
    from xuanpolicy_amd.policies import Basic_MLP, Categorical_AC_Policy, Gaussian_AC_Policy
    act = torch.nn.LeakyReLU
    rep = Basic_MLP((D,), [hidden], None, torch.nn.init.orthogonal_, act, DEV)
    cls = Categorical_AC_Policy if discrete else Gaussian_AC_Policy
    space = _Disc(A) if discrete else _Box((A,))
    return cls(space, rep, [hidden], [hidden], None, torch.nn.init.orthogonal_, act, DEV)


def _load(policy, g, prefix):
    sd = {k[len(prefix):]: torch.as_tensor(v) for k, v in g.items() if k.startswith(prefix)}
    policy.load_state_dict(sd)


def _check_sd(policy, g, prefix, rtol, atol):
    for k, v in policy.state_dict().items():
        np.testing.assert_allclose(v.detach().cpu().numpy(), g[prefix + k], rtol=rtol, atol=atol, err_msg=k)


@pytest.mark.parametrize("tag", ["ppo_gaussian_6", "ppo_gaussian_17", "ppo_categorical_2", "ppo_categorical_6",
                                 "a2c_gaussian_6", "a2c_categorical_6"])
def test_learner_update_matches_reference(golden, tag):
    from xuanpolicy_amd.learners import A2C_Learner, PPOCLIP_Learner
    g = golden("loss.npz")
    algo, dist, A = tag.split("_")
    A = int(A)
    D = g[tag + "/obs"].shape[1]
    pol = _policy(D, A, dist == "categorical")
    _load(pol, g, tag + "/sd0/")
    opt = torch.optim.Adam(pol.parameters(), 4e-4, eps=1e-5)
    sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.0, total_iters=1000)
    if algo == "ppo":
        lrn = PPOCLIP_Learner(pol, opt, sch, DEV, "./", vf_coef=0.25, ent_coef=0.01, clip_range=0.2,
                              clip_grad_norm=0.5, use_grad_clip=True)
        info = lrn.update(g[tag + "/obs"], g[tag + "/act"], g[tag + "/ret"], g[tag + "/val"], g[tag + "/adv"],
                          g[tag + "/old_logp"])
    else:
        lrn = A2C_Learner(pol, opt, sch, DEV, "./", 0.25, 0.01, 0.5)
        info = lrn.update(g[tag + "/obs"], g[tag + "/act"], g[tag + "/ret"], g[tag + "/adv"])
    for k in ("actor-loss", "critic-loss", "entropy", "predict_value", "learning_rate"):
        assert abs(info[k] - float(g[tag + "/info/" + k])) < 1e-5, (k, info[k], float(g[tag + "/info/" + k]))
    loss = info["actor-loss"] - 0.01 * info["entropy"] + 0.25 * info["critic-loss"]
    ref_loss = (float(g[tag + "/info/actor-loss"]) - 0.01 * float(g[tag + "/info/entropy"])
                + 0.25 * float(g[tag + "/info/critic-loss"]))
    assert abs(loss - ref_loss) < 1e-4
    _check_sd(pol, g, tag + "/sd1/", rtol=1e-4, atol=2e-6)


@pytest.mark.parametrize("name", ["agent_ppo_gauss.npz", "agent_a2c_cat.npz"])
def test_buffer_and_learner_replay_reference_agent(golden, name):
    """The reference's two recorded PPOCLIP_Agent / A2C_Agent iterations replayed through the drop-in
    DummyOnPolicyBuffer (store / finish_path / sample) and learners: GAE, adv-norm, every update's info
    dict and the final parameters."""
    from xuanpolicy_amd.buffer import DummyOnPolicyBuffer
    from xuanpolicy_amd.learners import A2C_Learner, PPOCLIP_Learner
    g = golden(name)
    N, T, D, A, n_epoch, n_mb, discrete, _, _ = (int(x) for x in g["config"])
    algo = "ppo" if "ppo" in name else "a2c"
    pol = _policy(D, A, bool(discrete))
    _load(pol, g, "sd0/")
    opt = torch.optim.Adam(pol.parameters(), 4e-4, eps=1e-5)
    sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.0, total_iters=10000)
    if algo == "ppo":
        lrn = PPOCLIP_Learner(pol, opt, sch, DEV, "./", vf_coef=0.25, ent_coef=0.01, clip_range=0.2,
                              clip_grad_norm=0.5, use_grad_clip=True)
    else:
        lrn = A2C_Learner(pol, opt, sch, DEV, "./", 0.25, 0.01, 0.5)
    aux = {"old_logp": ()} if algo == "ppo" else {}
    buf = DummyOnPolicyBuffer(_Box((D,)), _Disc(A) if discrete else _Box((A,)), aux, N, T, True, True, 0.99, 0.95,
                              device=DEV)
    B = N * T // n_mb
    u = 0
    for it in range(g["obs"].shape[0]):
        for t in range(T):
            buf.store(g["obs"][it][:, t], g["act"][it][:, t], g["rew"][it][:, t], g["val"][it][:, t],
                      g["term"][it][:, t], {"old_logp": g["logp"][it][:, t]} if algo == "ppo" else None)
            for i in np.nonzero(g["closed"][it][:, t])[0]:
                buf.finish_path(float(g["boot"][it][i, t]), i)
        np.testing.assert_allclose(buf.advantages.cpu().numpy(), g["adv"][it], rtol=1e-5, atol=2e-5)
        np.testing.assert_allclose(buf.returns.cpu().numpy(), g["ret"][it], rtol=1e-5, atol=2e-5)
        for e in range(n_epoch):
            perm = g["perms"][it * n_epoch + e]
            for s in range(0, N * T, B):
                o, a, r, v, ad, ax = buf.sample(perm[s:s + B])
                if algo == "ppo":
                    info = lrn.update(o, a, r, v, ad, ax["old_logp"])
                else:
                    info = lrn.update(o, a, r, ad)
                got = [info["actor-loss"], info["critic-loss"], info["entropy"], info["learning_rate"],
                       info["predict_value"]]
                np.testing.assert_allclose(got, g["infos"][u][:5], rtol=2e-4, atol=2e-5)
                u += 1
        buf.clear()
    _check_sd(pol, g, "sd1/", rtol=1e-3, atol=5e-5)


def test_fused_agent_rollout_step_parity():
    """Step the fused PPO agent one env step at a time and check each step's buffer column and state
    against the CPU restatement of the reference loop (RMS normalisation, sampled-action log-prob,
    env dynamics, reward normalisation, return tracker, ret_rms, closures)."""
    from xuanpolicy_amd.runner import build_synthbox_ppo
    N, T, D, A = 256, 16, 17, 6
    # per-step bootstraps (defer_bootstrap=False): every closed column's V(norm(final obs)) is written as the step runs
    agent = build_synthbox_ppo(n_envs=N, n_steps=T, obs_dim=D, act_dim=A, hidden=64, n_epoch=1, n_minibatch=2,
                               seed=5, device=DEV, max_episode_steps=6, defer_bootstrap=False)
    assert not agent.defer_boot
    env, mem = agent.envs, agent.memory
    obs_rms = cpu_ref.RunningMeanStdRef((D,))
    ret_rms = cpu_ref.RunningMeanStdRef(())
    returns = np.zeros(N, np.float32)
    cenv = synth_env.SynthBoxVec(N, D, A, seed=5, max_episode_steps=6)
    for t in range(T - 1):
        raw = env.obs.cpu().numpy().copy()
        state_steps = env.ep_step.cpu().numpy().copy()
        cenv.state, cenv.ep_step = raw.copy(), state_steps.astype(np.int64)
        cenv.episode = env.ep_index.cpu().numpy().astype(np.uint32)
        obs_rms.update(raw)
        obs_n = cpu_ref.process_observation(raw, obs_rms, 5.0)
        ret_std_before = ret_rms.std
        agent.train(1, log=False)
        np.testing.assert_allclose(agent.obs_mean.cpu().numpy(), obs_rms.mean, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(agent.obs_var.cpu().numpy(), obs_rms.var, rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(mem.observations[:, t].cpu().numpy(), obs_n, rtol=1e-4, atol=1e-4)
        act = mem.actions[:, t].cpu().numpy()
        with torch.no_grad():
            mu, logstd, v = agent.policy.heads(mem.observations[:, t].contiguous())
            lp = torch.distributions.Normal(mu, logstd.exp()).log_prob(mem.actions[:, t]).sum(-1)
        np.testing.assert_allclose(mem.auxiliary_infos["old_logp"][:, t].cpu().numpy(), lp.cpu().numpy(), rtol=1e-5,
                                   atol=1e-4)
        np.testing.assert_allclose(mem.values[:, t].cpu().numpy(), v.cpu().numpy(), rtol=1e-5, atol=1e-5)
        fin, r, te, tr, _ = cenv.step(act)
        np.testing.assert_allclose(env.final_obs.cpu().numpy(), fin, rtol=1e-4, atol=1e-5)
        np.testing.assert_array_equal(mem.terminals[:, t].cpu().numpy(), te.astype(np.float32))
        exp_rew = np.clip(r / np.clip(ret_std_before, 0.1, 100), -5, 5)
        np.testing.assert_allclose(mem.rewards[:, t].cpu().numpy(), exp_rew, rtol=1e-4, atol=1e-5)
        returns = (1 - te) * 0.99 * returns + r
        done = te | tr
        for i in np.nonzero(done)[0]:
            ret_rms.update(returns[i:i + 1])
        returns = np.where(done, 0, returns).astype(np.float32)
        np.testing.assert_allclose(agent.returns.cpu().numpy(), returns, rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(float(agent.ret_var), float(ret_rms.var), rtol=1e-4, atol=1e-6)
        closed = mem.closed[:, t].cpu().numpy().astype(bool)
        np.testing.assert_array_equal(closed, done)
        with torch.no_grad():
            vb = agent.policy.value(torch.as_tensor(cpu_ref.process_observation(fin, obs_rms, 5.0), device=DEV))
        exp_boot = np.where(done, np.where(te, 0, vb.cpu().numpy()), 0)
        np.testing.assert_allclose(mem.boot[:, t].cpu().numpy(), exp_boot, rtol=1e-4, atol=1e-4)


def test_fused_agent_iteration_matches_cpu_replay():
    """A whole fused iteration (rollout -> GAE -> n_epoch x n_minibatch fused updates) vs the CPU oracle
    learner replaying the same buffer with the same device permutations from the same weights."""
    from xuanpolicy_amd.runner import build_synthbox_ppo
    N, T, D, A = 128, 32, 17, 6
    agent = build_synthbox_ppo(n_envs=N, n_steps=T, obs_dim=D, act_dim=A, hidden=64, n_epoch=2, n_minibatch=4,
                               seed=9, device=DEV, ent_coef=0.01)
    pol = cpu_ref.build_actor_critic_ref(D, A, [64], [64], [64])
    pol.load_state_dict({k: v.cpu() for k, v in agent.policy.state_dict().items()})
    agent.train(T - 1, log=False)
    agent.train(1, log=False)  # last step: buffer full -> GAE -> updates
    mem = agent.memory
    adv, ret = cpu_ref.gae_rows(mem.rewards.cpu().numpy(), mem.values.cpu().numpy(), mem.terminals.cpu().numpy(),
                                mem.closed.cpu().numpy(), mem.boot.cpu().numpy(), 0.99, 0.95)
    np.testing.assert_allclose(mem.advantages.cpu().numpy(), adv, rtol=1e-5, atol=2e-5)
    opt = torch.optim.Adam(pol.parameters(), agent.config.learning_rate, eps=1e-5)
    sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.0, total_iters=agent.config.running_steps)
    lrn = cpu_ref.LearnerRef(pol, opt, sch, "ppo", 0.25, 0.01, 0.2, 0.5, True)
    buf = cpu_ref.BufferRef((D,), (A,), {"old_logp": ()}, N, T)
    buf.observations[:] = mem.observations.cpu().numpy()
    buf.actions[:] = mem.actions.cpu().numpy()
    buf.values[:] = mem.values.cpu().numpy()
    buf.returns[:], buf.advantages[:] = ret, adv
    buf.auxiliary_infos["old_logp"][:] = mem.auxiliary_infos["old_logp"].cpu().numpy()
    buf.size = T
    B = N * T // 4
    for e in range(2):
        perm = agent.epoch_permutation(N * T, counter=e).cpu().numpy()
        for s in range(0, N * T, B):
            o, a, r, v, ad, ax = buf.sample(perm[s:s + B])
            info = lrn.update(o, a, r, ad, ax["old_logp"])
    got = agent.infos[-1] if agent.infos else agent.learner._info(agent.last_info)
    for k in ("actor-loss", "critic-loss", "entropy", "predict_value"):
        assert abs(got[k] - info[k]) < 1e-3 * max(1.0, abs(info[k])), (k, got[k], info[k])
    for k, v in agent.policy.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), pol.state_dict()[k].numpy(), rtol=1e-3, atol=1e-4, err_msg=k)


def test_host_env_path_runs():
    """The agent over a host (numpy) VecEnv with reset_obs infos: same kernels, per-step copies."""
    from xuanpolicy_amd.runner import build_synthbox_ppo

    class HostVec:
        def __init__(self, N, D, A):
            self.v = synth_env.SynthBoxVec(N, D, A, seed=2, max_episode_steps=9)
            self.num_envs = N
            self.observation_space, self.action_space = _Box((D,)), _Box((A,))
            self.buf_obs = self.v.reset()

        def step(self, a):
            fin, r, te, tr, nxt = self.v.step(a)
            return fin, r, te, tr, [{"reset_obs": nxt[i]} for i in range(self.num_envs)]

    N, T = 32, 8
    import xuanpolicy_amd.runner as R
    cfg = R.get_arguments("ppo", "synthbox", "x")
    cfg.parallels, cfg.n_steps, cfg.n_epoch, cfg.n_minibatch = N, T, 1, 2
    cfg.representation_hidden_size = cfg.actor_hidden_size = cfg.critic_hidden_size = [32]
    agent = R.build_agent(cfg, DEV, envs=HostVec(N, 17, 6))
    agent.train(2 * T)
    assert len(agent.infos) == 2 and all(np.isfinite(v) for v in agent.infos[-1].values() if isinstance(v, float))
    del build_synthbox_ppo
