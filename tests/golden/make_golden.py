"""Capture golden vectors from the reference (XuanCe 1.0.5 fork at /root/reference).

Run in the build container only (the reference never travels to the GPU box):
    cd /tmp && python /root/repo/tests/golden/make_golden.py
Writes small .npz fixtures next to this file (data only: inputs and the reference's outputs).

Fixtures:
  gae.npz      G1/G2  DummyOnPolicyBuffer store/finish_path/sample (memory_tools.py:143-245) under the
                      agent's closure rules (ppoclip_agent.py:69-101): plain and Atari life-loss modes,
                      use_gae on/off, plus sample() of two minibatches with adv-norm.
  loss.npz     G3/G4  PPOCLIP_Learner.update / A2C_Learner.update (ppoclip_learner.py:24-65,
                      a2c_learner.py:19-50) on Gaussian (A=6, 17) and Categorical (K=2, 6) heads:
                      inputs, head outputs, d loss/d head (captured before grad clipping), info dict,
                      parameters before and after the Adam step.
  agent_*.npz  G5     two seeded iterations of PPOCLIP_Agent.train / A2C_Agent.train on SynthBox envs
                      (oracle/synth_env.py) in the reference's DummyVecEnv_Gym: every stored step,
                      every closure, the permutations, learner infos, initial and final parameters.
  rms.npz      G7     RunningMeanStd (statistic_tools.py:35-112) update sequences.
  atari_a2c.npz G8    two seeded iterations of A2C_Agent.train (a2c_agent.py:57-107) with env_name "Atari":
                      DummyOnPolicyBuffer_Atari (memory_tools.py:526-560, uint8 frames), AC_CNN_Atari
                      (cnn.py:45-93) + Categorical_AC_Policy, DummyVecEnv_Atari over SynthAtari envs
                      (oracle/synth_env.py; life losses keep the path open, game overs truncate).  Frames are
                      NOT stored: the test regenerates them by stepping the oracle env with the recorded
                      actions and checks them against the recorded per-step frame sums.
  perdqn.npz   G9     PerDQN_Learner.update (perdqn_learner.py:17-48) on BasicQnetwork (deterministic.py:148-182)
                      over a small Basic_CNN (cnn.py:5-40): 4 updates, sync_frequency 2 (target copies),
                      uint8 4x84x84 batches regenerated from a recorded numpy seed (PCG64), 18 actions:
                      |TD error| per sample, the info dict, and the parameters after every update.
  per.npz      G6     PerOffPolicyBuffer (memory_tools.py:369-492) + Sum/MinSegmentTree (segtree_tool.py):
                      store / sample(beta) / update_priorities rounds with every uniform random.random()
                      returned to the sampler recorded, the trees after every call, max priorities, the
                      sampled indices (incl. the uint8 wrap for n_size > 256), IS weights and batches.
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

import ref_loader  # noqa: E402

xuance = ref_loader.import_reference()
import torch  # noqa: E402
import gym  # noqa: E402  (stub)
from xuance.common.memory_tools import DummyOnPolicyBuffer  # noqa: E402
from xuance.common.statistic_tools import RunningMeanStd  # noqa: E402
from xuance.torch.representations import Basic_MLP  # noqa: E402
from xuance.torch.policies import Gaussian_AC_Policy, Categorical_AC_Policy  # noqa: E402
from xuance.torch.learners import PPOCLIP_Learner, A2C_Learner  # noqa: E402
from xuance.torch.agents import PPOCLIP_Agent, A2C_Agent  # noqa: E402
from xuance.environment.gym.gym_vec_env import DummyVecEnv_Gym, DummyVecEnv_Atari  # noqa: E402
from xuance.torch.representations import AC_CNN_Atari  # noqa: E402
from oracle.synth_env import SynthAtariEnv, SynthBoxEnv  # noqa: E402

torch.set_num_threads(1)


# ----------------------------------------------------------------------------------------------
def capture_gae(seed=0, N=64, T=128, obs_dim=3, act_dim=2):
    out = {}
    rng = np.random.default_rng(seed)
    for atari in (False, True):
        for use_gae in (True, False):
            tag = ("atari" if atari else "plain") + ("_gae" if use_gae else "_nogae")
            buf = DummyOnPolicyBuffer(gym.spaces.Box(-1, 1, (obs_dim,)), gym.spaces.Box(-1, 1, (act_dim,)),
                                      {"old_logp": ()}, N, T, use_gae, True, 0.99, 0.95)
            closed = np.zeros((N, T), np.uint8)
            boot = np.zeros((N, T), np.float32)
            term_all = rng.random((N, T)) < 0.01
            trunc_all = rng.random((N, T)) < 0.01
            boot_all = rng.normal(0, 1, (N, T)).astype(np.float32)
            for t in range(T):
                obs = rng.normal(0, 1, (N, obs_dim)).astype(np.float32)
                act = rng.normal(0, 1, (N, act_dim)).astype(np.float32)
                rew = rng.normal(0, 1, N).astype(np.float32)
                val = rng.normal(0, 1, N).astype(np.float32)
                lp = rng.normal(-3, 1, N).astype(np.float32)
                term, trunc = term_all[:, t], trunc_all[:, t]
                buf.store(obs, act, rew, val, term, {"old_logp": lp})
                if buf.full:
                    # ppoclip_agent.py:69-75: close every env's path at buffer-full.
                    for i in range(N):
                        v = 0.0 if term[i] else boot_all[i, t]
                        buf.finish_path(v, i)
                        closed[i, T - 1], boot[i, T - 1] = 1, v
                    break
                for i in range(N):  # ppoclip_agent.py:89-101
                    if term[i] or trunc[i]:
                        if atari and not trunc[i]:
                            continue  # life loss: masked d=1 mid-path, no closure
                        v = 0.0 if term[i] else boot_all[i, t]
                        buf.finish_path(v, i)
                        closed[i, t], boot[i, t] = 1, v
            out[tag + "/rew"] = buf.rewards.copy()
            out[tag + "/val"] = buf.values.copy()
            out[tag + "/term"] = buf.terminals.copy()
            out[tag + "/closed"] = closed
            out[tag + "/boot"] = boot
            out[tag + "/adv"] = buf.advantages.copy()
            out[tag + "/ret"] = buf.returns.copy()
            if tag == "plain_gae":
                out[tag + "/obs"] = buf.observations.copy()
                out[tag + "/act"] = buf.actions.copy()
                out[tag + "/logp"] = buf.auxiliary_infos["old_logp"].copy()
                perm = np.arange(N * T)
                rng.shuffle(perm)
                B = N * T // 4
                for k in range(2):
                    idx = perm[k * B:(k + 1) * B]
                    o, a, r, v, ad, ax = buf.sample(idx)
                    out["sample%d/idx" % k] = idx.astype(np.int64)
                    out["sample%d/obs" % k] = o
                    out["sample%d/act" % k] = a
                    out["sample%d/ret" % k] = r
                    out["sample%d/val" % k] = v
                    out["sample%d/adv" % k] = ad.astype(np.float32)
                    out["sample%d/logp" % k] = ax["old_logp"]
    np.savez_compressed(os.path.join(HERE, "gae.npz"), **out)
    print("gae.npz", len(out))


# ----------------------------------------------------------------------------------------------
def _policy(D, A, discrete, hidden=(64,), seed=0):
    torch.manual_seed(seed)
    act = torch.nn.LeakyReLU
    rep = Basic_MLP((D,), list(hidden), None, torch.nn.init.orthogonal_, act, "cpu")
    if discrete:
        return Categorical_AC_Policy(gym.spaces.Discrete(A), rep, list(hidden), list(hidden), None,
                                     torch.nn.init.orthogonal_, act, "cpu")
    return Gaussian_AC_Policy(gym.spaces.Box(-1, 1, (A,)), rep, list(hidden), list(hidden), None,
                              torch.nn.init.orthogonal_, act, "cpu")


def _sd(prefix, policy, out):
    for k, v in policy.state_dict().items():
        out[prefix + k] = v.detach().cpu().numpy().copy()


def capture_loss(B=512, D=11):
    out = {}
    cases = [("ppo", "gaussian", 6), ("ppo", "gaussian", 17), ("ppo", "categorical", 2), ("ppo", "categorical", 6),
             ("a2c", "gaussian", 6), ("a2c", "categorical", 6)]
    for ci, (algo, dist, A) in enumerate(cases):
        tag = "%s_%s_%d" % (algo, dist, A)
        discrete = dist == "categorical"
        policy = _policy(D, A, discrete, seed=100 + ci)
        rng = np.random.default_rng(200 + ci)
        obs = rng.normal(0, 1, (B, D)).astype(np.float32)
        with torch.no_grad():
            _, d0, v0 = policy(obs)
            act = d0.stochastic_sample()
            lp0 = d0.log_prob(act).numpy()
        act = act.numpy().astype(np.float32)
        old_logp = (lp0 + rng.normal(0, 0.3, B)).astype(np.float32)
        adv = rng.normal(0, 1, B).astype(np.float32)
        ret = rng.normal(0, 1, B).astype(np.float32)
        val = rng.normal(0, 1, B).astype(np.float32)
        _sd(tag + "/sd0/", policy, out)
        opt = torch.optim.Adam(policy.parameters(), 4e-4, eps=1e-5)
        sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.0, total_iters=1000)
        cap = {}
        head_mod = policy.actor.model if discrete else policy.actor.mu

        def hook_head(m, i, o):
            o.retain_grad()
            cap["head"] = o

        def hook_v(m, i, o):
            o.retain_grad()
            cap["v"] = o
        h1 = head_mod.register_forward_hook(hook_head)
        h2 = policy.critic.register_forward_hook(hook_v)
        if not discrete:
            h3 = policy.actor.logstd.register_hook(lambda g: cap.__setitem__("dlogstd", g.clone()))
        ent_coef = 0.01
        if algo == "ppo":
            learner = PPOCLIP_Learner(policy, opt, sch, "cpu", "./", vf_coef=0.25, ent_coef=ent_coef, clip_range=0.2,
                                      clip_grad_norm=0.5, use_grad_clip=True)
            info = learner.update(obs, act, ret, val, adv, old_logp)
        else:
            learner = A2C_Learner(policy, opt, sch, "cpu", "./", vf_coef=0.25, ent_coef=ent_coef, clip_grad=0.5)
            info = learner.update(obs, act, ret, adv)
        h1.remove()
        h2.remove()
        if not discrete:
            h3.remove()
            out[tag + "/dlogstd"] = cap["dlogstd"].numpy()
            out[tag + "/logstd0"] = out[tag + "/sd0/actor.logstd"]
        out[tag + "/obs"] = obs
        out[tag + "/act"] = act
        out[tag + "/old_logp"] = old_logp
        out[tag + "/adv"] = adv
        out[tag + "/ret"] = ret
        out[tag + "/val"] = val
        out[tag + "/head"] = cap["head"].detach().numpy()
        out[tag + "/dhead"] = cap["head"].grad.numpy()
        out[tag + "/v"] = cap["v"].detach().numpy()
        out[tag + "/dv"] = cap["v"].grad.numpy()
        for k, v in info.items():
            out[tag + "/info/" + k] = np.asarray(float(v))
        _sd(tag + "/sd1/", policy, out)
    np.savez_compressed(os.path.join(HERE, "loss.npz"), **out)
    print("loss.npz", len(out))


# ----------------------------------------------------------------------------------------------
def capture_agent(algo, discrete, D, A, N=8, T=128, iters=2, max_ep=50, seed=7):
    tag = "agent_%s_%s" % (algo, "cat" if discrete else "gauss")
    cfg = types.SimpleNamespace(render=False, n_steps=T, n_minibatch=4, n_epoch=2, gamma=0.99, gae_lambda=0.95,
                                env_name="SynthBox", use_gae=True, use_advnorm=True, device="cpu", model_dir="./models/",
                                log_dir="./logs/", vf_coef=0.25, ent_coef=0.01, clip_range=0.2, clip_grad_norm=0.5,
                                use_grad_clip=True, clip_grad=0.5, use_obsnorm=True, use_rewnorm=True,
                                obsnorm_range=5, rewnorm_range=5, seed=seed, logger="tensorboard", test_mode=False)
    np.random.seed(seed)
    torch.manual_seed(seed)
    spaces = (gym.spaces.Box(-1, 1, (D,)), gym.spaces.Discrete(A) if discrete else gym.spaces.Box(-1, 1, (A,)))
    envs = DummyVecEnv_Gym([(lambda i=i: SynthBoxEnv(D, A, seed=seed, env_index=i, discrete=discrete,
                                                     max_episode_steps=max_ep, spaces=spaces)) for i in range(N)])
    policy = _policy(D, A, discrete, seed=seed)
    out = {}
    _sd("sd0/", policy, out)
    opt = torch.optim.Adam(policy.parameters(), 4e-4, eps=1e-5)
    sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.0, total_iters=10000)
    Agent = PPOCLIP_Agent if algo == "ppo" else A2C_Agent
    agent = Agent(cfg, envs, policy, opt, sch, "cpu")
    envs.reset()
    rec = {"closed": np.zeros((iters, N, T), np.uint8), "boot": np.zeros((iters, N, T), np.float32)}
    snaps, perms, infos = [], [], []
    mem = agent.memory
    it = {"k": 0}
    orig_fp, orig_clear, orig_update = mem.finish_path, mem.clear, agent.learner.update
    orig_shuffle = np.random.shuffle

    def finish_path(val, i):
        end = mem.n_size if mem.full else mem.ptr
        if end > mem.start_ids[i] and it["k"] < iters:
            rec["closed"][it["k"], i, end - 1] = 1
            rec["boot"][it["k"], i, end - 1] = val
        return orig_fp(val, i)

    def clear():
        snaps.append({"obs": mem.observations.copy(), "act": mem.actions.copy(), "rew": mem.rewards.copy(),
                      "val": mem.values.copy(), "term": mem.terminals.copy(), "ret": mem.returns.copy(),
                      "adv": mem.advantages.copy(),
                      "logp": mem.auxiliary_infos["old_logp"].copy() if algo == "ppo" else np.zeros((N, T), np.float32)})
        it["k"] += 1
        return orig_clear()

    def update(*a):
        info = orig_update(*a)
        infos.append([float(info[k]) for k in ("actor-loss", "critic-loss", "entropy", "learning_rate",
                                                "predict_value")] + [float(info.get("clip_ratio", np.nan))])
        return info

    def shuffle(x):
        orig_shuffle(x)
        perms.append(x.copy())

    mem.finish_path, mem.clear, agent.learner.update = finish_path, clear, update
    np.random.shuffle = shuffle
    try:
        agent.train(iters * T)
    finally:
        np.random.shuffle = orig_shuffle
    for k in ("obs", "act", "rew", "val", "term", "ret", "adv", "logp"):
        out[k] = np.stack([s[k] for s in snaps])
    out["closed"], out["boot"] = rec["closed"], rec["boot"]
    out["perms"] = np.stack(perms).astype(np.int64)
    out["infos"] = np.asarray(infos, np.float64)
    out["config"] = np.asarray([N, T, D, A, cfg.n_epoch, cfg.n_minibatch, int(discrete), max_ep, seed], np.int64)
    _sd("sd1/", policy, out)
    np.savez_compressed(os.path.join(HERE, tag + ".npz"), **out)
    print(tag, len(out), "closures", int(out["closed"].sum()))


# ----------------------------------------------------------------------------------------------
def capture_rms(seed=3):
    rng = np.random.default_rng(seed)
    out = {}
    rms = RunningMeanStd((5,), comm=None, use_mpi=False)
    xs, means, vars_, counts = [], [], [], []
    for k in range(20):
        x = (rng.normal(0, 1, (64, 5)) * (1 + k % 3) + k * 0.1).astype(np.float32)
        rms.update(x)
        xs.append(x)
        means.append(rms.mean.copy())
        vars_.append(rms.var.copy())
        counts.append(rms.count)
    out["obs/x"], out["obs/mean"], out["obs/var"] = np.stack(xs), np.stack(means), np.stack(vars_)
    out["obs/count"] = np.asarray(counts, np.float64)
    ret = RunningMeanStd((), comm=None, use_mpi=False)
    rs = rng.normal(0, 3, 200).astype(np.float32)
    rm, rv = [], []
    for r in rs:
        ret.update(np.asarray([r], np.float32))
        rm.append(float(ret.mean))
        rv.append(float(ret.var))
    out["ret/x"], out["ret/mean"], out["ret/var"] = rs, np.asarray(rm), np.asarray(rv)
    np.savez_compressed(os.path.join(HERE, "rms.npz"), **out)
    print("rms.npz", len(out))


# ----------------------------------------------------------------------------------------------
def capture_per():
    import random
    import xuance.common.memory_tools as mt
    out = {}
    cases = [("small", 2, 100, 32, 0.6, [40, 40, 40], 0.4), ("wrap", 1, 300, 16, 0.5, [290, 20], 0.7)]
    for tag, n_envs, n_size, batch, alpha, stores, beta in cases:
        rng = np.random.default_rng(11)
        random.seed(5)
        uniforms = []
        orig = random.random

        def rec():
            u = orig()
            uniforms.append(u)
            return u
        mt.random.random = rec
        buf = mt.PerOffPolicyBuffer(gym.spaces.Box(-1, 1, (3,)), gym.spaces.Discrete(4), {}, n_envs, n_size, batch,
                                    alpha)
        cap = buf._it_sum[0]._capacity
        pre = "%s/" % tag
        out[pre + "config"] = np.asarray([n_envs, n_size, batch, cap], np.int64)
        out[pre + "alpha_beta"] = np.asarray([alpha, beta], np.float64)
        step_obs, step_act, step_rew, step_term, step_next = [], [], [], [], []
        for r, n_store in enumerate(stores):
            for _ in range(n_store):
                o = rng.normal(0, 1, (n_envs, 3)).astype(np.float32)
                a = rng.integers(0, 4, n_envs)
                rw = rng.normal(0, 1, n_envs).astype(np.float32)
                te = (rng.random(n_envs) < 0.1).astype(np.float32)
                nx = rng.normal(0, 1, (n_envs, 3)).astype(np.float32)
                buf.store(o, a, rw, te, nx)
                step_obs.append(o), step_act.append(a), step_rew.append(rw), step_term.append(te), step_next.append(nx)
            pr = "%sr%d/" % (pre, r)
            out[pr + "n_store"] = np.asarray(n_store)
            out[pr + "tree_sum_after_store"] = np.stack([np.asarray(t._value, np.float64) for t in buf._it_sum])
            out[pr + "tree_min_after_store"] = np.stack([np.asarray(t._value, np.float64) for t in buf._it_min])
            n_u = len(uniforms)
            ob, ac, rw, te, nx, w, idx = buf.sample(beta)
            out[pr + "uniforms"] = np.asarray(uniforms[n_u:], np.float64)
            out[pr + "step_choices"] = np.asarray(idx)
            out[pr + "weights"] = np.asarray(w, np.float64)
            out[pr + "obs"], out[pr + "act"], out[pr + "rew"] = ob, ac, rw
            out[pr + "term"], out[pr + "next"] = te, nx
            prio = (rng.random(batch) * 2.0).astype(np.float32)
            prio[::7] = 0.0
            out[pr + "priorities"] = prio
            # The sampled indices are uint8 (memory_tools.py:465).  Under the pinned NumPy 1.21,
            # `idx += capacity` in SegmentTree.__setitem__ promotes uint8 + int to int64; NumPy 2 raises
            # OverflowError once capacity > 255.  Pass the same (wrapped) values as int64 = NumPy 1.21.
            buf.update_priorities(np.asarray(idx).astype(np.int64), prio)
            out[pr + "tree_sum_after_update"] = np.stack([np.asarray(t._value, np.float64) for t in buf._it_sum])
            out[pr + "tree_min_after_update"] = np.stack([np.asarray(t._value, np.float64) for t in buf._it_min])
            out[pr + "max_priority"] = np.array(buf._max_priority, np.float64, copy=True)
            out[pr + "size_ptr"] = np.asarray([buf.size, buf.ptr], np.int64)
        out[pre + "obs"], out[pre + "act"] = np.stack(step_obs), np.stack(step_act)
        out[pre + "rew"], out[pre + "term"], out[pre + "next"] = np.stack(step_rew), np.stack(step_term), np.stack(step_next)
        mt.random.random = orig
    np.savez_compressed(os.path.join(HERE, "per.npz"), **out)
    print("per.npz", len(out))


# ----------------------------------------------------------------------------------------------
ATARI_NET = dict(filters=[8, 8], kernels=[8, 4], strides=[4, 2], fc_hidden_sizes=[32])  # a small AC_CNN_Atari
# the production nets (a2c/atari.yaml + ppo/atari.yaml's AC_CNN_Atari, perdqn/atari.yaml's Basic_CNN + q 512)
ATARI_PROD_NET = dict(filters=[32, 64, 64], kernels=[8, 4, 3], strides=[4, 2, 1], fc_hidden_sizes=[512])
PERDQN_PROD_NET = dict(filters=[32, 64, 64], kernels=[8, 4, 3], strides=[4, 2, 1], q_hidden=[512])


def _sd_compact(prefix, policy, out):
    """state_dict into out; tensors above fixture_init.BIG elements as every 16th row + per-row f64 sums."""
    from fixture_init import BIG
    for k, v in policy.state_dict().items():
        a = v.detach().cpu().numpy()
        if a.size > BIG:
            out[prefix + k + "::rows16"] = a[::16].copy()
            out[prefix + k + "::rowsum"] = a.reshape(a.shape[0], -1).astype(np.float64).sum(1)
        else:
            out[prefix + k] = a.copy()


def _uniform_init(policy, seed, out):
    """Overwrite the freshly built policy with fixture_init.uniform_state(seed); record seed + checksums."""
    from fixture_init import checksum, uniform_state
    sd = policy.state_dict()
    vals = uniform_state([(k, v.shape) for k, v in sd.items()], seed)
    policy.load_state_dict({k: torch.as_tensor(v) for k, v in vals.items()})
    out["init_seed"] = np.asarray(seed, np.int64)
    for k, v in vals.items():
        out["sd0sum/" + k] = checksum(v)


def capture_atari(N=4, T=16, iters=2, max_ep=20, n_actions=6, seed=5, net=ATARI_NET, n_minibatch=2, n_epoch=2,
                  fname="atari_a2c.npz", init_seed=None, algo="a2c"):
    """G8 / G8P (algo "a2c": a2c/atari.yaml's coefficients) and G12 / G12P (algo "ppo": PPOCLIP_Agent with env_name
    "Atari" and ppo/atari.yaml's lr 2.5e-4, clip_range 0.2, clip_grad_norm 0.5, vf 0.25, ent 0.01 —
    examples/ppo/ppo_atari.py's agent; the buffer's old_logp column and the clip_ratio info are recorded too)."""
    cfg = types.SimpleNamespace(render=False, n_steps=T, n_minibatch=n_minibatch, n_epoch=n_epoch, gamma=0.99,
                                gae_lambda=0.95, env_name="Atari", use_gae=True, use_advnorm=True, device="cpu", model_dir="./models/",
                                log_dir="./logs/", vf_coef=0.25, ent_coef=0.01, clip_grad=0.2, use_obsnorm=False,
                                use_rewnorm=False, obsnorm_range=5, rewnorm_range=5, seed=seed, logger="tensorboard",
                                test_mode=False, clip_range=0.2, clip_grad_norm=0.5, use_grad_clip=True)
    lr = 7e-4 if algo == "a2c" else 2.5e-4
    np.random.seed(seed)
    torch.manual_seed(seed)
    obs_space, act_space = gym.spaces.Box(0, 255, (84, 84, 4)), gym.spaces.Discrete(n_actions)

    class _Env(SynthAtariEnv):   # the reference's env contract: spaces on the instance
        observation_space, action_space = obs_space, act_space

        def close(self):
            pass

    envs = DummyVecEnv_Atari([(lambda i=i: _Env(i, seed=seed, n_actions=n_actions, max_episode_steps=max_ep))
                              for i in range(N)])
    torch.manual_seed(seed)
    rep = AC_CNN_Atari((84, 84, 4), net["kernels"], net["strides"], net["filters"], None,
                       torch.nn.init.orthogonal_, torch.nn.ReLU, "cpu", net["fc_hidden_sizes"])
    policy = Categorical_AC_Policy(act_space, rep, [], [], None, torch.nn.init.orthogonal_, torch.nn.ReLU, "cpu")
    out = {}
    if init_seed is None:
        _sd("sd0/", policy, out)
    else:
        _uniform_init(policy, init_seed, out)
    opt = torch.optim.Adam(policy.parameters(), lr, eps=1e-5)
    sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.0, total_iters=10000)
    agent = (A2C_Agent if algo == "a2c" else PPOCLIP_Agent)(cfg, envs, policy, opt, sch, "cpu")
    envs.reset()
    rec = {"closed": np.zeros((iters, N, T), np.uint8), "boot": np.zeros((iters, N, T), np.float32)}
    snaps, perms, infos, env_acts = [], [], [], []
    mem = agent.memory
    it = {"k": 0}
    orig_fp, orig_clear, orig_update, orig_step = mem.finish_path, mem.clear, agent.learner.update, envs.step
    orig_shuffle = np.random.shuffle

    def finish_path(val, i):
        end = mem.n_size if mem.full else mem.ptr
        if end > mem.start_ids[i] and it["k"] < iters:
            rec["closed"][it["k"], i, end - 1] = 1
            rec["boot"][it["k"], i, end - 1] = val
        return orig_fp(val, i)

    def clear():
        snaps.append({"act": mem.actions.copy(), "rew": mem.rewards.copy(), "val": mem.values.copy(),
                      "term": mem.terminals.copy(), "ret": mem.returns.copy(), "adv": mem.advantages.copy(),
                      "frame_sum": mem.observations.reshape(N, T, -1).astype(np.int64).sum(-1),
                      "obs_dtype_u8": np.asarray(mem.observations.dtype == np.uint8),
                      "old_logp": (mem.auxiliary_infos["old_logp"].copy() if algo == "ppo" else np.zeros(0))})
        it["k"] += 1
        return orig_clear()

    def update(*a):
        info = orig_update(*a)
        infos.append([float(info[k]) for k in ("actor-loss", "critic-loss", "entropy", "learning_rate",
                                                "predict_value") + (("clip_ratio",) if algo == "ppo" else ())])
        return info

    def shuffle(x):
        orig_shuffle(x)
        perms.append(x.copy())

    def step(acts):
        env_acts.append(np.asarray(acts).copy())
        return orig_step(acts)

    mem.finish_path, mem.clear, agent.learner.update, envs.step = finish_path, clear, update, step
    np.random.shuffle = shuffle
    try:
        agent.train(iters * T)
    finally:
        np.random.shuffle = orig_shuffle
    for k in ("act", "rew", "val", "term", "ret", "adv", "frame_sum") + (("old_logp",) if algo == "ppo" else ()):
        out[k] = np.stack([s_[k] for s_ in snaps])
    out["algo"] = np.asarray(0 if algo == "a2c" else 1, np.int64)
    out["hyper"] = np.asarray([lr, cfg.vf_coef, cfg.ent_coef, cfg.clip_range, cfg.clip_grad_norm], np.float64)
    assert all(bool(s_["obs_dtype_u8"]) for s_ in snaps)
    out["closed"], out["boot"] = rec["closed"], rec["boot"]
    out["env_actions"] = np.stack(env_acts).astype(np.int64)
    out["perms"] = np.stack(perms).astype(np.int64)
    out["infos"] = np.asarray(infos, np.float64)
    out["config"] = np.asarray([N, T, n_actions, cfg.n_epoch, cfg.n_minibatch, max_ep, seed], np.int64)
    out["net"] = np.asarray(net["filters"] + net["kernels"] + net["strides"] + net["fc_hidden_sizes"], np.int64)
    _sd_compact("sd1/", policy, out)
    np.savez_compressed(os.path.join(HERE, fname), **out)
    print(fname, len(out), "closures", int(out["closed"].sum()), "life-loss terminals", int(out["term"].sum()))


# ----------------------------------------------------------------------------------------------
PERDQN_NET = dict(filters=[8, 8], kernels=[8, 4], strides=[4, 2], q_hidden=[32])


def perdqn_batch(seed, k, B, A):
    """The k-th update's inputs, regenerated identically by the test (numpy PCG64 is stable)."""
    rng = np.random.default_rng(seed * 1000 + k)
    obs = rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)
    nxt = rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)
    act = rng.integers(0, A, B).astype(np.float32)
    rew = rng.normal(0, 1, B).astype(np.float32)
    term = (rng.random(B) < 0.2).astype(np.float32)
    return obs, act, rew, nxt, term


def capture_perdqn(B=32, A=18, n_updates=4, seed=9, sync=2, gamma=0.99, net=PERDQN_NET, fname="perdqn.npz",
                   every_sd=True):
    from xuance.torch.representations import Basic_CNN
    from xuance.torch.policies import BasicQnetwork
    from xuance.torch.learners import PerDQN_Learner
    torch.manual_seed(seed)
    rep = Basic_CNN((84, 84, 4), net["kernels"], net["strides"], net["filters"], None,
                    torch.nn.init.orthogonal_, torch.nn.ReLU, "cpu")
    policy = BasicQnetwork(gym.spaces.Discrete(A), rep, net["q_hidden"], None, torch.nn.init.orthogonal_,
                           torch.nn.ReLU, "cpu")
    out = {}
    _sd("sd0/", policy, out)
    opt = torch.optim.Adam(policy.parameters(), 1e-3, eps=1e-5)
    sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.5, total_iters=10)
    lrn = PerDQN_Learner(policy, opt, sch, "cpu", "./", gamma, sync)
    tds, infos, sums = [], [], []
    for k in range(n_updates):
        obs, act, rew, nxt, term = perdqn_batch(seed, k, B, A)
        sums.append([int(obs.astype(np.int64).sum()), int(nxt.astype(np.int64).sum())])
        td, info = lrn.update(obs, act, rew, nxt, term)
        tds.append(np.asarray(td, np.float32))
        infos.append([float(info["Qloss"]), float(info["learning_rate"]), float(info["predictQ"])])
        if every_sd or k == n_updates - 1:
            _sd("sd%d/" % (k + 1), policy, out)
    out["td_abs"] = np.stack(tds)
    out["infos"] = np.asarray(infos, np.float64)
    out["input_sums"] = np.asarray(sums, np.int64)
    out["config"] = np.asarray([B, A, n_updates, seed, sync], np.int64)
    out["gamma"] = np.asarray(gamma, np.float64)
    out["net"] = np.asarray(net["filters"] + net["kernels"] + net["strides"] + net["q_hidden"], np.int64)
    np.savez_compressed(os.path.join(HERE, fname), **out)
    print(fname, len(out))


def capture_perdqn_agent(N=4, n_size=128, batch=64, A=18, steps=48, seed=13, max_ep=60, net=PERDQN_PROD_NET,
                         fname="perdqn_agent.npz"):
    """G10: PerDQN_Agent.train (perdqn_agent.py:56-95) on N SynthAtari envs (18 actions, DummyVecEnv_Atari) with the
    production Basic_CNN + q 512: e-greedy draws from np.random (the MT19937 state before train() is recorded, so
    the replay makes the same draws), PerOffPolicyBuffer store / sample(beta) / update_priorities with every
    random.random() uniform recorded, PerDQN_Learner updates with target copies.  Records every env action, every
    update's sampled steps, |TD| priorities and info, the beta / epsilon schedules, the final trees and weights.
    update_priorities receives int64 indices and float64 priorities: the pinned NumPy 1.21 arithmetic
    (np.float32 ** float -> float64 leaves; uint8 + int -> int64), which NumPy 2 would otherwise change."""
    import random
    import xuance.common.memory_tools as mt
    from xuance.torch.representations import Basic_CNN
    from xuance.torch.policies import BasicQnetwork
    from xuance.torch.agents import PerDQN_Agent
    cfg = types.SimpleNamespace(render=False, training_frequency=1, start_training=64, start_greedy=0.5,
                                end_greedy=0.05, decay_step_greedy=200, PER_beta0=0.4, env_name="Atari",
                                n_size=n_size, batch_size=batch, PER_alpha=0.5, device="cpu", model_dir="./models/",
                                log_dir="./logs/", gamma=0.99, sync_frequency=5, use_obsnorm=False,
                                use_rewnorm=False, obsnorm_range=5, rewnorm_range=5, seed=seed, logger="tensorboard",
                                test_mode=False)
    obs_space, act_space = gym.spaces.Box(0, 255, (84, 84, 4)), gym.spaces.Discrete(A)

    class _Env(SynthAtariEnv):
        observation_space, action_space = obs_space, act_space

        def close(self):
            pass
    envs = DummyVecEnv_Atari([(lambda i=i: _Env(i, seed=seed, n_actions=A, max_episode_steps=max_ep))
                              for i in range(N)])
    torch.manual_seed(seed)
    rep = Basic_CNN((84, 84, 4), net["kernels"], net["strides"], net["filters"], None, torch.nn.init.orthogonal_,
                    torch.nn.ReLU, "cpu")
    policy = BasicQnetwork(act_space, rep, net["q_hidden"], None, torch.nn.init.orthogonal_, torch.nn.ReLU, "cpu")
    out = {}
    _sd("sd0/", policy, out)
    opt = torch.optim.Adam(policy.parameters(), 1e-4, eps=1e-5)
    sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.5, total_iters=100)
    agent = PerDQN_Agent(cfg, envs, policy, opt, sch, "cpu")
    envs.reset()
    mem = agent.memory
    uniforms, env_acts, upd = [], [], {"steps": [], "td": [], "info": [], "beta": [], "u0": []}
    sched = {"beta": [], "eps": []}
    orig_rand, orig_step = random.random, envs.step
    orig_sample, orig_update, orig_prio = mem.sample, agent.learner.update, mem.update_priorities

    def rec_rand():
        u = orig_rand()
        uniforms.append(u)
        return u

    def step(acts):
        env_acts.append(np.asarray(acts).astype(np.int64).copy())
        sched["beta"].append(agent.PER_beta)
        sched["eps"].append(agent.egreedy)
        return orig_step(acts)

    def sample(beta):
        upd["beta"].append(beta)
        upd["u0"].append(len(uniforms))
        res = orig_sample(beta)
        upd["steps"].append(np.asarray(res[-1]).astype(np.int64).copy())
        return res

    def update(*a):
        td, info = orig_update(*a)
        upd["td"].append(np.asarray(td, np.float32).copy())
        upd["info"].append([float(info["Qloss"]), float(info["learning_rate"]), float(info["predictQ"])])
        return td, info

    def update_priorities(idxes, priorities):
        return orig_prio(np.asarray(idxes).astype(np.int64), np.asarray(priorities).astype(np.float64))

    mt.random.random = rec_rand
    envs.step = step
    mem.sample, agent.learner.update, mem.update_priorities = sample, update, update_priorities
    np.random.seed(seed)
    st = np.random.get_state()
    out["np_state_keys"] = np.asarray(st[1], np.uint32)
    out["np_state_pos"] = np.asarray([st[2], st[3]], np.int64)
    out["np_state_gauss"] = np.asarray(st[4], np.float64)
    try:
        agent.train(steps)
    finally:
        mt.random.random = orig_rand
    n_up = len(upd["td"])
    assert n_up > 10, n_up
    b = batch // N
    out["env_actions"] = np.stack(env_acts)
    out["sched_beta"], out["sched_eps"] = np.asarray(sched["beta"]), np.asarray(sched["eps"])
    out["upd_steps"] = np.stack(upd["steps"])
    out["upd_td"] = np.stack(upd["td"])
    out["upd_info"] = np.asarray(upd["info"], np.float64)
    out["upd_beta"] = np.asarray(upd["beta"], np.float64)
    out["upd_uniforms"] = np.stack([np.asarray(uniforms[u0:u0 + batch], np.float64).reshape(N, b)
                                    for u0 in upd["u0"]])
    assert len(uniforms) == n_up * batch
    out["tree_sum"] = np.stack([np.asarray(t._value, np.float64) for t in mem._it_sum])
    out["tree_min"] = np.stack([np.asarray(t._value, np.float64) for t in mem._it_min])
    out["max_priority"] = np.array(mem._max_priority, np.float64, copy=True)
    out["size_ptr"] = np.asarray([mem.size, mem.ptr], np.int64)
    out["final_beta_eps"] = np.asarray([agent.PER_beta, agent.egreedy], np.float64)
    out["config"] = np.asarray([N, n_size, batch, A, steps, seed, max_ep, cfg.start_training, cfg.sync_frequency,
                                cfg.decay_step_greedy], np.int64)
    out["hyper"] = np.asarray([cfg.start_greedy, cfg.end_greedy, cfg.PER_beta0, cfg.PER_alpha, cfg.gamma, 1e-4, 0.5],
                              np.float64)
    out["net"] = np.asarray(net["filters"] + net["kernels"] + net["strides"] + net["q_hidden"], np.int64)
    _sd("sd1/", policy, out)
    np.savez_compressed(os.path.join(HERE, fname), **out)
    print(fname, len(out), "updates", n_up)


# ----------------------------------------------------------------------------------------------
# G11: the reference's own train() loop over its own host VecEnvs (round 5).  PPOCLIP_Agent.train / A2C_Agent.train
# (ppoclip_agent.py:59-111, a2c_agent.py:57-107) over DummyVecEnv_Gym / DummyVecEnv_Atari / SubprocVecEnv_Gym
# (gym_vec_env.py:40-231) of SynthBox / SynthAtari thunks, split into several train() calls whose boundaries fall on
# done steps.  Recorded: every action handed to envs.step (the oracle loop is fed them: the reference samples torch's
# CPU generator), and at every full-buffer point (mem.clear, after the learner's updates) the whole buffer, every
# closure and bootstrap, the obs / return RunningMeanStd state, the return tracker, and the post-update weights
# (the oracle loads them there, so the fixture pins the LOOP; the learner is pinned by G3-G5).  At the end: the RMS
# state and tracker again.
VEC_CASES = {
    # name: (algo, discrete, D / K, A, N, T, max_ep, obsnorm, calls, vec)
    "ppo_gauss_norm": ("ppo", False, 5, 3, 8, 16, 5, True, (5, 5, 6, 16), "dummy"),
    "ppo_gauss_raw": ("ppo", False, 5, 3, 8, 16, 5, False, (5, 5, 6, 16), "dummy"),
    "a2c_cat_norm": ("a2c", True, 5, 4, 8, 16, 5, True, (5, 5, 6, 16), "dummy"),
    "ppo_gauss_raw_subproc": ("ppo", False, 5, 3, 8, 16, 5, False, (5, 5, 6, 16), "subproc"),
    "atari_a2c": ("a2c", True, None, 6, 8, 32, 40, False, (17, 15, 32), "atari"),
}
VEC_ATARI_NET = dict(filters=[8, 8], kernels=[8, 4], strides=[4, 2], fc_hidden_sizes=[16])


class _VecBox(SynthBoxEnv):
    """SynthBoxEnv with the reference's env contract (spaces set by the ctor; close()); module level so that
    SubprocVecEnv_Gym's spawned workers can unpickle the thunks."""

    def close(self):
        pass


def _vec_box_thunk(D, A, seed, i, discrete, max_ep):
    spaces = (gym.spaces.Box(-1, 1, (D,)), gym.spaces.Discrete(A) if discrete else gym.spaces.Box(-1, 1, (A,)))
    return _VecBox(D, A, seed=seed, env_index=i, discrete=discrete, max_episode_steps=max_ep, spaces=spaces)


def capture_vecloop(name, seed=11):
    import functools
    algo, discrete, D, A, N, T, max_ep, obsnorm, calls, vec = VEC_CASES[name]
    atari = vec == "atari"
    cfg = types.SimpleNamespace(render=False, n_steps=T, n_minibatch=4, n_epoch=2, gamma=0.99, gae_lambda=0.95,
                                env_name="Atari" if atari else "SynthBox", use_gae=True, use_advnorm=True, device="cpu",
                                model_dir="./models/", log_dir="./logs/", vf_coef=0.25, ent_coef=0.01, clip_range=0.2,
                                clip_grad_norm=0.5, use_grad_clip=True, clip_grad=0.5, use_obsnorm=obsnorm,
                                use_rewnorm=obsnorm, obsnorm_range=5, rewnorm_range=5, seed=seed, logger="tensorboard",
                                test_mode=False)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if atari:
        obs_space, act_space = gym.spaces.Box(0, 255, (84, 84, 4)), gym.spaces.Discrete(A)

        class _Env(SynthAtariEnv):
            observation_space, action_space = obs_space, act_space

            def close(self):
                pass
        envs = DummyVecEnv_Atari([(lambda i=i: _Env(i, seed=seed, n_actions=A, max_episode_steps=max_ep))
                                  for i in range(N)])
        net = VEC_ATARI_NET
        rep = AC_CNN_Atari((84, 84, 4), net["kernels"], net["strides"], net["filters"], None,
                           torch.nn.init.orthogonal_, torch.nn.ReLU, "cpu", net["fc_hidden_sizes"])
        policy = Categorical_AC_Policy(act_space, rep, [], [], None, torch.nn.init.orthogonal_, torch.nn.ReLU, "cpu")
    else:
        thunks = [functools.partial(_vec_box_thunk, D, A, seed, i, discrete, max_ep) for i in range(N)]
        if vec == "subproc":
            from xuance.environment.gym.gym_vec_env import SubprocVecEnv_Gym
            envs = SubprocVecEnv_Gym(thunks)
        else:
            envs = DummyVecEnv_Gym(thunks)
        policy = _policy(D, A, discrete, seed=seed)
    out = {}
    _sd("sd0/", policy, out)
    opt = torch.optim.Adam(policy.parameters(), 4e-4, eps=1e-5)
    sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.0, total_iters=10000)
    agent = (PPOCLIP_Agent if algo == "ppo" else A2C_Agent)(cfg, envs, policy, opt, sch, "cpu")
    envs.reset()
    iters = sum(calls) // T
    rec = {"closed": np.zeros((iters, N, T), np.uint8), "boot": np.zeros((iters, N, T), np.float32)}
    snaps, env_acts = [], []
    mem = agent.memory
    it = {"k": 0}
    orig_fp, orig_clear, orig_step = mem.finish_path, mem.clear, envs.step

    def rms_state():
        return {"obs_mean": np.array(agent.obs_rms.mean, np.float64, copy=True),
                "obs_var": np.array(agent.obs_rms.var, np.float64, copy=True),
                "obs_count": np.asarray(agent.obs_rms.count, np.float64),
                "ret_mean": np.asarray(agent.ret_rms.mean, np.float64), "ret_var": np.asarray(agent.ret_rms.var, np.float64),
                "ret_count": np.asarray(agent.ret_rms.count, np.float64),
                "returns": np.array(agent.returns, np.float32, copy=True)}

    def finish_path(val, i):
        end = mem.n_size if mem.full else mem.ptr
        if end > mem.start_ids[i] and it["k"] < iters:
            rec["closed"][it["k"], i, end - 1] = 1
            rec["boot"][it["k"], i, end - 1] = val
        return orig_fp(val, i)

    def clear():
        s_ = {"act": mem.actions.copy(), "rew": mem.rewards.copy(), "val": mem.values.copy(),
              "term": mem.terminals.copy(), "ret": mem.returns.copy(), "adv": mem.advantages.copy(),
              "logp": mem.auxiliary_infos["old_logp"].copy() if algo == "ppo" else np.zeros((N, T), np.float32)}
        if atari:
            s_["frame_sum"] = mem.observations.reshape(N, T, -1).astype(np.int64).sum(-1)
        else:
            s_["obs"] = mem.observations.copy()
        s_.update(rms_state())
        for k_, v_ in policy.state_dict().items():
            s_["sd/" + k_] = v_.detach().cpu().numpy().copy()
        snaps.append(s_)
        it["k"] += 1
        return orig_clear()

    def step(acts):
        env_acts.append(np.asarray(acts).copy())
        return orig_step(acts)

    mem.finish_path, mem.clear, envs.step = finish_path, clear, step
    try:
        for k_ in calls:
            agent.train(k_)
    finally:
        if vec == "subproc":
            envs.close()
    assert len(snaps) == iters
    for k_ in snaps[0]:
        out["it/" + k_] = np.stack([s_[k_] for s_ in snaps])
    for k_, v_ in rms_state().items():
        out["end/" + k_] = v_
    out["closed"], out["boot"] = rec["closed"], rec["boot"]
    out["env_actions"] = np.stack(env_acts)
    out["calls"] = np.asarray(calls, np.int64)
    out["config"] = np.asarray([N, T, D or 0, A, max_ep, int(obsnorm), int(discrete), seed, cfg.n_epoch,
                                cfg.n_minibatch], np.int64)
    fname = "vecloop_%s.npz" % name
    np.savez_compressed(os.path.join(HERE, fname), **out)
    mid = (out["closed"][:, :, :T - 1] != 0) & (out["it/term"][:, :, :T - 1] == 0)
    print(fname, len(out), "closures", int(out["closed"].sum()), "mid truncations", int(mid.sum()),
          "terminals", int(out["it/term"].sum()))


if __name__ == "__main__":
    os.makedirs("/tmp/xref_run", exist_ok=True)
    os.chdir("/tmp/xref_run")
    which = set(sys.argv[1:]) or {"base"}
    if "base" in which:
        capture_gae()
        capture_loss()
        capture_agent("ppo", False, 17, 6)
        capture_agent("a2c", True, 4, 2)
        capture_rms()
        capture_per()
        capture_atari()
        capture_perdqn()
    if "prod" in which:   # round 3: the production CNN nets (G8P, G9P) and the PerDQN agent loop (G10)
        torch.set_num_threads(8)
        capture_atari(N=8, T=64, iters=2, max_ep=40, net=ATARI_PROD_NET, n_minibatch=2, n_epoch=2,
                      fname="atari_a2c_prod.npz", init_seed=21)
        capture_perdqn(B=2048, n_updates=3, seed=23, sync=2, net=PERDQN_PROD_NET, fname="perdqn_prod.npz",
                       every_sd=False)
        capture_perdqn_agent()
    if "ppo_atari" in which:   # round 6: G12 / G12P, examples/ppo/ppo_atari.py's PPOCLIP_Agent on Atari frames
        torch.set_num_threads(8)
        capture_atari(N=4, T=16, iters=2, max_ep=20, n_minibatch=4, n_epoch=4, fname="atari_ppo.npz", algo="ppo")
        capture_atari(N=8, T=64, iters=2, max_ep=40, net=ATARI_PROD_NET, n_minibatch=4, n_epoch=4,
                      fname="atari_ppo_prod.npz", init_seed=27, algo="ppo")
    if "vecloop" in which:   # round 5: G11
        for name in VEC_CASES:
            capture_vecloop(name)
