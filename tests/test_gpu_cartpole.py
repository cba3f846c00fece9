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
        agent.learner.small_updates = False   # the multi-kernel slot graphs (K30 has its own test)
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


def test_graphed_updates_ragged_last_minibatch():
    """N*T = 800 rows in minibatches of 133: six full slots and a ragged 2-row slot per epoch.  The agent keeps one
    gather buffer per minibatch size, so the slot graphs are keyed by stable pointers: 7 graphs after three
    iterations (no growth), and the parameters equal the eager run's."""
    from xuanpolicy_amd.runner import build_cartpole_ppo
    out = []
    for graphed in (False, True):
        agent = build_cartpole_ppo(n_envs=8, n_steps=100, hidden=64, seed=6, device=DEV, graph_update=graphed,
                                   n_minibatch=6, n_epoch=2)
        agent.learner.small_updates = False
        assert agent.batch_size == 133
        for _ in range(3):
            agent.train(100, log=False)
        torch.cuda.synchronize()
        graphs = getattr(agent.learner, "_slot_graphs", {})
        assert len(graphs) == (7 if graphed else 0), len(graphs)
        assert sum(isinstance(v, tuple) for v in graphs.values()) == (7 if graphed else 0)
        out.append([p.detach().cpu().numpy().copy() for p in agent.policy.parameters()])
    for a, b in zip(*out):
        np.testing.assert_allclose(b, a, rtol=1e-6, atol=1e-7)


def test_graph_capture_failure_falls_back_to_eager():
    """A launch failing inside the slot capture (after the backward queued its column-sum finalizes): the learner
    drops the aborted capture's queued work and workspaces, reruns the update eagerly and stays eager — the
    parameters equal the eager run's (stale finalizes must not be flushed into the eager update)."""
    from xuanpolicy_amd import ops
    from xuanpolicy_amd.runner import build_cartpole_ppo
    out = []
    for inject in (False, True):
        agent = build_cartpole_ppo(n_envs=8, n_steps=128, hidden=64, seed=4, device=DEV, graph_update=inject)
        agent.learner.small_updates = False
        if inject:
            fm = agent.learner._fused_mlp()
            real = ops.ColsumQueue.flush
            state = {"raised": 0}

            def flaky(self, *a, **k):
                if torch.cuda.is_current_stream_capturing() and not state["raised"]:
                    state["raised"] = 1
                    assert self.items, "the injected failure must find queued finalizes"
                    raise RuntimeError("injected capture failure")
                return real(self, *a, **k)
            fm._cq.flush = flaky.__get__(fm._cq)
        for _ in range(2):
            agent.train(128, log=False)
        torch.cuda.synchronize()
        if inject:
            assert state["raised"] == 1 and agent.learner._graph_failed
            assert not any(isinstance(v, tuple) for v in agent.learner._slot_graphs.values())
        out.append([p.detach().cpu().numpy().copy() for p in agent.policy.parameters()])
    for a, b in zip(*out):
        np.testing.assert_allclose(b, a, rtol=1e-6, atol=1e-7)


def test_epoch_graph_capture_failure_falls_back_to_slot_graphs():
    """a failure inside the whole-epoch capture (learners.update_epoch, after every slot graph exists)
    restores the learner's workspace / partial buffers and continues on the slot graphs — the parameters equal a run
    that never tried the epoch graph."""
    from xuanpolicy_amd import ops
    from xuanpolicy_amd.runner import build_cartpole_ppo
    out = []
    for inject in (False, True):
        agent = build_cartpole_ppo(n_envs=8, n_steps=100, hidden=64, seed=4, device=DEV, n_minibatch=6, n_epoch=4)
        agent.learner.small_updates = False
        fm = agent.learner._fused_mlp()
        state = {"raised": 0}
        if inject:
            real = ops.ColsumQueue.flush

            def flaky(self, *a, **k):
                slots = agent.learner.__dict__.get("_slot_graphs", {})
                if (torch.cuda.is_current_stream_capturing() and not state["raised"]
                        and sum(isinstance(v, tuple) for v in slots.values()) == 7):
                    state["raised"] = 1
                    raise RuntimeError("injected epoch-capture failure")
                return real(self, *a, **k)
            fm._cq.flush = flaky.__get__(fm._cq)
        else:
            agent.learner.graph_epochs = False
        for _ in range(2):
            agent.train(100, log=False)
        torch.cuda.synchronize()
        assert not agent.learner.graph_epochs
        assert not agent.learner.__dict__.get("_epoch_graphs")
        if inject:
            assert state["raised"] == 1 and not getattr(agent.learner, "_graph_failed", False)
        out.append([p.detach().cpu().numpy().copy() for p in agent.policy.parameters()])
    for a, b in zip(*out):
        np.testing.assert_allclose(b, a, rtol=1e-6, atol=1e-7)


def test_graphed_k9_schedule_windows(monkeypatch):
    """K9 captured in the slot graphs reads (lr, Adam step) from the device schedule (xpa_clip_adam_step_sched): with a
    24-update window the table is refilled five times inside two iterations (128 updates) and the LinearLR decay is
    live; the parameters, the Adam step count and the host learning rate equal the eager run's (host K9 arguments),
    and no launch ran past its window."""
    from xuanpolicy_amd import flat
    from xuanpolicy_amd.runner import build_cartpole_ppo
    monkeypatch.setattr(flat.FusedClipAdam, "SCHED_WINDOW", 24)
    out, lrs, steps = [], [], []
    for graphed in (False, True):
        agent = build_cartpole_ppo(n_envs=8, n_steps=128, hidden=64, seed=5, device=DEV, graph_update=graphed)
        agent.learner.small_updates = False
        for _ in range(2):
            agent.train(128, log=False)
        torch.cuda.synchronize()
        fo = agent.learner.fused_opt
        assert fo.sched_enabled == graphed
        if graphed:
            assert not fo.sched_overflow()
            assert sum(isinstance(v, tuple) for v in agent.learner._slot_graphs.values()) == 8
            assert len(agent.learner._epoch_graphs) == 1   # epochs 3-16 replay one whole-epoch graph
        out.append([p.detach().cpu().numpy().copy() for p in agent.policy.parameters()])
        lrs.append(agent.learner.optimizer.param_groups[0]["lr"])
        steps.append(fo.step_count)
    assert steps[0] == steps[1] == 128
    assert lrs[0] == lrs[1] and lrs[0] < agent.config.learning_rate
    for a, b in zip(*out):
        np.testing.assert_allclose(b, a, rtol=1e-6, atol=1e-7)


def test_small_mlp_update_matches_multi_kernel_path():
    """K30 (xpa_small_mlp_update: gather + forward + loss + backward + clip + Adam in one launch) against the
    multi-kernel update (K13 / hipBLASLt / K2 / K10 / K9) from the same start: every update's loss scalars and the
    parameters after one iteration (64 updates), within the f32 reassociation of the two paths."""
    from xuanpolicy_amd.runner import build_cartpole_ppo
    res = []
    for small in (True, False):
        agent = build_cartpole_ppo(n_envs=8, n_steps=128, hidden=64, seed=7, device=DEV)
        agent.learner.small_updates = small
        agent.update_log = []
        agent.train(128, log=False)
        torch.cuda.synchronize()
        assert agent.learner.small_update_ok(agent.memory.observations.reshape(1024, -1), 128) == small
        res.append(([u.cpu().numpy() for u in agent.update_log],
                    [p.detach().cpu().numpy().copy() for p in agent.policy.parameters()]))
    (log_s, par_s), (log_m, par_m) = res
    assert len(log_s) == len(log_m) == 64
    for u, (a, b) in enumerate(zip(log_s, log_m)):
        np.testing.assert_allclose(a[:6], b[:6], rtol=1e-4, atol=1e-5, err_msg="update %d" % u)
    for a, b in zip(par_s, par_m):
        np.testing.assert_allclose(a, b, rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("n_steps,n_mb", [(128, 8), (100, 7)])
def test_small_mlp_epoch_graphs_match_eager(n_steps, n_mb):
    """K30 epochs captured as one graph (learners.small_epoch: eager the first epoch of a layout, captured the second,
    replayed after) give the eager K30 run's parameters bit for bit — including a ragged last minibatch (800 rows in
    minibatches of 114: seven full ones and one of 2 rows) — and the schedule cursor never runs past its window."""
    from xuanpolicy_amd.runner import build_cartpole_ppo
    out = []
    for graphed in (False, True):
        agent = build_cartpole_ppo(n_envs=8, n_steps=n_steps, hidden=64, seed=4, device=DEV, graph_update=graphed,
                                   n_minibatch=n_mb, n_epoch=4)
        for _ in range(3):
            agent.train(n_steps, log=False)
        torch.cuda.synchronize()
        assert agent.learner.small_update_ok(agent.memory.observations.reshape(8 * n_steps, -1), agent.batch_size)
        graphs = getattr(agent.learner, "_small_graphs", {})
        assert sum(isinstance(v, tuple) for v in graphs.values()) == (1 if graphed else 0)
        assert not agent.learner.fused_opt.sched_overflow()
        out.append([p.detach().cpu().numpy().copy() for p in agent.policy.parameters()])
    for a, b in zip(*out):
        np.testing.assert_array_equal(b, a)


@pytest.mark.parametrize("agent_name,hidden,obsnorm,n_envs", [("PPO_Clip", 64, True, 8), ("A2C", 64, True, 8),
                                                               ("PPO_Clip", 32, True, 8), ("PPO_Clip", 64, False, 8),
                                                               ("PPO_Clip", 64, True, 100), ("A2C", 64, True, 256)])
def test_fused_rollout_matches_multi_kernel_steps(agent_name, hidden, obsnorm, n_envs):
    """K32 (xpa_small_rollout_cartpole: obs RMS + normalise + MLP forward + sample + CartPole step + K8 post in one
    launch) against the multi-kernel step (K5, obs_normalize, the torch forward, K3, K18, K8) from the same start:
    iteration 1's 128 steps as ONE K32 launch, then an update, then 127 single-step launches (time limit 40: mid-buffer
    truncations fill the deferred slots).  n_envs 100 / 256 run K32's N > 64 branches (the row-group obs-RMS sums and
    the block-sum ret_rms merge); A2C keeps the reset observations in its slots (a2c_agent.py:88-95) on both paths.
    Everything but the forward is the same arithmetic, so the actions, buffer
    observations, rewards / closures, slots, RMS statistics, returns and env state are bit-identical; the stored
    values / log-probs agree within the f32 reassociation of the two forwards."""
    from xuanpolicy_amd.runner import build_cartpole_ppo
    res = []
    for fused in (True, False):
        agent = build_cartpole_ppo(n_envs=n_envs, n_steps=128, hidden=hidden, seed=9, device=DEV, max_episode_steps=40,
                                   agent=agent_name, fused_rollout=fused, clip_grad=0.5, use_obsnorm=obsnorm)
        assert agent.defer_boot and agent.n_slots == 4
        agent.train(128 + 127, log=False)
        torch.cuda.synchronize()
        assert (agent._small_rollout() is not None) == fused
        mem, env = agent.memory, agent.envs
        logp = mem.auxiliary_infos["old_logp"] if agent.algo == "ppo" else agent.logp_scratch
        res.append({k: v.detach().cpu().numpy().copy() for k, v in dict(
            obs=mem.observations, act=mem.actions, rew=mem.rewards, term=mem.terminals, closed=mem.closed,
            boot=mem.boot, slot_t=agent.slot_t, slot_obs=agent.slot_obs, boot_obs=agent.boot_obs,
            obs_mean=agent.obs_mean, obs_var=agent.obs_var, obs_count=agent.obs_count, ret_mean=agent.ret_mean,
            ret_var=agent.ret_var, ret_count=agent.ret_count, returns=agent.returns, state=env.state,
            ep_index=env.ep_index, ep_score=env.ep_score, cursor=agent.cursor, obs_norm=agent.obs_norm,
            val=mem.values, logp=logp).items()})
    f, m = res
    assert (f["slot_t"] >= 0).sum() > 0 and f["closed"][:, :127].sum() > n_envs
    for k in f:
        if k in ("val", "logp"):
            np.testing.assert_allclose(f[k][:, :127], m[k][:, :127], rtol=1e-4, atol=1e-5, err_msg=k)
        else:
            np.testing.assert_array_equal(f[k], m[k], err_msg=k)


@pytest.mark.parametrize("n_steps,n_mb", [(128, 8), (100, 7)])
def test_small_mlp_split_matches_one_workgroup(n_steps, n_mb):
    """K30's split form (one workgroup per 32 minibatch rows writing partial gradients + a finalize launch that sums
    them in workgroup order, clips and steps Adam) against the one-workgroup form from the same start: every update's
    loss scalars and the parameters after two iterations, within the f32 reassociation of the row sums (128-row and
    ragged 114-row minibatches: 4 workgroups, the last with 18 rows)."""
    from xuanpolicy_amd.runner import build_cartpole_ppo
    res = []
    for split in (True, False):
        agent = build_cartpole_ppo(n_envs=8, n_steps=n_steps, hidden=64, seed=8, device=DEV, n_minibatch=n_mb)
        agent.learner.small_split = split
        agent.update_log = []
        for _ in range(2):
            agent.train(n_steps, log=False)
        torch.cuda.synchronize()
        res.append(([u.cpu().numpy() for u in agent.update_log],
                    [p.detach().cpu().numpy().copy() for p in agent.policy.parameters()]))
    (log_s, par_s), (log_o, par_o) = res
    assert len(log_s) == len(log_o) > 0
    for u, (a, b) in enumerate(zip(log_s, log_o)):
        np.testing.assert_allclose(a[:6], b[:6], rtol=1e-4, atol=1e-5, err_msg="update %d" % u)
    for a, b in zip(par_s, par_o):
        np.testing.assert_allclose(a, b, rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("small", [True, False])
def test_graphed_k9_follows_lr_changes_outside_the_scheduler(small):
    """the device (lr, Adam step) table read by the captured K9 (and by K30, eager or captured) is refilled
    when the learning rate changes outside scheduler.step() inside a live window — here an edited param_groups lr and
    a replaced scheduler after the first iteration.  Reference: the eager multi-kernel update, whose K9 takes the host
    lr every step.  The captured multi-kernel path must match it to rounding; K30 (other arithmetic) to 1e-2 — a stale
    table (the old, decayed lr for 64 updates) moves the weights by ~1e-2 absolute."""
    from xuanpolicy_amd.runner import build_cartpole_ppo
    out = []
    for sm, graphed in ((False, False), (small, True)):
        agent = build_cartpole_ppo(n_envs=8, n_steps=128, hidden=64, seed=5, device=DEV, graph_update=graphed)
        agent.learner.small_updates = sm
        agent.train(128, log=False)
        opt = agent.learner.optimizer
        for g in opt.param_groups:
            g["lr"] = 1e-3
        agent.learner.scheduler = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.25,
                                                                    total_iters=300)
        agent.train(128, log=False)
        torch.cuda.synchronize()
        fo = agent.learner.fused_opt
        if fo.sched_enabled:
            assert not fo.sched_overflow()
            assert fo._sched_lrs[fo.step_count - fo._sched_start] == opt.param_groups[0]["lr"]
        out.append(([p.detach().cpu().numpy().copy() for p in agent.policy.parameters()],
                    opt.param_groups[0]["lr"]))
    (pa, la), (pb, lb) = out
    assert la == lb and la < 1e-3
    for a, b in zip(pa, pb):
        if small:
            np.testing.assert_allclose(b, a, rtol=1e-2, atol=1e-3)
        else:
            np.testing.assert_allclose(b, a, rtol=1e-6, atol=1e-7)
