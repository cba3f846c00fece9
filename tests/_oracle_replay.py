"""Test helper: run an agent's last rollout step and check the whole iteration against the CPU oracle.

Used by the end-to-end GPU tests (tests/test_gpu_fastpath_e2e.py for the C2 fast path,
tests/test_gpu_cartpole.py for C1).  The caller has trained the agent up to one env step before the buffer is
full; this takes the iteration's weights / Adam / LinearLR state, runs the last step (deferred bootstraps +
GAE + n_epoch x n_minibatch updates on device), then checks against the oracle (f64 / f32 torch CPU):

  * rollout: every stored value and old log-prob against the oracle policy at the iteration's weights;
  * bootstraps: the last-step and mid-buffer truncation bootstraps against V(norm(final obs));
  * GAE: advantages / returns against the oracle's finish_path restatement (1e-5, north_star);
  * updates: the oracle learner (ppoclip_learner.py:24-65 / a2c_learner.py:19-50, torch CPU autograd,
    clip_grad_norm_, Adam, LinearLR) replays the same buffer with the device permutations; every update's loss
    scalars (total loss within 1e-4, north_star) and the final weights must match.
Reference: xuance/torch/agents/policy_gradient/ppoclip_agent.py:59-111, a2c_agent.py:57-107."""
import os

import numpy as np
import torch

from oracle import cpu_ref


def _load_by_order(pol, agent):
    """The agent's parameters into the oracle policy in state_dict order (the CNN oracle names its critic head
    differently from the reference; the order is the reference's)."""
    src = [v.detach().cpu() for v in agent.policy.state_dict().values()]
    keys = list(pol.state_dict().keys())
    assert len(src) == len(keys)
    pol.load_state_dict(dict(zip(keys, src)))


def _obs_input(obs):
    """Buffer observations as the oracle policy takes them: uint8 frames as numpy (the policy scales them), else f64."""
    return obs if obs.dtype == np.uint8 else torch.as_tensor(obs.astype(np.float64))


def replay_last_step_iteration(agent, D, A, hidden, discrete, algo, ent, n_epoch, n_mb, expect_mid_truncations=False,
                               pol=None, alias_cols=(), report=None, loss_tol=1e-4, w_atol=1e-4,
                               clip_tol=None, envelope=None, lockstep=False, free_run_updates=None):
    """lockstep: also snapshot the device's weights and (pre-clip) gradients at every update and replay each update from
    the device's own weights (replay_updates: every update's loss scalars at loss_tol and its gradient per tensor, with no
    drift carried over from earlier updates).  free_run_updates = n: the free-running replay (the oracle stepping its
    own weights) asserts only its first n updates and not the final weights.
    envelope: None, or a factor k — the updates after the first are then held to max(loss_tol, k x a MEASURED f64
    envelope) (replay_updates), the first one (identical starting weights) to loss_tol.
    pol: the oracle policy to replay with (default: the MLP actor-critic of `hidden`); it is loaded with the agent's
    weights here.  The deferred-bootstrap checks run when the agent defers them (device envs); a host VecEnv's
    per-step bootstraps are checked against the reference loop by tests/test_gpu_hostenv.py.  alias_cols: buffer
    columns whose stored observation is not the one the policy acted on (a host VecEnv's first store of a train() call
    without obs-norm aliases buf_obs after the step, ppoclip_agent.py:59-74): their values / old log-probs are not
    recomputed from the buffer here (tests/test_gpu_hostenv.py checks them against the reference loop)."""
    N, T = agent.n_envs, agent.n_steps
    cfg = agent.config
    if pol is None:
        pol = cpu_ref.build_actor_critic_ref(D, A, hidden, hidden, hidden, discrete=discrete,
                                             activation=getattr(cfg, "activation", "LeakyReLU"))
    _load_by_order(pol, agent)
    pol.double()
    # the optimizer / schedule state the updates of this iteration start from (Adam moments + step, LinearLR)
    opt_state = [{k: (v.detach().cpu().clone() if isinstance(v, torch.Tensor) else v)
                  for k, v in agent.learner.optimizer.state[p].items()}
                 for p in agent.policy.parameters()]   # in parameter order (= the oracle's)
    lr0 = agent.learner.optimizer.param_groups[0]["lr"]
    sched_epoch = agent.learner.scheduler.last_epoch
    perm_counter = agent._perm_counter
    agent.update_log = []
    snaps = None
    if lockstep:   # the weights each update starts from and the gradient it produced, before its clip + Adam step
        snaps = []
        lrn_dev = agent.learner
        orig_step = lrn_dev._sync_clip_step

        def snap_step(*a, **kw):
            snaps.append(([p.detach().clone() for p in agent.policy.parameters()],
                          [p.grad.detach().clone() for p in agent.policy.parameters()]))
            return orig_step(*a, **kw)
        lrn_dev._sync_clip_step = snap_step
    try:
        agent.train(1, log=False)             # last env step -> deferred bootstraps + GAE -> the updates
    finally:
        if lockstep:
            del lrn_dev._sync_clip_step
    torch.cuda.synchronize()
    mem = agent.memory
    gamma, lam = float(mem.gamma), float(mem.gae_lam)

    # ---- rollout: values and old log-probs at the iteration's weights (f64 oracle) ----
    obs_np = mem.observations.cpu().numpy()
    obs_shape = tuple(obs_np.shape[2:])
    act = mem.actions.cpu().numpy().astype(np.float64)
    with torch.no_grad():
        head, logstd, v = pol.heads(_obs_input(obs_np.reshape((N * T,) + obs_shape)))
        d = pol.dist(head, logstd)
        if discrete:
            lp = d.log_prob(torch.as_tensor(act.reshape(N * T)).long())
        else:
            lp = d.log_prob(torch.as_tensor(act.reshape(N * T, A))).sum(-1)
    keep = np.ones((N, T), bool)
    keep[:, list(alias_cols)] = False
    keep = keep.reshape(-1)
    np.testing.assert_allclose(mem.values.cpu().numpy().reshape(-1)[keep], v.numpy()[keep], rtol=1e-4, atol=1e-4)
    if algo == "ppo":
        np.testing.assert_allclose(mem.auxiliary_infos["old_logp"].cpu().numpy().reshape(-1)[keep], lp.numpy()[keep],
                                   rtol=1e-4, atol=2e-4)

    # ---- bootstraps ----
    term = mem.terminals.cpu().numpy()
    closed = mem.closed.cpu().numpy().astype(bool)
    boot = mem.boot.cpu().numpy()
    if agent.defer_boot:
        _check_deferred(agent, pol, N, T, term, closed, boot, expect_mid_truncations)

    # ---- GAE (north_star: 1e-5 on advantages / returns) ----
    adv, ret = cpu_ref.gae_rows(mem.rewards.cpu().numpy(), mem.values.cpu().numpy(), term, closed.astype(np.uint8),
                                boot, gamma, lam)
    np.testing.assert_allclose(mem.advantages.cpu().numpy(), adv, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(mem.returns.cpu().numpy(), ret, rtol=1e-5, atol=1e-5)
    replay_updates(agent, pol, opt_state, lr0, sched_epoch, perm_counter, adv, ret, discrete, A, algo, ent, n_epoch,
                   n_mb, report=report, loss_tol=loss_tol, w_atol=w_atol, clip_tol=clip_tol, envelope=envelope,
                   check_updates=free_run_updates)
    if snaps is not None:
        # the lockstep replay checks the update computation given the device's inputs: the device's own advantages /
        # returns (held to the f64 GAE above at 1e-5), so that a row whose ratio sits at a clip bound is classified from
        # the same advantage on both sides (r06: the f64 GAE's last-bit differences flipped such rows and moved a
        # first-layer gradient by 2e-3 relative L2 with no difference in the update itself)
        replay_updates_lockstep(agent, pol, snaps, mem.advantages.cpu().numpy().astype(np.float64),
                                mem.returns.cpu().numpy().astype(np.float64), discrete, A, algo, ent, n_epoch, n_mb,
                                perm_counter, loss_tol=loss_tol)


def _check_deferred(agent, pol, N, T, term, closed, boot, expect_mid_truncations):
    with torch.no_grad():
        v_last = pol.heads(torch.as_tensor(agent.boot_obs.cpu().numpy().astype(np.float64)))[2].numpy()
        v_slot = pol.heads(torch.as_tensor(agent.slot_obs.cpu().numpy().astype(np.float64)))[2].numpy()
    np.testing.assert_allclose(boot[:, T - 1], np.where(term[:, T - 1] != 0, 0.0, v_last), rtol=1e-4, atol=1e-4)
    mid = closed[:, :T - 1] & (term[:, :T - 1] == 0)
    rows, cols = np.nonzero(mid)
    if expect_mid_truncations:
        assert len(rows) > 0, "the case must exercise mid-buffer truncation bootstraps"
    # the k-th mid-buffer truncation of env n (in time order) was kept in slot k (row k N + n of slot_obs)
    S = agent.n_slots
    k_of = np.zeros(len(rows), np.int64)
    for j in range(len(rows)):
        k_of[j] = int(np.sum(mid[rows[j], :cols[j]]))
    assert (k_of < S).all(), "more mid-buffer truncations than deferred slots"
    np.testing.assert_allclose(boot[rows, cols], v_slot[k_of * N + rows], rtol=1e-4, atol=1e-4)


def replay_updates(agent, pol, opt_state, lr0, sched_epoch, perm_counter, adv, ret, discrete, A, algo, ent, n_epoch,
                   n_mb, report=None, loss_tol=1e-4, w_atol=1e-4, clip_tol=None, envelope=None, check_updates=None):
    """The oracle learner replays the agent's buffer (with adv / ret given) using the device permutations, from the
    Adam / LinearLR state the iteration's updates started from: every update's loss scalars and the final weights.

    envelope = k (no blanket tolerance for a drifting replay): the same updates are also replayed by an
    ensemble from the same state — in f64, and in f32 with every weight jittered by one ulp after each update (2 seeds:
    a stand-in for another correct f32 implementation, whose summation orders differ everywhere) —
    (tests/golden/make_envelopes.py's method, measured here on this run's inputs), and update u > 0 is held to
    max(loss_tol, k x the running maximum over updates <= u of the ensemble's largest distance from the f32 oracle) per
    scalar, the clip fraction to the f32-rounding rows + that envelope, the final weights to max(w_atol, k x the ensemble's
    per-tensor distance); update 0 (identical starting weights) to loss_tol.
    check_updates = n: assert only the first n updates and skip the final weights (the lockstep replay checks every update
    from the device's own weights instead)."""
    import copy
    N, T = agent.n_envs, agent.n_steps
    cfg, mem = agent.config, agent.memory
    members = ([("f64", copy.deepcopy(pol).double(), None)] +
               [("jit%d" % sd, copy.deepcopy(pol).float(), sd) for sd in (1, 2)]) if envelope else []
    pol.float()
    clip = cfg.clip_grad_norm if algo == "ppo" else cfg.clip_grad

    def learner(pl, dtype):
        opt = torch.optim.Adam(pl.parameters(), cfg.learning_rate, eps=1e-5)
        sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.0, total_iters=cfg.running_steps)
        # continue from the agent's Adam moments and LinearLR position (it steps once per update,
        # ppoclip_learner.py:50-51)
        params = list(pl.parameters())
        assert len(params) == len(opt_state)
        for p, st in zip(params, opt_state):
            if st:
                opt.state[p] = {"step": torch.tensor(float(st["step"])), "exp_avg": st["exp_avg"].to(dtype).clone(),
                                "exp_avg_sq": st["exp_avg_sq"].to(dtype).clone()}
        opt.param_groups[0]["lr"] = lr0
        sch.last_epoch = sched_epoch
        return cpu_ref.LearnerRef(pl, opt, sch, algo, cfg.vf_coef, ent, getattr(cfg, "clip_range", 0.2), clip, True)
    lrn = learner(pol, torch.float32)
    ens = [(learner(pl, next(pl.parameters()).dtype), pl,
            torch.Generator().manual_seed(sd) if sd is not None else None) for _, pl, sd in members]
    obs_np = mem.observations.cpu().numpy()
    buf = cpu_ref.BufferRef(obs_np.shape[2:], () if discrete else (A,), {"old_logp": ()} if algo == "ppo" else {}, N, T,
                            obs_dtype=obs_np.dtype)
    buf.observations[:] = obs_np
    buf.actions[:] = mem.actions.cpu().numpy()
    buf.values[:] = mem.values.cpu().numpy()
    buf.returns[:], buf.advantages[:] = ret, adv
    if algo == "ppo":
        buf.auxiliary_infos["old_logp"][:] = mem.auxiliary_infos["old_logp"].cpu().numpy()
    buf.size = T
    B = N * T // n_mb
    assert len(agent.update_log) == n_epoch * n_mb
    u = 0
    run_max = {}
    for e in range(n_epoch):
        perm = agent.epoch_permutation(N * T, counter=perm_counter + e).cpu().numpy()
        for s in range(0, N * T, B):
            o, a, r, _, ad, ax = buf.sample(perm[s:s + B])
            info = lrn.update(o, a, r, ad, ax.get("old_logp"))
            got = agent.update_log[u].cpu().numpy()   # ops.OUT_KEYS order
            ref_loss = info["actor-loss"] - ent * info["entropy"] + cfg.vf_coef * info["critic-loss"]
            env = {}
            for lr_e, pl, gen in ens:
                i_e = lr_e.update(o, a, r, ad, ax.get("old_logp"))
                l_e = i_e["actor-loss"] - ent * i_e["entropy"] + cfg.vf_coef * i_e["critic-loss"]
                d = {k: abs(float(info[k]) - float(i_e[k])) for k in i_e if k in info and k != "clip_boundary_rows"}
                d["loss"] = abs(ref_loss - l_e)
                for k, v in d.items():   # running maximum over the updates (make_envelopes.envelope_atari)
                    run_max[k] = max(run_max.get(k, 0.0), v)
                if gen is not None:      # one ulp up or down (or none) per weight: another f32 rounding of the step
                    with torch.no_grad():
                        for p in pl.parameters():
                            p.add_(torch.randint(-1, 2, p.shape, generator=gen).to(p.dtype)
                                   * p.abs().clamp_min(1e-30) * 2.0 ** -23)
            if ens:
                env = {k: envelope * v if u > 0 else 0.0 for k, v in run_max.items()}
            if report is None and check_updates is not None and u >= check_updates:
                u += 1
                continue
            if report is not None:   # diagnostics (tools/c4_drift.py): record instead of asserting
                report.append(("update", u, [float(got[j]) for j in range(6)],
                               [float(info[k]) for k in ("actor-loss", "critic-loss", "entropy")] + [float(ref_loss)]))
                u += 1
                continue
            # relative above 1, as its components below (C4's critic loss reaches ~35: 1e-4 absolute there is 3e-6
            # relative, inside the two f32 paths' summation-order noise)
            assert abs(got[3] - ref_loss) <= max(loss_tol * max(1.0, abs(ref_loss)), env.get("loss", 0.0)), \
                ("loss", u, got[3], ref_loss, env.get("loss"))
            for j, k in enumerate(("actor-loss", "critic-loss", "entropy")):
                assert abs(got[j] - info[k]) <= max(loss_tol * max(1.0, abs(info[k])), env.get(k, 0.0)), \
                    (k, u, got[j], info[k], env.get(k))
            assert abs(got[5] - info["predict_value"]) <= max(1e-4 * max(1.0, abs(info["predict_value"])),
                                                              env.get("predict_value", 0.0))
            if algo == "ppo":
                # rows within f32 rounding of a clip bound may land on either side (counted by the oracle)
                tol = (2.0 + info["clip_boundary_rows"]) / B + 1e-7 + env.get("clip_ratio", 0.0)
                if clip_tol is not None:   # a drifting replay (see the C4 test): rows near a bound beyond f32 rounding
                    tol = max(tol, clip_tol)
                assert abs(got[4] - info["clip_ratio"]) <= tol, ("clip_ratio", u, got[4], info["clip_ratio"], tol)
            u += 1
    if check_updates is not None and report is None:
        return
    refs_e = [list(pl.state_dict().values()) for _, pl, _ in ens]
    for j, ((k, val), ref) in enumerate(zip(agent.policy.state_dict().items(), pol.state_dict().values())):
        if report is not None:
            a, b = val.detach().cpu().double().numpy(), ref.double().numpy()
            report.append(("weight", k, float(np.abs(a - b).max()), float(np.abs(b).max())))
            continue
        atol = w_atol
        for r_e in refs_e:
            atol = max(atol, envelope * float((ref.double() - r_e[j].double()).abs().max()))
        np.testing.assert_allclose(val.detach().cpu().numpy(), ref.numpy(), rtol=1e-3, atol=atol, err_msg=k)


def replay_updates_lockstep(agent, pol, snaps, adv, ret, discrete, A, algo, ent, n_epoch, n_mb, perm_counter,
                            loss_tol=1e-4, grad_rtol=1e-3):
    """Every update of the iteration replayed from the device's own weights at that update (snaps[u] = (weights,
    pre-clip gradient) taken as the device update reached its clip + Adam step): the loss scalars within loss_tol, and
    each parameter's gradient within grad_rtol in relative L2 norm.  (Element-wise, a gradient can differ where the math
    is undecided in f32: a pre-activation within rounding of the LeakyReLU kink takes slope 1 or 0.01, a PPO ratio at a
    clip bound takes the 0 or the A branch of min() — r06 measured 2-4e-5 on single elements of C4's 376-wide W0 gradient
    of max 0.031 at update 0, on the library-GEMM path as on the split one; such isolated flips are far below 1e-3 of
    the tensor's norm, a wrong or missing row is not.  A whole row's unclipped gradient is not: one such row of C4's
    8192-row minibatch moved the first layer's gradient by 2.3e-3 — so the oracle's gradient may take or drop each
    clip-bound row's contribution, r06.)  No drift is carried between updates, so no envelope is needed
    (ppoclip_learner.py:24-65)."""
    N, T = agent.n_envs, agent.n_steps
    cfg, mem = agent.config, agent.memory
    pol.float()
    clip = cfg.clip_grad_norm if algo == "ppo" else cfg.clip_grad
    opt = torch.optim.SGD(pol.parameters(), lr=0.0)   # the step is irrelevant: weights are reloaded per update
    lrn = cpu_ref.LearnerRef(pol, opt, None, algo, cfg.vf_coef, ent, getattr(cfg, "clip_range", 0.2), clip, True)
    obs_np = mem.observations.cpu().numpy()
    buf = cpu_ref.BufferRef(obs_np.shape[2:], () if discrete else (A,), {"old_logp": ()} if algo == "ppo" else {}, N, T,
                            obs_dtype=obs_np.dtype)
    buf.observations[:] = obs_np
    buf.actions[:] = mem.actions.cpu().numpy()
    buf.values[:] = mem.values.cpu().numpy()
    buf.returns[:], buf.advantages[:] = ret, adv
    if algo == "ppo":
        buf.auxiliary_infos["old_logp"][:] = mem.auxiliary_infos["old_logp"].cpu().numpy()
    buf.size = T
    B = N * T // n_mb
    assert len(snaps) == n_epoch * n_mb == len(agent.update_log)
    params = list(pol.parameters())
    u = 0
    for e in range(n_epoch):
        perm = agent.epoch_permutation(N * T, counter=perm_counter + e).cpu().numpy()
        for s in range(0, N * T, B):
            w_dev, g_dev = snaps[u]
            with torch.no_grad():
                for p, w in zip(params, w_dev):
                    p.copy_(w.cpu().to(p.dtype))
            o, a, r, _, ad, ax = buf.sample(perm[s:s + B])
            info = lrn.update(o, a, r, ad, ax.get("old_logp"), capture_grads=True)
            got = agent.update_log[u].cpu().numpy()   # ops.OUT_KEYS order
            ref_loss = info["actor-loss"] - ent * info["entropy"] + cfg.vf_coef * info["critic-loss"]
            assert abs(got[3] - ref_loss) <= loss_tol * max(1.0, abs(ref_loss)), ("lockstep loss", u, got[3], ref_loss)
            for j, k in enumerate(("actor-loss", "critic-loss", "entropy")):
                assert abs(got[j] - info[k]) <= loss_tol * max(1.0, abs(info[k])), ("lockstep", k, u, got[j], info[k])
            # rows at a clip bound (LearnerRef.boundary_grads): the device may have taken the other branch for any of
            # them; each such row's unclipped gradient is added to / removed from the oracle's where that moves it
            # toward the device's (greedy over the rows, on the whole gradient), then every tensor is held to grad_rtol
            gr_all = [gr.double() for gr in lrn.last_grads]
            res = [gd.cpu().double() - gr for gd, gr in zip(g_dev, gr_all)]
            flips = 0
            for bg in getattr(lrn, "boundary_grads", []):
                bg = [b.double() for b in bg]
                n0 = sum(float((x * x).sum()) for x in res)
                best = None
                for sgn in (1.0, -1.0):
                    n1 = sum(float(((x - sgn * b) ** 2).sum()) for x, b in zip(res, bg))
                    if n1 < n0 and (best is None or n1 < best[0]):
                        best = (n1, sgn)
                if best is not None:
                    res = [x - best[1] * b for x, b in zip(res, bg)]
                    flips += 1
            for name, rr, gr in zip((n for n, _ in pol.named_parameters()), res, gr_all):
                l2 = float(rr.norm()) / (float(gr.norm()) + 1e-30)
                if os.environ.get("XPA_LOCKSTEP_REPORT"):
                    print("LOCKSTEP", u, name, "%.3e" % l2, "flips", flips)
                    continue
                assert l2 <= grad_rtol, ("lockstep grad (relative L2)", u, name, l2, "boundary flips", flips)
            u += 1
