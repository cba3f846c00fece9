"""GPU: K14F (r06) — the env-fused policy head launch with K8's deferred, normalised post step and the next step's
obs_rms.update in its tail (csrc/rollout.hip xpa_rollout_step_synthbox), against the five-launch step it replaces
(K14E, then K8 = xpa_rollout_post_deferred_norm, then the next step's standalone xpa_rms_update).

Two agents from one seed run the same steps; every buffer and running statistic the post step writes is compared.
The only arithmetic that differs is the order of the f64 sums behind ret_rms / obs_rms (block partials of 4 envs in
two ticketed levels instead of K8's 256-env blocks and K5's 256-row blocks), so the f32 statistics agree to f64
rounding and everything downstream of them to a few f32 ulps; integer and flag columns are exact.  Mid-buffer
truncations (max_episode_steps < n_steps) exercise the kept slot rows; ragged env counts leave idle waves in the last
block (they must still reach the tickets); 4096 envs is C2's XCD-mapped grid (1024 blocks, 16 ticket groups).  The
end-to-end oracle replays in test_gpu_fastpath_e2e.py run with K14F on (the default)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _run(monkeypatch, fused, n_envs, steps, agent_kind="PPO_Clip", max_ep=7):
    import xuanpolicy_amd.agents as ag
    from xuanpolicy_amd.runner import build_synthbox_ppo
    monkeypatch.setattr(ag, "FUSE_POST", fused)
    monkeypatch.setattr(ag, "FOLD_RMS", False)
    agent = build_synthbox_ppo(n_envs=n_envs, n_steps=16, obs_dim=17, act_dim=6, hidden=256, n_epoch=1, n_minibatch=4,
                               seed=11, device="cuda:0", max_episode_steps=max_ep, agent=agent_kind)
    assert agent._k14f_on() == fused
    agent.train(steps, log=False)
    if not fused and agent.use_obsnorm:   # K14F has merged the observation the last step produced; the standalone
        agent._rms_update(agent.envs.obs)   # path merges it at the next step's start: catch up before comparing
    torch.cuda.synchronize()
    m = agent.memory
    t = min(steps % 16 or 16, 16)
    out = {
        "obs_mean": agent.obs_mean, "obs_var": agent.obs_var, "obs_count": agent.obs_count,
        "ret_mean": agent.ret_mean, "ret_var": agent.ret_var, "ret_count": agent.ret_count, "returns": agent.returns,
        "rewards": m.rewards[:, :t], "terminals": m.terminals[:, :t], "closed": m.closed[:, :t], "boot": m.boot[:, :t],
        "observations": m.observations[:, :t], "actions": m.actions[:, :t], "values": m.values[:, :t],
        "slot_t": agent.slot_t, "slot_obs": agent.slot_obs, "boot_obs": agent.boot_obs, "cursor": agent.cursor,
        "overflow": agent.slot_overflow, "env_obs": agent.envs.obs,
    }
    if agent_kind == "PPO_Clip":
        out["old_logp"] = m.auxiliary_infos["old_logp"][:, :t]
    out = {k: v.clone() for k, v in out.items()}
    if fused:
        part, tickets = agent._k14f_ws[1]
        out["tickets"] = tickets.clone()
    del agent
    return out


EXACT = ("obs_count", "ret_count", "terminals", "closed", "slot_t", "cursor", "overflow")


def _compare(f, u):
    assert int(f["tickets"].abs().sum()) == 0, "K14F left a ticket non-zero"
    for k in EXACT:
        assert torch.equal(f[k], u[k]), k
    for k in ("obs_mean", "obs_var", "ret_mean", "ret_var"):
        assert torch.allclose(f[k], u[k], rtol=2e-7, atol=1e-9), (k, f[k], u[k])
    # downstream of the statistics: a few f32 ulps of the normalisations / reward scaling, carried through the policy
    for k in ("returns", "rewards", "boot", "observations", "slot_obs", "boot_obs", "env_obs"):
        assert torch.allclose(f[k], u[k], rtol=1e-5, atol=1e-6), (k, (f[k] - u[k]).abs().max().item())
    for k in ("actions", "values") + (("old_logp",) if "old_logp" in f else ()):
        assert torch.allclose(f[k], u[k], rtol=1e-4, atol=1e-5), (k, (f[k] - u[k]).abs().max().item())


@pytest.mark.parametrize("n_envs,steps", [(1000, 16 + 7), (1002, 13), (4096, 16 + 16), (5, 9)])
def test_k14f_matches_k14e_k8_rms(monkeypatch, n_envs, steps):
    f = _run(monkeypatch, True, n_envs, steps)
    u = _run(monkeypatch, False, n_envs, steps)
    # the runs must have kept truncation rows (max_episode_steps 7 < 16 steps per rollout)
    assert int((u["slot_t"] >= 0).sum()) + int((u["closed"] != 0).sum()) > 0
    _compare(f, u)


def test_k14f_a2c_keeps_next_observation_rows(monkeypatch):
    """A2C (boot_from_reset): K14F keeps the env's next (reset) observation as the truncation row, as K8's slot_src."""
    f = _run(monkeypatch, True, 600, 12, agent_kind="A2C")
    u = _run(monkeypatch, False, 600, 12, agent_kind="A2C")
    assert int((u["slot_t"] >= 0).sum()) > 0
    _compare(f, u)
