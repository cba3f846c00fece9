"""End-to-end parity of the exact pipeline bench.py times (C2 nets: [256] LeakyReLU, ppo/mujoco.yaml).

One full fused iteration on the fast path — K13 trunk with the observation normalisation fused in, the
paired hidden GEMM + K14E (heads, sampling, buffer store and the SynthBox env step in one launch), K8
with deferred truncation bootstraps, the compact GAE scan (bootstrap fix-up fused), then n_epoch x
n_minibatch updates of K4 gather -> K13 -> K16 actor / critic (hidden GEMM on fp32 MFMA + loss + head
backward) -> split-K dW -> dX -> K13 backward -> batched column-sum finalize with the merged loss
finalize -> K9 clip + Adam from producer partials — checked against the CPU oracle:

  * rollout: every stored value and old log-prob against the oracle policy at the iteration's weights;
  * bootstraps: the last-step and mid-buffer truncation bootstraps against V(norm(final obs));
  * GAE: advantages / returns against the oracle's finish_path restatement (1e-5, north_star);
  * updates: the oracle learner (ppoclip_learner.py:24-65 / a2c_learner.py:19-50, torch CPU autograd,
    clip_grad_norm_, Adam, LinearLR) replays the same buffer with the device permutations; every
    update's loss scalars (total loss within 1e-4, north_star) and the final weights must match.

Reference: xuance/torch/agents/policy_gradient/ppoclip_agent.py:59-111, a2c_agent.py:57-107.
"""
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


CASES = [
    # (agent, discrete, act_dim, ent_coef): the bench configuration first
    ("PPO_Clip", False, 6, 0.0),
    ("PPO_Clip", False, 6, 0.01),
    ("A2C", True, 18, 0.01),
]


@pytest.mark.parametrize("agent_name,discrete,A,ent", CASES)
def test_fast_path_iteration_matches_oracle(agent_name, discrete, A, ent):
    from xuanpolicy_amd.runner import build_synthbox_ppo
    N, T, D, H = 512, 64, 17, 256
    n_epoch, n_mb = 2, 4
    agent = build_synthbox_ppo(n_envs=N, n_steps=T, obs_dim=D, act_dim=A, hidden=H, n_epoch=n_epoch,
                               n_minibatch=n_mb, seed=13, device=DEV, agent=agent_name, discrete=discrete,
                               ent_coef=ent, max_episode_steps=T + 17)
    algo = "ppo" if agent_name == "PPO_Clip" else "a2c"
    fm = agent.learner._fused_mlp()
    # the bench's path, not a fallback
    assert fm is not None and fm.fused_heads and fm.gemm_heads and fm.thin0 and fm.pair is not None
    assert agent.defer_boot and agent.use_graph
    assert agent._env_fused(fm) == (not discrete)

    agent.train(T, log=False)             # iteration 1 (episodes start together; time limit at step 81)
    agent.train(T - 1, log=False)         # iteration 2's rollout but its last step
    # free-running over every update at 1e-4, and (r06) lockstep from the device's own weights: loss + gradients
    replay_last_step_iteration(agent, D, A, [H], discrete, algo, ent, n_epoch, n_mb, expect_mid_truncations=not discrete,
                               lockstep=True)


@pytest.mark.parametrize("agent_name,discrete,A", [("PPO_Clip", False, 6), ("A2C", True, 8)])
def test_fast_path_iteration_with_k16w_matches_oracle(agent_name, discrete, A, monkeypatch):
    """The same end-to-end replay with the heads on K16W (xpa_head_gemm_ws_*: wave-specialised, the epilogue of one
    tile overlapped with the next tile's GEMM) instead of K16 — the adv moments, the loss finalize, the partial rows
    beyond its grid."""
    from xuanpolicy_amd import ops
    from xuanpolicy_amd.runner import build_synthbox_ppo
    monkeypatch.setattr(ops, "K16W_ENABLED", True)
    N, T, D, H = 512, 64, 17, 256
    agent = build_synthbox_ppo(n_envs=N, n_steps=T, obs_dim=D, act_dim=A, hidden=H, n_epoch=2, n_minibatch=4,
                               seed=21, device=DEV, agent=agent_name, discrete=discrete, ent_coef=0.01,
                               max_episode_steps=T + 17)
    fm = agent.learner._fused_mlp()
    assert fm is not None and fm.gemm_heads
    agent.train(T, log=False)
    agent.train(T - 1, log=False)
    replay_last_step_iteration(agent, D, A, [H], discrete, "ppo" if agent_name == "PPO_Clip" else "a2c", 0.01, 2, 4,
                               expect_mid_truncations=not discrete)


@pytest.mark.parametrize("agent_name,discrete,A,heads,crit", [("PPO_Clip", False, 6, "s3", False),
                                                              ("A2C", True, 18, "s3", False),
                                                              ("PPO_Clip", False, 6, "s3p", False),
                                                              ("A2C", True, 8, "s3q", False),
                                                              ("A2C", True, 8, "s3q", True),
                                                              ("PPO_Clip", False, 6, "s3q", True)])
def test_fast_path_iteration_with_split_gemms_matches_oracle(agent_name, discrete, A, heads, crit, monkeypatch):
    """The same end-to-end replay with the update's hidden-layer GEMMs on the bf16 matrix cores by the three-way
    split (ops.S3_GEMMS: K16S heads, K40 dX, K41 dW slices into the f64 finalize): every update's loss within 1e-4
    and the final weights, as for the f32 MFMA path.  crit: the factored critic backward (r05, the default with the
    K16Q heads: K41P / K42C, dz_critic never stored) instead of K41V / K42S on the whole dz_pair."""
    from xuanpolicy_amd import ops
    from xuanpolicy_amd.fused_mlp import FusedActorCritic
    from xuanpolicy_amd.runner import build_synthbox_ppo
    monkeypatch.setattr(ops, "S3_GEMMS", True)
    monkeypatch.setattr(ops, "S3_HEADS", heads)
    monkeypatch.setattr(FusedActorCritic, "CRIT_FACTORED", crit)
    N, T, D, H = 512, 64, 17, 256
    agent = build_synthbox_ppo(n_envs=N, n_steps=T, obs_dim=D, act_dim=A, hidden=H, n_epoch=2, n_minibatch=4,
                               seed=21, device=DEV, agent=agent_name, discrete=discrete, ent_coef=0.01,
                               max_episode_steps=T + 17)
    fm = agent.learner._fused_mlp()
    assert fm is not None and fm.gemm_heads and fm.pair is not None
    agent.train(T, log=False)
    agent.train(T - 1, log=False)
    if crit:
        assert any(k[0] == "wgrad_pair" for k in fm._partials if isinstance(k, tuple)), "K41P not used"
        assert any(k[0] == "crit" for k in fm._partials if isinstance(k, tuple)), "the factored critic not used"
    else:
        assert any(k[0] == "s3wgrad" for k in fm._partials if isinstance(k, tuple)), "K41 not used"
    assert any(k[0] == "s3split" for k in fm._partials if isinstance(k, tuple)), "K40 not used"
    if heads in ("s3p", "s3q"):
        assert any(k[:2] == ("s3split", "s3p_a") for k in fm._partials if isinstance(k, tuple)), "K16P not used"
        assert any(k[0] == "hsign" for k in fm._partials if isinstance(k, tuple)), "K16R / K42S not used"
    assert any(k[0] == "k42" for k in fm._partials if isinstance(k, tuple)), "K42 not used"
    replay_last_step_iteration(agent, D, A, [H], discrete, "ppo" if agent_name == "PPO_Clip" else "a2c", 0.01, 2, 4,
                               expect_mid_truncations=not discrete)


@pytest.mark.parametrize("mode", ["direct", "gather", "off"])
def test_c4_shape_iteration_matches_oracle(mode, monkeypatch):
    """C4's per-shard shapes (BASELINE.json configs[3]: SynthBox(obs=376, act=17), ppo/mujoco.yaml, [256] nets) at a
    reduced N x T: the 376-wide trunk (no K13: the first layer is a library GEMM), the non-K14E rollout (K14 policy
    head + the separate env GEMM + K7), the 1024-thread K5 for wide observations, the KMAX-18 K16 bucket (A = 17)
    and the K9 step — one whole iteration replayed against the oracle (values, old log-probs, bootstraps, GAE,
    every update's loss scalars, final weights)."""
    from xuanpolicy_amd.fused_mlp import FusedActorCritic
    from xuanpolicy_amd.runner import build_synthbox_ppo
    # r05: the wide trunk layer on K40F / K42W (or K42C's dz form) / K41V with the transposed finalize; off = the
    # library GEMM trunk of r04
    wide = mode != "off"
    monkeypatch.setattr(FusedActorCritic, "WIDE_TRUNK", wide)
    monkeypatch.setattr(FusedActorCritic, "WIDE_DIRECT", mode == "direct")   # rows through idx, or the pitched gather
    N, T, D, A, H = 512, 64, 376, 17, 256
    n_epoch, n_mb = 2, 4
    agent = build_synthbox_ppo(n_envs=N, n_steps=T, obs_dim=D, act_dim=A, hidden=H, n_epoch=n_epoch,
                               n_minibatch=n_mb, seed=17, device=DEV, max_episode_steps=T + 17)
    fm = agent.learner._fused_mlp()
    assert fm is not None and fm.fused_heads and fm.gemm_heads and not fm.thin0 and fm.pair is not None
    assert agent.defer_boot and agent.n_slots == 1 and not agent._env_fused(fm)
    agent.train(T, log=False)
    agent.train(T - 1, log=False)
    # tolerances (r06): every update is replayed from the device's own weights at that update (lockstep) — its loss
    # scalars at north_star's 1e-4 and each parameter's pre-clip gradient at 1e-4 of the tensor's scale (+ the share of
    # rows at a clip bound).  The free-running replay (the oracle stepping its own weights) is asserted at update 0 only,
    # which starts from identical weights: later updates drift apart through Adam — r06 measured the device at 2.1e-4
    # on update 5's actor loss where an f64 + jittered-f32 ensemble of oracle replays stayed within 1e-6 (a ratio at a
    # clip bound flips its min() branch; c4_drift.jsonl: 0 vs 2e-4 by seed), so no envelope of the oracle's own spread
    # covers it, while the lockstep replay shows every update computed to 1e-4
    replay_last_step_iteration(agent, D, A, [H], False, "ppo", 0.0, n_epoch, n_mb, expect_mid_truncations=True,
                               loss_tol=1e-4, w_atol=1e-4, lockstep=True, free_run_updates=1)
    assert fm._wide_on() == wide
    keys = {k[0] for k in fm._partials if isinstance(k, tuple)}
    assert ("wide_bwd" in keys) == wide and ("wide_x" in keys) == (mode == "gather"), keys


def test_deferred_bootstraps_with_several_truncations_per_rollout():
    """A time limit shorter than the rollout (max_episode_steps 20 < n_steps 64): every env truncates up to
    ceil(63 / 20) = 4 times before the last step.  K8 keeps one deferred slot per truncation (agent.n_slots = 4), the
    fix-up writes each slot's V(norm(final obs)) at its own step, and the iteration replays against the oracle
    (ppoclip_agent.py:95-101 closes every truncated path with its own bootstrap)."""
    from xuanpolicy_amd.runner import build_synthbox_ppo
    N, T, D, A, H = 256, 64, 17, 6, 256
    agent = build_synthbox_ppo(n_envs=N, n_steps=T, obs_dim=D, act_dim=A, hidden=H, n_epoch=2, n_minibatch=4,
                               seed=19, device=DEV, max_episode_steps=20)
    assert agent.defer_boot and agent.n_slots == 4
    agent.train(T, log=False)
    agent.train(T - 1, log=False)
    replay_last_step_iteration(agent, D, A, [H], False, "ppo", 0.0, 2, 4, expect_mid_truncations=True)
    mem = agent.memory
    mid = (mem.closed[:, :T - 1] != 0) & (mem.terminals[:, :T - 1] == 0)
    assert int(mid.sum(1).max()) >= 3              # several truncations of one env inside one rollout
    assert int(agent.slot_overflow) == 0 and int(agent.slot_t.max()) == -1


@pytest.mark.parametrize("agent_name,discrete,A", [("PPO_Clip", False, 6), ("A2C", True, 18)])
def test_fast_path_iteration_with_f32_gemms_matches_oracle(agent_name, discrete, A, monkeypatch):
    """The r03 update path (ops.S3_GEMMS off: K16 heads on the f32 MFMA, hipBLASLt dX and split-K dW) replayed the same
    way — the A/B partner of the default split GEMMs (bench.py --gemm f32)."""
    from xuanpolicy_amd import ops
    from xuanpolicy_amd.runner import build_synthbox_ppo
    monkeypatch.setattr(ops, "S3_GEMMS", False)
    N, T, D, H = 512, 64, 17, 256
    agent = build_synthbox_ppo(n_envs=N, n_steps=T, obs_dim=D, act_dim=A, hidden=H, n_epoch=2, n_minibatch=4,
                               seed=21, device=DEV, agent=agent_name, discrete=discrete, ent_coef=0.01,
                               max_episode_steps=T + 17)
    fm = agent.learner._fused_mlp()
    assert fm is not None and fm.gemm_heads and fm.pair is not None
    agent.train(T, log=False)
    agent.train(T - 1, log=False)
    assert not any(isinstance(k, tuple) and k[0] in ("s3split", "s3wgrad") for k in fm._partials)
    replay_last_step_iteration(agent, D, A, [H], discrete, "ppo" if agent_name == "PPO_Clip" else "a2c", 0.01, 2, 4,
                               expect_mid_truncations=not discrete)


def test_trunk_heads_iteration_equals_k13_k16(monkeypatch):
    """The K16X learner wiring (fused_mlp.use_trunk_heads: the gather-only K13 form, xpa_head_gemm_trunk_actor writing
    h, plain K16 critic on that h, dW GEMM and K13 backward on it) against the default K13 forward + K16: one whole C2
    fast-path iteration from the same seed, every parameter and every update's loss scalars bit for bit.  K16X exists on
    the f32 MFMA only: both runs take the f32 GEMMs (ops.S3_GEMMS off)."""
    from xuanpolicy_amd import ops
    from xuanpolicy_amd.runner import build_synthbox_ppo
    monkeypatch.setattr(ops, "S3_GEMMS", False)
    runs = []
    for on in (False, True):
        agent = build_synthbox_ppo(n_envs=256, n_steps=32, obs_dim=17, act_dim=6, hidden=256, n_epoch=2,
                                   n_minibatch=4, seed=3, device="cuda:0")
        fm = agent.learner._fused_mlp()
        assert fm is not None and fm.trunk_heads and not fm.use_trunk_heads
        fm.use_trunk_heads = on
        agent.train(32)
        torch.cuda.synchronize()
        runs.append(([p.detach().clone() for p in agent.policy.parameters()], [dict(i) for i in agent.infos]))
    (p0, i0), (p1, i1) = runs
    assert len(p0) == len(p1) and all(torch.equal(a, b) for a, b in zip(p0, p1))
    assert i0 == i1


def test_s3r_trunk_iteration_equals_k13_k16p(monkeypatch):
    """The trunk's h and act' three ways, one whole C2 fast-path iteration each from the same seed: K13's forward +
    K16P + K42 on h (reference), K13 writing h's sign bits + K16P + K42S (the default, fused_mlp.SIGN_BITS), and the
    K16R wiring (fused_mlp.TRUNK_S3R: the gather-only K13 form; h formed inside both split-GEMM head launches, the actor
    writing h and its sign bits; K41 on that h; K42S) — every parameter and every update's loss scalars bit for bit."""
    from xuanpolicy_amd import ops
    from xuanpolicy_amd.fused_mlp import FusedActorCritic
    from xuanpolicy_amd.runner import build_synthbox_ppo
    monkeypatch.setattr(ops, "S3_GEMMS", True)
    monkeypatch.setattr(ops, "S3_HEADS", "s3p")
    runs = []
    for s3r, sign in ((False, False), (False, True), (True, True)):
        monkeypatch.setattr(FusedActorCritic, "TRUNK_S3R", s3r)
        monkeypatch.setattr(FusedActorCritic, "SIGN_BITS", sign)
        agent = build_synthbox_ppo(n_envs=256, n_steps=32, obs_dim=17, act_dim=6, hidden=256, n_epoch=2,
                                   n_minibatch=4, seed=3, device="cuda:0")
        fm = agent.learner._fused_mlp()
        assert fm is not None and fm.trunk_heads and fm._s3r_on() == s3r
        agent.train(32)
        torch.cuda.synchronize()
        assert any(isinstance(k, tuple) and k[0] == "hsign" for k in fm._partials) == (s3r or sign)
        runs.append(([p.detach().clone() for p in agent.policy.parameters()], [dict(i) for i in agent.infos]))
    p0, i0 = runs[0]
    for p1, i1 in runs[1:]:
        assert len(p0) == len(p1) and all(torch.equal(a, b) for a, b in zip(p0, p1))
        assert i0 == i1
