"""CPU checks of the round-5 host-side plans (no GPU, no kernel launches):
  * FusedActorCritic recognises C4's 376-wide trunk layer as the wide form (not the thin K13 one) and pads it as the
    split kernels read it (K40F: 16-k chunks to 384; K41V: 128-row tiles to 384);
  * the rollout buffer's observations carry zeroed slack in the same allocation (what the row-index K40F / K41V read
    past a row's end);
  * the obs-RMS fold into K8 is an opt-in (default off: the reference's update order)."""
import pytest
import torch
import torch.nn as nn

from oracle import cpu_ref


def test_c4_policy_plans_the_wide_trunk():
    from xuanpolicy_amd import ops
    from xuanpolicy_amd.fused_mlp import FusedActorCritic
    pol = cpu_ref.build_actor_critic_ref(376, 17, [256], [256], [256])
    fm = FusedActorCritic(pol)
    assert fm.wide0 and not fm.thin0 and fm.fused_heads
    assert fm._wide_mpad(376) == 384 and (376 + 15) // 16 * 16 == 384
    # without the flat parameter placement (no paired layer) or the split GEMMs, the wide path does not apply
    assert not fm._wide_on()
    c2 = FusedActorCritic(cpu_ref.build_actor_critic_ref(17, 6, [256], [256], [256]))
    assert c2.thin0 and not c2.wide0
    assert ops.S3_GEMMS


@pytest.mark.parametrize("d,wide", [(376, True), (100, True), (64, False), (378, False)])
def test_wide_form_needs_float4_rows(d, wide):
    """d % 4 == 0 (16-B row vectors) and d > 64 (below: K13's thin form)."""
    from xuanpolicy_amd.fused_mlp import FusedActorCritic
    fm = FusedActorCritic(cpu_ref.build_actor_critic_ref(d, 6, [256], [256], [256]))
    assert fm.wide0 == wide


def test_observation_buffer_has_zeroed_slack():
    from xuanpolicy_amd import buffer as bf

    class Box:
        shape = (376,)

    class Act:
        shape = (17,)

    mem = bf.DummyOnPolicyBuffer(Box(), Act(), {"old_logp": ()}, 8, 16, device="cpu")
    obs = mem.observations
    assert tuple(obs.shape) == (8, 16, 376) and obs.is_contiguous()
    st = obs.untyped_storage().nbytes() // obs.element_size()
    assert st >= obs.storage_offset() + obs.numel() + bf.OBS_SLACK
    tail = torch.empty(0, dtype=obs.dtype).set_(obs.untyped_storage(), obs.storage_offset() + obs.numel(),
                                                (bf.OBS_SLACK,))
    assert torch.count_nonzero(tail) == 0


def test_rms_fold_is_opt_in():
    import xuanpolicy_amd.agents as ag
    assert ag.FOLD_RMS is False


def test_relu_critic_keeps_thin_plan():
    """A ReLU net plans the same forms (act code 1, slope 0)."""
    from xuanpolicy_amd.fused_mlp import FusedActorCritic
    pol = cpu_ref.build_actor_critic_ref(376, 17, [256], [256], [256], activation="ReLU")
    fm = FusedActorCritic(pol)
    assert fm.wide0 and fm.rep[0][1] == 1 and fm.rep[0][2] == 0.0
    assert isinstance(pol.representation.model[1], nn.ReLU)


@pytest.mark.parametrize("d,B,direct", [(376, 65536, True), (1024, 65536, False), (1024, 49152, True),
                                        (2048, 24576, True), (2048, 24577, False), (4096, 12289, False)])
def test_wide_direct_respects_k41v_index_stage(d, B, direct):
    """the row-index forms only where K41V-IDX's per-slice rows (ceil(B / S) to 32) fit its 1536-row LDS
    index stage (csrc/sgemm3.hip kVIdxMax); beyond it the pitched gather (no limit) runs instead of a mid-update
    hipErrorInvalidValue."""
    from xuanpolicy_amd import buffer as bf
    from xuanpolicy_amd.fused_mlp import FusedActorCritic, Rows
    fm = FusedActorCritic(cpu_ref.build_actor_critic_ref(d, 6, [256], [256], [256]))
    flat = torch.zeros(B + bf.OBS_SLACK // d + 2, d)[:B]   # slack after the last row, as the rollout buffer has
    x = Rows(flat, torch.zeros(B, dtype=torch.int64))
    assert fm._wide_direct_ok(x, d) == direct
    S = fm._wide_slices(fm._wide_mpad(d))
    per = -(-B // S)
    assert (-(-per // 32) * 32 <= fm.WIDE_VIDX_MAX) == direct


def test_trunk_backward_form_and_crit_plan_share_one_predicate():
    """the factored critic is planned only where the fused trunk backward form applies (one predicate,
    _trunk_bwd_form), and the planned backward raises instead of being stripped under python -O."""
    import inspect
    from xuanpolicy_amd.fused_mlp import FusedActorCritic
    src = inspect.getsource(FusedActorCritic.loss_backward)
    assert "assert self._trunk_bwd_fused" not in src and "RuntimeError" in src
    assert "_trunk_bwd_form" in inspect.getsource(FusedActorCritic._crit_plan)
    fm = FusedActorCritic(cpu_ref.build_actor_critic_ref(17, 6, [256], [256], [256]))
    x = torch.zeros(8, 17)
    assert fm._trunk_bwd_form(torch.zeros(8, 256), x, [torch.zeros(8, 256)]) is None   # no paired layer: no fused form
