"""GPU: the critic's factored backward (r05) — K16Q critic with mask / dv outputs, K42C, K41P (csrc/head.hip,
csrc/sgemm3.hip).

With a LeakyReLU critic hidden layer and one output unit, dz_c[r, c] = dv[r] wc[c] (slope + (1 - slope) m[r, c]),
m = [h_c > 0], so the critic's halves of the paired hidden layer's dX and dW are masked GEMMs whose mask operand is
exact in bf16 (three split products instead of six) and dz_c is never stored.  Checked here:
  * the mask-writing critic head reproduces the dz-writing one bit for bit (every partial), and dz_c rebuilt from its
    mask / dv equals the dz it no longer writes, bit for bit;
  * K42C against an f64 restatement of K42S on the unfactored dz_pair (the trunk layer's dW1 / db1);
  * K41P against f64 products of dz_a^T h and dz_c^T h, within the f32 GEMM's own error;
  * the learner with the factored path against the unfactored one (every gradient, the loss scalars)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _words(m):
    """bool [rows, 256] -> int32 [rows, 8]: bit c & 31 of word c >> 5 = m[row, c] (the critic head's mask layout)."""
    a = m.cpu().numpy().reshape(m.shape[0], 8, 32).astype(np.uint64)
    w = (a << np.arange(32, dtype=np.uint64)).sum(-1).astype(np.uint32)
    return torch.from_numpy(w.view(np.int32).copy()).to(DEV)


def _sign_k42(h):
    """K42S's h_sign layout: byte b bit j = h[row, 32 j + b] > 0."""
    rows = h.shape[0]
    bits = (h > 0).view(rows, 8, 32).to(torch.int32)
    sign = (bits << torch.arange(8, device=DEV, dtype=torch.int32).view(1, 8, 1)).sum(1).to(torch.uint8)
    return sign.contiguous().view(torch.int32).view(rows, 8)


@pytest.mark.parametrize("B,code", [(65536, 1), (777, 1), (4133, 1)])
def test_critic_mask_head_equals_dz_form(B, code):
    from xuanpolicy_amd import ops
    L, s = ops.lib(), ops._stream()
    g = torch.Generator(device=DEV).manual_seed(B + 11)
    H, R = 256, B + 300
    x = torch.randn(B, H, device=DEV, generator=g)
    wh_c = torch.randn(H, H, device=DEV, generator=g) / 16
    bh_c = torch.randn(H, device=DEV, generator=g) * 0.1
    w_c = torch.randn(1, H, device=DEV, generator=g) / 16
    b_c = torch.randn(1, device=DEV, generator=g) * 0.1
    idx = torch.randperm(R, device=DEV, generator=g)[:B].contiguous()
    idx[B // 2] = -1
    ret = torch.randn(R, device=DEV, generator=g)
    wsc = ops.s3_split(wh_c.t())
    G = int(L.xpa_head_fused_num_partials(B))
    W = int(L.xpa_loss_partial_width(6))
    p = ops._p
    slope = 0.01

    def run(mask_form):
        assert L.xpa_lds_poison(s) == 0
        dz = torch.full((B, 2 * H), 777.0, device=DEV)
        parts = [torch.full((G, n), 555.0, device=DEV) for n in (H, H, 1)]
        lp = torch.zeros(G, W, device=DEV)
        mask = torch.full((B, 8), -7, dtype=torch.int32, device=DEV)
        dv = torch.full((B,), 333.0, device=DEV)
        if mask_form:
            assert L.xpa_head_gemm_s3q_critic_mask(code, B, H, p(x), H, p(wsc), p(bh_c), 2 * H, p(w_c), p(b_c), slope,
                                                   p(idx), R, p(ret), 0.25, None, p(parts[0]), p(parts[1]),
                                                   p(parts[2]), p(lp), W, s, p(mask), p(dv)) == 0
        else:
            assert L.xpa_head_gemm_s3q_critic(code, B, H, p(x), H, p(wsc), p(bh_c), 2 * H, p(w_c), p(b_c), slope,
                                              p(idx), R, p(ret), 0.25, p(dz[:, H:]), p(parts[0]), p(parts[1]),
                                              p(parts[2]), p(lp), W, s) == 0
        torch.cuda.synchronize()
        return dz, parts, lp, mask, dv

    dz, parts_ref, lp_ref, _, _ = run(False)
    dz2, parts, lp, mask, dv = run(True)
    for i, (a_, b_) in enumerate(zip(parts_ref, parts)):
        assert torch.equal(a_, b_), i
    assert torch.equal(lp_ref, lp)
    assert torch.equal(dz2, torch.full_like(dz2, 777.0)), "the mask form must not write dz"
    m = (mask.cpu().numpy().view(np.uint32)[:, :, None] >> np.arange(32, dtype=np.uint32)) & 1
    m = torch.from_numpy(m.reshape(B, 256).astype(bool)).to(DEV)
    rebuilt = (dv[:, None] * w_c[0][None, :]) * torch.where(m, torch.ones((), device=DEV),
                                                            torch.full((), slope, device=DEV))
    assert torch.equal(rebuilt, dz[:, H:]), "dz_c rebuilt from mask / dv"
    # the mask is the sign of the critic's hidden activations: rows where dv == 0 carry no information in dz, so check
    # it against an f64 hidden pre-activation away from zero
    z = x.double() @ wh_c.double().t() + bh_c.double()
    clear = z.abs() > 1e-4
    assert torch.equal(m[clear], (z > 0)[clear])


@pytest.mark.parametrize("rows,din,act", [(65536, 17, 1), (4133, 17, 1), (300, 5, 0), (77, 32, 1)])
def test_trunk_bwd_crit_matches_f64(rows, din, act):
    """K42C: g = dz_a Wh_a + dz_c Wh_c with dz_c = dv wc (slope_c + (1 - slope_c) m), then the trunk layer's backward
    from its sign bits (K42S's epilogue) — against f64 on the unfactored dz_c, within 2e-5 of the output scale."""
    from xuanpolicy_amd import ops
    g = torch.Generator(device=DEV).manual_seed(rows + din + 5)
    H = 256
    dz_a = torch.randn(rows, 2 * H, device=DEV, generator=g)[:, :H] * 1e-3   # row stride 512, as the learner's
    wa = torch.randn(H, 256, device=DEV, generator=g) / 16
    whc = torch.randn(H, 256, device=DEV, generator=g) / 16
    wc = torch.randn(H, device=DEV, generator=g) / 16
    slope_c, slope = 0.01, 0.01
    m = torch.rand(rows, H, device=DEV, generator=g) > 0.45
    dv = torch.randn(rows, device=DEV, generator=g) * 1e-3
    x = torch.randn(rows, din, device=DEV, generator=g)
    pre = torch.randn(rows, 256, device=DEV, generator=g)
    sign = _sign_k42(pre)
    pair = torch.cat([wa, whc], 0)
    buf = torch.empty(int(ops.lib().xpa_s3_split_bytes(2 * H, 256)), dtype=torch.uint8, device=DEV)
    cs = torch.empty(256, device=DEV)
    ops.s3_split_batch([(pair, buf)], scales=[(wc, 1.0 - slope_c, H)], cs=(cs, slope_c))
    pdw, pdb = ops.s3_gemm_trunk_bwd_crit(dz_a, buf, H, H, _words(m), dv, cs, sign, x, act, slope)
    torch.cuda.synchronize()
    d = lambda t: t.double()   # noqa: E731
    s_c = torch.where(m, 1.0, slope_c).double()
    dz_c = d(dv)[:, None] * d(wc)[None, :] * s_c
    gg = d(dz_a) @ d(wa) + dz_c @ d(whc)
    gp = torch.where(pre > 0, 1.0, slope).double() if act == 1 else torch.ones_like(gg)
    dz1 = gg * gp
    ref_dw, ref_db = (dz1.t() @ d(x)).reshape(-1), dz1.sum(0)
    got_dw, got_db = pdw.double().sum(0), pdb.double().sum(0)
    assert torch.isfinite(pdw).all() and torch.isfinite(pdb).all()
    ref_cs = slope_c * (d(wc) @ d(whc))
    assert (d(cs) - ref_cs).abs().max().item() <= 1e-6 * ref_cs.abs().max().item()
    for got, ref, what in ((got_dw, ref_dw, "dW1"), (got_db, ref_db, "db1")):
        scale = ref.abs().max().item()
        err = (got - ref).abs().max().item()
        assert err <= 2e-5 * scale, (what, err, scale)


@pytest.mark.parametrize("rows", [65536, 4133, 300, 77])
def test_wgrad_pair_matches_f32_gemm_error(rows):
    """K41P: the actor's slices sum to dz_a^T h and the critic's to dz_c^T h (dz_c = dv wc (slope + (1 - slope) m))
    within 2x the f32 GEMM's own error against f64 (+ a 2^-24-relative floor), as K41V's test."""
    from xuanpolicy_amd import ops
    g = torch.Generator(device=DEV).manual_seed(rows * 7 + 1)
    H, slope = 256, 0.01
    dz_a = (torch.randn(rows, 2 * H, device=DEV, generator=g)
            * torch.exp(2 * torch.randn(rows, 2 * H, device=DEV, generator=g)))[:, :H]
    h = torch.randn(rows, H, device=DEV, generator=g)
    m = torch.rand(rows, H, device=DEV, generator=g) > 0.45
    dv = torch.randn(rows, device=DEV, generator=g) * torch.exp(torch.randn(rows, device=DEV, generator=g))
    wc = torch.randn(H, device=DEV, generator=g) / 16
    pa, pc = ops.s3_wgrad_pair(dz_a, h, _words(m), dv, wc, slope)
    torch.cuda.synchronize()
    assert torch.isfinite(pa).all() and torch.isfinite(pc).all()
    s_c = torch.where(m, torch.ones((), device=DEV), torch.full((), slope, device=DEV))
    dz_c = (dv[:, None] * wc[None, :]) * s_c            # the head's own f32 arithmetic
    for got, a, what in ((pa.double().sum(0), dz_a, "actor"), (pc.double().sum(0), dz_c, "critic")):
        ref = a.double().t() @ h.double()
        native = torch.mm(a.t(), h)
        torch.cuda.synchronize()
        scale = ref.abs().max().item()
        err = (got - ref).abs().max().item()
        err_f32 = (native.double() - ref).abs().max().item()
        assert err <= 2 * err_f32 + 2 ** -24 * scale, (what, err, err_f32, scale)


def test_learner_factored_critic_matches_unfactored():
    """One C2-shaped update through FusedActorCritic (the bench's nets, B = 8192) with the factored critic backward and
    with it switched off: every parameter gradient and the loss scalars agree within the f32 GEMM's error."""
    from xuanpolicy_amd.fused_mlp import FusedActorCritic
    from xuanpolicy_amd.runner import build_synthbox_ppo
    agent = build_synthbox_ppo(n_envs=256, n_steps=32, obs_dim=17, act_dim=6, hidden=256, n_epoch=1, n_minibatch=1,
                               seed=9, device="cuda:0")
    agent.train(32)   # a buffer to sample from (and one update, which also compiles every path)
    torch.cuda.synchronize()
    lrn = agent.learner
    fm = lrn._fused_mlp()
    assert fm is not None
    res = []
    for flag in (True, False):
        FusedActorCritic.CRIT_FACTORED = flag
        try:
            grads, sc = _one_update_grads(agent)
        finally:
            FusedActorCritic.CRIT_FACTORED = True
        res.append((grads, sc))
    (ga, sa), (gb, sb) = res
    # both are f32 sums over 8192 rows with heavy cancellation (a minibatch mean of noisy terms): two summation orders
    # differ by up to ~1e-4 of the output scale (the kernels are held to f64 above); a wiring error would be O(1)
    for i, (a_, b_) in enumerate(zip(ga, gb)):
        scale = b_.abs().max().item()
        assert (a_ - b_).abs().max().item() <= 2e-4 * scale + 1e-12, i
    assert np.allclose(sa, sb, rtol=1e-5, atol=1e-6)


def _one_update_grads(agent):
    """Gradients of one update on a fixed minibatch (the learner's fused forward / backward, no optimizer step)."""
    from xuanpolicy_amd.fused_mlp import Rows
    lrn = agent.learner
    fm = lrn._fused_mlp()
    mem = agent.memory
    N, T = mem.n_envs, mem.n_size
    g = torch.Generator(device=DEV).manual_seed(1)
    idx = torch.randperm(N * T, device=DEV, generator=g)
    flat_obs = mem.observations.view(N * T, -1)
    adv, ret = mem.advantages.view(-1), mem.returns.view(-1)
    act = mem.actions.reshape(-1)
    old = mem.auxiliary_infos["old_logp"].view(-1)
    part = torch.empty((int(fm_num_partials(idx.numel())), 2), dtype=torch.float64, device=DEV)
    for p_ in lrn.policy.parameters():
        p_.grad.zero_()
    ctx = fm.forward_hidden(Rows(flat_obs, idx), adv=adv, adv_partials=part)
    sc = fm.loss_backward(ctx, "ppo", "gaussian", act, adv, ret, old_logp=old, idx=idx, adv_partials=part,
                          clip_range=0.2, vf_coef=0.25, ent_coef=0.0)
    torch.cuda.synchronize()
    return [p_.grad.detach().clone() for p_ in lrn.policy.parameters()], sc.cpu().numpy()


def fm_num_partials(rows):
    from xuanpolicy_amd import ops
    return ops.lib().xpa_gather_num_partials(rows)
