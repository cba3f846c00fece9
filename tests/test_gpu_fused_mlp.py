"""GPU: the explicit actor-critic backward (fused_mlp + K10) equals torch autograd through the same
policy, for Gaussian and Categorical heads, LeakyReLU / ReLU / Tanh, with and without a trunk."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


class _Box:
    def __init__(self, n):
        self.shape = (n,)


class _Disc:
    def __init__(self, n):
        self.n, self.shape = n, ()


def _policy(D, A, discrete, act, rep_hidden):
    from xuanpolicy_amd.policies import Basic_Identical, Basic_MLP, Categorical_AC_Policy, Gaussian_AC_Policy
    rep = Basic_MLP((D,), rep_hidden, None, torch.nn.init.orthogonal_, act, DEV) if rep_hidden else \
        Basic_Identical((D,), DEV)
    cls = Categorical_AC_Policy if discrete else Gaussian_AC_Policy
    return cls(_Disc(A) if discrete else _Box(A), rep, [256], [256], None, torch.nn.init.orthogonal_, act, DEV)


def _colsum_check():
    from xuanpolicy_amd import ops
    L = ops.lib()
    for rows, cols, code in [(65536, 256, 1), (1000, 6, 0), (4097, 1, 0), (300, 12, 2), (513, 20, 1)]:
        g = torch.randn(rows, cols, device=DEV)
        h = torch.randn(rows, cols, device=DEV)
        exp = g.clone()
        if code == 1:
            exp = torch.where(h > 0, g, g * 0.01)
        elif code == 2:
            exp = g * (1 - h * h)
        part = torch.empty(int(L.xpa_act_bwd_num_partials(rows)), cols, device=DEV)
        out = torch.empty(cols, device=DEV)
        s = ops._stream()
        assert L.xpa_act_bwd_colsum(code, ops._p(g), ops._p(h), rows, cols, 0.01, ops._p(g) if code else None,
                                    ops._p(part), s) == 0
        assert L.xpa_colsum_finalize(ops._p(part), part.shape[0], cols, ops._p(out), s) == 0
        torch.testing.assert_close(g, exp, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(out, exp.double().sum(0).float(), rtol=1e-5, atol=1e-3)


def test_act_bwd_colsum_kernel():
    _colsum_check()


@pytest.mark.parametrize("discrete,act,rep_hidden", [(False, torch.nn.LeakyReLU, [256]), (True, torch.nn.LeakyReLU, [256]),
                                                     (False, torch.nn.Tanh, [64]), (True, torch.nn.ReLU, []),
                                                     (False, torch.nn.LeakyReLU, [])])
def test_explicit_backward_matches_autograd(discrete, act, rep_hidden):
    from xuanpolicy_amd.flat import FlatState
    from xuanpolicy_amd.fused_mlp import FusedActorCritic
    torch.manual_seed(0)
    D, A, B = 17, 6, 65536
    p1 = _policy(D, A, discrete, act, rep_hidden)
    p2 = _policy(D, A, discrete, act, rep_hidden)
    p2.load_state_dict(p1.state_dict())
    x = torch.randn(B, D, device=DEV)
    dh = torch.randn(B, A, device=DEV) * 1e-3
    dv = torch.randn(B, device=DEV) * 1e-3
    head, logstd, v = p1.heads(x)
    tensors, grads = [head, v], [dh, dv]
    torch.autograd.backward(tensors, grads)
    fs = FlatState(p2.parameters())
    fm = FusedActorCritic(p2)
    h2, ls2, v2, ctx = fm.forward(x)
    torch.testing.assert_close(h2, head.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(v2, v.detach(), rtol=1e-5, atol=1e-5)
    fs.flat.fill_(123.0)   # every gradient must be overwritten
    if ls2 is not None:
        ls2.grad.zero_()   # logstd's gradient comes from the loss finalize, not from this backward
    fm.backward(ctx, dh.clone(), dv.clone())
    for (n1, a), (n2, b) in zip(p1.named_parameters(), p2.named_parameters()):
        if n1.endswith("logstd"):
            continue
        ga, gb = a.grad.double(), b.grad.double()
        scale = ga.abs().max().item() + 1e-12
        assert (ga - gb).abs().max().item() <= 2e-5 * scale, (n1, (ga - gb).abs().max().item(), scale)


@pytest.mark.parametrize("algo,discrete,act,rep_hidden,ent", [
    ("ppo", False, torch.nn.LeakyReLU, [256], 0.0), ("ppo", True, torch.nn.LeakyReLU, [256], 0.01),
    ("a2c", False, torch.nn.Tanh, [64], 0.005), ("a2c", True, torch.nn.ReLU, [], 0.01),
    ("ppo", False, torch.nn.LeakyReLU, [], 0.0)])
def test_fused_heads_match_loss_kernel_path(algo, discrete, act, rep_hidden, ent):
    """K12 (heads + loss + head backward in one pass) == K2 loss kernel + explicit backward, which the
    drop-in tests pin to the reference's fixtures: loss scalars and every parameter gradient."""
    from xuanpolicy_amd import ops
    from xuanpolicy_amd.flat import FlatState
    from xuanpolicy_amd.fused_mlp import FusedActorCritic
    torch.manual_seed(1)
    D, A, B, R = 17, 6, 8192 + 37, 20000
    p1 = _policy(D, A, discrete, act, rep_hidden)
    p2 = _policy(D, A, discrete, act, rep_hidden)
    p2.load_state_dict(p1.state_dict())
    fs1, fs2 = FlatState(p1.parameters()), FlatState(p2.parameters())
    fm1, fm2 = FusedActorCritic(p1), FusedActorCritic(p2)
    assert fm2.fused_heads
    obs_all = torch.randn(R, D, device=DEV)
    idx = torch.randperm(R, device=DEV)[:B].contiguous()
    idx[5] = R + 3          # invalid rows contribute nothing
    idx[B - 1] = -1
    adv = torch.randn(R, device=DEV)
    ret = torch.randn(R, device=DEV)
    if discrete:
        act_buf = torch.randint(0, A, (R,), device=DEV).float()
    else:
        act_buf = torch.randn(R, A, device=DEV)
    with torch.no_grad():
        h0, _, _ = p1.heads(obs_all)
        if discrete:
            old = torch.distributions.Categorical(logits=h0).log_prob(act_buf.long())
        else:
            old = torch.distributions.Normal(h0, p1.actor.logstd.exp()).log_prob(act_buf).sum(-1)
        old = (old + 0.05 * torch.randn(R, device=DEV)).contiguous()   # ratios on both sides of the clip
    obs, part = ops.gather_minibatch(idx.clamp(0, R - 1), obs_all, adv=adv)
    # both paths read the same adv-norm partials
    dist = "categorical" if discrete else "gaussian"
    kw = dict(old_logp=old if algo == "ppo" else None, idx=idx, adv_partials=part, clip_range=0.2, vf_coef=0.25,
              ent_coef=ent)
    fs1.flat.fill_(7.0)
    fs2.flat.fill_(-7.0)
    head, logstd, v, ctx = fm1.forward(obs)
    s1, dh, _, dv = ops.policy_loss(algo, dist, head, logstd, v, act_buf, adv, ret,
                                    d_logstd_out=logstd.grad if logstd is not None else None, **kw)
    fm1.backward(ctx, dh, dv)
    ctx2 = fm2.forward_hidden(obs)
    s2 = fm2.loss_backward(ctx2, algo, dist, act_buf, adv, ret, **kw)
    torch.cuda.synchronize()
    a, b = s1.double().cpu(), s2.double().cpu()
    assert torch.allclose(a, b, rtol=2e-5, atol=2e-6), (a, b)
    for (n1, x1), (n2, x2) in zip(p1.named_parameters(), p2.named_parameters()):
        ga, gb = x1.grad.double(), x2.grad.double()
        scale = ga.abs().max().item() + 1e-12
        assert (ga - gb).abs().max().item() <= 5e-5 * scale, (n1, (ga - gb).abs().max().item(), scale)
        assert not bool((x2.grad == -7.0).any()), n2   # every gradient written
