"""Diagnostic: K16 dz vs a torch fp32 recomputation on the failing categorical test case — are the
differences isolated elements whose pre-activation sits at the LeakyReLU kink (|z| ~ rounding)?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from test_gpu_fused_mlp import DEV, _policy  # noqa: E402


def main():
    from xuanpolicy_amd import ops
    from xuanpolicy_amd.flat import FlatState
    from xuanpolicy_amd.fused_mlp import FusedActorCritic, head_placement
    torch.manual_seed(1)
    D, A, B, R = 17, 6, 8192 + 37, 20000
    p2 = _policy(D, A, True, torch.nn.LeakyReLU, [256])
    p1 = _policy(D, A, True, torch.nn.LeakyReLU, [256])
    p2.load_state_dict(p1.state_dict())
    fs2 = FlatState(p2.parameters(), placement=head_placement(p2))
    fm2 = FusedActorCritic(p2, flat=fs2)
    obs_all = torch.randn(R, D, device=DEV)
    idx = torch.randperm(R, device=DEV)[:B].contiguous()
    adv = torch.randn(R, device=DEV)
    ret = torch.randn(R, device=DEV)
    act_buf = torch.randint(0, A, (R,), device=DEV).float()
    with torch.no_grad():
        h0, _, _ = p1.heads(obs_all)
        old = torch.distributions.Categorical(logits=h0).log_prob(act_buf.long())
        old = (old + 0.05 * torch.randn(R, device=DEV)).contiguous()
    obs, part = ops.gather_minibatch(idx, obs_all, adv=adv)
    kw = dict(old_logp=old, idx=idx, adv_partials=part, clip_range=0.2, vf_coef=0.25, ent_coef=0.01)
    ctx2 = fm2.forward_hidden(obs)
    fm2.loss_backward(ctx2, "ppo", "categorical", act_buf, adv, ret, **kw)
    torch.cuda.synchronize()
    dz16 = fm2._hws.dz_pair[:, :256].double()
    # torch fp32 recomputation of the actor hidden layer and its dz from K2's d head
    with torch.no_grad():
        s = p2.representation(obs)["state"]
        lin = p2.actor.model[0]
        z = F.linear(s, lin.weight, lin.bias)
        z64 = F.linear(s.double(), lin.weight.double(), lin.bias.double())
        h = F.leaky_relu(z, 0.01)
        out = p2.actor.model[2]
        head = F.linear(h, out.weight, out.bias)
        v = p2.critic.model[2](F.leaky_relu(p2.critic.model[0](s), 0.01))[:, 0]
        _, dh, _, dv = ops.policy_loss("ppo", "categorical", head.contiguous(), None, v.contiguous(), act_buf, adv,
                                       ret, **kw)
        dz = (dh @ out.weight) * torch.where(z > 0, 1.0, 0.01)
        lc = p2.critic.model[0]
        zc = F.linear(s, lc.weight, lc.bias)
        dzc = (dv.reshape(-1, 1) @ p2.critic.model[2].weight) * torch.where(zc > 0, 1.0, 0.01)
    dzc16 = fm2._hws.dz_pair[:, 256:].double()
    dc = (dzc16 - dzc.double()).abs()
    print("critic dz scale %.3e max diff %.3e (%.2e of scale); K16 dv-path vs torch" % (
        dzc.abs().max().item(), dc.max().item(), dc.max().item() / dzc.abs().max().item()))
    bc = dc > 1e-3 * dzc.abs().max().item()
    if bc.any():
        r, c = bc.nonzero()[:10].T
        for i in range(len(r)):
            print("critic row %d col %d zc %.3e dz16 %.3e dz %.3e" % (r[i], c[i], zc[r[i], c[i]], dzc16[r[i], c[i]],
                                                                     dzc[r[i], c[i]]))
    diff = (dz16 - dz.double()).abs()
    scale = dz.abs().max().item()
    bad = diff > 1e-3 * scale
    print("dz scale %.3e  max diff %.3e  elements > 1e-3 scale: %d of %d" % (scale, diff.max().item(),
                                                                            int(bad.sum()), bad.numel()))
    if bad.any():
        r, c = bad.nonzero()[:10].T
        for i in range(len(r)):
            print("row %d col %d  z32 %.3e  z64 %.3e  dz16 %.3e  dz %.3e" % (r[i], c[i], z[r[i], c[i]], z64[r[i], c[i]],
                                                                        dz16[r[i], c[i]], dz[r[i], c[i]]))
    rest = diff.masked_fill(bad, 0).max().item()
    print("max diff outside those: %.3e (%.2e of scale)" % (rest, rest / scale))


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def grads_all():
    """The failing test's body, every parameter's gradient error printed, K16 on and off."""
    from xuanpolicy_amd import ops
    from xuanpolicy_amd.flat import FlatState
    from xuanpolicy_amd.fused_mlp import FusedActorCritic, head_placement
    for gemm in (True, False):
        torch.manual_seed(1)
        D, A, B, R = 17, 6, 8192 + 37, 20000
        p1 = _policy(D, A, True, torch.nn.LeakyReLU, [256])
        p2 = _policy(D, A, True, torch.nn.LeakyReLU, [256])
        p2.load_state_dict(p1.state_dict())
        fs1 = FlatState(p1.parameters())
        fs2 = FlatState(p2.parameters(), placement=head_placement(p2))
        fm1, fm2 = FusedActorCritic(p1), FusedActorCritic(p2, flat=fs2)
        fm2.gemm_heads = gemm
        obs_all = torch.randn(R, D, device=DEV)
        idx = torch.randperm(R, device=DEV)[:B].contiguous()
        idx[5] = R + 3
        idx[B - 1] = -1
        adv = torch.randn(R, device=DEV)
        ret = torch.randn(R, device=DEV)
        act_buf = torch.randint(0, A, (R,), device=DEV).float()
        with torch.no_grad():
            h0, _, _ = p1.heads(obs_all)
            old = torch.distributions.Categorical(logits=h0).log_prob(act_buf.long())
            old = (old + 0.05 * torch.randn(R, device=DEV)).contiguous()
        obs, part = ops.gather_minibatch(idx.clamp(0, R - 1), obs_all, adv=adv)
        kw = dict(old_logp=old, idx=idx, adv_partials=part, clip_range=0.2, vf_coef=0.25, ent_coef=0.01)
        fs1.flat.fill_(7.0)
        fs2.flat.fill_(-7.0)
        head, logstd, v, ctx = fm1.forward(obs)
        s1, dh, _, dv = ops.policy_loss("ppo", "categorical", head, logstd, v, act_buf, adv, ret, **kw)
        fm1.backward(ctx, dh, dv)
        ctx2 = fm2.forward_hidden(obs)
        fm2.loss_backward(ctx2, "ppo", "categorical", act_buf, adv, ret, **kw)
        torch.cuda.synchronize()
        for (n1, x1), (n2, x2) in zip(p1.named_parameters(), p2.named_parameters()):
            ga, gb = x1.grad.double(), x2.grad.double()
            scale = ga.abs().max().item() + 1e-12
            d = (ga - gb).abs()
            print("gemm=%d %-34s err/scale %.2e  argmax %s" % (gemm, n1, d.max().item() / scale,
                                                              tuple(int(u) for u in (d == d.max()).nonzero()[0])))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "grads":
    grads_all()
