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
    import copy
    p3 = copy.deepcopy(p1).double()   # fp64 truth for the gradient check
    rep3 = p3.representation.model if rep_hidden else torch.nn.Identity()   # Basic_MLP casts to f32: run
    s3 = rep3(x.double())                                                 # the Sequential chains directly
    h3 = (p3.actor.model if discrete else p3.actor.mu)(s3)
    v3 = p3.critic.model(s3)[:, 0]
    torch.autograd.backward([h3, v3], [dh.double(), dv.double()])
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
    # random-sign head gradients summed over 65536 rows cancel heavily, so two fp32 summation orders
    # differ well above 1e-5 relative; the bar is: no further from the fp64 gradient than torch's own
    # fp32 autograd (x2), or within 2e-5 of the gradient's scale
    for (n1, a), (n2, b), (n3, c) in zip(p1.named_parameters(), p2.named_parameters(), p3.named_parameters()):
        if n1.endswith("logstd"):
            continue
        ga, gb, gc = a.grad.double(), b.grad.double(), c.grad
        scale = gc.abs().max().item() + 1e-12
        e_torch = (ga - gc).abs().max().item()
        e_ours = (gb - gc).abs().max().item()
        assert e_ours <= max(2 * e_torch, 2e-5 * scale), (n1, e_ours, e_torch, scale)


@pytest.mark.parametrize("algo,discrete,act,rep_hidden,ent,paired,D,A", [
    ("ppo", False, torch.nn.LeakyReLU, [256], 0.0, True, 17, 6), ("ppo", False, torch.nn.LeakyReLU, [256], 0.0, False, 17, 6),
    ("ppo", True, torch.nn.LeakyReLU, [256], 0.01, True, 17, 6), ("a2c", False, torch.nn.Tanh, [64], 0.005, True, 17, 6),
    ("a2c", True, torch.nn.ReLU, [], 0.01, False, 17, 6), ("ppo", False, torch.nn.LeakyReLU, [], 0.0, True, 17, 6),
    ("ppo", False, torch.nn.LeakyReLU, [256], 0.0, True, 376, 17),     # C4 shapes (KMAX 18 bucket)
    ("ppo", True, torch.nn.LeakyReLU, [256], 0.01, True, 33, 18), ("a2c", False, torch.nn.Tanh, [256], 0.01, False, 20, 9)])
def test_fused_heads_match_loss_kernel_path(algo, discrete, act, rep_hidden, ent, paired, D, A):
    """K12 (heads + loss + head backward in one pass) == K2 loss kernel + explicit backward, which the
    drop-in tests pin to the reference's fixtures: loss scalars and every parameter gradient."""
    from xuanpolicy_amd import ops
    from xuanpolicy_amd.flat import FlatState
    from xuanpolicy_amd.fused_mlp import FusedActorCritic
    torch.manual_seed(1)
    B, R = 8192 + 37, 20000
    p1 = _policy(D, A, discrete, act, rep_hidden)
    p2 = _policy(D, A, discrete, act, rep_hidden)
    p2.load_state_dict(p1.state_dict())
    from xuanpolicy_amd.fused_mlp import head_placement
    fs1 = FlatState(p1.parameters())
    fs2 = FlatState(p2.parameters(), placement=head_placement(p2) if paired else None)
    fm1, fm2 = FusedActorCritic(p1), FusedActorCritic(p2, flat=fs2)
    assert fm2.fused_heads and (fm2.pair is not None) == paired
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
    if act is not torch.nn.Tanh:
        # At a ReLU / LeakyReLU kink the derivative is a step: a hidden pre-activation within fp32 rounding
        # of 0 takes either branch depending on the GEMM's summation order (K16's MFMA k-order vs
        # hipBLASLt), moving one unit's gradient by a whole row's contribution.  Such rows are made
        # invalid (idx = -1: both paths give them no gradient) so the comparison is unambiguous.
        with torch.no_grad():
            s_ = p1.representation(obs_all[idx.clamp(0, R - 1)])["state"]
            seq = p1.actor.model if discrete else p1.actor.mu
            near = torch.zeros(B, dtype=torch.bool, device=DEV)
            for lin in (seq[0], p1.critic.model[0]):
                near |= (torch.nn.functional.linear(s_, lin.weight, lin.bias).abs() < 1e-6).any(1)
        assert int(near.sum()) < B // 50
        idx[near] = -1
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
    # the clip norm's squared-sum partials written beside the gradients (xpa_clip_adam_step_partials)
    if fm2.sq_ready is not None:
        buf, cnt = fm2.sq_ready
        sq_fused = float(buf[:cnt].sum())
        sq_true = sum(float((x.grad.double() ** 2).sum()) for x in p2.parameters())
        assert abs(sq_fused - sq_true) <= 1e-9 * sq_true, (sq_fused, sq_true)
    else:   # the C2 / C4 fast path (paired heads on a [256] thin trunk) must cover every gradient
        assert not (paired and rep_hidden == [256] and D <= 64)


@pytest.mark.parametrize("rows,din,code", [(1000, 17, 1), (65536 + 5, 17, 1), (77, 4, 2), (4096, 33, 0),
                                           (3000, 64, 1), (129, 8, 2)])
def test_thin_first_layer_kernels(rows, din, code):
    """K13 forward / backward vs torch fp32 (F.linear + activation, autograd)."""
    from xuanpolicy_amd import ops
    L = ops.lib()
    torch.manual_seed(rows + din)
    slope = 0.01
    x = torch.randn(rows, din, device=DEV)
    lin = torch.nn.Linear(din, 256).to(DEV)
    act = {0: lambda z: z, 1: lambda z: torch.nn.functional.leaky_relu(z, slope), 2: torch.tanh}[code]
    xr = x.clone().requires_grad_(False)
    h_ref = act(torch.nn.functional.linear(xr, lin.weight, lin.bias))
    h = torch.empty(rows, 256, device=DEV)
    s = ops._stream()
    assert L.xpa_thin_linear_act_fwd(code, ops._p(x), din, rows, din, 256, ops._p(lin.weight), ops._p(lin.bias),
                                     slope, ops._p(h), 256, s) == 0
    torch.testing.assert_close(h, h_ref.detach(), rtol=1e-5, atol=1e-5)
    g = torch.randn(rows, 256, device=DEV) * 1e-2
    h_ref.backward(g)
    G = int(L.xpa_thin_bwd_num_partials(rows))
    pdw = torch.empty(G, 256 * din, device=DEV)
    pdb = torch.empty(G, 256, device=DEV)
    dw = torch.empty(256, din, device=DEV)
    db = torch.empty(256, device=DEV)
    assert L.xpa_thin_linear_act_bwd(code, ops._p(g), 256, ops._p(h), 256, rows, ops._p(x), din, din, 256, slope,
                                     ops._p(pdw), ops._p(pdb), s) == 0
    assert L.xpa_colsum_finalize(ops._p(pdw), G, 256 * din, ops._p(dw), s) == 0
    assert L.xpa_colsum_finalize(ops._p(pdb), G, 256, ops._p(db), s) == 0
    for got, exp in ((dw, lin.weight.grad), (db, lin.bias.grad)):
        scale = exp.abs().max().item()
        assert (got - exp).abs().max().item() <= 2e-5 * scale + 1e-6
    # invalid arguments launch nothing
    assert L.xpa_thin_linear_act_fwd(code, ops._p(x), din, rows, 65, 256, ops._p(lin.weight), ops._p(lin.bias),
                                     slope, ops._p(h), 256, s) != 0


@pytest.mark.parametrize("rows,din,code", [(4096, 17, 1), (1001, 8, 2), (77, 33, 0)])
def test_thin_forward_with_fused_normalisation(rows, din, code):
    """xpa_thin_linear_act_fwd_norm == xpa_obs_normalize (into xn and the buffer column) followed by
    xpa_thin_linear_act_fwd: identical normalised rows, h within fp32 rounding."""
    from xuanpolicy_amd import ops
    torch.manual_seed(rows + din)
    X = torch.randn(rows, din + 3, device=DEV) * 3 + 1
    x = X[:, :din]
    mean, var = torch.randn(din, device=DEV), torch.rand(din, device=DEV) + 0.1
    W, b = torch.randn(256, din, device=DEV) * 0.2, torch.randn(256, device=DEV) * 0.1
    T = 5
    cur = torch.tensor([3, 0, 0, 0], dtype=torch.int32, device=DEV)
    L = ops.lib()
    s = ops._stream()
    outs = []
    for fused in (False, True):
        xn = torch.zeros(rows, din, device=DEV)
        col = torch.zeros(rows, T, din, device=DEV)
        h = torch.empty(rows, 256, device=DEV)
        if fused:
            assert L.xpa_thin_linear_act_fwd_norm(code, ops._p(x), x.stride(0), rows, din, 256, ops._p(W), ops._p(b),
                                                   0.01, ops._p(h), 256, ops._p(mean), ops._p(var), 5.0, ops._p(xn),
                                                   din, ops._p(col), T * din, ops._p(cur), s) == 0
        else:
            ops.obs_normalize(x, mean, var, 5.0, xn, col_out=col, col_ld=T * din, cursor=cur)
            assert L.xpa_thin_linear_act_fwd(code, ops._p(xn), din, rows, din, 256, ops._p(W), ops._p(b), 0.01,
                                             ops._p(h), 256, s) == 0
        outs.append((xn, col, h))
    (xa, ca, ha), (xb, cb, hb) = outs
    assert torch.equal(xa, xb) and torch.equal(ca, cb)
    torch.testing.assert_close(hb, ha, rtol=1e-6, atol=1e-6)


def test_colsum_finalize_batch_matches_single():
    """xpa_colsum_finalize_batch == per-segment xpa_colsum_finalize (bitwise: same fixed-order f64 sums),
    more segments than one launch holds."""
    from xuanpolicy_amd import ops
    L = ops.lib()
    torch.manual_seed(3)
    shapes = [(512, 1536), (512, 6), (256, 4352), (1, 3), (700, 1), (64, 256)] * 3
    q = ops.ColsumQueue()
    outs, refs = [], []
    s = ops._stream()
    for G, C in shapes:
        part = torch.randn(G, C, device=DEV)
        out = torch.full((C,), 9.0, device=DEV)
        ref = torch.empty(C, device=DEV)
        assert L.xpa_colsum_finalize(ops._p(part), G, C, ops._p(ref), s) == 0
        q.add(part, out)
        outs.append(out)
        refs.append(ref)
    q.flush()
    q.add(torch.zeros(2, 2, device=DEV), torch.zeros(2, device=DEV))
    q.flush()                      # a second plan
    for o, r in zip(outs, refs):
        assert torch.equal(o, r)


@pytest.mark.parametrize("discrete,act,D,A", [(False, torch.nn.LeakyReLU, 17, 6), (True, torch.nn.LeakyReLU, 17, 6),
                                              (False, torch.nn.Tanh, 17, 6), (False, torch.nn.LeakyReLU, 376, 17),
                                              (True, torch.nn.LeakyReLU, 40, 18)])
def test_rollout_policy_head_matches_sample_kernel(discrete, act, D, A):
    """K14 (trunk + paired hidden GEMM + heads + sample/store) == policy_heads (nn modules) + K3 on the
    same cursor/seed: same RNG draws, so actions / log-probs / values agree to fp32 rounding."""
    from xuanpolicy_amd import ops
    from xuanpolicy_amd.flat import FlatState
    from xuanpolicy_amd.fused_mlp import FusedActorCritic, head_placement
    from xuanpolicy_amd.policies import policy_heads
    torch.manual_seed(5)
    N, T = 4096 + 3, 8
    pol = _policy(D, A, discrete, act, [256])
    fs = FlatState(pol.parameters(), placement=head_placement(pol))
    fm = FusedActorCritic(pol, flat=fs)
    assert fm.rollout_ok
    x = torch.randn(N, D, device=DEV)
    cur = torch.tensor([3, 77, 0, 0], dtype=torch.int32, device=DEV)
    dist = "categorical" if discrete else "gaussian"
    bufs = []
    for path in ("k3", "k14"):
        ba = torch.zeros((N, T) if discrete else (N, T, A), device=DEV)
        bl, bv = torch.zeros(N, T, device=DEV), torch.zeros(N, T, device=DEV)
        env_in = torch.zeros(N, A, device=DEV)
        if path == "k3":
            with torch.no_grad():
                head, logstd, v = policy_heads(pol, x)
            ops.rollout_sample(dist, head.contiguous(), logstd, v.contiguous(), cur, 1234, ba, bl, bv, env_in)
        else:
            fm.rollout_act(x, dist, cur, 1234, ba, bl, bv, env_in)
        bufs.append((ba, bl, bv, env_in))
    (a1, l1, v1, e1), (a2, l2, v2, e2) = bufs
    torch.testing.assert_close(v2, v1, rtol=1e-5, atol=1e-5)
    if discrete:   # inverse-CDF picks agree except where u sits within rounding of a CDF boundary
        assert (a1 != a2).float().mean().item() < 1e-3
        same = (a1 == a2)
        torch.testing.assert_close(l2[same], l1[same], rtol=1e-5, atol=1e-5)
    else:
        torch.testing.assert_close(a2, a1, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(l2, l1, rtol=1e-5, atol=1e-4)
        torch.testing.assert_close(e2, e1, rtol=1e-5, atol=1e-5)
    vb = fm.rollout_value(x)
    with torch.no_grad():
        torch.testing.assert_close(vb, policy_heads(pol, x)[2], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("D,A,act", [(17, 6, torch.nn.LeakyReLU), (64, 3, torch.nn.Tanh), (5, 17, torch.nn.LeakyReLU)])
def test_rollout_head_with_fused_env_step(D, A, act):
    """K14 with the SynthBox env step fused in (xpa_rollout_policy_head_synthbox) == K14 followed by the env's
    own step (env GEMM + K7): the buffers bitwise, the env's outputs to fp32 rounding of its pre-activation
    (a fixed-order chain instead of the GEMM), its flags and episode counters exactly away from the
    termination threshold."""
    from xuanpolicy_amd.envs import SynthBoxVecEnv
    from xuanpolicy_amd.flat import FlatState
    from xuanpolicy_amd.fused_mlp import FusedActorCritic, head_placement
    from oracle import synth_env
    torch.manual_seed(7)
    N, T = 4096 + 3, 8
    pol = _policy(D, A, False, act, [256])
    fs = FlatState(pol.parameters(), placement=head_placement(pol))
    fm = FusedActorCritic(pol, flat=fs)
    envs = [SynthBoxVecEnv(N, D, A, seed=3, max_episode_steps=4, device=DEV) for _ in range(2)]
    for step in range(6):
        x = envs[0].obs.clone()
        cur = torch.tensor([step % T, 100 + step, 0, 0], dtype=torch.int32, device=DEV)
        outs = []
        for fused, env in zip((False, True), envs):
            ba = torch.zeros(N, T, A, device=DEV)
            bl, bv = torch.zeros(N, T, device=DEV), torch.zeros(N, T, device=DEV)
            if fused:
                assert env.fusable_with_policy_step("gaussian")
                fm.rollout_act(x, "gaussian", cur, 99, ba, bl, bv, env.act_in, env=env)
            else:
                fm.rollout_act(x, "gaussian", cur, 99, ba, bl, bv, env.act_in)
                env.step_device()
            outs.append((ba, bl, bv, env))
        (a1, l1, v1, e1), (a2, l2, v2, e2) = outs
        assert torch.equal(a1, a2) and torch.equal(l1, l2) and torch.equal(v1, v2)
        assert torch.equal(e1.act_in, e2.act_in)
        torch.testing.assert_close(e2.final_obs, e1.final_obs, rtol=1e-5, atol=2e-6)
        torch.testing.assert_close(e2.rew, e1.rew, rtol=1e-5, atol=1e-6)
        near = (e1.final_obs[:, 0] - synth_env.TERM_THRESH).abs() < 1e-5
        assert torch.equal(e1.term[~near], e2.term[~near]) and torch.equal(e1.trunc, e2.trunc)
        assert torch.equal(e1.ep_step[~near], e2.ep_step[~near])
        e2.X.copy_(e1.X)   # re-sync the states (tanh dynamics amplify ulps over steps)
        for name in ("ep_step", "ep_index", "ep_score", "ep_last_score", "ep_last_len"):
            getattr(e2, name).copy_(getattr(e1, name))
    assert int(envs[0].ep_index.sum()) > 0


@pytest.mark.parametrize("nseg,dist", [(3, 0), (17, 0), (3, 1), (0, 0)])
def test_colsum_queue_deferred_loss_finalize(nseg, dist):
    """ColsumQueue.defer_loss: the loss finalize run as the batched finalize's extra block (one plan) or on
    its own ahead of it (more segments than one launch holds) == xpa_policy_loss_finalize_sq called
    directly: loss scalars and d logstd bitwise, and the clip-norm total = the outputs' squares + d logstd's."""
    from xuanpolicy_amd import ops
    L, s = ops.lib(), ops._stream()
    torch.manual_seed(nseg + dist)
    B, K, G = 65536, 6, 512
    W = int(L.xpa_loss_partial_width(K))
    lp = torch.randn(G, W, device=DEV) * 0.01
    sc_ref, dls_ref = torch.zeros(ops.N_OUT, device=DEV), torch.zeros(K, device=DEV)
    sq_ref = torch.zeros(1, dtype=torch.float64, device=DEV)
    assert L.xpa_policy_loss_finalize_sq(0, dist, B, K, ops._p(lp), G, 0.25, 0.01, ops._p(sc_ref), ops._p(dls_ref),
                                         ops._p(sq_ref), s) == 0
    q = ops.ColsumQueue()
    outs = []
    for i in range(nseg):
        part = torch.randn(8 if i % 2 else 64, 300 + i, device=DEV)
        out = torch.empty(300 + i, device=DEV)
        q.add(part, out)
        outs.append(out)
    sc, dls = torch.zeros(ops.N_OUT, device=DEV), torch.zeros(K, device=DEV)
    sq = torch.zeros(16384, dtype=torch.float64, device=DEV)
    q.defer_loss(0, dist, B, K, lp, 0.25, 0.01, sc, dls)
    total, written = q.flush(DEV, sq=sq)
    torch.cuda.synchronize()
    assert torch.equal(sc, sc_ref)
    if dist == 0:
        assert torch.equal(dls, dls_ref)
    assert float(sq[0]) == float(sq_ref[0])
    assert written == sum(o.numel() for o in outs) and q.loss is None
    if nseg == 0:   # nothing queued but the loss: it still runs, no norm total
        assert total is None
    elif nseg <= ops.ColsumQueue.MAX_SEGS:
        exp = sum(float((o.double() ** 2).sum()) for o in outs) + float(sq_ref[0])
        assert total is not None and abs(float(total) - exp) <= 1e-9 * max(exp, 1.0)
    else:
        assert total is None


@pytest.mark.parametrize("algo,dist,K,B,code,form", [
    ("a2c", "categorical", 18, 777, 0, "k16"),    # the r01 aperture-violation configuration
    ("ppo", "gaussian", 17, 4133, 1, "k16"),      # C4 head width, ragged tail (4133 = 64 * 64 + 37)
    ("ppo", "categorical", 18, 193, 2, "k16"),
    ("a2c", "gaussian", 6, 65, 1, "k16"),
    ("ppo", "gaussian", 6, 64, 0, "k16"),
    # K16W: ragged tails, one tile, a grid below the tile count (20037 rows = 314 tiles on 256 blocks: partial rows
    # 256..313 written as zeros), 8-wide heads
    ("ppo", "gaussian", 6, 4133, 1, "ws"),
    ("a2c", "categorical", 8, 777, 0, "ws"),
    ("ppo", "categorical", 4, 64, 2, "ws"),
    ("ppo", "gaussian", 6, 20037, 1, "ws"),
    ("a2c", "gaussian", 8, 33, 1, "ws"),
    # K16S (the GEMM by the bf16 three-way split): the K16 case matrix's shapes
    ("a2c", "categorical", 18, 777, 0, "s3"),
    ("ppo", "gaussian", 17, 4133, 1, "s3"),
    ("ppo", "categorical", 18, 193, 2, "s3"),
    ("ppo", "gaussian", 6, 20037, 1, "s3"),
    ("a2c", "gaussian", 6, 65, 1, "s3"),
    # K16P (Wh's planes split once, DMA'd)
    ("ppo", "gaussian", 6, 4133, 1, "s3p"),
    ("a2c", "categorical", 18, 777, 0, "s3p"),
    ("ppo", "categorical", 8, 193, 2, "s3p"),
    ("ppo", "gaussian", 17, 4133, 1, "s3p"),   # C4's head on the production split form
])
@pytest.mark.parametrize("poison", [False, True])
def test_head_gemm_kernels_vs_fp64_autograd(algo, dist, K, B, code, form, poison):
    """K16 (xpa_head_gemm_actor / _critic), K16W (xpa_head_gemm_ws_*) or K16S (xpa_head_gemm_s3_*) through the C ABI against float64 autograd
    of the same head:
    z = x Wh^T + bh, h = act(z), head = h W^T + b, the PPO-Clip / A2C loss with Gaussian / Categorical
    log-prob + entropy (ppoclip_learner.py:32-44, a2c_learner.py:24-31) and the critic's value loss.
    Checked: dz (d loss / d z), the summed per-block partials (dW_out, db_out, db_hidden, loss sums) and
    untouched memory around every output (canaries on both sides of dz and the partials).  poison: every CU's LDS
    filled with NaN bit patterns first (xpa_lds_poison) — a kernel reading LDS it did not write shows it (r04: the
    critic's phase 2 read the unwritten pad slot of d head)."""
    from xuanpolicy_amd import ops
    L, s = ops.lib(), ops._stream()
    g = torch.Generator(device=DEV).manual_seed(B + K)
    H, R = 256, B + 300
    slope = 0.01
    x = torch.randn(B, H, device=DEV, generator=g)
    wh_a, wh_c = (torch.randn(H, H, device=DEV, generator=g) / 16 for _ in range(2))
    bh_a, bh_c = (torch.randn(H, device=DEV, generator=g) * 0.1 for _ in range(2))
    w_a = torch.randn(K, H, device=DEV, generator=g) / 16
    b_a = torch.randn(K, device=DEV, generator=g) * 0.1
    w_c = torch.randn(1, H, device=DEV, generator=g) / 16
    b_c = torch.randn(1, device=DEV, generator=g) * 0.1
    logstd = (-1 + 0.1 * torch.randn(K, device=DEV, generator=g)) if dist == "gaussian" else None
    idx = torch.randperm(R, device=DEV, generator=g)[:B].contiguous()
    idx[B // 2] = -1           # invalid rows contribute nothing
    idx[B - 1] = R + 5
    adv = torch.randn(R, device=DEV, generator=g)
    ret = torch.randn(R, device=DEV, generator=g)
    if dist == "gaussian":
        act = torch.randn(R, K, device=DEV, generator=g) * 0.5
    else:
        act = torch.randint(0, K, (R,), device=DEV, generator=g).float()
    old = -1.5 + 0.3 * torch.randn(R, device=DEV, generator=g) if algo == "ppo" else None
    if code != 2:   # kinks: rows with a pre-activation within rounding of 0 take either branch -> invalid
        with torch.no_grad():
            near = ((x @ wh_a.t() + bh_a).abs() < 1e-5).any(1) | ((x @ wh_c.t() + bh_c).abs() < 1e-5).any(1)
        idx[near] = -1
    G = int(L.xpa_head_fused_num_partials(B))
    W = int(L.xpa_loss_partial_width(K))
    pad = 64
    dz_buf = torch.full((B * 2 * H + 2 * pad,), 777.0, device=DEV)   # canaries around the [B, 512] pair
    dz = dz_buf[pad:pad + B * 2 * H].view(B, 2 * H)

    def canary(n):
        return torch.full((n + 2 * pad,), 555.0, device=DEV)
    p_dw_a, p_dbh_a, p_dbo_a = canary(G * K * H), canary(G * H), canary(G * K)
    p_dw_c, p_dbh_c, p_dbo_c = canary(G * H), canary(G * H), canary(G)
    lp = torch.zeros(G * W + 2 * pad, device=DEV)
    lp[:pad] = 555.0
    lp[pad + G * W:] = 555.0
    v = lambda t: ops._p(t[pad:])   # noqa: E731
    algo_c, dist_c = ops.ALGO[algo], ops.DIST[dist]
    ent, clip, vf = 0.01, 0.2, 0.25
    pre = {"k16": "xpa_head_gemm_", "ws": "xpa_head_gemm_ws_", "s3": "xpa_head_gemm_s3_", "s3p": "xpa_head_gemm_s3p_"}[form]
    fa, fc = getattr(L, pre + "actor"), getattr(L, pre + "critic")
    if poison:
        torch.cuda.synchronize()
        assert L.xpa_lds_poison(s) == 0
    if form == "s3p":   # the hidden weights as Wh^T's three bf16 planes
        wh_a_arg, wh_c_arg = ops.s3_split(wh_a.t()), ops.s3_split(wh_c.t())
    else:
        wh_a_arg, wh_c_arg = wh_a, wh_c
    assert fa(algo_c, dist_c, code, B, K, H, ops._p(x), H, ops._p(wh_a_arg), ops._p(bh_a), 2 * H,
              ops._p(w_a), ops._p(b_a), slope, ops._p(logstd) if logstd is not None else None,
              ops._p(idx), R, ops._p(act), ops._p(old) if old is not None else None, ops._p(adv),
              None, 0, clip, ent, ops._p(dz), v(p_dw_a), v(p_dbh_a), v(p_dbo_a), v(lp), W, s) == 0
    if poison:   # the critic launch behind fresh poison too (else it sees the actor's leftovers)
        assert L.xpa_lds_poison(s) == 0
    assert fc(code, B, H, ops._p(x), H, ops._p(wh_c_arg), ops._p(bh_c), 2 * H, ops._p(w_c),
              ops._p(b_c), slope, ops._p(idx), R, ops._p(ret), vf, ops._p(dz[:, H:]), v(p_dw_c),
              v(p_dbh_c), v(p_dbo_c), v(lp), W, s) == 0
    torch.cuda.synchronize()
    for t in (p_dw_a, p_dbh_a, p_dbo_a, p_dw_c, p_dbh_c, p_dbo_c):
        assert bool((t[:pad] == 555.0).all()) and bool((t[-pad:] == 555.0).all()), "partials written out of bounds"
    assert bool((lp[:pad] == 555.0).all()) and bool((lp[-pad:] == 555.0).all()), "loss partials out of bounds"
    assert bool((dz_buf[:pad] == 777.0).all()) and bool((dz_buf[-pad:] == 777.0).all()), "dz out of bounds"

    # float64 autograd reference
    d = lambda t: t.detach().double().cpu()   # noqa: E731
    act_fn = {0: lambda z: z, 1: lambda z: torch.nn.functional.leaky_relu(z, slope), 2: torch.tanh}[code]
    idx_c = idx.cpu()
    valid = (idx_c >= 0) & (idx_c < R)
    rows = idx_c.clamp(0, R - 1)
    A_n = d(adv)[rows]
    za = (d(x) @ d(wh_a).t() + d(bh_a)).requires_grad_(True)
    zc = (d(x) @ d(wh_c).t() + d(bh_c)).requires_grad_(True)
    wa, ba, wc, bc = (d(t).requires_grad_(True) for t in (w_a, b_a, w_c, b_c))
    head = act_fn(za) @ wa.t() + ba
    vv = (act_fn(zc) @ wc.t() + bc)[:, 0]
    ls = d(logstd).requires_grad_(True) if logstd is not None else None
    if dist == "gaussian":
        nd = torch.distributions.Normal(head, ls.exp())
        logp = nd.log_prob(d(act)[rows]).sum(-1)
        entr = nd.entropy().sum(-1)
    else:
        cd = torch.distributions.Categorical(logits=head)
        logp = cd.log_prob(d(act)[rows].long())
        entr = cd.entropy()
    m = valid.double()
    if algo == "ppo":
        ratio = (logp - d(old)[rows]).exp()
        surr = torch.minimum(ratio.clamp(1 - clip, 1 + clip) * A_n, ratio * A_n)
    else:
        surr = A_n * logp
    actor_loss = -(surr * m).sum() / B
    entropy = (entr * m).sum() / B
    critic = ((vv - d(ret)[rows]) ** 2 * m).sum() / B
    total = actor_loss - ent * entropy + vf * critic
    total.backward()

    def close(got, exp, what, rel=2e-5):
        scale = exp.abs().max().item() + 1e-12
        err = (got.double().cpu() - exp).abs().max().item()
        assert err <= rel * scale + 1e-9, (what, err, scale)
    close(dz[:, :H], za.grad, "dz actor")
    close(dz[:, H:], zc.grad, "dz critic")
    close(p_dw_a[pad:-pad].view(G, K * H).double().sum(0).view(K, H), wa.grad, "dW_out actor")
    close(p_dbo_a[pad:-pad].view(G, K).double().sum(0), ba.grad, "db_out actor")
    close(p_dbh_a[pad:-pad].view(G, H).double().sum(0), za.grad.sum(0), "db_hidden actor")
    close(p_dw_c[pad:-pad].view(G, H).double().sum(0).view(1, H), wc.grad, "dW_out critic")
    close(p_dbo_c[pad:-pad].view(G, 1).double().sum(0), bc.grad, "db_out critic")
    close(p_dbh_c[pad:-pad].view(G, H).double().sum(0), zc.grad.sum(0), "db_hidden critic")
    sc = torch.zeros(ops.N_OUT, device=DEV)
    dls = torch.zeros(K, device=DEV)
    assert L.xpa_policy_loss_finalize(algo_c, dist_c, B, K, v(lp), G, vf, ent, ops._p(sc), ops._p(dls), s) == 0
    torch.cuda.synchronize()
    got = sc.double().cpu()
    assert abs(got[0] - actor_loss.item()) < 1e-5 and abs(got[1] - critic.item() * 1.0 / 1.0) < 1e-5
    assert abs(got[2] - entropy.item()) < 1e-5 and abs(got[3] - total.item()) < 1e-5
    if ls is not None:
        close(dls, ls.grad, "d logstd", rel=1e-5)


@pytest.mark.parametrize("algo,dist,K,B", [("ppo", "gaussian", 6, 65536), ("a2c", "categorical", 4, 20037),
                                          ("ppo", "gaussian", 6, 3000), ("ppo", "categorical", 8, 130)])
def test_head_gemm_ws_equals_k16(algo, dist, K, B):
    """K16W (wave-specialised) against K16 on the same inputs: dz bit for bit (the same GEMM k order, the same epilogue
    chains, only the thread running each changes) and the per-block partials summed over their rows to f32 rounding
    (the two grids group the tiles into blocks differently); every partial row K16W's grid does not own is 0."""
    from xuanpolicy_amd import ops
    L, s = ops.lib(), ops._stream()
    g = torch.Generator(device=DEV).manual_seed(B * 3 + K)
    H, R = 256, B + 100
    x = torch.randn(B, H, device=DEV, generator=g)
    wh_a, wh_c = (torch.randn(H, H, device=DEV, generator=g) / 16 for _ in range(2))
    bh_a, bh_c = (torch.randn(H, device=DEV, generator=g) * 0.1 for _ in range(2))
    w_a, b_a = torch.randn(K, H, device=DEV, generator=g) / 16, torch.randn(K, device=DEV, generator=g) * 0.1
    w_c, b_c = torch.randn(1, H, device=DEV, generator=g) / 16, torch.randn(1, device=DEV, generator=g) * 0.1
    logstd = (-1 + 0.1 * torch.randn(K, device=DEV, generator=g)) if dist == "gaussian" else None
    idx = torch.randperm(R, device=DEV, generator=g)[:B].contiguous()
    adv, ret = torch.randn(R, device=DEV, generator=g), torch.randn(R, device=DEV, generator=g)
    act = (torch.randn(R, K, device=DEV, generator=g) * 0.5 if dist == "gaussian"
           else torch.randint(0, K, (R,), device=DEV, generator=g).float())
    old = -1.5 + 0.3 * torch.randn(R, device=DEV, generator=g) if algo == "ppo" else None
    G = int(L.xpa_head_fused_num_partials(B))
    Wd = int(L.xpa_loss_partial_width(K))
    outs = []
    for ws in (False, True):
        dz = torch.full((B, 2 * H), 123.0, device=DEV)
        parts = [torch.full((G, n), 9.0, device=DEV) for n in (K * H, H, K, H, H, 1)]
        lp = torch.zeros(G, Wd, device=DEV)
        fa = L.xpa_head_gemm_ws_actor if ws else L.xpa_head_gemm_actor
        fc = L.xpa_head_gemm_ws_critic if ws else L.xpa_head_gemm_critic
        assert fa(ops.ALGO[algo], ops.DIST[dist], 1, B, K, H, ops._p(x), H, ops._p(wh_a), ops._p(bh_a), 2 * H,
                  ops._p(w_a), ops._p(b_a), 0.01, ops._p(logstd), ops._p(idx), R, ops._p(act), ops._p(old),
                  ops._p(adv), None, 0, 0.2, 0.01, ops._p(dz), ops._p(parts[0]), ops._p(parts[1]), ops._p(parts[2]),
                  ops._p(lp), Wd, s) == 0
        assert fc(1, B, H, ops._p(x), H, ops._p(wh_c), ops._p(bh_c), 2 * H, ops._p(w_c), ops._p(b_c), 0.01,
                  ops._p(idx), R, ops._p(ret), 0.25, ops._p(dz[:, H:]), ops._p(parts[3]), ops._p(parts[4]),
                  ops._p(parts[5]), ops._p(lp), Wd, s) == 0
        torch.cuda.synchronize()
        outs.append((dz, parts, lp))
    (dz0, p0, l0), (dz1, p1, l1) = outs
    assert torch.equal(dz0, dz1), "dz differs from K16"
    gw = int(L.xpa_head_gemm_ws_grid(B))
    assert gw == min(G, 256)
    for a, b in zip(p0 + [l0], p1 + [l1]):
        if G > gw:
            assert bool((b[gw:] == 0).all()), "rows beyond K16W's grid must be zero"
        torch.testing.assert_close(b.double().sum(0), a.double().sum(0), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("rows,n_rows,din", [(65536, 524288, 17), (1000, 5000, 4), (77, 300, 17)])
def test_thin_gather_forms_equal_k4_then_k13(rows, n_rows, din):
    """K13 with K4's gather folded in (xpa_thin_linear_act_fwd_gather / _bwd_gather) == xpa_gather_minibatch then
    the plain K13 forms, bit for bit: h, the gathered rows (x_out), the adv-moment partials, and the dW / db
    partials; out-of-range indices give zero rows and add nothing."""
    import torch
    from xuanpolicy_amd import _lib, ops
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(rows)
    flat = torch.randn(n_rows, din, generator=g).to(dev)
    adv = torch.randn(n_rows, generator=g).to(dev)
    idx = torch.randint(0, n_rows, (rows,), generator=g)
    idx[::97] = -3            # masked rows
    idx[5::131] = n_rows + 7
    idx = idx.to(dev)
    lin = torch.nn.Linear(din, 256).to(dev)
    L, st = ops.lib(), ops._stream(dev)
    xg, part = ops.gather_minibatch(idx, flat, adv=adv)
    h_ref = torch.empty(rows, 256, device=dev)
    _lib.check(L.xpa_thin_linear_act_fwd(1, ops._p(xg), din, rows, din, 256, ops._p(lin.weight), ops._p(lin.bias),
                                         0.01, ops._p(h_ref), 256, st), "fwd")
    h = torch.empty(rows, 256, device=dev)
    part2 = torch.empty_like(part)
    xo = torch.empty(rows, din, device=dev)
    _lib.check(L.xpa_thin_linear_act_fwd_gather(1, ops._p(flat), din, n_rows, ops._p(idx), rows, din, 256,
                                                ops._p(lin.weight), ops._p(lin.bias), 0.01, ops._p(h), 256, ops._p(adv),
                                                ops._p(part2), ops._p(xo), st), "fwd_gather")
    assert torch.equal(h, h_ref) and torch.equal(part2, part) and torch.equal(xo, xg)
    gr = torch.randn(rows, 256, generator=g).to(dev)
    G = int(L.xpa_thin_bwd_num_partials(rows))
    pw, pb = torch.empty(G, 256 * din, device=dev), torch.empty(G, 256, device=dev)
    pw2, pb2 = torch.empty_like(pw), torch.empty_like(pb)
    _lib.check(L.xpa_thin_linear_act_bwd(1, ops._p(gr), 256, ops._p(h), 256, rows, ops._p(xg), din, din, 256, 0.01,
                                         ops._p(pw), ops._p(pb), st), "bwd")
    _lib.check(L.xpa_thin_linear_act_bwd_gather(1, ops._p(gr), 256, ops._p(h), 256, rows, ops._p(flat), din, n_rows,
                                                ops._p(idx), din, 256, 0.01, ops._p(pw2), ops._p(pb2), st), "bwd_gather")
    assert torch.equal(pw, pw2) and torch.equal(pb, pb2)


@pytest.mark.parametrize("algo,dist,K,B,code,din", [
    ("ppo", "gaussian", 6, 4133, 1, 17),    # the C2 head and trunk widths, ragged tail (4133 = 64 * 64 + 37)
    ("a2c", "categorical", 4, 777, 0, 4),
    ("ppo", "categorical", 8, 193, 2, 20),
    ("a2c", "gaussian", 6, 64, 1, 17),
])
def test_head_gemm_trunk_kernels_equal_k13_then_k16(algo, dist, K, B, code, din):
    """K16X (xpa_head_gemm_trunk_actor / _critic: the trunk layer Linear(d_in, 256) + act formed in the prologue)
    against K13 (xpa_thin_linear_act_fwd) followed by K16 on the same inputs, bit for bit: the h the launches write
    (same fmaf chain as K13), dz, every per-block partial and the loss partials (same k loop and epilogue as K16);
    canaries around h, dz and the partials.  (K16 itself is checked against float64 autograd above.)"""
    from xuanpolicy_amd import ops
    L, s = ops.lib(), ops._stream()
    g = torch.Generator(device=DEV).manual_seed(B + K + din)
    H, R = 256, B + 300
    slope = 0.01
    xr = torch.randn(B, din, device=DEV, generator=g)
    w0 = torch.randn(H, din, device=DEV, generator=g) / 4
    b0 = torch.randn(H, device=DEV, generator=g) * 0.1
    wh_a, wh_c = (torch.randn(H, H, device=DEV, generator=g) / 16 for _ in range(2))
    bh_a, bh_c = (torch.randn(H, device=DEV, generator=g) * 0.1 for _ in range(2))
    w_a = torch.randn(K, H, device=DEV, generator=g) / 16
    b_a = torch.randn(K, device=DEV, generator=g) * 0.1
    w_c = torch.randn(1, H, device=DEV, generator=g) / 16
    b_c = torch.randn(1, device=DEV, generator=g) * 0.1
    logstd = (-1 + 0.1 * torch.randn(K, device=DEV, generator=g)) if dist == "gaussian" else None
    idx = torch.randperm(R, device=DEV, generator=g)[:B].contiguous()
    idx[B // 2] = -1
    adv = torch.randn(R, device=DEV, generator=g)
    ret = torch.randn(R, device=DEV, generator=g)
    act = (torch.randn(R, K, device=DEV, generator=g) * 0.5 if dist == "gaussian"
           else torch.randint(0, K, (R,), device=DEV, generator=g).float())
    old = -1.5 + 0.3 * torch.randn(R, device=DEV, generator=g) if algo == "ppo" else None
    h_ref = torch.empty(B, H, device=DEV)
    assert L.xpa_thin_linear_act_fwd(code, ops._p(xr), din, B, din, H, ops._p(w0), ops._p(b0), slope, ops._p(h_ref), H,
                                     s) == 0
    G = int(L.xpa_head_fused_num_partials(B))
    W = int(L.xpa_loss_partial_width(K))
    pad = 64
    algo_c, dist_c = ops.ALGO[algo], ops.DIST[dist]
    ent, clip, vf = 0.01, 0.2, 0.25

    def run(trunk):
        cz = lambda n, v=555.0: torch.full((n + 2 * pad,), v, device=DEV)   # noqa: E731
        out = dict(dz=cz(B * 2 * H, 777.0), h=cz(B * H, 333.0), p_dw_a=cz(G * K * H), p_dbh_a=cz(G * H),
                   p_dbo_a=cz(G * K), p_dw_c=cz(G * H), p_dbh_c=cz(G * H), p_dbo_c=cz(G), lp=cz(G * W))
        out["lp"][pad:-pad] = 0.0
        v = lambda k: ops._p(out[k][pad:])   # noqa: E731
        dz = out["dz"][pad:pad + B * 2 * H].view(B, 2 * H)
        p_ls = ops._p(logstd) if logstd is not None else None
        p_old = ops._p(old) if old is not None else None
        if trunk:
            assert L.xpa_head_gemm_trunk_actor(
                algo_c, dist_c, code, B, K, H, ops._p(xr), din, din, ops._p(w0), ops._p(b0), slope, v("h"), H,
                ops._p(wh_a), ops._p(bh_a), 2 * H, ops._p(w_a), ops._p(b_a), slope, p_ls, ops._p(idx), R, ops._p(act),
                p_old, ops._p(adv), None, 0, clip, ent, ops._p(dz), v("p_dw_a"), v("p_dbh_a"), v("p_dbo_a"), v("lp"),
                W, s) == 0
            h2 = torch.empty(B, H, device=DEV)
            assert L.xpa_head_gemm_trunk_critic(
                code, B, H, ops._p(xr), din, din, ops._p(w0), ops._p(b0), slope, ops._p(h2), H, ops._p(wh_c), ops._p(bh_c),
                2 * H, ops._p(w_c), ops._p(b_c), slope, ops._p(idx), R, ops._p(ret), vf, ops._p(dz[:, H:]),
                v("p_dw_c"), v("p_dbh_c"), v("p_dbo_c"), v("lp"), W, s) == 0
        else:
            assert L.xpa_head_gemm_actor(algo_c, dist_c, code, B, K, H, ops._p(h_ref), H, ops._p(wh_a), ops._p(bh_a),
                                         2 * H, ops._p(w_a), ops._p(b_a), slope, p_ls, ops._p(idx), R, ops._p(act),
                                         p_old, ops._p(adv), None, 0, clip, ent, ops._p(dz), v("p_dw_a"), v("p_dbh_a"),
                                         v("p_dbo_a"), v("lp"), W, s) == 0
            assert L.xpa_head_gemm_critic(code, B, H, ops._p(h_ref), H, ops._p(wh_c), ops._p(bh_c), 2 * H,
                                          ops._p(w_c), ops._p(b_c), slope, ops._p(idx), R, ops._p(ret), vf,
                                          ops._p(dz[:, H:]), v("p_dw_c"), v("p_dbh_c"), v("p_dbo_c"), v("lp"), W,
                                          s) == 0
        torch.cuda.synchronize()
        for k, t in out.items():
            fill = {"dz": 777.0, "h": 333.0}.get(k, 555.0)
            assert bool((t[:pad] == fill).all()) and bool((t[-pad:] == fill).all()), k + " written out of bounds"
        return {k: t[pad:-pad] for k, t in out.items()}

    ref, got = run(False), run(True)
    assert torch.equal(got["h"].view(B, H), h_ref), "h differs from K13's"
    for k in ("dz", "p_dw_a", "p_dbh_a", "p_dbo_a", "p_dw_c", "p_dbh_c", "p_dbo_c", "lp"):
        assert torch.equal(got[k], ref[k]), k   # same h, same k loop and epilogue: bit for bit


@pytest.mark.parametrize("algo,dist,K,B,code,din", [
    ("ppo", "gaussian", 6, 4133, 1, 17),    # the C2 head and trunk widths, ragged tail (4133 = 64 * 64 + 37)
    ("a2c", "categorical", 4, 777, 0, 4),
    ("ppo", "categorical", 8, 193, 2, 20),   # tanh: h written, no sign bits
    ("a2c", "gaussian", 6, 64, 1, 17),
    ("ppo", "gaussian", 6, 20037, 1, 17),
])
def test_head_gemm_s3r_equals_k13_then_k16p(algo, dist, K, B, code, din):
    """K16R (xpa_head_gemm_s3r_*: h formed from the gathered rows in the k loop of the split-GEMM heads) against K13
    (xpa_thin_linear_act_fwd) followed by K16P on the same inputs, bit for bit: the h the actor writes (K13's fmaf
    chain), its sign bits, dz, every partial and the loss partials; canaries around every output."""
    from xuanpolicy_amd import ops
    L, s = ops.lib(), ops._stream()
    g = torch.Generator(device=DEV).manual_seed(B + K + din + 1)
    H, R = 256, B + 300
    slope = 0.01
    xr = torch.randn(B, din, device=DEV, generator=g)
    w0 = torch.randn(H, din, device=DEV, generator=g) / 4
    b0 = torch.randn(H, device=DEV, generator=g) * 0.1
    wh_a, wh_c = (torch.randn(H, H, device=DEV, generator=g) / 16 for _ in range(2))
    bh_a, bh_c = (torch.randn(H, device=DEV, generator=g) * 0.1 for _ in range(2))
    w_a = torch.randn(K, H, device=DEV, generator=g) / 16
    b_a = torch.randn(K, device=DEV, generator=g) * 0.1
    w_c = torch.randn(1, H, device=DEV, generator=g) / 16
    b_c = torch.randn(1, device=DEV, generator=g) * 0.1
    logstd = (-1 + 0.1 * torch.randn(K, device=DEV, generator=g)) if dist == "gaussian" else None
    idx = torch.randperm(R, device=DEV, generator=g)[:B].contiguous()
    idx[B // 2] = -1
    adv = torch.randn(R, device=DEV, generator=g)
    ret = torch.randn(R, device=DEV, generator=g)
    act = (torch.randn(R, K, device=DEV, generator=g) * 0.5 if dist == "gaussian"
           else torch.randint(0, K, (R,), device=DEV, generator=g).float())
    old = -1.5 + 0.3 * torch.randn(R, device=DEV, generator=g) if algo == "ppo" else None
    h_ref = torch.empty(B, H, device=DEV)
    assert L.xpa_thin_linear_act_fwd(code, ops._p(xr), din, B, din, H, ops._p(w0), ops._p(b0), slope, ops._p(h_ref), H,
                                     s) == 0
    wsa, wsc = ops.s3_split(wh_a.t()), ops.s3_split(wh_c.t())
    G = int(L.xpa_head_fused_num_partials(B))
    W = int(L.xpa_loss_partial_width(K))
    pad = 64
    algo_c, dist_c = ops.ALGO[algo], ops.DIST[dist]
    ent, clip, vf = 0.01, 0.2, 0.25
    use_sign = code in (0, 1)

    def run(trunk):
        assert L.xpa_lds_poison(s) == 0
        cz = lambda n, v=555.0: torch.full((n + 2 * pad,), v, device=DEV)   # noqa: E731
        out = dict(dz=cz(B * 2 * H, 777.0), h=cz(B * H, 333.0), sg=cz(B * 8, 0.5), p_dw_a=cz(G * K * H),
                   p_dbh_a=cz(G * H), p_dbo_a=cz(G * K), p_dw_c=cz(G * H), p_dbh_c=cz(G * H), p_dbo_c=cz(G),
                   lp=cz(G * W))
        out["lp"][pad:-pad] = 0.0
        v = lambda k: ops._p(out[k][pad:])   # noqa: E731
        dz = out["dz"][pad:pad + B * 2 * H].view(B, 2 * H)
        p_ls = ops._p(logstd) if logstd is not None else None
        p_old = ops._p(old) if old is not None else None
        if trunk:
            assert L.xpa_head_gemm_s3r_actor(
                algo_c, dist_c, code, B, K, H, ops._p(xr), din, din, ops._p(w0), ops._p(b0), slope, v("h"), H,
                v("sg") if use_sign else None, ops._p(wsa), ops._p(bh_a), 2 * H, ops._p(w_a), ops._p(b_a), slope, p_ls,
                ops._p(idx), R, ops._p(act), p_old, ops._p(adv), None, 0, clip, ent, ops._p(dz), v("p_dw_a"),
                v("p_dbh_a"), v("p_dbo_a"), v("lp"), W, s) == 0
            assert L.xpa_head_gemm_s3r_critic(
                code, B, H, ops._p(xr), din, din, ops._p(w0), ops._p(b0), slope, ops._p(wsc), ops._p(bh_c), 2 * H,
                ops._p(w_c), ops._p(b_c), slope, ops._p(idx), R, ops._p(ret), vf, ops._p(dz[:, H:]), v("p_dw_c"),
                v("p_dbh_c"), v("p_dbo_c"), v("lp"), W, s) == 0
        else:
            assert L.xpa_head_gemm_s3p_actor(algo_c, dist_c, code, B, K, H, ops._p(h_ref), H, ops._p(wsa),
                                             ops._p(bh_a), 2 * H, ops._p(w_a), ops._p(b_a), slope, p_ls, ops._p(idx),
                                             R, ops._p(act), p_old, ops._p(adv), None, 0, clip, ent, ops._p(dz),
                                             v("p_dw_a"), v("p_dbh_a"), v("p_dbo_a"), v("lp"), W, s) == 0
            assert L.xpa_head_gemm_s3p_critic(code, B, H, ops._p(h_ref), H, ops._p(wsc), ops._p(bh_c), 2 * H,
                                              ops._p(w_c), ops._p(b_c), slope, ops._p(idx), R, ops._p(ret), vf,
                                              ops._p(dz[:, H:]), v("p_dw_c"), v("p_dbh_c"), v("p_dbo_c"), v("lp"), W,
                                              s) == 0
        torch.cuda.synchronize()
        for k, t in out.items():
            fill = {"dz": 777.0, "h": 333.0, "sg": 0.5}.get(k, 555.0)
            assert bool((t[:pad] == fill).all()) and bool((t[-pad:] == fill).all()), k + " written out of bounds"
        return {k: t[pad:-pad] for k, t in out.items()}

    ref, got = run(False), run(True)
    assert torch.equal(got["h"].view(B, H), h_ref), "h differs from K13's"
    if use_sign:
        bits = (h_ref > 0).view(B, 8, 32).to(torch.int32)                      # [row, j, byte b]
        want = (bits << torch.arange(8, device=DEV, dtype=torch.int32).view(1, 8, 1)).sum(1).to(torch.uint8)
        assert torch.equal(got["sg"].view(torch.uint8).view(B, 32), want), "sign bits"
    for k in ("dz", "p_dw_a", "p_dbh_a", "p_dbo_a", "p_dw_c", "p_dbh_c", "p_dbo_c", "lp"):
        assert torch.equal(got[k], ref[k]), k   # same h, same k loop and epilogue: bit for bit


@pytest.mark.parametrize("rows,din,code", [(4133, 17, 1), (65536, 17, 1), (777, 4, 0), (300, 20, 1)])
def test_trunk_bwd_sign_equals_h_form(rows, din, code):
    """K42S (act' from K16R's sign bits) == K42 (act' from h) bit for bit: the same factor per element."""
    from xuanpolicy_amd import ops
    g = torch.Generator(device=DEV).manual_seed(rows + din)
    xr = torch.randn(rows, din, device=DEV, generator=g)
    h = torch.randn(rows, 256, device=DEV, generator=g)
    if code == 1:
        h = torch.where(h > 0, h, 0.01 * h)
    h[5, 7] = 0.0   # a zero activation takes the slope branch in both forms
    dz = torch.randn(rows, 512, device=DEV, generator=g)
    w = torch.randn(512, 256, device=DEV, generator=g) / 16
    bs = ops.s3_split(w)
    bits = (h > 0).view(rows, 8, 32).to(torch.int32)
    sign = (bits << torch.arange(8, device=DEV, dtype=torch.int32).view(1, 8, 1)).sum(1).to(torch.uint8)
    sign = sign.contiguous().view(torch.int32).view(rows, 8)
    ref = ops.s3_gemm_trunk_bwd(dz, bs, 512, h, xr, code, 0.01)
    got = ops.s3_gemm_trunk_bwd(dz, bs, 512, None, xr, code, 0.01, h_sign=sign)
    torch.cuda.synchronize()
    assert torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1])


@pytest.mark.parametrize("rows,n_rows,din,code", [(4133, 5000, 17, 1), (65536, 70000, 17, 1), (200, 300, 4, 0)])
def test_thin_gather_sign_form(rows, n_rows, din, code):
    """xpa_thin_linear_act_fwd_gather_sign: h, the gathered rows and the adv moments bit for bit the gather form's,
    plus h's sign bits in K42S's byte layout (byte b of a row, bit j = h[row, 32 j + b] > 0)."""
    from xuanpolicy_amd import ops
    L, st = ops.lib(), ops._stream()
    g = torch.Generator(device=DEV).manual_seed(rows + din)
    flat = torch.randn(n_rows, din, device=DEV, generator=g)
    idx = torch.randperm(n_rows, device=DEV, generator=g)[:rows].contiguous()
    idx[rows // 3] = -1
    w = torch.randn(256, din, device=DEV, generator=g) / 4
    b = torch.randn(256, device=DEV, generator=g) * 0.1
    b[3] = -1e9   # a column that is never positive
    adv = torch.randn(n_rows, device=DEV, generator=g)
    tiles = (rows + 63) // 64
    outs = []
    for sign in (False, True):
        h = torch.full((rows, 256), 7.0, device=DEV)
        xo = torch.full((rows, din), 7.0, device=DEV)
        ap = torch.zeros(2 * tiles, dtype=torch.float64, device=DEV)
        sg = torch.full((rows + 2, 8), 12345, dtype=torch.int32, device=DEV)
        args = [code, ops._p(flat), din, n_rows, ops._p(idx), rows, din, 256, ops._p(w), ops._p(b), 0.01, ops._p(h), 256,
                ops._p(adv), ops._p(ap), ops._p(xo)]
        if sign:
            assert L.xpa_thin_linear_act_fwd_gather_sign(*args, ops._p(sg), st) == 0
        else:
            assert L.xpa_thin_linear_act_fwd_gather(*args, st) == 0
        torch.cuda.synchronize()
        outs.append((h, xo, ap, sg))
    (h0, x0, a0, _), (h1, x1, a1, sg) = outs
    assert torch.equal(h0, h1) and torch.equal(x0, x1) and torch.equal(a0, a1)
    bits = (h1 > 0).view(rows, 8, 32).to(torch.int32)
    want = (bits << torch.arange(8, device=DEV, dtype=torch.int32).view(1, 8, 1)).sum(1).to(torch.uint8)
    assert torch.equal(sg[:rows].contiguous().view(torch.uint8).view(rows, 32), want)
    assert bool((sg[rows:] == 12345).all()), "sign rows past the batch written"


@pytest.mark.parametrize("algo,dist,K,B,code", [("ppo", "gaussian", 6, 4133, 1), ("a2c", "categorical", 8, 777, 0),
                                                ("ppo", "gaussian", 6, 65536, 1), ("ppo", "categorical", 4, 193, 2)])
def test_head_gemm_s3q_equals_s3p(algo, dist, K, B, code):
    """K16Q (32 x 128 wave tiles) == K16P bit for bit: dz and every partial (each output's accumulation chain and the
    epilogue are the same, only which wave computes it differs)."""
    from xuanpolicy_amd import ops
    L, s = ops.lib(), ops._stream()
    g = torch.Generator(device=DEV).manual_seed(B + K + 7)
    H, R = 256, B + 300
    x = torch.randn(B, H, device=DEV, generator=g)
    wh_a, wh_c = (torch.randn(H, H, device=DEV, generator=g) / 16 for _ in range(2))
    bh_a, bh_c = (torch.randn(H, device=DEV, generator=g) * 0.1 for _ in range(2))
    w_a = torch.randn(K, H, device=DEV, generator=g) / 16
    b_a = torch.randn(K, device=DEV, generator=g) * 0.1
    w_c = torch.randn(1, H, device=DEV, generator=g) / 16
    b_c = torch.randn(1, device=DEV, generator=g) * 0.1
    logstd = (-1 + 0.1 * torch.randn(K, device=DEV, generator=g)) if dist == "gaussian" else None
    idx = torch.randperm(R, device=DEV, generator=g)[:B].contiguous()
    idx[B // 2] = -1
    adv, ret = torch.randn(R, device=DEV, generator=g), torch.randn(R, device=DEV, generator=g)
    act = (torch.randn(R, K, device=DEV, generator=g) * 0.5 if dist == "gaussian"
           else torch.randint(0, K, (R,), device=DEV, generator=g).float())
    old = -1.5 + 0.3 * torch.randn(R, device=DEV, generator=g) if algo == "ppo" else None
    wsa, wsc = ops.s3_split(wh_a.t()), ops.s3_split(wh_c.t())
    G = int(L.xpa_head_fused_num_partials(B))
    W = int(L.xpa_loss_partial_width(K))
    p = ops._p

    def run(form):
        assert L.xpa_lds_poison(s) == 0
        dz = torch.full((B, 2 * H), 777.0, device=DEV)
        parts = [torch.full((G, n), 555.0, device=DEV) for n in (K * H, H, K, H, H, 1)]
        lp = torch.zeros(G, W, device=DEV)
        fa, fc = getattr(L, "xpa_head_gemm_%s_actor" % form), getattr(L, "xpa_head_gemm_%s_critic" % form)
        assert fa(ops.ALGO[algo], ops.DIST[dist], code, B, K, H, p(x), H, p(wsa), p(bh_a), 2 * H, p(w_a), p(b_a), 0.01,
                  p(logstd) if logstd is not None else None, p(idx), R, p(act), p(old) if old is not None else None,
                  p(adv), None, 0, 0.2, 0.01, p(dz), p(parts[0]), p(parts[1]), p(parts[2]), p(lp), W, s) == 0
        assert fc(code, B, H, p(x), H, p(wsc), p(bh_c), 2 * H, p(w_c), p(b_c), 0.01, p(idx), R, p(ret), 0.25,
                  p(dz[:, H:]), p(parts[3]), p(parts[4]), p(parts[5]), p(lp), W, s) == 0
        torch.cuda.synchronize()
        return [dz] + parts + [lp]

    ref, got = run("s3p"), run("s3q")
    for i, (a_, b_) in enumerate(zip(ref, got)):
        assert torch.equal(a_, b_), i


@pytest.mark.parametrize("rows,din,code", [(65536, 17, 1), (4133, 17, 1), (300, 4, 0), (20, 17, 1)])
def test_trunk_bwd_sign_lookahead_equals_default(rows, din, code):
    """K42S's lookahead form (xpa_s3_probe bit 128: 4-stage ring, chunk c + 1's A split between chunk c's MFMA blocks)
    and its ping-pong form (bit 256: the two waves of a SIMD one phase apart) == the default form bit for bit (same products, same order per accumulator), including 1- and 2-chunk tails."""
    from xuanpolicy_amd import ops
    L = ops.lib()
    g = torch.Generator(device=DEV).manual_seed(rows + 3 * din)
    xr = torch.randn(rows, din, device=DEV, generator=g)
    h = torch.randn(rows, 256, device=DEV, generator=g)
    for k in (512, 32, 16):
        dz = torch.randn(rows, k, device=DEV, generator=g)
        w = torch.randn(k, 256, device=DEV, generator=g) / 16
        bs = ops.s3_split(w)
        bits = (h > 0).view(rows, 8, 32).to(torch.int32)
        sign = (bits << torch.arange(8, device=DEV, dtype=torch.int32).view(1, 8, 1)).sum(1).to(torch.uint8)
        sign = sign.contiguous().view(torch.int32).view(rows, 8)
        ref = ops.s3_gemm_trunk_bwd(dz, bs, k, None, xr, code, 0.01, h_sign=sign)
        for form in (128, 256):   # 256: the ping-pong k loop (r05)
            try:
                assert L.xpa_s3_probe(form) == 0
                got = ops.s3_gemm_trunk_bwd(dz, bs, k, None, xr, code, 0.01, h_sign=sign)
                torch.cuda.synchronize()
            finally:
                L.xpa_s3_probe(0)
            assert torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1]), (k, form)
