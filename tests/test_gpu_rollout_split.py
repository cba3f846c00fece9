"""GPU: K40R (r05), the rollout's paired hidden layer on the split GEMM (csrc/sgemm3.hip xpa_s3_gemm_rows_pair).

  * every output equals K40's (xpa_s3_gemm on the same half) + bias, bit for bit, on ragged row counts;
  * a C2-shaped rollout with K40R against the f32 library GEMM's: actions, log-probs and values within the f32 GEMM's
    error (the end-to-end oracle replays in test_gpu_fastpath_e2e.py run with K40R on, the default)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("M", [4096, 777, 64, 5, 65536])
def test_rows_pair_equals_k40_halves(M):
    from xuanpolicy_amd import ops
    g = torch.Generator(device=DEV).manual_seed(M)
    x = torch.randn(M, 256, device=DEV, generator=g) * torch.exp(torch.randn(M, 1, device=DEV, generator=g))
    wa = torch.randn(256, 256, device=DEV, generator=g) / 16
    wc = torch.randn(256, 256, device=DEV, generator=g) / 16
    b = torch.randn(512, device=DEV, generator=g)
    sa, sc = ops.s3_split(wa.t()), ops.s3_split(wc.t())
    z = torch.full((M, 512), 777.0, device=DEV)
    ops.s3_gemm_rows_pair(x, sa, sc, b, out=z)
    za = ops.s3_gemm(x, sa, 256) + b[:256]
    zc = ops.s3_gemm(x, sc, 256) + b[256:]
    torch.cuda.synchronize()
    assert torch.equal(z[:, :256], za)
    assert torch.equal(z[:, 256:], zc)
    # and close to the f64 product (the split's f32 accuracy)
    ref = x.double() @ torch.cat([wa, wc], 0).double().t() + b.double()
    bound = 4e-6 * (x.double().abs() @ torch.cat([wa, wc], 0).double().abs().t()) + 1e-6
    assert bool(((z.double() - ref).abs() <= bound).all())


def test_rollout_with_k40r_matches_library_gemm(monkeypatch):
    """Two agents from one seed, one rollout each: K40R (default) vs the f32 library GEMM (ROLLOUT_SPLIT off)."""
    from xuanpolicy_amd.fused_mlp import FusedActorCritic
    from xuanpolicy_amd.runner import build_synthbox_ppo
    outs = []
    for split in (True, False):
        monkeypatch.setattr(FusedActorCritic, "ROLLOUT_SPLIT", split)
        agent = build_synthbox_ppo(n_envs=512, n_steps=16, obs_dim=17, act_dim=6, hidden=256, n_epoch=1,
                                   n_minibatch=4, seed=5, device="cuda:0")
        agent.train(15, log=False)   # stops before the update: the buffers hold the rollout
        fm = agent.learner._fused_mlp()
        assert (getattr(fm, "_roll_split", None) is not None) == split
        m = agent.memory
        outs.append((m.actions[:, :15].clone(), m.auxiliary_infos["old_logp"][:, :15].clone(),
                     m.values[:, :15].clone()))
        del agent
    for a, b in zip(*outs):
        scale = b.abs().max().item()
        assert (a - b).abs().max().item() <= 1e-4 * max(scale, 1.0)


def test_fold_rms_matches_standalone_update(monkeypatch):
    """r05: the next step's obs_rms.update folded into K8 (xpa_rollout_post_deferred_norm_rms) against the standalone
    per-step update (xpa_rms_update): the running statistics and the stored normalised observations after a rollout
    and a half (the fold's block partials sum the same rows in another fixed order: f64 rounding only)."""
    import xuanpolicy_amd.agents as ag
    from xuanpolicy_amd.runner import build_synthbox_ppo
    outs = []
    monkeypatch.setattr(ag, "FUSE_POST", False)   # r06: K14F would fold the update in both arms
    for fold in (True, False):
        monkeypatch.setattr(ag, "FOLD_RMS", fold)
        agent = build_synthbox_ppo(n_envs=1000, n_steps=16, obs_dim=17, act_dim=6, hidden=256, n_epoch=1,
                                   n_minibatch=4, seed=9, device="cuda:0", max_episode_steps=7)
        assert agent._rms_fold_ok() == fold
        agent.train(16 + 7, log=False)   # one rollout + update, then 7 steps of the next
        stored = (agent.memory.observations[:, :7].clone(), agent.memory.values[:, :7].clone())
        if not fold:   # the fold has merged the observation the last step produced already; the standalone path
            agent._rms_update(agent.envs.obs)   # merges it at the next step: catch up before comparing
        torch.cuda.synchronize()
        outs.append((agent.obs_mean.clone(), agent.obs_var.clone(), agent.obs_count.clone()) + stored)
        del agent
    (m1, v1, c1, o1, val1), (m0, v0, c0, o0, val0) = outs
    assert torch.equal(c1, c0)
    assert torch.allclose(m1, m0, rtol=1e-6, atol=1e-7) and torch.allclose(v1, v0, rtol=1e-6, atol=1e-7)
    assert torch.allclose(o1, o0, rtol=1e-5, atol=1e-6)
    assert torch.allclose(val1, val0, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("M,act", [(8192, 1), (777, 1), (64, 0), (5, 2), (65536, 1)])
def test_gemm_value_matches_f64(M, act):
    """r06, K40V: v = act(x Wh^T + bh) . w_out + b_out in one launch (the split GEMM with the value head in its
    epilogue) against f64, within the f32 GEMM's error carried through the output layer."""
    from xuanpolicy_amd import ops
    g = torch.Generator(device=DEV).manual_seed(M + act)
    x = torch.randn(M, 256, device=DEV, generator=g)
    wh = torch.randn(256, 256, device=DEV, generator=g) / 16
    bh = torch.randn(256, device=DEV, generator=g) * 0.1
    wo = torch.randn(1, 256, device=DEV, generator=g) / 16
    bo = torch.randn(1, device=DEV, generator=g)
    slope = 0.01
    v = ops.s3_gemm_value(x, ops.s3_split(wh.t()), 256, bh, act, slope, wo.view(-1), bo)
    torch.cuda.synchronize()
    z = x.double() @ wh.double().t() + bh.double()
    if act == 1:
        hz = torch.where(z > 0, z, z * slope)
    elif act == 2:
        hz = torch.tanh(z)
    else:
        hz = z
    ref = hz @ wo.double().view(-1) + bo.double()
    # the hidden layer's f32 error (4e-6 of sum |x w| per element) through |w_out|, plus the 256-term output sum's
    bound = (4e-6 * (x.double().abs() @ wh.double().abs().t())) @ wo.double().abs().view(-1) + \
        1e-6 * (hz.abs() @ wo.double().abs().view(-1)) + 1e-6
    err = (v.double() - ref).abs()
    assert torch.isfinite(v).all()
    assert bool((err <= bound).all()), (err / bound).max().item()


def test_deferred_bootstraps_k40v_equal_reference_critic(monkeypatch):
    """The deferred bootstrap rows through K40V (opt-in, agents.VALUE_GEMM) against the reference-shaped critic
    (trunk, library GEMM, K14's value head) on the same rows with the rollout's weights, to f32 accuracy; the update
    phase then takes the K40V + compact-scan form (the e2e oracle replays run it end to end)."""
    from xuanpolicy_amd.runner import build_synthbox_ppo
    agent = build_synthbox_ppo(n_envs=1024, n_steps=16, obs_dim=17, act_dim=6, hidden=256, n_epoch=1, n_minibatch=4,
                               seed=21, device="cuda:0", max_episode_steps=20)   # one slot: the fused scans apply
    agent.value_gemm = True
    agent.train(15, log=False)   # stops one step before the update: the rollout's weights and planes still current
    fm = agent._rollout_mlp()
    agent._boot_pair.normal_()   # any rows
    v_k40v = fm.rollout_value_split(agent._boot_pair)
    v_ref = fm.rollout_value(agent._boot_pair)
    torch.cuda.synchronize()
    assert v_k40v is not None
    scale = v_ref.abs().max().item()
    assert (v_k40v - v_ref).abs().max().item() <= 2e-5 * max(scale, 1.0)
    agent.train(1, log=False)    # the last step + the update phase: K40V + the compact scan is the form taken
    assert agent.gae_form == "compact" and agent.value_gemm


@pytest.mark.parametrize("M,din,code,with_col", [(4096, 17, 1, True), (1000, 17, 1, False), (777, 5, 2, True),
                                                 (37, 18, 0, True), (65536, 17, 1, True)])
def test_rows_pair_trunk_equals_two_launches(M, din, code, with_col):
    """r06, K40T: the trunk (obs normalisation + thin first layer) formed inside K40R's launch equals the two-launch form
    (xpa_thin_linear_act_fwd_norm, then xpa_s3_gemm_rows_pair on its h) bit for bit: z, the normalised rows in xn and
    the rollout buffer column; ragged and XCD-mapped (M % 512 == 0) row counts, d_in forms 8 / 18, every activation."""
    from xuanpolicy_amd import ops
    g = torch.Generator(device=DEV).manual_seed(M + din)
    X = torch.randn(M, din + 3, device=DEV, generator=g) * 3 + 1
    x = X[:, :din]                       # strided rows, as the env's observation view
    mean = torch.randn(din, device=DEV, generator=g)
    var = torch.rand(din, device=DEV, generator=g) + 0.1
    W = torch.randn(256, din, device=DEV, generator=g) * 0.2
    b = torch.randn(256, device=DEV, generator=g) * 0.1
    wa = torch.randn(256, 256, device=DEV, generator=g) / 16
    wc = torch.randn(256, 256, device=DEV, generator=g) / 16
    bias = torch.randn(512, device=DEV, generator=g)
    sa, sc = ops.s3_split(wa.t()), ops.s3_split(wc.t())
    T = 5
    cur = torch.tensor([3, 0, 0, 0], dtype=torch.int32, device=DEV)
    L = ops.lib()
    outs = []
    for fused in (False, True):
        xn = torch.full((M, din), 55.0, device=DEV)
        col = torch.full((M, T, din), 66.0, device=DEV) if with_col else None
        if fused:
            z = ops.s3_gemm_rows_pair_trunk(x, W, b, code, 0.01, mean, var, 5.0, xn, col, T * din, cur, sa, sc, bias)
        else:
            h = torch.empty(M, 256, device=DEV)
            assert L.xpa_thin_linear_act_fwd_norm(code, ops._p(x), x.stride(0), M, din, 256, ops._p(W), ops._p(b),
                                                   0.01, ops._p(h), 256, ops._p(mean), ops._p(var), 5.0, ops._p(xn),
                                                   din, ops._p(col) if with_col else None, T * din, ops._p(cur),
                                                   ops._stream()) == 0
            z = ops.s3_gemm_rows_pair(h, sa, sc, bias)
        outs.append((z, xn, col))
    torch.cuda.synchronize()
    (z0, xn0, c0), (z1, xn1, c1) = outs
    assert torch.equal(z1, z0)
    assert torch.equal(xn1, xn0)
    if with_col:
        assert torch.equal(c1, c0)


def test_rollout_with_k40t_bit_equal(monkeypatch):
    """A C2-shaped rollout with the trunk inside K40R's launch (FusedActorCritic.ROLLOUT_TRUNK, opt-in) and with
    K13-norm + K40R: the rollout buffers (observations, actions, log-probs, values) and the obs statistics are equal."""
    from xuanpolicy_amd import ops
    from xuanpolicy_amd.fused_mlp import FusedActorCritic
    from xuanpolicy_amd.runner import build_synthbox_ppo
    calls = []
    k40t = ops.s3_gemm_rows_pair_trunk

    def counted(*a, **k):
        calls.append(1)
        return k40t(*a, **k)
    monkeypatch.setattr(ops, "s3_gemm_rows_pair_trunk", counted)
    outs = []
    for trunk in (True, False):
        monkeypatch.setattr(FusedActorCritic, "ROLLOUT_TRUNK", trunk)
        n0 = len(calls)
        agent = build_synthbox_ppo(n_envs=1024, n_steps=16, obs_dim=17, act_dim=6, hidden=256, n_epoch=1,
                                   n_minibatch=4, seed=11, device="cuda:0", max_episode_steps=9)
        agent.train(16 + 15, log=False)   # a rollout + update, then 15 steps of the next rollout
        assert (len(calls) > n0) == trunk     # K40T is the form the rollout took (captured or eager)
        m = agent.memory
        torch.cuda.synchronize()
        outs.append((m.observations[:, :15].clone(), m.actions[:, :15].clone(),
                     m.auxiliary_infos["old_logp"][:, :15].clone(), m.values[:, :15].clone(), agent.obs_mean.clone(),
                     agent.obs_var.clone()))
        del agent
    for a, b in zip(*outs):
        assert torch.equal(a, b)
