"""GPU parity tests: every HIP kernel through the C ABI vs the CPU oracle / reference golden vectors.
Run on the MI355X box (pytest -m gpu)."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref, synth_env

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cpu_ref.build_oracle()
    from xuanpolicy_amd import _lib
    _lib.load()


def _gae_close(got, ref):
    """GAE advantages / returns against the oracle at north_star's 1e-5 (absolute, plus 1e-5 relative), widened by
    2^-20 of the row's largest |value|: the scan reassociates the discounted sum, and its f32 rounding is relative to the
    largest partial sum of the row, not to the element (a return of 0.12 in a row that peaks at 13 carries ~1e-5 of
    the row's rounding).  On unit-scale rows the extra term is below 1e-6."""
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    row = np.abs(ref).max(axis=-1, keepdims=True) if ref.ndim > 1 else np.abs(ref).max()
    tol = 1e-5 + 1e-5 * np.abs(ref) + 2.0 ** -20 * row
    bad = np.abs(got - ref) > tol
    assert not bad.any(), ("GAE mismatch", int(bad.sum()), float(np.abs(got - ref)[bad].max()))


def _d(x, dtype=None):
    t = torch.as_tensor(np.ascontiguousarray(x))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(DEV)


def _h(t):
    return t.detach().cpu().numpy()


# ---------------------------------------------------------------------------------------------- K1
@pytest.mark.parametrize("tag", ["plain_gae", "plain_nogae", "atari_gae", "atari_nogae"])
def test_gae_kernel_golden(golden, tag):
    from xuanpolicy_amd import ops
    g = golden("gae.npz")
    use_gae = tag.endswith("_gae")
    adv, ret = ops.gae_scan(_d(g[tag + "/rew"]), _d(g[tag + "/val"]), _d(g[tag + "/term"]), _d(g[tag + "/closed"]),
                            _d(g[tag + "/boot"]), 0.99, 0.95, use_gae)
    np.testing.assert_allclose(_h(adv), g[tag + "/adv"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(_h(ret), g[tag + "/ret"], rtol=1e-5, atol=1e-5)


def _random_gae_case(rng, N, T, p_close=0.02, p_term=0.02, close_last=True):
    rew = rng.normal(0, 1, (N, T)).astype(np.float32)
    val = rng.normal(0, 1, (N, T)).astype(np.float32)
    term = (rng.random((N, T)) < p_term).astype(np.float32)
    closed = (rng.random((N, T)) < p_close).astype(np.uint8)
    if close_last:
        closed[:, -1] = 1
    boot = np.where(closed > 0, rng.normal(0, 1, (N, T)), 0).astype(np.float32)
    boot[term > 0] = 0.0
    return rew, val, term, closed, boot


@pytest.mark.parametrize("N,T", [(1, 1), (7, 63), (64, 128), (33, 129), (5, 1024), (130, 4), (3, 257), (1000, 128),
                                 (9, 36), (2, 64), (70, 96), (11, 200), (6, 516), (5, 256)])
@pytest.mark.parametrize("use_gae", [True, False])
def test_gae_kernel_random_shapes(N, T, use_gae):
    from xuanpolicy_amd import ops
    rng = np.random.default_rng(N * 1000 + T)
    # open tails: about a third of the rows are not closed at T-1
    rew, val, term, closed, boot = _random_gae_case(rng, N, T, close_last=False)
    closed[rng.random(N) < 0.66, -1] = 1
    ref_adv = np.full((N, T), -7.0, np.float32)
    ref_ret = np.full((N, T), -7.0, np.float32)
    cpu_ref.gae_rows(rew, val, term, closed, boot, 0.99, 0.95, use_gae, adv=ref_adv, ret=ref_ret)
    adv = torch.full((N, T), -7.0, device=DEV)
    ret = torch.full((N, T), -7.0, device=DEV)
    ops.gae_scan(_d(rew), _d(val), _d(term), _d(closed), _d(boot), 0.99, 0.95, use_gae, adv=adv, ret=ret)
    # north_star: 1e-5 on advantages / returns (unit-scale rewards and values; rtol 1e-5 covers the returns of long
    # undiscounted-looking paths, |ret| up to ~30 here)
    _gae_close(_h(adv), ref_adv)
    _gae_close(_h(ret), ref_ret)


def _compact_case(rng, N, T, p_term=0.02, p_slot=0.3):
    rew = rng.normal(0, 1, (N, T)).astype(np.float32)
    val = rng.normal(0, 1, (N, T)).astype(np.float32)
    term = (rng.random((N, T)) < p_term).astype(np.float32)
    term[rng.random(N) < 0.1, -1] = 1.0                        # some rows end on a terminal
    slot = np.where(rng.random(N) < p_slot, rng.integers(0, max(T - 1, 1), N), -1).astype(np.int32)
    if T > 1:
        slot[:: 7] = T - 2                                    # truncation right before the last step
        term[np.arange(N)[slot >= 0], slot[slot >= 0]] = 0.0  # a truncation slot is not a terminal (K8)
    vboot = rng.normal(0, 1, 2 * N).astype(np.float32)
    # the equivalent dense closure record (K8 flags + xpa_rollout_bootstrap_fixup)
    closed = (term > 0).astype(np.uint8)
    closed[:, -1] = 1
    boot = np.zeros((N, T), np.float32)
    rows = np.nonzero(slot >= 0)[0]
    closed[rows, slot[rows]] = 1
    boot[rows, slot[rows]] = vboot[rows]
    boot[:, -1] = np.where(term[:, -1] > 0, 0.0, vboot[N:])
    return rew, val, term, slot, vboot, closed, boot


@pytest.mark.parametrize("N,T", [(1000, 128), (4096, 128), (33, 36), (5, 516), (7, 130), (3, 20), (11, 256), (2, 1)])
@pytest.mark.parametrize("use_gae", [True, False])
def test_gae_compact_matches_fixup_plus_scan(N, T, use_gae):
    """xpa_gae_scan_compact (the fused agent's form) == xpa_rollout_bootstrap_fixup + xpa_gae_scan ==
    the oracle, including the boot column it writes and the slot reset."""
    from xuanpolicy_amd import ops
    rng = np.random.default_rng(N * 7 + T)
    rew, val, term, slot, vboot, closed, boot = _compact_case(rng, N, T)
    ref_adv, ref_ret = cpu_ref.gae_rows(rew, val, term, closed, boot, 0.99, 0.95, use_gae)
    slot_d = _d(slot)
    boot_d = torch.zeros(N, T, device=DEV)
    adv, ret = ops.gae_scan_compact(_d(rew), _d(val), _d(term), slot_d, _d(vboot), 0.99, 0.95, use_gae,
                                    boot=boot_d)
    _gae_close(_h(adv), ref_adv)
    _gae_close(_h(ret), ref_ret)
    np.testing.assert_array_equal(_h(boot_d), boot)
    assert (_h(slot_d) == -1).all()
    # the dense path on the same record agrees to the bit pattern of the scan order
    a2, r2 = ops.gae_scan(_d(rew), _d(val), _d(term), _d(closed), _d(boot), 0.99, 0.95, use_gae)
    np.testing.assert_allclose(_h(adv), _h(a2), rtol=0, atol=1e-6)
    np.testing.assert_allclose(_h(ret), _h(r2), rtol=0, atol=1e-6)


@pytest.mark.parametrize("N,T", [(4096, 128), (1000, 128), (777, 64), (33, 36), (5, 516), (7, 260), (11, 256)])
@pytest.mark.parametrize("act", [0, 1, 2])
def test_gae_value_fused_matches_value_head_plus_compact(N, T, act):
    """xpa_gae_scan_value (value head inside the scan) == xpa_value_head + xpa_gae_scan_compact bit for bit (adv,
    ret, the boot column, the slot reset), and the values it bootstraps with == the oracle's act(z) . w + b."""
    from xuanpolicy_amd import ops
    rng = np.random.default_rng(N * 13 + T + act)
    rew, val, term, slot, _, closed, _ = _compact_case(rng, N, T)
    H, slope = 256, 0.01
    z = rng.normal(0, 1, (2 * N, H)).astype(np.float32)
    w = (rng.normal(0, 1, (1, H)) / 16).astype(np.float32)
    b = rng.normal(0, 1, (1,)).astype(np.float32)
    z_d, w_d, b_d = _d(z), _d(w), _d(b)
    vboot = ops.value_head(z_d, (act, slope), w_d, b_d)
    boot_a, slot_a = torch.zeros(N, T, device=DEV), _d(slot)
    adv_a, ret_a = ops.gae_scan_compact(_d(rew), _d(val), _d(term), slot_a, vboot, 0.99, 0.95, True, boot=boot_a)
    boot_b, slot_b = torch.zeros(N, T, device=DEV), _d(slot)
    adv_b = torch.full((N, T), -7.0, device=DEV)
    ret_b = torch.full((N, T), -7.0, device=DEV)
    ops.gae_scan_value(_d(rew), _d(val), _d(term), slot_b, z_d, (act, slope), w_d, b_d, 0.99, 0.95, True,
                       adv=adv_b, ret=ret_b, boot=boot_b)
    np.testing.assert_array_equal(_h(adv_b), _h(adv_a))
    np.testing.assert_array_equal(_h(ret_b), _h(ret_a))
    np.testing.assert_array_equal(_h(boot_b), _h(boot_a))
    assert (_h(slot_b) == -1).all()
    # the oracle: V in f64 from the same z, then the dense-closure GAE restatement
    h = z.astype(np.float64)
    h = np.where(h > 0, h, h * slope) if act == 1 else (np.tanh(h) if act == 2 else h)
    v = (h @ w[0].astype(np.float64) + b[0]).astype(np.float32)
    np.testing.assert_allclose(_h(vboot), v, rtol=1e-5, atol=1e-5)
    ref_boot = np.zeros((N, T), np.float32)
    rows = np.nonzero(slot >= 0)[0]
    ref_boot[rows, slot[rows]] = v[rows]
    ref_boot[:, -1] = np.where(term[:, -1] > 0, 0.0, v[N:])
    ref_adv, ref_ret = cpu_ref.gae_rows(rew, val, term, closed, ref_boot, 0.99, 0.95, True)
    _gae_close(_h(adv_b), ref_adv)
    _gae_close(_h(ret_b), ref_ret)


def test_gae_kernel_unaligned_views():
    """float4 path needs 16-B alignment; an offset view must take the scalar path and stay correct."""
    from xuanpolicy_amd import ops
    rng = np.random.default_rng(5)
    N, T = 17, 128
    rew, val, term, closed, boot = _random_gae_case(rng, N, T)
    big = torch.zeros(N * T + 1, device=DEV)
    r_view = big[1:].view(N, T)
    r_view.copy_(_d(rew))
    adv, ret = ops.gae_scan(r_view, _d(val), _d(term), _d(closed), _d(boot), 0.98, 0.9)
    ref_adv, ref_ret = cpu_ref.gae_rows(rew, val, term, closed, boot, 0.98, 0.9)
    _gae_close(_h(adv), ref_adv)
    _gae_close(_h(ret), ref_ret)


def test_gae_kernel_full_size_properties():
    """BASELINE sizes (4096 x 128 and 262144 x 128): sampled rows vs the oracle, plus the
    size-independent identity ret = adv + v."""
    from xuanpolicy_amd import ops
    for N in (4096, 262144):
        T = 128
        g = torch.Generator(device=DEV).manual_seed(N)
        rew = torch.randn(N, T, device=DEV, generator=g)
        val = torch.randn(N, T, device=DEV, generator=g)
        term = (torch.rand(N, T, device=DEV, generator=g) < 0.01).float()
        closed = (torch.rand(N, T, device=DEV, generator=g) < 0.001).to(torch.uint8)
        closed[:, -1] = 1
        boot = torch.randn(N, T, device=DEV, generator=g) * closed
        adv, ret = ops.gae_scan(rew, val, term, closed, boot, 0.99, 0.95)
        np.testing.assert_allclose(_h(ret), _h(adv + val), rtol=0, atol=1e-6)
        rows = torch.randint(0, N, (256,), generator=torch.Generator().manual_seed(1)).to(DEV)
        ra, rr = cpu_ref.gae_rows(_h(rew[rows]), _h(val[rows]), _h(term[rows]), _h(closed[rows]), _h(boot[rows]),
                                  0.99, 0.95)
        np.testing.assert_allclose(_h(adv[rows]), ra, rtol=1e-5, atol=1e-5)


# ---------------------------------------------------------------------------------------------- K2
LOSS_CASES = ["ppo_gaussian_6", "ppo_gaussian_17", "ppo_categorical_2", "ppo_categorical_6", "a2c_gaussian_6",
              "a2c_categorical_6"]


@pytest.mark.parametrize("tag", LOSS_CASES)
def test_loss_kernel_golden(golden, tag):
    from xuanpolicy_amd import ops
    g = golden("loss.npz")
    algo, dist, _ = tag.split("_")
    sc, dh, dls, dv = ops.policy_loss(algo, dist, _d(g[tag + "/head"]),
                                      _d(g[tag + "/logstd0"]) if dist == "gaussian" else None, _d(g[tag + "/v"]),
                                      _d(g[tag + "/act"]), _d(g[tag + "/adv"]), _d(g[tag + "/ret"]),
                                      old_logp=_d(g[tag + "/old_logp"]) if algo == "ppo" else None,
                                      clip_range=0.2, vf_coef=0.25, ent_coef=0.01)
    sc = _h(sc)
    info = {k: float(g[tag + "/info/" + k]) for k in ("actor-loss", "critic-loss", "entropy", "predict_value")}
    assert abs(sc[0] - info["actor-loss"]) < 1e-5
    assert abs(sc[1] - info["critic-loss"]) < 1e-5
    assert abs(sc[2] - info["entropy"]) < 1e-5
    assert abs(sc[5] - info["predict_value"]) < 1e-6
    loss = info["actor-loss"] - 0.01 * info["entropy"] + 0.25 * info["critic-loss"]
    assert abs(sc[3] - loss) < 1e-4
    if algo == "ppo":
        assert abs(sc[4] - float(g[tag + "/info/clip_ratio"])) < 1e-7
    np.testing.assert_allclose(_h(dh), g[tag + "/dhead"], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(_h(dv), g[tag + "/dv"], rtol=1e-4, atol=1e-8)
    if dist == "gaussian":
        np.testing.assert_allclose(_h(dls), g[tag + "/dlogstd"], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("algo,dist,A,B", [("ppo", "gaussian", 17, 65536), ("ppo", "categorical", 18, 4097),
                                           ("a2c", "gaussian", 6, 1000), ("a2c", "categorical", 6, 257)])
def test_loss_kernel_indexed_advnorm(algo, dist, A, B):
    """idx-gathered inputs + per-minibatch adv-norm from the gather kernel's moments vs the oracle."""
    from xuanpolicy_amd import ops
    rng = np.random.default_rng(A * 7 + B)
    rows = 3 * B
    head = rng.normal(0, 0.5, (B, A)).astype(np.float32)
    logstd = (-1 + rng.normal(0, 0.1, A)).astype(np.float32)
    v = rng.normal(0, 1, B).astype(np.float32)
    if dist == "gaussian":
        act_all = rng.normal(0, 0.6, (rows, A)).astype(np.float32)
    else:
        act_all = rng.integers(0, A, rows).astype(np.float32)
    adv_all = (rng.normal(0.3, 2.0, rows)).astype(np.float32)
    ret_all = rng.normal(0, 1, rows).astype(np.float32)
    logp_all = rng.normal(-3, 1, rows).astype(np.float32)
    idx = rng.permutation(rows)[:B].astype(np.int64)
    obs_all = rng.normal(0, 1, (rows, 5)).astype(np.float32)
    idx_d = _d(idx)
    obs_mb, part = ops.gather_minibatch(idx_d, _d(obs_all), adv=_d(adv_all))
    np.testing.assert_array_equal(_h(obs_mb), obs_all[idx])
    a = adv_all[idx].astype(np.float64)
    np.testing.assert_allclose(_h(part).sum(0), [a.sum(), (a * a).sum()], rtol=1e-9)
    sc, dh, dls, dv = ops.policy_loss(algo, dist, _d(head), _d(logstd) if dist == "gaussian" else None, _d(v),
                                      _d(act_all), _d(adv_all), _d(ret_all), old_logp=_d(logp_all), idx=idx_d,
                                      adv_partials=part, clip_range=0.2, vf_coef=0.5, ent_coef=0.01)
    adv_n = (adv_all[idx] - adv_all[idx].mean()) / (adv_all[idx].std() + 1e-8)
    if dist == "gaussian":
        # old_logp near the current logp so ratios straddle the clip range
        sc_s = np.exp(logstd)
        lp = (-(act_all[idx] - head) ** 2 / (2 * sc_s ** 2) - logstd - 0.5 * np.log(2 * np.pi)).sum(-1)
        logp_all[idx] = lp + rng.normal(0, 0.3, B)
        sc, dh, dls, dv = ops.policy_loss(algo, dist, _d(head), _d(logstd), _d(v), _d(act_all), _d(adv_all),
                                          _d(ret_all), old_logp=_d(logp_all), idx=idx_d, adv_partials=part,
                                          clip_range=0.2, vf_coef=0.5, ent_coef=0.01)
    info, rdh, rdls, rdv = cpu_ref.loss_grads_ref(algo, dist, head, logstd, v, act_all[idx], adv_n, ret_all[idx],
                                                  logp_all[idx], 0.2, 0.5, 0.01)
    sc = _h(sc)
    assert abs(sc[3] - info["loss"]) < 1e-4, (sc, info)
    assert abs(sc[0] - info["actor-loss"]) < 1e-4
    np.testing.assert_allclose(_h(dh), rdh, rtol=2e-4, atol=1e-8)
    np.testing.assert_allclose(_h(dv), rdv, rtol=1e-4, atol=1e-9)
    if dist == "gaussian":
        np.testing.assert_allclose(_h(dls), rdls, rtol=2e-4, atol=1e-5)
    if algo == "ppo":
        assert abs(sc[4] - info["clip_ratio"]) < 2.0 / B


@pytest.mark.parametrize("algo,A,B,advnorm", [
    ("ppo", 6, 1024 * 256 * 2 + 77, False),   # pipelined K2: > 2 tiles per block, a ragged last tile
    ("ppo", 6, 65536, True),                   # C2 minibatch, in order, adv-norm
    ("a2c", 2, 256 * 1024 + 256, False),       # A2C slot count (2A + 3), exactly one extra tile
    ("ppo", 8, 300, False),                    # one full tile + a 44-row tail
    ("ppo", 1, 259, True),                     # 1-float rows; 3-row tail
    ("a2c", 5, 1, False),                      # a single row (the generic kernel: B < one tile)
    ("ppo", 17, 5000, False),                  # C4 head width (the straight-line K2, A > 8)
])
def test_loss_kernel_in_order_rows(algo, A, B, advnorm):
    """K2 with the minibatch rows in order (idx = None: the LDS-DMA pipelined form for A <= 8) against the
    oracle's closed-form loss and gradients (ppoclip_learner.py:32-44, a2c_learner.py:24-31)."""
    from xuanpolicy_amd import ops
    rng = np.random.default_rng(A * 13 + B)
    head = rng.normal(0, 0.5, (B, A)).astype(np.float32)
    logstd = (-1 + rng.normal(0, 0.1, A)).astype(np.float32)
    v = rng.normal(0, 1, B).astype(np.float32)
    act = (head + np.exp(logstd) * rng.normal(0, 1, (B, A))).astype(np.float32)
    adv = rng.normal(0.3, 2.0, B).astype(np.float32)
    ret = rng.normal(0, 1, B).astype(np.float32)
    sc_s = np.exp(logstd)
    lp = (-(act - head) ** 2 / (2 * sc_s ** 2) - logstd - 0.5 * np.log(2 * np.pi)).sum(-1)
    old = (lp + rng.normal(0, 0.3, B)).astype(np.float32)
    part = None
    if advnorm:
        a = adv.astype(np.float64)
        part = torch.tensor([[a.sum(), (a * a).sum()]], dtype=torch.float64, device=DEV)
    sc, dh, dls, dv = ops.policy_loss(algo, "gaussian", _d(head), _d(logstd), _d(v), _d(act), _d(adv), _d(ret),
                                      old_logp=_d(old) if algo == "ppo" else None, adv_partials=part,
                                      clip_range=0.2, vf_coef=0.5, ent_coef=0.01)
    adv_n = (adv - adv.mean()) / (adv.std() + 1e-8) if advnorm else adv
    info, rdh, rdls, rdv = cpu_ref.loss_grads_ref(algo, "gaussian", head, logstd, v, act, adv_n, ret,
                                                  old if algo == "ppo" else None, 0.2, 0.5, 0.01)
    sc = _h(sc)
    assert abs(sc[3] - info["loss"]) < 1e-4, (sc, info)
    assert abs(sc[0] - info["actor-loss"]) < 1e-4
    np.testing.assert_allclose(_h(dh), rdh, rtol=2e-4, atol=1e-8)
    np.testing.assert_allclose(_h(dv), rdv, rtol=1e-4, atol=1e-9)
    np.testing.assert_allclose(_h(dls), rdls, rtol=2e-4, atol=1e-5)
    if algo == "ppo":
        assert abs(sc[4] - info["clip_ratio"]) < 2.0 / B


def test_loss_kernel_out_of_range_idx_is_inert():
    from xuanpolicy_amd import ops
    B, A = 64, 3
    head = torch.randn(B, A, device=DEV)
    idx = torch.arange(B, device=DEV)
    idx[5] = 10_000
    idx[9] = -3
    sc, dh, dls, dv = ops.policy_loss("a2c", "gaussian", head, torch.zeros(A, device=DEV), torch.zeros(B, device=DEV),
                                      torch.zeros(B * A, device=DEV), torch.ones(B, device=DEV),
                                      torch.zeros(B, device=DEV), idx=idx)
    assert float(dh[5].abs().sum()) == 0.0 and float(dh[9].abs().sum()) == 0.0
    assert torch.isfinite(sc).all()


# ---------------------------------------------------------------------------------------------- K5
def test_rms_kernel_golden(golden):
    from xuanpolicy_amd import ops
    g = golden("rms.npz")
    mean = torch.zeros(5, device=DEV)
    var = torch.ones(5, device=DEV)
    cnt = torch.full((1,), 1e-4, dtype=torch.float64, device=DEV)
    for k in range(g["obs/x"].shape[0]):
        ops.rms_update(_d(g["obs/x"][k]), mean, var, cnt)
        np.testing.assert_allclose(_h(mean), g["obs/mean"][k], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(_h(var), g["obs/var"][k], rtol=1e-5, atol=1e-6)
        assert abs(float(cnt) - g["obs/count"][k]) < 1e-6


@pytest.mark.parametrize("N,D", [(4096, 17), (1000, 376), (3, 2)])
def test_rms_and_normalize_strided(N, D):
    from xuanpolicy_amd import ops
    rng = np.random.default_rng(N + D)
    X = _d(rng.normal(1.0, 3.0, (N, D + 5)).astype(np.float32))
    x = X[:, :D]
    ref = cpu_ref.RunningMeanStdRef((D,))
    mean = torch.zeros(D, device=DEV)
    var = torch.ones(D, device=DEV)
    cnt = torch.full((1,), 1e-4, dtype=torch.float64, device=DEV)
    for _ in range(3):
        ops.rms_update(x, mean, var, cnt)
        ref.update(_h(x))
    np.testing.assert_allclose(_h(mean), ref.mean, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(_h(var), ref.var, rtol=1e-4, atol=1e-5)
    out = torch.empty(N, D, device=DEV)
    T = 4
    col = torch.zeros(N, T, D, device=DEV)
    cur = torch.tensor([2, 0, 0, 0], dtype=torch.int32, device=DEV)
    ops.obs_normalize(x, mean, var, 5.0, out, col_out=col, col_ld=T * D, cursor=cur)
    exp = np.clip((_h(x) - _h(mean)) / (np.sqrt(_h(var)) + 1e-8), -5, 5)
    np.testing.assert_allclose(_h(out), exp, rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(_h(col[:, 2]), _h(out))
    assert float(col[:, [0, 1, 3]].abs().sum()) == 0.0


@pytest.mark.parametrize("N,D", [(4096, 17), (1000, 376), (3, 2), (70000, 5)])
def test_rms_update_single_launch_equals_two_launch(N, D):
    """xpa_rms_update (last-arriving block merges, ticket) == xpa_rms_partials + xpa_rms_merge, bit for
    bit, over consecutive updates; the ticket is back at zero after every launch."""
    from xuanpolicy_amd import ops
    rng = np.random.default_rng(N * 3 + D)
    X = _d(rng.normal(1.0, 3.0, (N, D + 3)).astype(np.float32))
    x = X[:, :D]
    st = [(torch.zeros(D, device=DEV), torch.ones(D, device=DEV),
           torch.full((1,), 1e-4, dtype=torch.float64, device=DEV)) for _ in range(2)]
    ticket = torch.zeros(1, dtype=torch.int32, device=DEV)
    for k in range(4):
        xk = x * (1.0 + 0.1 * k)
        ops.rms_update(xk, *st[0])
        ops.rms_update(xk, *st[1], ticket=ticket)
        for a, b in zip(st[0], st[1]):
            assert torch.equal(a, b)
        assert int(ticket.item()) == 0


# ---------------------------------------------------------------------------------------------- K7
@pytest.mark.parametrize("D,A,discrete", [(17, 6, False), (376, 17, False), (4, 2, True)])
def test_synthbox_step_matches_oracle(D, A, discrete):
    from xuanpolicy_amd.envs import SynthBoxVecEnv
    N = 512
    env = SynthBoxVecEnv(N, D, A, seed=11, discrete=discrete, max_episode_steps=7, device=DEV)
    ref = synth_env.SynthBoxVec(N, D, A, seed=11, discrete=discrete, max_episode_steps=7)
    np.testing.assert_array_equal(_h(env.obs), ref.state)
    rng = np.random.default_rng(0)
    for step in range(12):
        acts = rng.integers(0, A, N) if discrete else rng.normal(0, 1, (N, A)).astype(np.float32)
        ref.state = _h(env.obs).copy()  # re-sync: compare one step at a time (tanh dynamics amplify ulps)
        fin, r, te, tr, nxt = ref.step(acts)
        g_fin, g_r, g_te, g_tr, _ = env.step(acts)
        np.testing.assert_allclose(g_fin, fin, rtol=1e-5, atol=2e-6)
        np.testing.assert_allclose(g_r, r, rtol=1e-5, atol=1e-6)
        near = np.abs(fin[:, 0] - synth_env.TERM_THRESH) < 1e-5
        np.testing.assert_array_equal(g_te[~near], te[~near])
        np.testing.assert_array_equal(g_tr, tr)
        done = te | tr
        np.testing.assert_array_equal(_h(env.obs)[done & ~near], nxt[done & ~near])  # reset states are exact
    assert int(env.ep_index.sum()) > 0


# ---------------------------------------------------------------------------------------------- K3
def test_rollout_sample_gaussian_and_categorical():
    from xuanpolicy_amd import ops
    N, T, A = 20000, 4, 3
    cur = torch.tensor([1, 77, 0, 0], dtype=torch.int32, device=DEV)
    mu = torch.randn(N, A, device=DEV) * 0.3
    logstd = torch.tensor([-1.0, -0.5, 0.2], device=DEV)
    v = torch.randn(N, device=DEV)
    act = torch.zeros(N, T, A, device=DEV)
    logp = torch.zeros(N, T, device=DEV)
    val = torch.zeros(N, T, device=DEV)
    env_in = torch.zeros(N, A + 2, device=DEV)
    ops.rollout_sample("gaussian", mu, logstd, v, cur, 5, act, logp, val, env_in[:, :A], act_clip=1.0)
    a1 = act[:, 1]
    eps = (a1 - mu) / torch.exp(logstd)
    assert abs(float(eps.mean())) < 0.02 and abs(float(eps.std()) - 1.0) < 0.02
    ref_lp = torch.distributions.Normal(mu, torch.exp(logstd)).log_prob(a1).sum(-1)
    np.testing.assert_allclose(_h(logp[:, 1]), _h(ref_lp), rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(_h(val[:, 1]), _h(v))
    np.testing.assert_array_equal(_h(env_in[:, :A]), np.clip(_h(a1), -1, 1))
    assert float(act[:, [0, 2, 3]].abs().sum()) == 0.0
    # same cursor.step -> same draws; different step -> different draws
    act2 = torch.zeros_like(act)
    ops.rollout_sample("gaussian", mu, logstd, v, cur, 5, act2, logp, val, env_in[:, :A])
    assert torch.equal(act2[:, 1], a1)
    K = 5
    logits = torch.randn(N, K, device=DEV)
    cact = torch.zeros(N, T, device=DEV)
    onehot = torch.zeros(N, K, device=DEV)
    ops.rollout_sample("categorical", logits, None, v, cur, 9, cact, logp, val, onehot)
    k = cact[:, 1].long()
    np.testing.assert_allclose(_h(logp[:, 1]), _h(torch.log_softmax(logits, -1).gather(1, k[:, None])[:, 0]),
                               rtol=1e-5, atol=1e-5)
    assert torch.equal(onehot.argmax(1), k) and torch.equal(onehot.sum(1), torch.ones(N, device=DEV))
    freq = torch.bincount(k, minlength=K).float() / N
    np.testing.assert_allclose(_h(freq), _h(torch.softmax(logits, -1).mean(0)), atol=0.015)


# ---------------------------------------------------------------------------------------------- K8
@pytest.mark.parametrize("algo,atari,mid", [("ppo", False, False), ("a2c", False, False), ("ppo", True, False),
                                            ("a2c", False, True)])
def test_rollout_post_matches_reference_rules(algo, atari, mid):
    """mid: a second bootstrap array v_boot_mid for the closures before the last step (A2C's V(norm(reset_obs)),
    a2c_agent.py:88-95); the last step's closures keep v_boot."""
    from xuanpolicy_amd import ops
    rng = np.random.default_rng(3)
    N, T = 300, 5
    returns = rng.normal(0, 1, N).astype(np.float32)
    ret_rms = cpu_ref.RunningMeanStdRef(())
    ret_rms.mean, ret_rms.var, ret_rms.count = np.float32(0.3), np.float32(2.0), 17.0
    rm = torch.tensor([0.3], device=DEV)
    rv = torch.tensor([2.0], device=DEV)
    rc = torch.tensor([17.0], dtype=torch.float64, device=DEV)
    rt = _d(returns)
    bufs = {k: torch.zeros(N, T, device=DEV) for k in ("rew", "term", "boot")}
    closed = torch.zeros(N, T, dtype=torch.uint8, device=DEV)
    cur = torch.tensor([0, 0, 0, 0], dtype=torch.int32, device=DEV)
    for t in range(T):
        rew = rng.normal(0, 2, N).astype(np.float32)
        term = rng.random(N) < 0.2
        trunc = rng.random(N) < 0.1
        vb = rng.normal(0, 1, N).astype(np.float32)
        vm = rng.normal(0, 1, N).astype(np.float32)
        # reference rules (agent.py:118-123, ppoclip_agent.py:69-101 / a2c_agent.py:84)
        exp_rew = np.clip(rew / np.clip(np.sqrt(ret_rms.var), 0.1, 100), -5, 5)
        if algo == "ppo":
            returns = (1 - term) * 0.99 * returns + rew
        else:
            returns = 0.99 * returns + rew
        done = term | trunc
        for i in np.nonzero(done)[0]:
            ret_rms.update(returns[i:i + 1])
        returns = np.where(done, 0, returns).astype(np.float32)
        last = t == T - 1
        close = np.full(N, True) if last else (done & ~(atari & ~trunc))
        exp_boot = np.where(close, np.where(term, 0, vm if (mid and not last) else vb), 0)
        ops.rollout_post(_d(rew), _d(term.astype(np.uint8)), _d(trunc.astype(np.uint8)), _d(vb), cur, rm, rv, rc, rt,
                         bufs["rew"], bufs["term"], closed, bufs["boot"], 0.99, mask_returns=(algo == "ppo"),
                         use_rewnorm=True, rew_range=5.0, atari_lifeloss=atari, v_boot_mid=_d(vm) if mid else None)
        np.testing.assert_allclose(_h(bufs["rew"][:, t]), exp_rew, rtol=1e-5, atol=1e-6)
        np.testing.assert_array_equal(_h(bufs["term"][:, t]), term.astype(np.float32))
        np.testing.assert_array_equal(_h(closed[:, t]).astype(bool), close)
        np.testing.assert_allclose(_h(bufs["boot"][:, t]), exp_boot, rtol=0, atol=0)
        np.testing.assert_allclose(_h(rt), returns, rtol=1e-5, atol=1e-5)
        assert abs(float(rm) - float(ret_rms.mean)) < 1e-5 * max(1, abs(float(ret_rms.mean)))
        assert abs(float(rv) - float(ret_rms.var)) < 1e-4 * max(1, abs(float(ret_rms.var)))
        assert abs(float(rc) - ret_rms.count) < 1e-9
    assert _h(cur)[0] == 0 and _h(cur)[1] == T


@pytest.mark.parametrize("slot_src", [False, True])
def test_rollout_post_deferred_slot_rows(slot_src):
    """xpa_rollout_post_deferred_norm: a mid-buffer truncation keeps norm(final obs) in its slot, or with slot_src
    (A2C: the env's next, reset, observations) norm(slot_src); the last step's boot rows are norm(final obs) either
    way.  Row-strided sources (a column block of a wider matrix, as the device envs hold them)."""
    from xuanpolicy_amd import ops
    rng = np.random.default_rng(5)
    N, T, D, S = 97, 4, 17, 3
    mean = rng.normal(0, 0.3, D).astype(np.float32)
    var = rng.uniform(0.5, 2.0, D).astype(np.float32)

    def norm(x):
        return np.clip((x - mean) / (np.sqrt(var) + np.float32(1e-8)), -5, 5).astype(np.float32)
    rm, rv = torch.zeros(1, device=DEV), torch.ones(1, device=DEV)
    rc = torch.full((1,), 1e-4, dtype=torch.float64, device=DEV)
    rt = torch.zeros(N, device=DEV)
    bufs = {k: torch.zeros(N, T, device=DEV) for k in ("rew", "term", "boot")}
    closed = torch.zeros(N, T, dtype=torch.uint8, device=DEV)
    cur = torch.zeros(4, dtype=torch.int32, device=DEV)
    slot_obs = torch.zeros(S * N, D, device=DEV)
    slot_t = torch.full((S * N,), -1, dtype=torch.int32, device=DEV)
    over = torch.zeros(1, dtype=torch.int32, device=DEV)
    boot_norm = torch.zeros(N, D, device=DEV)
    kept = {}
    for t in range(T):
        fin = rng.normal(0, 1, (N, D + 3)).astype(np.float32)
        nxt = rng.normal(0, 1, (N, D + 5)).astype(np.float32)
        trunc = (rng.random(N) < 0.3) if t < T - 1 else np.zeros(N, bool)
        term = np.zeros(N, bool)
        deferred = (_d(fin)[:, :D], slot_obs, slot_t, over, _d(mean), _d(var), 5.0, boot_norm)
        if slot_src:
            deferred += (_d(nxt)[:, :D],)
        ops.rollout_post(_d(np.zeros(N, np.float32)), _d(term.astype(np.uint8)), _d(trunc.astype(np.uint8)), None, cur,
                         rm, rv, rc, rt, bufs["rew"], bufs["term"], closed, bufs["boot"], 0.99, deferred=deferred)
        for n in np.nonzero(trunc)[0]:
            k = sum(1 for (m, _) in kept if m == n)
            kept[(n, k)] = (t, norm((nxt if slot_src else fin)[n, :D]))
        if t == T - 1:
            np.testing.assert_allclose(_h(boot_norm), norm(fin[:, :D]), rtol=1e-6, atol=1e-6)
    assert len(kept) > N // 3 and int(over) == 0
    st, so = _h(slot_t), _h(slot_obs)
    for (n, k), (t, row) in kept.items():
        assert st[k * N + n] == t
        np.testing.assert_allclose(so[k * N + n], row, rtol=1e-6, atol=1e-6)


# ---------------------------------------------------------------------------------------------- K9
@pytest.mark.parametrize("max_norm", [0.5, None, 0.0, 1e9])
def test_fused_clip_adam_matches_torch(max_norm):
    """xpa_clip_adam_step == clip_grad_norm_ + torch.optim.Adam (foreach) over several steps, with
    optimizer.state_dict() still describing the moments.  None = use_grad_clip False (no clip); 0.0 clips
    to a zero gradient exactly as torch.nn.utils.clip_grad_norm_(params, 0) does."""
    from xuanpolicy_amd.flat import FlatState, FusedClipAdam
    torch.manual_seed(0)
    net_a = torch.nn.Sequential(torch.nn.Linear(17, 33), torch.nn.LeakyReLU(), torch.nn.Linear(33, 7)).to(DEV)
    net_b = torch.nn.Sequential(torch.nn.Linear(17, 33), torch.nn.LeakyReLU(), torch.nn.Linear(33, 7)).to(DEV)
    net_b.load_state_dict(net_a.state_dict())
    opt_a = torch.optim.Adam(net_a.parameters(), 4e-4, eps=1e-5, foreach=True)
    opt_b = torch.optim.Adam(net_b.parameters(), 4e-4, eps=1e-5)
    fs = FlatState(net_b.parameters())
    fused = FusedClipAdam(opt_b, fs)
    for step in range(6):
        x = torch.randn(64, 17, device=DEV)
        opt_a.zero_grad()
        (net_a(x) ** 2).mean().backward()
        if max_norm is not None:
            torch.nn.utils.clip_grad_norm_(net_a.parameters(), max_norm)
        opt_a.step()
        fs.zero_()
        (net_b(x) ** 2).mean().backward()
        fused.step(max_norm)
        for pa, pb in zip(net_a.parameters(), net_b.parameters()):
            np.testing.assert_allclose(_h(pb), _h(pa), rtol=1e-5, atol=1e-7)
    sa, sb = opt_a.state_dict()["state"], opt_b.state_dict()["state"]
    for k in sa:
        np.testing.assert_allclose(_h(sb[k]["exp_avg"]), _h(sa[k]["exp_avg"]), rtol=1e-5, atol=1e-9)
        np.testing.assert_allclose(_h(sb[k]["exp_avg_sq"]), _h(sa[k]["exp_avg_sq"]), rtol=1e-4, atol=1e-10)
        assert float(sb[k]["step"]) == float(sa[k]["step"]) == 6.0


def test_splitk_linear_matches_linear():
    from xuanpolicy_amd.policies import FastLinear
    torch.manual_seed(1)
    for (n_in, n_out) in [(17, 256), (256, 256), (256, 6), (256, 1)]:
        lin = FastLinear(n_in, n_out).to(DEV)
        ref = torch.nn.Linear(n_in, n_out).to(DEV)
        ref.load_state_dict(lin.state_dict())
        x = torch.randn(65536, n_in, device=DEV, requires_grad=True)
        gy = torch.randn(65536, n_out, device=DEV)
        lin(x).backward(gy)
        gx = x.grad.clone()
        x.grad = None
        ref(x).backward(gy)
        np.testing.assert_allclose(_h(gx), _h(x.grad), rtol=1e-5, atol=1e-5)
        # fp32 sums over K = 65536 in a different order: compare relative to the gradient's scale
        for a, b in ((lin.weight.grad, ref.weight.grad), (lin.bias.grad, ref.bias.grad)):
            a, b = _h(a).astype(np.float64), _h(b).astype(np.float64)
            assert np.abs(a - b).max() <= 2e-5 * np.abs(b).max(), (np.abs(a - b).max(), np.abs(b).max())


@pytest.mark.parametrize("row_shape,dtype", [((4, 84, 84), torch.uint8), ((17,), torch.float32), ((3,), torch.uint8),
                                             ((1024,), torch.float32), ((4, 84, 84), torch.float32)])
def test_gather_minibatch_row_shapes(row_shape, dtype):
    """K4 for narrow rows, 4-byte and byte rows and the wide-row path (>= 4 KiB, Atari frames), with
    out-of-range indices zeroed and the adv moments computed alongside."""
    from xuanpolicy_amd import ops
    g = torch.Generator(device="cuda").manual_seed(1)
    R, B = 3000, 777
    if dtype == torch.uint8:
        src = torch.randint(0, 256, (R,) + row_shape, generator=g, device="cuda", dtype=torch.int64).to(torch.uint8)
    else:
        src = torch.randn((R,) + row_shape, generator=g, device="cuda")
    idx = torch.randint(0, R, (B,), generator=g, device="cuda")
    idx[3] = R + 1
    idx[10] = -5
    adv = torch.randn(R, generator=g, device="cuda")
    out, part = ops.gather_minibatch(idx, src, adv=adv)
    ok = (idx >= 0) & (idx < R)
    exp = torch.zeros_like(out)
    exp[ok] = src[idx[ok]]
    assert torch.equal(out, exp)
    a = adv[idx[ok]].double()
    np.testing.assert_allclose(part[:, 0].sum().item(), a.sum().item(), rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(part[:, 1].sum().item(), (a * a).sum().item(), rtol=1e-12)


@pytest.mark.parametrize("n", [1, 2, 7, 1000, 524288, 65536 * 8 + 3])
def test_random_permutation_is_a_bijection(n):
    from xuanpolicy_amd import ops
    p0 = ops.random_permutation(n, 1, 0)
    assert torch.equal(torch.sort(p0).values, torch.arange(n, device=p0.device))
    if n >= 1000:
        p1 = ops.random_permutation(n, 1, 1)
        assert not torch.equal(p0, p1)                                   # a new epoch reshuffles
        assert torch.equal(p0, ops.random_permutation(n, 1, 0))          # deterministic per (seed, counter)
        # no positional structure: correlation between position and value is small
        pos = torch.arange(n, device=p0.device, dtype=torch.float64)
        c = torch.corrcoef(torch.stack([pos, p0.double()]))[0, 1].item()
        assert abs(c) < 0.05
