"""GPU: the C3 update's convolution kernels at the size the bench runs them — one minibatch of B = 16 384 frames
(a2c/atari.yaml: 1024 envs x 128 steps / 8 minibatches; AC_CNN_Atari cnn.py:45-93) — against float64 torch
convolutions (the kernel tests stopped at B <= 2048, so grid and indexing at 7.2 M output rows per launch
ran only inside the bench).  The production forms (the library defaults): K25B conv1 forward from uint8, K26B conv1
weight gradient, K27B conv2 data gradient, K28 conv2 / conv3 forward and conv3 data gradient, K29 conv2 / conv3
weight gradient.  Per-image outputs (forward, data gradient) are checked on sampled images — the first, the last 16 and
random ones in between — against f64 convolutions of those images; weight gradients (reductions over every row) against
the f64 gradient summed over 2048-frame chunks."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
B = 16384


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _ops():
    from xuanpolicy_amd import _lib, ops
    return _lib, ops


def _sample(n=B, k=32, seed=0):
    rng = np.random.default_rng(seed)
    mid = rng.choice(np.arange(1, n - 16), k, replace=False)
    return torch.as_tensor(np.sort(np.concatenate([[0], mid, np.arange(n - 16, n)])), device=DEV)


def _chunks(n=B, c=2048):
    return [(i, min(n, i + c)) for i in range(0, n, c)]


def test_conv1_u8_forward_at_c3_batch():
    """K25B (the default conv1 form): [16384, 84, 84, 4] uint8 -> [16384, 21, 21, 32] with bias + ReLU."""
    _l, ops = _ops()
    L = ops.lib()
    assert L.xpa_conv1_form(-1) & 1, "K25B is the default conv1 forward"
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randint(0, 256, (B, 84, 84, 4), device=DEV, dtype=torch.int32, generator=g).to(torch.uint8)
    w = torch.randn(32, 4, 8, 8, device=DEV, generator=g) * 0.05
    b = torch.randn(32, device=DEV, generator=g) * 0.1
    y = torch.full((B, 21, 21, 32), float("nan"), device=DEV)
    _l.check(L.xpa_conv1_u8_fwd(1, ops._p(x), B, 84, 84, 4, 8, 4, 2, ops._p(w), ops._p(b), 32, 0.0, ops._p(y),
                                ops._stream(DEV)), "conv1_u8")
    assert not torch.isnan(y).any()
    s = _sample()
    ref = F.relu(F.conv2d((x[s].double() / 255.0).permute(0, 3, 1, 2), w.double(), b.double(), 4, 2)).permute(0, 2, 3, 1)
    torch.testing.assert_close(y[s].double(), ref, rtol=1e-5, atol=2e-5)


def test_conv1_u8_weight_gradient_at_c3_batch():
    """K26B (the default conv1 weight gradient): dW [32, 4, 8, 8] over 16384 x 441 rows, f64 column-sum finalize."""
    _l, ops = _ops()
    L, st = ops.lib(), ops._stream(DEV)
    assert L.xpa_conv1_form(-1) & 2, "K26B is the default conv1 weight gradient"
    g = torch.Generator(device=DEV).manual_seed(2)
    x = torch.randint(0, 256, (B, 84, 84, 4), device=DEV, dtype=torch.int32, generator=g).to(torch.uint8)
    dz = torch.randn(B, 21, 21, 32, device=DEV, generator=g)
    G = int(L.xpa_conv1_u8_wgrad_num_partials())
    part = torch.full((G, 8192), float("nan"), device=DEV)
    _l.check(L.xpa_conv1_u8_wgrad(ops._p(dz), ops._p(x), B, 84, 84, 4, 8, 4, 2, 32, ops._p(part), st), "wgrad")
    dw = torch.empty(32, 4, 8, 8, device=DEV)
    _l.check(L.xpa_colsum_finalize(ops._p(part), G, 8192, ops._p(dw), st), "finalize")
    ref = torch.zeros(32, 4, 8, 8, dtype=torch.float64, device=DEV)
    for i, j in _chunks():
        ref += torch.nn.grad.conv2d_weight((x[i:j].double() / 255.0).permute(0, 3, 1, 2), (32, 4, 8, 8),
                                           dz[i:j].double().permute(0, 3, 1, 2), 4, 2)
    tol = 2e-6 * float(ref.abs().max()) + 1e-6 * (B * 441) ** 0.5
    torch.testing.assert_close(dw.double(), ref, rtol=1e-5, atol=tol)


def test_conv2_data_gradient_at_c3_batch():
    """K27B (the default conv2 data gradient): dX [16384, 21, 21, 32] from dY [16384, 10, 10, 64], 4x4 stride 2 pad 1."""
    _l, ops = _ops()
    L = ops.lib()
    assert L.xpa_conv1_form(-1) & 4, "K27B is the default conv2 data gradient"
    g = torch.Generator(device=DEV).manual_seed(3)
    dy = torch.randn(B, 10, 10, 64, device=DEV, generator=g)
    w = torch.randn(64, 32, 4, 4, device=DEV, generator=g) * 0.1
    dx = torch.full((B, 21, 21, 32), float("nan"), device=DEV)
    _l.check(L.xpa_conv_dgrad_s2k(ops._p(dy), B, 10, 10, 64, ops._p(w), 32, 4, 2, 1, 21, 21, ops._p(dx),
                                  ops._stream(DEV)), "dgrad")
    assert not torch.isnan(dx).any()
    s = _sample(seed=3)
    ref = torch.nn.grad.conv2d_input((len(s), 32, 21, 21), w.double(), dy[s].double().permute(0, 3, 1, 2), 2, 1)
    torch.testing.assert_close(dx[s].double(), ref.permute(0, 2, 3, 1), rtol=1e-5, atol=1e-5)


# (H, Cin, Cout, k, s): AC_CNN_Atari's conv2 (21 -> 10) and conv3 (10 -> 10)
CONVS = [(21, 32, 64, 4, 2), (10, 64, 64, 3, 1)]


@pytest.mark.parametrize("H,Cin,Cout,k,s", CONVS)
def test_igemm_forward_at_c3_batch(H, Cin, Cout, k, s):
    """K28 (the default form) with bias + ReLU at B = 16384."""
    _l, ops = _ops()
    L = ops.lib()
    p = (k - s) // 2
    OH = (H + 2 * p - k) // s + 1
    g = torch.Generator(device=DEV).manual_seed(4 + k)
    x = torch.rand(B, H, H, Cin, device=DEV, generator=g)
    w = torch.randn(Cout, Cin, k, k, device=DEV, generator=g) / np.sqrt(Cin * k * k)
    b = torch.randn(Cout, device=DEV, generator=g) * 0.1
    y = torch.full((B, OH, OH, Cout), float("nan"), device=DEV)
    _l.check(L.xpa_conv_fwd(1, ops._p(x), B, H, H, Cin, ops._p(w), ops._p(b), Cout, k, s, p, 0.0, ops._p(y),
                            ops._stream(DEV)), "xpa_conv_fwd")
    assert not torch.isnan(y).any()
    sm = _sample(seed=k)
    ref = F.relu(F.conv2d(x[sm].double().permute(0, 3, 1, 2), w.double(), b.double(), s, p)).permute(0, 2, 3, 1)
    scale = float(ref.abs().max())
    torch.testing.assert_close(y[sm].double(), ref, rtol=0, atol=2e-6 * max(scale, 1.0))


def test_igemm_conv3_data_gradient_at_c3_batch():
    """K28's data gradient of conv3 (3x3 stride 1) with conv2's ReLU backward and bias gradient fused, B = 16384."""
    _l, ops = _ops()
    L = ops.lib()
    H, Cin, Cout, k, s, p = 10, 64, 64, 3, 1, 1
    g = torch.Generator(device=DEV).manual_seed(6)
    w = torch.randn(Cout, Cin, k, k, device=DEV, generator=g) / np.sqrt(Cin * k * k)
    dz = torch.randn(B, H, H, Cout, device=DEV, generator=g)
    y_prev = torch.relu(torch.randn(B, H, H, Cin, device=DEV, generator=g))
    dx = torch.full((B, H, H, Cin), float("nan"), device=DEV)
    G = int(L.xpa_conv_dgrad_num_partials(B, H, H))
    part = torch.full((G, Cin), float("nan"), device=DEV)
    _l.check(L.xpa_conv_dgrad(ops._p(dz), B, H, H, Cout, ops._p(w), Cin, k, s, p, H, H, 1, ops._p(y_prev), 0.0,
                              ops._p(dx), ops._p(part), ops._stream(DEV)), "xpa_conv_dgrad")
    db = torch.empty(Cin, device=DEV)
    _l.check(L.xpa_colsum_finalize(ops._p(part), G, Cin, ops._p(db), ops._stream(DEV)), "finalize")
    sm = _sample(seed=6)
    ref = torch.nn.grad.conv2d_input((len(sm), Cin, H, H), w.double(), dz[sm].double().permute(0, 3, 1, 2), s, p)
    ref = ref.permute(0, 2, 3, 1) * (y_prev[sm].double() > 0)
    scale = float(ref.abs().max())
    torch.testing.assert_close(dx[sm].double(), ref, rtol=0, atol=2e-6 * max(scale, 1.0))
    db_ref = torch.zeros(Cin, dtype=torch.float64, device=DEV)
    for i, j in _chunks():
        d = torch.nn.grad.conv2d_input((j - i, Cin, H, H), w.double(), dz[i:j].double().permute(0, 3, 1, 2), s, p)
        db_ref += (d.permute(0, 2, 3, 1) * (y_prev[i:j].double() > 0)).sum((0, 1, 2))
    torch.testing.assert_close(db.double(), db_ref, rtol=1e-5, atol=1e-5 * (B * H * H) ** 0.5)


@pytest.mark.parametrize("H,Cin,Cout,k,s", CONVS)
def test_igemm_weight_gradient_at_c3_batch(H, Cin, Cout, k, s):
    """K29 (the LDS-slab form the C3 update runs) with the block's own ReLU backward folded in and its bias gradient,
    B = 16384: dW over every output row against the f64 gradient."""
    _l, ops = _ops()
    L = ops.lib()
    p = (k - s) // 2
    OH = (H + 2 * p - k) // s + 1
    g = torch.Generator(device=DEV).manual_seed(7 + k)
    x = torch.rand(B, H, H, Cin, device=DEV, generator=g)
    gr = torch.randn(B, OH, OH, Cout, device=DEV, generator=g)
    y = torch.relu(torch.randn(B, OH, OH, Cout, device=DEV, generator=g))
    G = int(L.xpa_conv_wgrad_num_partials())
    cols = Cout * Cin * k * k
    part = torch.full((G, cols), float("nan"), device=DEV)
    bpart = torch.full((G, Cout), float("nan"), device=DEV)
    _l.check(L.xpa_conv_wgrad(1, ops._p(gr), ops._p(y), 0.0, ops._p(x), B, H, H, Cin, Cout, k, s, p, ops._p(part),
                              ops._p(bpart), ops._stream(DEV)), "xpa_conv_wgrad")
    dw = torch.empty(Cout, Cin, k, k, device=DEV)
    _l.check(L.xpa_colsum_finalize(ops._p(part), G, cols, ops._p(dw), ops._stream(DEV)), "finalize")
    db = torch.empty(Cout, device=DEV)
    _l.check(L.xpa_colsum_finalize(ops._p(bpart), G, Cout, ops._p(db), ops._stream(DEV)), "finalize")
    dw_ref = torch.zeros(Cout, Cin, k, k, dtype=torch.float64, device=DEV)
    db_ref = torch.zeros(Cout, dtype=torch.float64, device=DEV)
    for i, j in _chunks():
        dz = gr[i:j].double() * (y[i:j] > 0)
        dw_ref += torch.nn.grad.conv2d_weight(x[i:j].double().permute(0, 3, 1, 2), (Cout, Cin, k, k),
                                              dz.permute(0, 3, 1, 2), s, p)
        db_ref += dz.sum((0, 1, 2))
    rows = B * OH * OH
    tol = 2e-6 * float(dw_ref.abs().max()) + 1e-6 * rows ** 0.5
    torch.testing.assert_close(dw.double(), dw_ref, rtol=1e-5, atol=tol)
    torch.testing.assert_close(db.double(), db_ref, rtol=1e-5, atol=1e-5 * rows ** 0.5)
