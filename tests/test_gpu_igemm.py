"""GPU: K28 / K29 (csrc/igemm.hip), the generic NHWC implicit-GEMM convolutions of the CNN trunks, against float64
torch convolutions of the same operands (cnn_block, xuance/torch/utils/layers.py:27-57: padding (k - s) // 2):
forward with bias + activation, the data gradient (stride 1 and the masked stride-2 form) with the previous block's
activation backward and bias gradient fused, the weight gradient with and without the block's own activation backward
folded in.  Shapes: the production C3 / C5 convs (32 -> 64 4x4 s2, 64 -> 64 3x3 s1), the small-channel test nets
(4 -> 8 8x8 s4, 8 -> 8 4x4 s2) and ragged batches."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

# (B, H, W, Cin, Cout, k, s)
SHAPES = [(37, 21, 21, 32, 64, 4, 2), (29, 10, 10, 64, 64, 3, 1), (5, 84, 84, 4, 8, 8, 4), (11, 21, 21, 8, 8, 4, 2),
          (300, 10, 10, 64, 64, 3, 1)]


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture(params=[1, 3, 0], ids=["k28b", "k28b_mt3", "k28"])
def ig_form(request):
    """r05: K28 on the bf16 matrix cores (K28B, opt-in, where the GEMM's input channels are a multiple of 16; mt3: its
    3-tile waves, forward only) and the fp32-MFMA K28 (the default)."""
    from xuanpolicy_amd import ops
    L = ops.lib()
    prev = L.xpa_conv_igemm_form(-1)
    L.xpa_conv_igemm_form(request.param)
    yield request.param
    L.xpa_conv_igemm_form(prev)


def _data(B, H, W, Cin, Cout, k, s, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(B, H, W, Cin, generator=g)
    w = torch.randn(Cout, Cin, k, k, generator=g) / np.sqrt(Cin * k * k)
    b = torch.randn(Cout, generator=g) * 0.1
    return x, w, b


@pytest.mark.parametrize("shape", SHAPES)
def test_conv_fwd_matches_f64(shape, ig_form):
    from xuanpolicy_amd import _lib, ops
    B, H, W, Cin, Cout, k, s = shape
    p = (k - s) // 2
    x, w, b = _data(*shape, seed=1)
    ref = F.relu(F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), b.double(), s, p)).permute(0, 2, 3, 1)
    OH, OW = ref.shape[1], ref.shape[2]
    assert ops.lib().xpa_conv_igemm_ok(Cin, Cout, k)
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
    y = torch.full((B, OH, OW, Cout), float("nan"), device=DEV)
    _lib.check(ops.lib().xpa_conv_fwd(1, ops._p(xd), B, H, W, Cin, ops._p(wd), ops._p(bd), Cout, k, s, p, 0.0,
                                      ops._p(y), ops._stream(DEV)), "xpa_conv_fwd")
    scale = float(ref.abs().max())
    np.testing.assert_allclose(y.cpu().double().numpy(), ref.numpy(), rtol=0, atol=2e-6 * max(scale, 1.0))


@pytest.mark.parametrize("shape", SHAPES)
def test_conv_dgrad_matches_f64(shape, ig_form):
    """dX of the conv from dZ, times act'(y_prev) of the previous block (ReLU from its output), and that block's bias
    gradient (the column sums of the result)."""
    from xuanpolicy_amd import _lib, ops
    B, H, W, Cin, Cout, k, s = shape
    p = (k - s) // 2
    if not ops.lib().xpa_conv_igemm_ok(Cout, Cin, k) or s > 2:
        pytest.skip("data gradient taken by K28 for stride <= 2 and a weight image that fits the LDS")
    x, w, _ = _data(*shape, seed=2)
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    g = torch.Generator().manual_seed(3)
    dz = torch.randn(B, OH, OW, Cout, generator=g)
    y_prev = torch.relu(torch.randn(B, H, W, Cin, generator=g))          # the previous block's ReLU output
    xr = torch.zeros(B, Cin, H, W, dtype=torch.float64, requires_grad=True)
    out = F.conv2d(xr, w.double(), None, s, p)
    out.backward(dz.double().permute(0, 3, 1, 2))
    dx_ref = xr.grad.permute(0, 2, 3, 1) * (y_prev.double() > 0)
    db_ref = dx_ref.sum((0, 1, 2))
    dzd, wd, ypd = dz.to(DEV), w.to(DEV), y_prev.to(DEV)
    dx = torch.full((B, H, W, Cin), float("nan"), device=DEV)
    G = int(ops.lib().xpa_conv_dgrad_num_partials(B, H, W))
    part = torch.full((G, Cin), float("nan"), device=DEV)
    _lib.check(ops.lib().xpa_conv_dgrad(ops._p(dzd), B, OH, OW, Cout, ops._p(wd), Cin, k, s, p, H, W, 1, ops._p(ypd),
                                        0.0, ops._p(dx), ops._p(part), ops._stream(DEV)), "xpa_conv_dgrad")
    db = torch.empty(Cin, device=DEV)
    _lib.check(ops.lib().xpa_colsum_finalize(ops._p(part), G, Cin, ops._p(db), ops._stream(DEV)), "finalize")
    scale = float(dx_ref.abs().max())
    np.testing.assert_allclose(dx.cpu().double().numpy(), dx_ref.detach().numpy(), rtol=0, atol=2e-6 * max(scale, 1))
    np.testing.assert_allclose(db.cpu().double().numpy(), db_ref.detach().numpy(), rtol=1e-5,
                               atol=1e-5 * float(dx_ref.abs().sum((0, 1, 2)).max()))


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("fold_act", [False, True])
@pytest.mark.parametrize("form", ["slab", "stream"])
def test_conv_wgrad_matches_f64(shape, fold_act, form):
    """dW = sum over output pixels of dz x; fold_act: the operand is g * act'(y) and the bias gradient comes too.  Both
    K29 forms: the LDS-slab one (every shape here) and the streaming one (forced)."""
    from xuanpolicy_amd import _lib, ops
    ops.lib().xpa_conv_wgrad_force_stream(1 if form == "stream" else 0)
    B, H, W, Cin, Cout, k, s = shape
    p = (k - s) // 2
    x, w, b = _data(*shape, seed=4)
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    gen = torch.Generator().manual_seed(5)
    gr = torch.randn(B, OH, OW, Cout, generator=gen)
    y = torch.relu(torch.randn(B, OH, OW, Cout, generator=gen))
    dz = gr * (y > 0) if fold_act else gr
    wr = w.double().clone().requires_grad_(True)
    F.conv2d(x.double().permute(0, 3, 1, 2), wr, None, s, p).backward(dz.double().permute(0, 3, 1, 2))
    dw_ref = wr.grad
    L = ops.lib()
    G = int(L.xpa_conv_wgrad_num_partials())
    cols = Cout * Cin * k * k
    part = torch.full((G, cols), float("nan"), device=DEV)
    bpart = torch.full((G, Cout), float("nan"), device=DEV)
    xd, gd, yd = x.to(DEV), gr.to(DEV), y.to(DEV)
    try:
        _lib.check(L.xpa_conv_wgrad(1 if fold_act else -1, ops._p(gd), ops._p(yd) if fold_act else None, 0.0,
                                    ops._p(xd), B, H, W, Cin, Cout, k, s, p, ops._p(part),
                                    ops._p(bpart) if fold_act else None, ops._stream(DEV)), "xpa_conv_wgrad")
    finally:
        L.xpa_conv_wgrad_force_stream(0)
    dw = torch.empty(Cout, Cin, k, k, device=DEV)
    _lib.check(L.xpa_colsum_finalize(ops._p(part), G, cols, ops._p(dw), ops._stream(DEV)), "finalize")
    tol = 2e-6 * float(dw_ref.abs().max()) + 1e-6 * (B * OH * OW) ** 0.5
    np.testing.assert_allclose(dw.cpu().double().numpy(), dw_ref.numpy(), rtol=1e-5, atol=tol)
    if fold_act:
        db = torch.empty(Cout, device=DEV)
        _lib.check(L.xpa_colsum_finalize(ops._p(bpart), G, Cout, ops._p(db), ops._stream(DEV)), "finalize")
        np.testing.assert_allclose(db.cpu().double().numpy(), dz.double().sum((0, 1, 2)).numpy(), rtol=1e-5,
                                   atol=1e-5 * (B * OH * OW) ** 0.5)


def test_conv_igemm_rejects_bad_shapes():
    from xuanpolicy_amd import ops
    L = ops.lib()
    assert not L.xpa_conv_igemm_ok(3, 32, 3)      # in_c not a multiple of 4
    assert not L.xpa_conv_igemm_ok(64, 64, 5)     # weight image over 160 KiB
    assert not L.xpa_conv_igemm_ok(128, 64, 3)
    assert L.xpa_conv_fwd(1, None, 1, 10, 10, 64, None, None, 64, 3, 1, 1, 0.0, None, None) == 1


@pytest.mark.parametrize("shape", [(2048, 21, 21, 32, 64, 4, 2), (2048, 10, 10, 64, 64, 3, 1)])
def test_conv_fwd_bf16_form_error_vs_fp32_form(shape):
    """K28B against K28 at C3's conv2 / conv3 shapes: both against the f64 conv, K28B's error no larger than 2x K28's."""
    from xuanpolicy_amd import _lib, ops
    L = ops.lib()
    B, H, W, Cin, Cout, k, s = shape
    p = (k - s) // 2
    x, w, b = _data(*shape, seed=4)
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), b.double(), s, p).permute(0, 2, 3, 1)
    OH, OW = ref.shape[1], ref.shape[2]
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
    prev = L.xpa_conv_igemm_form(-1)
    errs = []
    try:
        for form in (1, 0):
            L.xpa_conv_igemm_form(form)
            y = torch.full((B, OH, OW, Cout), float("nan"), device=DEV)
            _lib.check(L.xpa_conv_fwd(0, ops._p(xd), B, H, W, Cin, ops._p(wd), ops._p(bd), Cout, k, s, p, 0.0, ops._p(y),
                                      ops._stream(DEV)), "xpa_conv_fwd")
            errs.append(float((y.cpu().double() - ref).abs().max()))
    finally:
        L.xpa_conv_igemm_form(prev)
    assert errs[0] <= 2 * errs[1] + 1e-9, errs
