"""GPU: the C3 CNN trunk kernels (K20 frames -> f32, K21 bias + activation, K22 activation backward + bias
gradient) against their PyTorch definitions, and the explicit AC_CNN_Atari actor-critic forward/backward
(fused_cnn.FusedCNNActorCritic) against autograd through the reference-layout modules."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _lib():
    from xuanpolicy_amd import _lib, ops
    return _lib, ops


@pytest.mark.parametrize("n", [1, 15, 16, 17, 1000, 28224 * 3 + 5, 28224 * 64])
def test_frames_to_f32_is_the_reference_division(n):
    """K20 == float32(uint8 / 255.0 in float64) (cnn.py:89-92, NumPy semantics) bit for bit, ragged tails and an
    unaligned source included."""
    _l, ops = _lib()
    g = torch.Generator(device="cpu").manual_seed(n)
    x = torch.randint(0, 256, (n + 1,), generator=g, dtype=torch.int32).to(torch.uint8)
    for src in (x[:n], x[1:]):
        xd = src.to(DEV)
        out = torch.full((n,), -1.0, device=DEV)
        _l.check(ops.lib().xpa_frames_to_f32(ops._p(xd), n, ops._p(out), ops._stream(DEV)), "frames")
        ref = (src.numpy() / 255.0).astype(np.float32)
        np.testing.assert_array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("rows,cols", [(7, 32), (4096, 64), (100003, 32), (333, 512), (64, 4)])
@pytest.mark.parametrize("act,slope", [(0, 0.0), (1, 0.0), (1, 0.01), (2, 0.0)])
def test_bias_act_and_backward(rows, cols, act, slope):
    _l, ops = _lib()
    g = torch.Generator(device="cpu").manual_seed(rows + cols + act)
    z = torch.randn(rows, cols, generator=g).to(DEV)
    b = torch.randn(cols, generator=g).to(DEV)
    y = z.clone()
    _l.check(ops.lib().xpa_bias_act(act, ops._p(y), rows, cols, ops._p(b), slope, ops._stream(DEV)), "bias_act")
    zb = z + b
    ref = {0: zb, 1: torch.nn.functional.leaky_relu(zb, slope), 2: torch.tanh(zb)}[act]
    torch.testing.assert_close(y, ref, rtol=1e-6, atol=1e-6)
    # backward: dz = dh * act'(y), bias gradient = column sums of dz (f64 finalize)
    dh = torch.randn(rows, cols, generator=g).to(DEV)
    G = int(ops.lib().xpa_act_bwd_bias_num_partials(rows, cols))
    part = torch.empty(G, cols, device=DEV)
    dz = dh.clone()
    _l.check(ops.lib().xpa_act_bwd_bias(act, ops._p(dz), ops._p(y), rows, cols, slope, ops._p(dz), ops._p(part),
                                        ops._stream(DEV)), "act_bwd_bias")
    db = torch.empty(cols, device=DEV)
    _l.check(ops.lib().xpa_colsum_finalize(ops._p(part), G, cols, ops._p(db), ops._stream(DEV)), "finalize")
    if act == 0:
        rdz = dh
    elif act == 1:
        rdz = torch.where(y > 0, dh, dh * slope)
    else:
        rdz = dh * (1 - y * y)
    if act == 1:
        torch.testing.assert_close(dz, rdz, rtol=0, atol=0)
    elif act == 2:   # dh * (1 - h^2): fp-contraction differs from torch's by an ulp
        torch.testing.assert_close(dz, rdz, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(db.double(), rdz.double().sum(0), rtol=1e-5, atol=1e-4)


def _c3_policy(K=6, seed=0):
    from xuanpolicy_amd.policies import AC_CNN_Atari, Categorical_AC_Policy

    class _Disc:
        n, shape = K, ()
    torch.manual_seed(seed)
    rep = AC_CNN_Atari((84, 84, 4), [8, 4, 3], [4, 2, 1], [32, 64, 64], None, torch.nn.init.orthogonal_,
                       torch.nn.ReLU, DEV, [512])
    return Categorical_AC_Policy(_Disc(), rep, [], [], None, torch.nn.init.orthogonal_, torch.nn.ReLU, DEV)


@pytest.mark.parametrize("B", [96, 257])
def test_fused_cnn_matches_autograd(B, conv_path):
    """FusedCNNActorCritic forward (logits, v) and every parameter gradient for given d logits / d v == autograd
    through the reference-layout modules (AC_CNN_Atari: uint8 / 255, NCHW convs with bias, ReLU, Flatten in
    (C, H, W) order, fc, heads)."""
    from xuanpolicy_amd.fused_cnn import FusedCNNActorCritic
    pol = _c3_policy()
    # non-trivial biases so the bias paths are exercised
    with torch.no_grad():
        for n, p in pol.named_parameters():
            if n.endswith("bias"):
                p.normal_(0, 0.1)
    g = torch.Generator(device="cpu").manual_seed(B)
    x = torch.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=torch.int32).to(torch.uint8).to(DEV)
    d_head = (torch.randn(B, 6, generator=g) / B).to(DEV)
    d_v = (torch.randn(B, generator=g) / B).to(DEV)
    # explicit path
    fc = FusedCNNActorCritic(pol)
    for p in pol.parameters():
        p.grad = torch.full_like(p, float("nan"))   # every gradient must be overwritten
    h2, _, v2, ctx = fc.forward(x)
    (hs, _, flat, fouts), s_state, _, _ = ctx
    # float64 CPU reference through the reference-layout modules (NCHW convs with bias, Flatten in (C, H, W)
    # order).  Its ReLUs take their masks from the explicit path's own activations: a unit within an ulp of the
    # kink may flip between two f32 paths (different conv algorithms), which would move that unit's whole
    # gradient contribution — the arithmetic under test is the backward, not the kink's side.
    import copy
    pol64 = copy.deepcopy(pol).to("cpu").double()
    masks = [(y > 0).permute(0, 3, 1, 2).cpu().double() for y in hs[1:]] + [(f > 0).cpu().double() for f in fouts]
    h = (x.cpu().double() / 255.0).permute(0, 3, 1, 2)
    relu_plain = h.new_zeros(())
    k = 0
    for mod in pol64.representation.model:
        if isinstance(mod, torch.nn.ReLU):
            plain = torch.relu(h)
            relu_plain = torch.maximum(relu_plain, (plain - h * masks[k]).abs().max().detach())
            h = h * masks[k]
            k += 1
        else:
            h = mod(h)
    l64, v64 = pol64.actor.model(h), pol64.critic(h)
    torch.testing.assert_close(h2.cpu().double(), l64.detach(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(v2.cpu().double(), v64.detach(), rtol=1e-4, atol=1e-5)
    assert float(relu_plain) < 1e-5   # the borrowed masks differ from f64's own only at near-zero units
    pol64.zero_grad()
    torch.autograd.backward([l64, v64], [d_head.cpu().double(), d_v.cpu().double()])
    ref = {n: p.grad.detach() for n, p in pol64.named_parameters()}
    fc.backward(ctx, d_head, d_v)
    bad = []
    for n, p in pol.named_parameters():
        scale = float(ref[n].abs().max()) + 1e-12
        err = float((p.grad.cpu().double() - ref[n]).abs().max())
        if not err <= 2e-5 * scale + 1e-8:
            bad.append((n, err, scale))
    assert not bad, bad


@pytest.mark.parametrize("B,HW,C", [(5, 100, 64), (2048, 100, 64), (3, 7, 32)])
def test_global_maxpool_and_backward_match_torch(B, HW, C):
    """K23 == torch's AdaptiveMaxPool2d((1, 1)) values and indices (first maximum wins: ties planted, incl. all-zero
    ReLU channels), K24 == its backward routed through the ReLU, with the bias column sums."""
    _l, ops = _lib()
    g = torch.Generator(device="cpu").manual_seed(B + HW)
    h = torch.relu(torch.randn(B, HW, C, generator=g))
    h[:, :, 0] = 0.0                                 # dead channel: every position ties at 0
    h[:, HW // 2, 1] = h[:, 0, 1] = 5.0              # a tie between two positions: the first must win
    hd = h.to(DEV)
    out = torch.empty(B, C, device=DEV)
    am = torch.empty(B, C, dtype=torch.int32, device=DEV)
    _l.check(ops.lib().xpa_global_maxpool(ops._p(hd), B, HW, C, ops._p(out), ops._p(am), ops._stream(DEV)), "maxpool")
    x = hd.permute(0, 2, 1).reshape(B, C, HW, 1)     # NCHW view of the NHWC data, W = 1
    ref, ridx = torch.nn.functional.adaptive_max_pool2d(x, (1, 1), return_indices=True)
    torch.testing.assert_close(out, ref.view(B, C), rtol=0, atol=0)
    assert torch.equal(am.long(), ridx.view(B, C))
    dout = torch.randn(B, C, generator=g).to(DEV)
    G = int(ops.lib().xpa_act_bwd_bias_num_partials(B * HW, C))
    part = torch.empty(G, C, device=DEV)
    dz = torch.empty(B, HW, C, device=DEV)
    _l.check(ops.lib().xpa_maxpool_act_bwd_bias(1, ops._p(dout), ops._p(am), ops._p(hd), B, HW, C, 0.0, ops._p(dz),
                                                ops._p(part), None, ops._stream(DEV)), "maxpool_bwd")
    db = torch.empty(C, device=DEV)
    _l.check(ops.lib().xpa_colsum_finalize(ops._p(part), G, C, ops._p(db), ops._stream(DEV)), "finalize")
    xr = x.clone().requires_grad_(True)
    torch.autograd.backward(torch.nn.functional.adaptive_max_pool2d(xr, (1, 1)), dout.view(B, C, 1, 1))
    rdz = (xr.grad.view(B, C, HW).permute(0, 2, 1) * (hd > 0)).contiguous()
    torch.testing.assert_close(dz, rdz, rtol=0, atol=0)
    torch.testing.assert_close(db.double(), rdz.double().sum((0, 1)), rtol=1e-5, atol=1e-5)   # f32 block sums


@pytest.mark.parametrize("B", [64, 300])
def test_fused_qnetwork_matches_autograd(B):
    """FusedQNetwork (Basic_CNN + Q head, C5): evalQ, targetQ and every eval-parameter gradient for a given d evalQ ==
    float64 autograd through the reference-layout modules (ReLU masks and max-pool positions borrowed from the f32
    path, as in test_fused_cnn_matches_autograd)."""
    import copy
    from xuanpolicy_amd.fused_cnn import FusedQNetwork
    from xuanpolicy_amd.policies import Basic_CNN, BasicQnetwork

    class _Disc:
        n, shape = 18, ()
    torch.manual_seed(B)
    rep = Basic_CNN((84, 84, 4), [8, 4, 3], [4, 2, 1], [32, 64, 64], None, torch.nn.init.orthogonal_, torch.nn.ReLU,
                    DEV)
    pol = BasicQnetwork(_Disc(), rep, [512], None, torch.nn.init.orthogonal_, torch.nn.ReLU, DEV)
    with torch.no_grad():
        for n, p in pol.named_parameters():
            if n.endswith("bias"):
                p.normal_(0, 0.1)
    pol.copy_target()
    g = torch.Generator(device="cpu").manual_seed(B)
    x = torch.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=torch.int32).to(torch.uint8).to(DEV)
    dq = (torch.randn(B, 18, generator=g) / B).to(DEV)
    fq = FusedQNetwork(pol)
    q, ctx = fq.forward(x)
    tq = fq.target(x)
    torch.testing.assert_close(tq, q, rtol=1e-6, atol=1e-6)   # target = deep copy of eval at construction
    (hs, am, _, _), s, outs = ctx
    pol64 = copy.deepcopy(pol).to("cpu").double()
    masks = [(y > 0).permute(0, 3, 1, 2).cpu().double() for y in hs[1:]]
    h = (x.cpu().double() / 255.0).permute(0, 3, 1, 2)
    k = 0
    for mod in pol64.representation.model:
        if isinstance(mod, torch.nn.ReLU):
            h = h * masks[k]
            k += 1
        elif isinstance(mod, torch.nn.AdaptiveMaxPool2d):
            Bc, Cc = h.shape[0], h.shape[1]
            h = torch.gather(h.reshape(Bc, Cc, -1), 2, am.cpu().long().view(Bc, Cc, 1)).view(Bc, Cc, 1, 1)
        else:
            h = mod(h)
    q64 = pol64.eval_Qhead(h)
    torch.testing.assert_close(q.cpu().double(), q64.detach(), rtol=1e-4, atol=1e-5)
    torch.autograd.backward(q64, dq.cpu().double())
    fq.backward(ctx, dq)
    bad = []
    for (n, p), (n64, p64) in zip(pol.named_parameters(), pol64.named_parameters()):
        if n.startswith("target"):
            continue
        scale = float(p64.grad.abs().max()) + 1e-12
        err = float((p.grad.cpu().double() - p64.grad).abs().max())
        if not err <= 2e-5 * scale + 1e-8:
            bad.append((n, err, scale))
    assert not bad, bad


@pytest.fixture(params=[1, 0], ids=["k25b", "k25"])
def conv1_form(request):
    """r05: the conv1 forward on the bf16 matrix cores (K25B, the default) and on fp32 MFMA (K25)."""
    _l, ops = _lib()
    L = ops.lib()
    prev = L.xpa_conv1_form(-1)
    L.xpa_conv1_form((prev & ~1) | request.param)
    yield request.param
    L.xpa_conv1_form(prev)


@pytest.mark.parametrize("B,act,slope,H,s,p", [(3, 1, 0.0, 84, 4, 2), (17, 0, 0.0, 84, 4, 2), (64, 1, 0.01, 84, 4, 2),
                                             (5, 2, 0.0, 84, 4, 2), (4, 1, 0.0, 85, 3, 1), (3, 0, 0.0, 86, 4, 1),
                                             (1, 0, 0.0, 84, 4, 2), (2, 1, 0.0, 83, 4, 2)])
def test_conv1_u8_matches_conv2d(B, act, slope, H, s, p, conv1_form):
    """K25 (the first conv block straight from uint8 frames on fp32 MFMA) == conv2d(K20 frames) + bias + act within
    fp32 summation-order rounding, at the AC_CNN_Atari / Basic_CNN shape (84 x 84 x 4, 8 x 8 stride 4 pad 2 -> 32)."""
    _l, ops = _lib()
    g = torch.Generator(device="cpu").manual_seed(B)
    OH = (H + 2 * p - 8) // s + 1   # 84 / 4 / 2: the 8-B pixel-pair form; odd width / stride / pad: the dword form
    x = torch.randint(0, 256, (B, H, H, 4), generator=g, dtype=torch.int32).to(torch.uint8).to(DEV)
    w = (torch.randn(32, 4, 8, 8, generator=g) * 0.05).to(DEV)
    b = (torch.randn(32, generator=g) * 0.1).to(DEV)
    y = torch.full((B, OH, OH, 32), float("nan"), device=DEV)
    _l.check(ops.lib().xpa_conv1_u8_fwd(act, ops._p(x), B, H, H, 4, 8, s, p, ops._p(w), ops._p(b), 32, slope,
                                        ops._p(y), ops._stream(DEV)), "conv1_u8")
    xf = x.double() / 255.0
    z = torch.nn.functional.conv2d(xf.permute(0, 3, 1, 2), w.double(), b.double(), s, p).permute(0, 2, 3, 1)
    ref = {0: z, 1: torch.nn.functional.leaky_relu(z, slope), 2: torch.tanh(z)}[act]
    torch.testing.assert_close(y.double(), ref, rtol=1e-5, atol=2e-5)


def test_conv1_u8_scale_within_one_rounding(conv1_form):
    """K25 scales by 1/255 on the weight side (sum x (w / 255)): with one-hot weights (output n reads tap
    (c, ky, kx) = (n % 4, 2 + n // 8, 2 + n % 8 // 4 * 3) with weight 1) every output is x * float32(1 / 255), within
    one f32 rounding of the reference's float32(x / 255.0) (K20), for all 256 byte values.  K25B (bf16 matrix cores,
    w / 255 split three ways): within one ulp of x * float32(1 / 255)."""
    _l, ops = _lib()
    B = 8
    x = (torch.arange(B * 84 * 84 * 4, dtype=torch.int64) * 2654435761 % 256).to(torch.uint8).reshape(B, 84, 84, 4)
    x = x.to(DEV)
    w = torch.zeros(32, 4, 8, 8)
    taps = [(n % 4, 2 + n // 8, 2 + (n % 8) // 4 * 3) for n in range(32)]
    for n, (c, ky, kx) in enumerate(taps):
        w[n, c, ky, kx] = 1.0
    w, b = w.to(DEV), torch.zeros(32, device=DEV)
    y = torch.empty((B, 21, 21, 32), device=DEV)
    _l.check(ops.lib().xpa_conv1_u8_fwd(0, ops._p(x), B, 84, 84, 4, 8, 4, 2, ops._p(w), ops._p(b), 32, 0.0, ops._p(y),
                                        ops._stream(DEV)), "conv1_u8")
    f = torch.empty((B, 84, 84, 4), device=DEV)
    _l.check(ops.lib().xpa_frames_to_f32(ops._p(x), x.numel(), ops._p(f), ops._stream(DEV)), "frames")
    yc, fc, xc = y.cpu(), f.cpu(), x.cpu()
    for n, (c, ky, kx) in enumerate(taps):
        iy = torch.arange(21) * 4 - 2 + ky   # taps chosen inside the frame for every output position
        ix = torch.arange(21) * 4 - 2 + kx
        xs = xc[:, iy][:, :, ix][..., c].float()
        ref = xs * torch.tensor(1.0 / 255.0, dtype=torch.float32)
        if conv1_form == 0:
            assert torch.equal(yc[..., n], ref), n
            torch.testing.assert_close(yc[..., n], fc[:, iy][:, :, ix][..., c], rtol=1.2e-7, atol=0)
        else:   # K25B: x lo + x mid is exact, the add of x hi rounds in the bf16 MFMA's accumulator (not RNE on
            # every input): within one ulp of the correctly rounded product
            ulp = (yc[..., n].view(torch.int32) - ref.view(torch.int32)).abs().max().item()
            assert ulp <= 1, (n, ulp)
            torch.testing.assert_close(yc[..., n], fc[:, iy][:, :, ix][..., c], rtol=2.4e-7, atol=0)
    assert len(torch.unique(xc)) == 256


def test_conv1_u8_bf16_form_error_vs_fp32_form():
    """K25B against K25 at the C3 update's row count scale (B = 1024 frames): both within f32 summation-order
    rounding of the f64 conv, and K25B's error no larger than 2x K25's (the split keeps every term to one rounding)."""
    _l, ops = _lib()
    L = ops.lib()
    B = 1024
    g = torch.Generator(device="cpu").manual_seed(11)
    x = torch.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=torch.int32).to(torch.uint8).to(DEV)
    w = (torch.randn(32, 4, 8, 8, generator=g) * 0.05).to(DEV)
    b = (torch.randn(32, generator=g) * 0.1).to(DEV)
    prev = L.xpa_conv1_form(-1)
    ys = []
    try:
        for form in (1, 0):
            L.xpa_conv1_form((prev & ~1) | form)
            y = torch.full((B, 21, 21, 32), float("nan"), device=DEV)
            _l.check(L.xpa_conv1_u8_fwd(0, ops._p(x), B, 84, 84, 4, 8, 4, 2, ops._p(w), ops._p(b), 32, 0.0, ops._p(y),
                                        ops._stream(DEV)), "conv1_u8")
            ys.append(y.double())
    finally:
        L.xpa_conv1_form(prev)
    ref = torch.nn.functional.conv2d((x.double() / 255.0).permute(0, 3, 1, 2), w.double(), b.double(), 4,
                                     2).permute(0, 2, 3, 1)
    e_b, e_f = (ys[0] - ref).abs().max().item(), (ys[1] - ref).abs().max().item()
    assert e_b <= 2 * e_f + 1e-7, (e_b, e_f)
    assert e_b <= 1e-5


@pytest.fixture(params=[4, 0], ids=["k27b", "k27"])
def dgrad_form(request):
    """r05: the conv2 data gradient on the bf16 matrix cores (K27B, the default) and on fp32 MFMA (K27)."""
    _l, ops = _lib()
    L = ops.lib()
    prev = L.xpa_conv1_form(-1)
    L.xpa_conv1_form((prev & ~4) | request.param)
    yield request.param
    L.xpa_conv1_form(prev)


@pytest.mark.parametrize("B,H,k,s,p", [(7, 21, 4, 2, 1), (64, 21, 4, 2, 1), (3, 20, 4, 2, 0), (5, 19, 4, 2, 3),
                                       (2, 9, 2, 1, 0), (4, 11, 2, 1, 1), (1, 21, 4, 2, 1)])
def test_conv_dgrad_s2k_matches_conv2d_input(B, H, k, s, p, dgrad_form):
    """K27 (data gradient of a 2s x 2s stride-s conv, 32 -> 64 channels, one implicit GEMM per residue class) ==
    torch.nn.grad.conv2d_input in float64, odd / even sizes, padding 0 .. 3 and stride 1 included."""
    _l, ops = _lib()
    g = torch.Generator(device="cpu").manual_seed(B * 100 + H)
    OH = (H + 2 * p - k) // s + 1
    dy = torch.randn(B, OH, OH, 64, generator=g).to(DEV)
    w = (torch.randn(64, 32, k, k, generator=g) * 0.1).to(DEV)
    dx = torch.full((B, H, H, 32), float("nan"), device=DEV)
    _l.check(ops.lib().xpa_conv_dgrad_s2k(ops._p(dy), B, OH, OH, 64, ops._p(w), 32, k, s, p, H, H, ops._p(dx),
                                          ops._stream(DEV)), "dgrad")
    ref = torch.nn.grad.conv2d_input((B, 32, H, H), w.double(), dy.double().permute(0, 3, 1, 2), s, p)
    torch.testing.assert_close(dx.double(), ref.permute(0, 2, 3, 1), rtol=1e-5, atol=1e-5)


@pytest.fixture(params=[2, 0], ids=["k26b", "k26"])
def conv1_wform(request):
    """r05: the conv1 weight gradient on the bf16 matrix cores (K26B, the default) and on fp32 MFMA (K26)."""
    _l, ops = _lib()
    L = ops.lib()
    prev = L.xpa_conv1_form(-1)
    L.xpa_conv1_form((prev & ~2) | request.param)
    yield request.param
    L.xpa_conv1_form(prev)


@pytest.mark.parametrize("B,H,s,p", [(1, 84, 4, 2), (6, 84, 4, 2), (33, 84, 4, 2), (5, 85, 3, 1), (2, 83, 4, 2)])
def test_conv1_u8_wgrad_matches_conv2d_weight(B, H, s, p, conv1_wform):
    """K26 partials + the f64 column-sum finalize == torch.nn.grad.conv2d_weight on (x / 255) in float64 (odd row
    counts: the last row pair half empty)."""
    _l, ops = _lib()
    L, st = ops.lib(), ops._stream(DEV)
    g = torch.Generator(device="cpu").manual_seed(7 * B)
    OH = (H + 2 * p - 8) // s + 1   # 84 / 4 / 2: the 8-B pixel-pair form; 85 / 3 / 1: the dword form
    x = torch.randint(0, 256, (B, H, H, 4), generator=g, dtype=torch.int32).to(torch.uint8).to(DEV)
    dz = torch.randn(B, OH, OH, 32, generator=g).to(DEV)
    part = torch.full((int(L.xpa_conv1_u8_wgrad_num_partials()), 8192), float("nan"), device=DEV)
    _l.check(L.xpa_conv1_u8_wgrad(ops._p(dz), ops._p(x), B, H, H, 4, 8, s, p, 32, ops._p(part), st), "wgrad")
    dw = torch.empty(32, 4, 8, 8, device=DEV)
    _l.check(L.xpa_colsum_finalize(ops._p(part), part.shape[0], 8192, ops._p(dw), st), "finalize")
    ref = torch.nn.grad.conv2d_weight((x.double() / 255.0).permute(0, 3, 1, 2), (32, 4, 8, 8),
                                      dz.double().permute(0, 3, 1, 2), s, p)
    torch.testing.assert_close(dw.double(), ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("act,slope", [(1, 0.0), (1, 0.01), (2, 0.0), (0, 0.0)])
def test_conv1_u8_wgrad_act_matches_k22_then_k26(act, slope, conv1_wform):
    """xpa_conv1_u8_wgrad_act (K26 with the activation backward + bias gradient folded in) == K22 on the conv's output
    then K26: the same weight gradient (bitwise: the same dz values in the same order) and the bias gradient within
    f32 summation-order rounding."""
    _l, ops = _lib()
    L, st = ops.lib(), ops._stream(DEV)
    B = 9
    g = torch.Generator(device="cpu").manual_seed(act * 10 + int(slope * 100))
    x = torch.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=torch.int32).to(torch.uint8).to(DEV)
    y = torch.randn(B, 21, 21, 32, generator=g).to(DEV)
    y = torch.tanh(y) if act == 2 else (torch.relu(y) if act == 1 and slope == 0 else y)
    dh = torch.randn(B, 21, 21, 32, generator=g).to(DEV)
    G = int(L.xpa_conv1_u8_wgrad_num_partials())
    pw, pb = torch.empty(G, 8192, device=DEV), torch.empty(G, 32, device=DEV)
    _l.check(L.xpa_conv1_u8_wgrad_act(act, ops._p(dh), ops._p(y), slope, ops._p(x), B, 84, 84, 4, 8, 4, 2, 32,
                                      ops._p(pw), ops._p(pb), st), "wgrad_act")
    dw, db = torch.empty(8192, device=DEV), torch.empty(32, device=DEV)
    _l.check(L.xpa_colsum_finalize(ops._p(pw), G, 8192, ops._p(dw), st), "f")
    _l.check(L.xpa_colsum_finalize(ops._p(pb), G, 32, ops._p(db), st), "f")
    dz = dh.clone()
    rows = B * 441
    kp = torch.empty(int(L.xpa_act_bwd_bias_num_partials(rows, 32)), 32, device=DEV)
    _l.check(L.xpa_act_bwd_bias(act, ops._p(dz), ops._p(y), rows, 32, slope, ops._p(dz), ops._p(kp), st), "k22")
    db_ref = torch.empty(32, device=DEV)
    _l.check(L.xpa_colsum_finalize(ops._p(kp), kp.shape[0], 32, ops._p(db_ref), st), "f")
    pw2 = torch.empty_like(pw)
    _l.check(L.xpa_conv1_u8_wgrad(ops._p(dz), ops._p(x), B, 84, 84, 4, 8, 4, 2, 32, ops._p(pw2), st), "wgrad")
    dw_ref = torch.empty(8192, device=DEV)
    _l.check(L.xpa_colsum_finalize(ops._p(pw2), G, 8192, ops._p(dw_ref), st), "f")
    assert torch.equal(dw, dw_ref)
    torch.testing.assert_close(db, db_ref, rtol=1e-5, atol=1e-4)


def test_conv1_u8_wgrad_bf16_form_error_vs_fp32_form():
    """K26B against K26 at B = 1024 frames (451 584 rows): both against the f64 weight gradient, K26B's error no larger
    than 2x K26's (dz split three ways, the frames exact: every product exact in f32)."""
    _l, ops = _lib()
    L, st = ops.lib(), ops._stream(DEV)
    B = 1024
    g = torch.Generator(device="cpu").manual_seed(12)
    x = torch.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=torch.int32).to(torch.uint8).to(DEV)
    dz = torch.randn(B, 21, 21, 32, generator=g).to(DEV)
    G = int(L.xpa_conv1_u8_wgrad_num_partials())
    prev = L.xpa_conv1_form(-1)
    outs = []
    try:
        for form in (2, 0):
            L.xpa_conv1_form((prev & ~2) | form)
            part = torch.full((G, 8192), float("nan"), device=DEV)
            _l.check(L.xpa_conv1_u8_wgrad(ops._p(dz), ops._p(x), B, 84, 84, 4, 8, 4, 2, 32, ops._p(part), st), "wgrad")
            dw = torch.empty(32, 4, 8, 8, device=DEV)
            _l.check(L.xpa_colsum_finalize(ops._p(part), G, 8192, ops._p(dw), st), "finalize")
            outs.append(dw.double())
    finally:
        L.xpa_conv1_form(prev)
    ref = torch.nn.grad.conv2d_weight((x.double() / 255.0).permute(0, 3, 1, 2), (32, 4, 8, 8),
                                      dz.double().permute(0, 3, 1, 2), 4, 2)
    e_b, e_f = (outs[0] - ref).abs().max().item(), (outs[1] - ref).abs().max().item()
    assert e_b <= 2 * e_f + 1e-9, (e_b, e_f)
    assert e_b <= 1e-5 * ref.abs().max().item() + 1e-4


def test_conv_dgrad_s2k_bf16_form_error_vs_fp32_form():
    """K27B against K27 at B = 2048 (the C3 conv2 shape): both against the f64 data gradient, K27B's error no larger
    than 2x K27's (the six-product split: f32-GEMM accuracy)."""
    _l, ops = _lib()
    L = ops.lib()
    B = 2048
    g = torch.Generator(device="cpu").manual_seed(13)
    dy = torch.randn(B, 10, 10, 64, generator=g).to(DEV)
    w = (torch.randn(64, 32, 4, 4, generator=g) * 0.1).to(DEV)
    prev = L.xpa_conv1_form(-1)
    outs = []
    try:
        for form in (4, 0):
            L.xpa_conv1_form((prev & ~4) | form)
            dx = torch.full((B, 21, 21, 32), float("nan"), device=DEV)
            _l.check(L.xpa_conv_dgrad_s2k(ops._p(dy), B, 10, 10, 64, ops._p(w), 32, 4, 2, 1, 21, 21, ops._p(dx),
                                          ops._stream(DEV)), "dgrad")
            outs.append(dx.double())
    finally:
        L.xpa_conv1_form(prev)
    ref = torch.nn.grad.conv2d_input((B, 32, 21, 21), w.double(), dy.double().permute(0, 3, 1, 2), 2, 1)
    ref = ref.permute(0, 2, 3, 1)
    e_b, e_f = (outs[0] - ref).abs().max().item(), (outs[1] - ref).abs().max().item()
    assert e_b <= 2 * e_f + 1e-9, (e_b, e_f)
    assert e_b <= 1e-5


def test_fc_act_fused_backward_equals_k22_path(monkeypatch):
    """r05: the fc data gradient with the last conv block's activation backward + bias partials in its epilogue
    (xpa_s3_gemm_group_act) against the K40G data gradient + K22: every gradient bit for bit except that block's bias
    (the same values summed in another order: f32 rounding)."""
    from xuanpolicy_amd import fused_cnn
    from xuanpolicy_amd.fused_cnn import FusedCNNActorCritic
    monkeypatch.setattr(fused_cnn._Trunk, "igemm_min_rows", 0)
    monkeypatch.setattr(fused_cnn._Trunk, "fc_split_min_rows", 0)
    B = 300
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=torch.int32).to(torch.uint8).to(DEV)
    d_head = (torch.randn(B, 6, generator=g) / B).to(DEV)
    d_v = (torch.randn(B, generator=g) / B).to(DEV)
    grads = []
    for fuse in (True, False):
        monkeypatch.setattr(fused_cnn._Trunk, "fc_fuse_act", fuse)
        pol = _c3_policy()
        with torch.no_grad():
            for n, p in pol.named_parameters():
                if n.endswith("bias"):
                    p.normal_(0, 0.1, generator=torch.Generator(device=p.device).manual_seed(len(n)))
        fc = FusedCNNActorCritic(pol)
        for p in pol.parameters():
            p.grad = torch.full_like(p, float("nan"))
        assert fc.trunk_._fc_fuse_ok(B) == fuse
        _, _, _, ctx = fc.forward(x)
        fc.backward(ctx, d_head, d_v)
        torch.cuda.synchronize()
        grads.append({n: p.grad.clone() for n, p in pol.named_parameters()})
        last = [n for n, p in pol.named_parameters() if p is fc.trunk_.convs[-1][0].bias]
    assert len(last) == 1
    for n in grads[0]:
        a, b = grads[0][n], grads[1][n]
        assert torch.isfinite(a).all(), n
        if n == last[0]:
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6 * float(b.abs().max()) + 1e-9, msg=n)
        else:
            assert torch.equal(a, b), n
