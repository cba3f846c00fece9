"""GPU: K40, the f32 GEMM on the bf16 matrix cores by a three-way operand split (csrc/sgemm3.hip).

The split must be exact (hi + mid + lo == x for every f32 operand element), and the GEMM must carry the f32 GEMM's
own error: against an f64 product of the same f32 operands, K40's max abs error stays within 2x (+ a 2^-24-relative
floor) of torch's f32 GEMM on the same device (hipBLASLt on the f32 matrix cores), on operands whose magnitudes
span ~8 decades (exp of a normal), so every split plane is exercised."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _wide(shape, g, scale=1.0):
    return (torch.randn(shape, device=DEV, generator=g) * torch.exp(2 * torch.randn(shape, device=DEV, generator=g))
            * scale)


def _planes(split, k):
    """Decode xpa_s3_split_b's layout back to three [k, 256] f64 planes (for the exactness check)."""
    raw = split.view(torch.int16).cpu().numpy().astype(np.uint16).astype(np.uint32) << 16
    v = raw.view(np.float32).astype(np.float64).reshape(k // 16, 3, 8, 2, 32, 8)
    out = np.zeros((3, k, 256))
    for h in range(2):
        for j in range(8):
            kk = 4 * h + j + (4 if j >= 4 else 0)
            for cb in range(8):
                out[:, kk::16, cb * 32:(cb + 1) * 32] = v[:, :, cb, h, :, j].transpose(1, 0, 2)
    return out


@pytest.mark.parametrize("k,transposed", [(512, False), (256, True), (16, False)])
def test_split_is_exact(k, transposed):
    from xuanpolicy_amd import ops
    g = torch.Generator(device=DEV).manual_seed(k)
    src = _wide((256, k) if transposed else (k, 256), g)
    b = src.t() if transposed else src
    sp = ops.s3_split(b)
    torch.cuda.synchronize()
    pl = _planes(sp, k)
    want = b.double().cpu().numpy()
    assert np.array_equal(pl.sum(0), want)
    # each plane is the round-to-nearest bf16 of what the previous ones leave
    hi = b.to(torch.bfloat16).double().cpu().numpy()
    assert np.array_equal(pl[0], hi)


@pytest.mark.parametrize("form", [0, 8])
@pytest.mark.parametrize("m,k,lda_pad,t_b", [(65536, 512, 0, False), (1000, 512, 0, False), (4097, 256, 8, True),
                                             (300, 256, 0, True), (1, 16, 0, False), (257, 32, 4, False)])
def test_gemm_matches_f32_gemm_error(m, k, lda_pad, t_b, form):
    """form 0: one 8-wave block per CU, 3-stage ring; form 8: two 4-wave blocks per CU, 2 stages (xpa_s3_probe)."""
    from xuanpolicy_amd import ops
    L = ops.lib()
    assert L.xpa_s3_probe(form) == 0
    try:
        _gemm_case(m, k, lda_pad, t_b)
    finally:
        L.xpa_s3_probe(0)


def _gemm_case(m, k, lda_pad, t_b):
    from xuanpolicy_amd import ops
    g = torch.Generator(device=DEV).manual_seed(m + k)
    abuf = _wide((m, k + lda_pad), g)
    a = abuf[:, :k]
    w = torch.randn(256, k, device=DEV, generator=g) / 16 if t_b else torch.randn(k, 256, device=DEV, generator=g) / 16
    b = w.t() if t_b else w
    out = torch.full((m, 256), float("nan"), device=DEV)
    ops.s3_gemm(a, ops.s3_split(b), k, out=out)
    native = torch.mm(a, b)
    torch.cuda.synchronize()
    ref = a.double() @ b.double()
    scale = ref.abs().max().item()
    err = (out.double() - ref).abs().max().item()
    err_f32 = (native.double() - ref).abs().max().item()
    assert torch.isfinite(out).all()
    assert err <= 2 * err_f32 + 2 ** -24 * scale, (err, err_f32, scale)
    # rms error: no systematic bias from the dropped terms
    rms = (out.double() - ref).pow(2).mean().sqrt().item()
    rms_f32 = (native.double() - ref).pow(2).mean().sqrt().item()
    assert rms <= 2 * rms_f32 + 1e-30


def test_gemm_rejects_bad_shapes():
    from xuanpolicy_amd import _lib, ops
    a = torch.randn(64, 24, device=DEV)
    with pytest.raises(_lib.XpaError):
        ops.s3_split(torch.randn(24, 256, device=DEV))          # k % 16
    with pytest.raises(_lib.XpaError):
        ops.s3_split(torch.randn(32, 128, device=DEV))          # n != 256
    sp = ops.s3_split(torch.randn(32, 256, device=DEV))
    with pytest.raises(_lib.XpaError):
        ops.s3_gemm(a, sp, 24)
    torch.cuda.synchronize()


@pytest.mark.parametrize("form", [0, 32])
@pytest.mark.parametrize("rows,m,lda_pad,slices", [(65536, 512, 0, None), (65536, 256, 0, None), (4133, 512, 8, None),
                                                   (100, 128, 0, 1), (1000, 256, 4, 7), (33, 128, 0, 2), (77, 128, 3, 2)])
def test_wgrad_matches_f32_gemm_error(rows, m, lda_pad, slices, form):
    """K41V (form 0, production) / the register-staged K41 (32): the slices' sum of dz^T x against an f64 product,
    within the f32 GEMM's own error (torch's dz^T x on the device); ragged slices (rows not a multiple of the slice count
    or of 32), strided rows, and an odd row stride (lda = m + 3: K41V's float4 staging does not apply, K41 runs)."""
    from xuanpolicy_amd import ops
    L = ops.lib()
    g = torch.Generator(device=DEV).manual_seed(rows + m)
    a = _wide((rows, m + lda_pad), g)[:, :m]
    b = torch.randn(rows, 256, device=DEV, generator=g)
    assert L.xpa_s3_probe(form) == 0
    try:
        part = ops.s3_wgrad(a, b, slices=slices)
        torch.cuda.synchronize()
    finally:
        L.xpa_s3_probe(0)
    S = part.shape[0]
    assert S == (slices or ops.s3_wgrad_slices(rows, m))
    got = part.double().sum(0)
    native = torch.mm(a.t(), b)
    torch.cuda.synchronize()
    ref = a.double().t() @ b.double()
    scale = ref.abs().max().item()
    err = (got - ref).abs().max().item()
    err_f32 = (native.double() - ref).abs().max().item()
    assert torch.isfinite(part).all()
    assert err <= 2 * err_f32 + 2 ** -24 * scale, (err, err_f32, scale)


@pytest.mark.parametrize("rows,m,slices", [(65536, 512, None), (4133, 256, 5), (100, 128, 1)])
def test_wgrad_wave_specialised_equals_k41(rows, m, slices):
    """K41W (producer / consumer waves, xpa_s3_probe form bit 8) writes the register-staged K41's partials (bit 32) bit
    for bit: the same LDS image, products and k order per accumulator."""
    from xuanpolicy_amd import ops
    L = ops.lib()
    g = torch.Generator(device=DEV).manual_seed(rows * 3 + m)
    a = _wide((rows, m), g)
    b = torch.randn(rows, 256, device=DEV, generator=g)
    try:
        assert L.xpa_s3_probe(32) == 0
        p0 = ops.s3_wgrad(a, b, slices=slices)
        assert L.xpa_s3_probe(8) == 0
        p1 = ops.s3_wgrad(a, b, slices=slices)
        torch.cuda.synchronize()
    finally:
        L.xpa_s3_probe(0)
    assert torch.equal(p0, p1)


@pytest.mark.parametrize("m,k", [(65536, 512), (4133, 256), (100, 32)])
def test_gemm_wave_specialised_equals_k40(m, k):
    """K40W (producer / consumer waves, form bit 16), K40's two-block form (bit 8), its 64 x 128 wave tile (bit 32) and
    its ping-pong k loop (bit 256, r05) write K40's output bit for bit:
    the same split, the same six products in the same order per accumulator, the same k order."""
    from xuanpolicy_amd import ops
    L = ops.lib()
    g = torch.Generator(device=DEV).manual_seed(m + 7 * k)
    a = _wide((m, k), g)
    sp = ops.s3_split(torch.randn(k, 256, device=DEV, generator=g) / 16)
    ref = ops.s3_gemm(a, sp, k)
    try:
        for form in (8, 16, 32, 256):
            assert L.xpa_s3_probe(form) == 0
            out = ops.s3_gemm(a, sp, k)
            torch.cuda.synchronize()
            assert torch.equal(out, ref), form
    finally:
        L.xpa_s3_probe(0)


@pytest.mark.parametrize("m,in_f,out_f", [(16384, 6400, 512), (777, 512, 256), (3, 544, 256)])
def test_gemm_group_equals_k40(m, in_f, out_f):
    """K40G (r05): one launch of the fc layer's problems — forward k halves x 256-column blocks and data-gradient
    column blocks (the last aligned to the end, overlapping its neighbour) — each output equal to its own K40 launch
    bit for bit; the overlapped columns come out identical from both blocks."""
    from xuanpolicy_amd import ops
    g = torch.Generator(device=DEV).manual_seed(m + in_f)
    x = _wide((m, in_f), g)
    w = torch.randn(out_f, in_f, device=DEV, generator=g) / 16
    kh = in_f // 2
    part = torch.full((2, m, out_f), float("nan"), device=DEV)
    fwd = []
    for j in range(out_f // 256):
        for p in range(2):
            fwd.append((x[:, p * kh:(p + 1) * kh], ops.s3_split(w[j * 256:(j + 1) * 256, p * kh:(p + 1) * kh].t()),
                        part[p, :, j * 256:(j + 1) * 256]))
    ops.s3_gemm_group(fwd, kh)
    for a, b, c in fwd:
        assert torch.equal(c, ops.s3_gemm(a, b, kh))
    gz = _wide((m, out_f), g)
    dx = torch.full((m, in_f), float("nan"), device=DEV)
    c0s = [min(c, in_f - 256) for c in range(0, in_f, 256)]
    dgr = [(gz, ops.s3_split(w[:, c0:c0 + 256]), dx[:, c0:c0 + 256]) for c0 in c0s]
    ops.s3_gemm_group(dgr, out_f)
    ref = gz.double() @ w.double()
    for (a, b, _), c0 in zip(dgr, c0s):
        assert torch.equal(dx[:, c0:c0 + 256], ops.s3_gemm(a, b, out_f))
    bound = 4e-6 * (gz.double().abs() @ w.double().abs()) + 1e-6
    assert bool(((dx.double() - ref).abs() <= bound).all())


@pytest.mark.parametrize("rows,m,lda_pad,slices", [(65536, 512, 0, None), (4133, 256, 8, 5), (100, 128, 0, 1),
                                                   (33, 128, 4, 2)])
def test_wgrad_vector_staged_matches_f32_gemm_error(rows, m, lda_pad, slices):
    """K41V (form bit 16: float4 staging, k-major planes read back with ds_read_b64_tr_b16): the slices' sum within
    the f32 GEMM's own error against an f64 product, like K41 (a different k order inside a step, so not K41's bits)."""
    from xuanpolicy_amd import ops
    L = ops.lib()
    g = torch.Generator(device=DEV).manual_seed(rows + 5 * m)
    a = _wide((rows, m + lda_pad), g)[:, :m]
    b = torch.randn(rows, 256, device=DEV, generator=g)
    assert L.xpa_s3_probe(16) == 0
    try:
        part = ops.s3_wgrad(a, b, slices=slices)
        torch.cuda.synchronize()
    finally:
        L.xpa_s3_probe(0)
    got = part.double().sum(0)
    native = torch.mm(a.t(), b)
    ref = a.double().t() @ b.double()
    scale = ref.abs().max().item()
    assert torch.isfinite(part).all()
    err = (got - ref).abs().max().item()
    err_f32 = (native.double() - ref).abs().max().item()
    assert err <= 2 * err_f32 + 2 ** -24 * scale, (err, err_f32, scale)


@pytest.mark.parametrize("rows,m,lda_pad,slices", [(65536, 512, 0, None), (4133, 256, 8, 5), (33, 128, 4, 2)])
def test_wgrad_interleaved_schedule_equals_k41v(rows, m, lda_pad, slices):
    """K41V's interleaved schedule (the default: the next stage's split placed between the MFMA blocks, the last
    chunks' staging unconditional) writes the partials of hipcc's own schedule (xpa_s3_probe bit 64) bit for bit: the
    same products per accumulator in the same order; so does the ping-pong form (bit 256, r05)."""
    from xuanpolicy_amd import ops
    L = ops.lib()
    g = torch.Generator(device=DEV).manual_seed(rows + 11 * m)
    a = _wide((rows, m + lda_pad), g)[:, :m]
    b = torch.randn(rows, 256, device=DEV, generator=g)
    ref = ops.s3_wgrad(a, b, slices=slices)
    for form in (64, 256):   # 256: the ping-pong form (r05)
        try:
            assert L.xpa_s3_probe(form) == 0
            got = ops.s3_wgrad(a, b, slices=slices)
            torch.cuda.synchronize()
        finally:
            L.xpa_s3_probe(0)
        assert torch.equal(ref, got), form


def test_split_batch_equals_single_splits():
    """xpa_s3_split_batch (the update's one split launch: Wh_pair, Wh_actor^T, Wh_critic^T) == xpa_s3_split_b each."""
    from xuanpolicy_amd import ops
    g = torch.Generator(device=DEV).manual_seed(3)
    mats = [torch.randn(512, 256, device=DEV, generator=g), torch.randn(256, 256, device=DEV, generator=g).t(),
            _wide((256, 256), g).t(), torch.randn(32, 256, device=DEV, generator=g)]
    outs = [torch.empty(int(ops.lib().xpa_s3_split_bytes(m.shape[0], 256)), dtype=torch.uint8, device=DEV)
            for m in mats]
    ops.s3_split_batch(list(zip(mats, outs)))
    torch.cuda.synchronize()
    for m, o in zip(mats, outs):
        assert torch.equal(o, ops.s3_split(m))


@pytest.mark.parametrize("rows,din,act", [(65536, 17, 1), (4133, 17, 2), (300, 5, 0), (77, 32, 1)])
def test_gemm_trunk_bwd_matches_f64(rows, din, act):
    """K42 (the dX GEMM with the first layer's backward in its epilogue) against an f64 restatement of K40 + K13's
    backward: g = dz W, dz1 = g act'(h) (LeakyReLU 0.01 / tanh / identity on the layer's output h), dW1 = dz1^T x,
    db1 = sum dz1 — the partial rows summed, within 2e-5 of the output scale (f32 GEMM + f32 partial sums)."""
    from xuanpolicy_amd import ops
    g = torch.Generator(device=DEV).manual_seed(rows + din)
    K = 512
    dz = torch.randn(rows, K, device=DEV, generator=g) * 1e-3
    w = torch.randn(K, 256, device=DEV, generator=g) / 16
    x = torch.randn(rows, din, device=DEV, generator=g)
    pre = torch.randn(rows, 256, device=DEV, generator=g)
    slope = 0.01
    h = {0: pre, 1: torch.nn.functional.leaky_relu(pre, slope), 2: torch.tanh(pre)}[act]
    h = h.clone()
    h[::7, ::5] = 0.0   # exact zeros: the LeakyReLU branch h > 0 is false there
    pdw, pdb = ops.s3_gemm_trunk_bwd(dz, ops.s3_split(w), K, h, x, act, slope)
    torch.cuda.synchronize()
    d = lambda t: t.double()   # noqa: E731
    gg = d(dz) @ d(w)
    gp = {0: lambda hh: torch.ones_like(hh), 1: lambda hh: torch.where(hh > 0, 1.0, slope),
          2: lambda hh: 1.0 - hh * hh}[act](d(h))
    dz1 = gg * gp
    ref_dw = (dz1.t() @ d(x)).reshape(-1)
    ref_db = dz1.sum(0)
    got_dw, got_db = pdw.double().sum(0), pdb.double().sum(0)
    assert torch.isfinite(pdw).all() and torch.isfinite(pdb).all()
    for got, ref, what in ((got_dw, ref_dw, "dW1"), (got_db, ref_db, "db1")):
        scale = ref.abs().max().item()
        err = (got - ref).abs().max().item()
        assert err <= 2e-5 * scale, (what, err, scale)


@pytest.mark.parametrize("act,slope,channels,m", [(1, 0.0, 64, 16384), (1, 0.01, 32, 777), (2, 0.0, 64, 300),
                                                  (0, 0.0, 32, 5)])
def test_gemm_group_act_equals_group_then_k22(act, slope, channels, m):
    """xpa_s3_gemm_group_act (r05): the stored values equal K40G's output passed through K22 (xpa_act_bwd_bias) bit
    for bit, and its per-channel bias partials sum (f64 finalize) to K22's bias gradient within f32 order rounding."""
    from xuanpolicy_amd import _lib, ops
    L, st = ops.lib(), ops._stream(DEV)
    g = torch.Generator(device=DEV).manual_seed(m + 3 * act)
    in_f, out_f = 1024, 512
    gz = _wide((m, out_f), g, 1e-2)
    w = torch.randn(out_f, in_f, device=DEV, generator=g) / 16
    y = torch.randn(m, in_f, device=DEV, generator=g)
    y = torch.tanh(y) if act == 2 else (torch.where(y > 0, y, y * slope) if act == 1 else y)
    c0s = list(range(0, in_f, 256))
    planes = [ops.s3_split(w[:, c0:c0 + 256]) for c0 in c0s]
    dz = torch.full((m, in_f), float("nan"), device=DEV)
    G = int(L.xpa_s3_gemm_group_act_num_partials(len(c0s), m))
    part = torch.full((G, channels), float("nan"), device=DEV)
    ops.s3_gemm_group_act([(gz, p, dz[:, c0:c0 + 256]) for p, c0 in zip(planes, c0s)], out_f,
                          [y[:, c0:c0 + 256] for c0 in c0s], act, slope, channels, part)
    db = torch.empty(channels, device=DEV)
    _lib.check(L.xpa_colsum_finalize(ops._p(part), G, channels, ops._p(db), st), "finalize")
    dx = torch.full((m, in_f), float("nan"), device=DEV)
    ops.s3_gemm_group([(gz, p, dx[:, c0:c0 + 256]) for p, c0 in zip(planes, c0s)], out_f)
    rows = m * in_f // channels
    kp = torch.empty(int(L.xpa_act_bwd_bias_num_partials(rows, channels)), channels, device=DEV)
    _lib.check(L.xpa_act_bwd_bias(act, ops._p(dx), ops._p(y), rows, channels, slope, ops._p(dx), ops._p(kp), st), "k22")
    db_ref = torch.empty(channels, device=DEV)
    _lib.check(L.xpa_colsum_finalize(ops._p(kp), kp.shape[0], channels, ops._p(db_ref), st), "finalize")
    torch.cuda.synchronize()
    assert torch.equal(dz, dx)
    torch.testing.assert_close(db, db_ref, rtol=1e-5, atol=1e-5 * float(dx.abs().sum(0).max()) + 1e-9)


@pytest.mark.parametrize("rows,width", [(16384, 3136), (2051, 3136), (300, 100)])
def test_wgrad_padded_rows_match_f32_gemm_error(rows, width):
    """r06, xpa_s3_wgrad_padded (a fc weight gradient whose input width is not a multiple of 128, e.g. the Nature CNN's 3136, read as 128-row tiles): the kept output
    rows (< width) of the slices' sum against f64 within the f32 GEMM's error; the rows past the width read the next row
    (or the slack after the last row, here filled with NaN: it may reach only the dropped rows)."""
    from xuanpolicy_amd import ops
    g = torch.Generator(device=DEV).manual_seed(rows + width)
    m = (width + 127) // 128 * 128
    buf = torch.full((rows * width + (m - width),), float("nan"), device=DEV)
    a = buf[:rows * width].view(rows, width)
    a.copy_(_wide((rows, width), g))
    b = torch.randn(rows, 2 * 256, device=DEV, generator=g)[:, 256:]   # a column half of g [rows, 512] (ld 512)
    part = ops.s3_wgrad(a, b, m=m)
    torch.cuda.synchronize()
    got = part.double().sum(0)[:width]
    ref = a.double().t() @ b.double()
    native = torch.mm(a.t(), b)
    scale = ref.abs().max().item()
    err = (got - ref).abs().max().item()
    err_f32 = (native.double() - ref).abs().max().item()
    assert torch.isfinite(part[:, :width]).all()
    assert err <= 2 * err_f32 + 2 ** -24 * scale, (err, err_f32, scale)
    with pytest.raises(ValueError):   # no slack after the last row
        ops.s3_wgrad(a.clone(), b, m=m)


def test_fc_weight_gradient_split_matches_library(monkeypatch):
    """r06: the C3 trunk's first fc weight gradient on K41V (fused_cnn._fc0_wgrad_split, at the update's B = 16384 and
    the production AC_CNN_Atari) against the hipBLASLt f32 GEMM it replaces, both against f64: within 2x its error."""
    from xuanpolicy_amd import fused_cnn
    from xuanpolicy_amd.policies import AC_CNN_Atari, Categorical_AC_Policy

    class _Disc:
        n, shape = 6, ()
    torch.manual_seed(0)
    rep = AC_CNN_Atari((84, 84, 4), [8, 4, 3], [4, 2, 1], [32, 64, 64], None, torch.nn.init.orthogonal_, torch.nn.ReLU,
                       DEV, [512])
    pol = Categorical_AC_Policy(_Disc(), rep, [], [], None, torch.nn.init.orthogonal_, torch.nn.ReLU, DEV)
    fc = fused_cnn.FusedCNNActorCritic(pol)
    tr = fc.trunk_
    B = 16384
    x = torch.randint(0, 256, (B, 84, 84, 4), dtype=torch.int32, device=DEV).to(torch.uint8)
    s, ctx = tr.forward(x)
    hs, am, flat, fouts = ctx
    assert tr._fc_wsplit_rows(B)
    g = torch.randn(B, 512, device=DEV) * 1e-3
    tr._dw_tmp = torch.empty_like(tr.fc[0][0].weight)
    assert tr._fc0_wgrad_split(g, flat)
    got = tr._dw_tmp.double().clone()
    native = torch.mm(g.t(), flat)
    torch.cuda.synchronize()
    ref = g.double().t() @ flat.double()
    scale = ref.abs().max().item()
    err = (got - ref).abs().max().item()
    err_f32 = (native.double() - ref).abs().max().item()
    assert err <= 2 * err_f32 + 2 ** -24 * scale, (err, err_f32, scale)
