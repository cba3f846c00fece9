"""GPU: the wide representation layer on the split GEMMs (r05; C4's Linear(376, 256) + LeakyReLU, csrc/sgemm3.hip,
csrc/rollout.hip, csrc/mlp.hip).

  * the pitched gather writes the minibatch rows into a zero-padded [B, 384] buffer (pad untouched, the advantage
    moments equal to K4's);
  * K40F (the split GEMM with bias + activation + the sign bits in its epilogue) against an f64 product of the same f32
    operands, within the f32 GEMM's error, and its sign bits equal to its own output's signs;
  * K42W (dX GEMM + act' from sign bits -> dz1, db1 partials) and K42C's dz form against f64;
  * the finalize's output map (K41V's padded dW^T slices straight into W [256, 376]) against the f64 slice sum, with
    the clip-norm partial over exactly the kept entries."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _sign_k42(h):
    """K42S's h_sign layout: byte b bit j = h[row, 32 j + b] > 0."""
    rows = h.shape[0]
    bits = (h > 0).view(rows, 8, 32).to(torch.int32)
    sign = (bits << torch.arange(8, device=DEV, dtype=torch.int32).view(1, 8, 1)).sum(1).to(torch.uint8)
    return sign.contiguous().view(torch.int32).view(rows, 8)


def _words(m):
    a = m.cpu().numpy().reshape(m.shape[0], 8, 32).astype(np.uint64)
    w = (a << np.arange(32, dtype=np.uint64)).sum(-1).astype(np.uint32)
    return torch.from_numpy(w.view(np.int32).copy()).to(DEV)


@pytest.mark.parametrize("B,n_rows,d", [(65536, 70000, 376), (777, 5000, 376), (64, 100, 100)])
def test_gather_pitched(B, n_rows, d):
    from xuanpolicy_amd import ops
    g = torch.Generator(device=DEV).manual_seed(B + d)
    obs = torch.randn(n_rows, d, device=DEV, generator=g)
    adv = torch.randn(n_rows, device=DEV, generator=g)
    idx = torch.randint(0, n_rows, (B,), device=DEV, generator=g)
    kp = (d + 15) // 16 * 16
    out = torch.zeros(B, kp, device=DEV)
    part = torch.empty(ops.gather_num_partials(B), 2, dtype=torch.float64, device=DEV)
    ops.gather_minibatch_pitched(idx, obs, out, adv=adv, adv_partials=part)
    ref, ref_part = ops.gather_minibatch(idx, obs, adv=adv)
    torch.cuda.synchronize()
    assert torch.equal(out[:, :d], ref)
    assert torch.equal(out[:, d:], torch.zeros_like(out[:, d:]))
    assert torch.equal(part, ref_part)


@pytest.mark.parametrize("M,d,act", [(65536, 376, 1), (4133, 376, 1), (300, 376, 0), (77, 100, 2), (1000, 64, 1)])
def test_gemm_bias_act_matches_f64(M, d, act):
    """K40F on the zero-padded rows and W^T's padded split: h = act(x W^T + b) within the f32 GEMM's error bound
    (4e-6 of sum |x_k w_k| per element), sign bits = its own output's signs."""
    from xuanpolicy_amd import ops
    g = torch.Generator(device=DEV).manual_seed(M + d + act)
    kp = (d + 15) // 16 * 16
    x = torch.randn(M, d, device=DEV, generator=g) * torch.exp(torch.randn(M, 1, device=DEV, generator=g))
    xp = torch.zeros(M, kp, device=DEV)
    xp[:, :d] = x
    w = torch.randn(256, d, device=DEV, generator=g) / d ** 0.5
    b = torch.randn(256, device=DEV, generator=g) * 0.1
    slope = 0.01
    ws = ops.s3_split_padded(w.t(), kp)
    sign = torch.full((M, 8), -1, dtype=torch.int32, device=DEV) if act != 2 else None
    h = ops.s3_gemm_bias_act(xp, ws, kp, b, act, slope, sign=sign)
    torch.cuda.synchronize()
    z = x.double() @ w.double().t() + b.double()
    bound = 4e-6 * (x.double().abs() @ w.double().abs().t()) + 1e-30
    if act == 1:
        ref = torch.where(z > 0, z, z * slope)
        bound = torch.where(z > 0, bound, bound * slope) + 1e-9 * bound
    elif act == 2:
        ref = torch.tanh(z)
        bound = bound + 1e-6
    else:
        ref = z
    err = (h.double() - ref).abs()
    assert torch.isfinite(h).all()
    assert bool((err <= bound).all()), (err / bound).max().item()
    if sign is not None:
        assert torch.equal(sign, _sign_k42(h))


@pytest.mark.parametrize("rows,crit", [(65536, False), (65536, True), (4133, True), (300, False), (77, True)])
def test_trunk_bwd_dz_matches_f64(rows, crit):
    """K42W: dz1 = (dz Wh_pair) act'(h) and db1 partials; with crit, K42C's factored critic half in the k loop."""
    from xuanpolicy_amd import ops
    g = torch.Generator(device=DEV).manual_seed(rows + (7 if crit else 0))
    H = 256
    dz = torch.randn(rows, 2 * H, device=DEV, generator=g) * 1e-3
    wa = torch.randn(H, 256, device=DEV, generator=g) / 16
    whc = torch.randn(H, 256, device=DEV, generator=g) / 16
    wc = torch.randn(H, device=DEV, generator=g) / 16
    slope_c, slope = 0.01, 0.01
    pre = torch.randn(rows, 256, device=DEV, generator=g)
    sign = _sign_k42(pre)
    pair = torch.cat([wa, whc], 0)
    buf = torch.empty(int(ops.lib().xpa_s3_split_bytes(2 * H, 256)), dtype=torch.uint8, device=DEV)
    G = int(ops.lib().xpa_s3_gemm_trunk_bwd_num_partials(rows))
    dz1 = torch.full((rows, 256), 555.0, device=DEV)
    pdb = torch.full((G, 256), 555.0, device=DEV)
    d = lambda t: t.double()   # noqa: E731
    if crit:
        m = torch.rand(rows, H, device=DEV, generator=g) > 0.45
        dv = torch.randn(rows, device=DEV, generator=g) * 1e-3
        cs = torch.empty(256, device=DEV)
        ops.s3_split_batch([(pair, buf)], scales=[(wc, 1.0 - slope_c, H)], cs=(cs, slope_c))
        ops.s3_gemm_trunk_bwd_dz(dz[:, :H], buf, 2 * H, sign, 1, slope, dz1, pdb,
                                 crit=(H, H, _words(m), dv, cs))
        dz_c = d(dv)[:, None] * d(wc)[None, :] * torch.where(m, 1.0, slope_c).double()
        gg = d(dz[:, :H]) @ d(wa) + dz_c @ d(whc)
    else:
        ops.s3_split_batch([(pair, buf)])
        ops.s3_gemm_trunk_bwd_dz(dz, buf, 2 * H, sign, 1, slope, dz1, pdb)
        gg = d(dz) @ d(pair)
    torch.cuda.synchronize()
    ref = gg * torch.where(pre > 0, 1.0, slope).double()
    scale = ref.abs().max().item()
    assert (d(dz1) - ref).abs().max().item() <= 2e-5 * scale
    ref_db = ref.sum(0)
    assert (d(pdb).sum(0) - ref_db).abs().max().item() <= 2e-5 * ref_db.abs().max().item() + 1e-5 * scale


@pytest.mark.parametrize("S,kp,d", [(85, 384, 376), (64, 128, 100), (3, 256, 256), (300, 128, 124)])
def test_finalize_output_map(S, kp, d):
    """Partials [S, kp * 256] (column r * 256 + i = row r of x^T dz, output unit i) finalized into W [256, d]
    (W[i, r] = the f64 slice sum, rows r >= d dropped) — and the clip-norm total over exactly W's entries."""
    from xuanpolicy_amd import ops
    g = torch.Generator(device=DEV).manual_seed(S + kp + d)
    part = torch.randn(S, kp, 256, device=DEV, generator=g)
    w = torch.full((256, d), 123.0, device=DEV)
    other = torch.randn(S, 300, device=DEV, generator=g)
    o2 = torch.empty(300, device=DEV)
    q = ops.ColsumQueue()
    q.add(part.view(S, -1), w, tmap=(256, d, d))
    q.add(other, o2)
    sq = torch.zeros(4096, dtype=torch.float64, device=DEV)
    total, written = q.flush(DEV, sq=sq)
    torch.cuda.synchronize()
    ref = part.double().sum(0)[:d].t()
    assert written == 256 * d + 300
    assert torch.isfinite(total).all()
    # f64 sums in the finalize's fixed order, rounded once to f32: within an f32 rounding of the f64 reference
    assert ((w.double() - ref).abs() <= 1e-6 * ref.abs() + 1e-6).all()
    assert ((o2.double() - other.double().sum(0)).abs() <= 1e-6 * other.double().sum(0).abs() + 1e-6).all()
    want = (w.double() ** 2).sum() + (o2.double() ** 2).sum()
    assert abs(total.item() - want.item()) <= 1e-9 * want.item()


@pytest.mark.parametrize("M,n_rows,d", [(65536, 70000, 376), (777, 5000, 376), (300, 400, 100)])
def test_row_index_forms_equal_gathered(M, n_rows, d):
    """r05: K40F and K41V reading the minibatch rows through idx from a buffer with zeroed slack equal their forms on
    the gathered, zero-padded rows bit for bit (K41V: the rows below the layer width, the rest is dropped)."""
    from xuanpolicy_amd import ops
    g = torch.Generator(device=DEV).manual_seed(M + d + 1)
    kp, mp = (d + 15) // 16 * 16, (d + 127) // 128 * 128
    store = torch.zeros(n_rows * d + 128, device=DEV)
    flat = store[:n_rows * d].view(n_rows, d)
    flat.copy_(torch.randn(n_rows, d, device=DEV, generator=g))
    idx = torch.randint(0, n_rows, (M,), device=DEV, generator=g)
    xp = torch.zeros(M, mp, device=DEV)
    xp[:, :d] = flat[idx]
    w = torch.randn(256, d, device=DEV, generator=g) / d ** 0.5
    b = torch.randn(256, device=DEV, generator=g) * 0.1
    ws = ops.s3_split_padded(w.t(), kp)
    s1, s2 = torch.empty((M, 8), dtype=torch.int32, device=DEV), torch.empty((M, 8), dtype=torch.int32, device=DEV)
    h1 = ops.s3_gemm_bias_act(flat, ws, kp, b, 1, 0.01, sign=s1, ridx=idx)
    h2 = ops.s3_gemm_bias_act(xp[:, :kp].contiguous(), ws, kp, b, 1, 0.01, sign=s2)
    dz = torch.randn(M, 256, device=DEV, generator=g)
    S = max(1, 256 // (mp // 128))
    p1 = ops.s3_wgrad(flat, dz, slices=S, aidx=idx, m=mp)
    p2 = ops.s3_wgrad(xp, dz, slices=S)
    torch.cuda.synchronize()
    assert torch.equal(h1, h2) and torch.equal(s1, s2)
    assert torch.equal(p1[:, :d], p2[:, :d])


@pytest.mark.parametrize("d", [376, 100])
def test_row_index_form_ignores_the_next_rows_values(d):
    """r06: K40F's row-index form reads a row's padded columns d .. kp - 1 from the NEXT buffer row; those
    columns are zeroed before the split, so a non-finite value there (inf / nan in the next observation) leaves this row's
    outputs equal to the gathered form's — only the row that holds it goes non-finite, as in the reference."""
    from xuanpolicy_amd import ops
    g = torch.Generator(device=DEV).manual_seed(d)
    n_rows, M = 600, 512
    kp = (d + 15) // 16 * 16
    store = torch.zeros(n_rows * d + 128, device=DEV)
    flat = store[:n_rows * d].view(n_rows, d)
    flat.copy_(torch.randn(n_rows, d, device=DEV, generator=g))
    flat[101, :16] = float("inf")     # the row after row 100
    flat[201, :16] = float("nan")     # the row after row 200
    idx = torch.randint(0, n_rows, (M,), device=DEV, generator=g)
    idx[0], idx[1], idx[2] = 100, 200, 101
    xp = torch.zeros(M, kp, device=DEV)
    xp[:, :d] = flat[idx]
    w = torch.randn(256, d, device=DEV, generator=g) / d ** 0.5
    b = torch.randn(256, device=DEV, generator=g) * 0.1
    ws = ops.s3_split_padded(w.t(), kp)
    h1 = ops.s3_gemm_bias_act(flat, ws, kp, b, 1, 0.01, ridx=idx)
    h2 = ops.s3_gemm_bias_act(xp, ws, kp, b, 1, 0.01)
    torch.cuda.synchronize()
    ok = (idx != 101) & (idx != 201)   # the rows that hold the inf / nan themselves go non-finite in both forms
    assert torch.isfinite(h1[ok]).all(), "a row's outputs picked up the next row's non-finite values"
    assert torch.equal(h1[ok], h2[ok])
    assert not torch.isfinite(h1[2]).all()   # the row that holds the inf is non-finite, as in the gathered form
