"""CPU model of the three-way bf16 split that K40 / K41 / K16S / K16P run on the bf16 matrix cores (csrc/s3_split.h).

The device claims rest on two facts checked here in numpy / torch-CPU arithmetic:
  * the split is exact: x = hi + mid + lo for f32 x, each part the round-to-nearest bf16 of what the earlier ones leave;
  * the six kept products (hi.hi, hi.mid, mid.hi, mid.mid, hi.lo, lo.hi), each exact in f32 and accumulated into one f32
    running sum once per 16-k group (the v_mfma_f32_32x32x16_bf16 step), give an error against the f64 product no larger
    than the f32 MFMA order (one f32 rounding per 2-k group, v_mfma_f32_32x32x2_f32) up to a small factor."""
import numpy as np
import torch


def _bf16(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(torch.bfloat16).float().numpy()


def _split3(x):
    hi = _bf16(x)
    r1 = (x - hi).astype(np.float32)
    mid = _bf16(r1)
    r2 = (r1 - mid).astype(np.float32)
    return hi, mid, _bf16(r2)


def _acc(parts_a, parts_b, group):
    """f32 running sum rounded once per `group` k of each product (the product terms summed exactly, in f64)."""
    M, K = parts_a[0].shape
    N = parts_b[0].shape[1]
    c = np.zeros((M, N), np.float32)
    for k0 in range(0, K, group):
        for a, b in zip(parts_a, parts_b):
            c = (c.astype(np.float64) + a[:, k0:k0 + group].astype(np.float64) @ b[k0:k0 + group].astype(np.float64)
                 ).astype(np.float32)
    return c


def test_split_is_exact_over_the_f32_range():
    """Exact for every finite |x| below bf16's largest finite value (3.39e38; above it hi rounds to inf) down to
    ~2^-100 (below, lo falls into bf16's subnormals and drops bits below 2^-24 of x)."""
    rng = np.random.default_rng(0)
    x = (rng.standard_normal(200000) * np.exp(rng.uniform(-60, 60, 200000))).astype(np.float32)
    x = np.concatenate([x, np.float32([0.0, -0.0, 1.0, 3.38e38, -3.3e38, 1e-30, 2.0 ** -100])])
    hi, mid, lo = _split3(x)
    assert np.array_equal(hi.astype(np.float64) + mid + lo, x.astype(np.float64))
    assert np.array_equal(hi, _bf16(x))


def test_six_products_carry_the_f32_gemm_error():
    rng = np.random.default_rng(1)
    M, K, N = 96, 512, 64
    A = (rng.standard_normal((M, K)) * np.exp(rng.standard_normal((M, K)))).astype(np.float32)
    B = (rng.standard_normal((K, N)) / 16).astype(np.float32)
    ref = A.astype(np.float64) @ B.astype(np.float64)
    ah, am, al = _split3(A)
    bh, bm, bl = _split3(B)
    # the device order: smallest terms first into the one accumulator (s3_split.h xpa_mfma_s3)
    emu = _acc([am, ah, al, ah, am, ah], [bm, bl, bh, bm, bh, bh], 16)
    f32 = _acc([A], [B], 2)
    scale = np.abs(ref).max()
    e_emu, e_f32 = np.abs(emu - ref).max() / scale, np.abs(f32 - ref).max() / scale
    assert e_emu <= 2 * e_f32 + 2.0 ** -24, (e_emu, e_f32)
    # dropping the mid / lo cross terms (two-way split, 3 products) is NOT f32-accurate: the third plane is needed
    two = _acc([ah, ah, am], [bh, bm, bh], 16)
    assert np.abs(two - ref).max() / scale > 10 * e_f32
