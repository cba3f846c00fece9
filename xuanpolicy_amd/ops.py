"""Torch-tensor front end of the C ABI (include/xuanpolicy_amd.h).

Every op validates device/dtype/shape/contiguity on the host (a wrong shape never reaches a kernel),
passes raw device pointers plus torch's current hipStream_t, and raises XpaError on any failure.
There is no CPU path: tensors must live on a ROCm device.
"""
import ctypes

import torch

from . import _lib

ALGO = {"ppo": 0, "a2c": 1}
DIST = {"gaussian": 0, "categorical": 1}
N_OUT = 6
OUT_KEYS = ("actor-loss", "critic-loss", "entropy", "loss", "clip_ratio", "predict_value")


def lib():
    return _lib.load()


class KernelTimer:
    """Optional per-launch HIP-event timing of the hot kernels on the stream they are launched on
    (bench.py's live roofline).  Disabled by default: no events in the hot loop."""

    def __init__(self):
        self.enabled = False
        self.only = None          # optional set of names to time (others pass through untimed)
        self.events = {}
        self.hip_pairs = {}
        # GPU spin (clock cycles) queued before the start event, so the kernel is already enqueued when
        # the start event completes and the host launch latency is not counted as kernel time.
        self.pad_cycles = {}

    def _on(self, name):
        return self.enabled and (self.only is None or name in self.only)

    def start(self, name):
        if not self._on(name):
            return None
        pad = self.pad_cycles.get(name, 0)
        if pad:
            torch.cuda._sleep(pad)
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        return e0

    def stop(self, name, e0):
        if e0 is None:
            return
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        self.events.setdefault(name, []).append((e0, e1))

    # ---- dispatch-attached events (hipExtLaunchKernel): the kernel's own start / end ---------------
    _rt = None

    @classmethod
    def _hip(cls):
        if cls._rt is None:
            rt = ctypes.CDLL("libamdhip64.so.7")   # the HIP runtime torch already loaded (same SONAME)
            rt.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
            rt.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
            rt.hipEventSynchronize.argtypes = [ctypes.c_void_p]
            rt.hipEventDestroy.argtypes = [ctypes.c_void_p]
            cls._rt = rt
        return cls._rt

    def kernel_events(self, name):
        """(start, stop) hipEvent_t handles for a launch whose kernel records them itself, or None when
        timing is off."""
        if not self._on(name):
            return None
        rt = self._hip()
        pair = []
        for _ in range(2):
            ev = ctypes.c_void_p()
            if rt.hipEventCreate(ctypes.byref(ev)) != 0:
                raise RuntimeError("hipEventCreate failed")
            pair.append(ev)
        self.hip_pairs.setdefault(name, []).append(tuple(pair))
        return pair

    def reset(self):
        self.events = {}
        rt = self._rt
        for pairs in getattr(self, "hip_pairs", {}).values():
            for a, b in pairs:
                rt.hipEventDestroy(a)
                rt.hipEventDestroy(b)
        self.hip_pairs = {}

    def mean_ms(self, name):
        pairs = getattr(self, "hip_pairs", {}).get(name, [])
        if pairs:
            rt = self._hip()
            tot = 0.0
            for a, b in pairs:
                rt.hipEventSynchronize(b)
                ms = ctypes.c_float()
                if rt.hipEventElapsedTime(ctypes.byref(ms), a, b) != 0:
                    raise RuntimeError("hipEventElapsedTime failed")
                tot += ms.value
            return tot / len(pairs)
        ev = self.events.get(name, [])
        if not ev:
            return None
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in ev) / len(ev)

    def count(self, name):
        return len(getattr(self, "hip_pairs", {}).get(name, [])) or len(self.events.get(name, []))


TIMER = KernelTimer()


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _req(t, name, dtype, shape=None, contiguous=True):
    if not isinstance(t, torch.Tensor):
        raise TypeError("%s must be a torch.Tensor" % name)
    if t.device.type != "cuda":
        raise ValueError("%s must be on a ROCm device (got %s); xuanpolicy_amd has no CPU path" % (name, t.device))
    if t.dtype != dtype:
        raise TypeError("%s must be %s (got %s)" % (name, dtype, t.dtype))
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError("%s must have shape %s (got %s)" % (name, tuple(shape), tuple(t.shape)))
    if contiguous and not t.is_contiguous():
        raise ValueError("%s must be contiguous" % name)
    return t


def _row_stride(t, name, cols):
    """2-D float tensor whose rows may be strided (e.g. a column block of a wider matrix)."""
    if t.dim() != 2 or t.stride(1) != 1 or t.shape[1] != cols or t.stride(0) < cols:
        raise ValueError("%s must be 2-D [n, %d] with unit column stride" % (name, cols))
    return t.stride(0)


# ------------------------------------------------------------------------------------------------
def s3_split(b, out=None):
    """K40: the three bf16 planes of the f32 GEMM operand b [k, 256] (any strides; e.g. W.t() for x W^T), in the
    layout xpa_s3_gemm reads.  Returns a uint8 device tensor of xpa_s3_split_bytes(k, 256) bytes."""
    _req(b, "b", torch.float32, contiguous=False)
    k, n = b.shape
    nbytes = int(lib().xpa_s3_split_bytes(k, n))
    if out is None:
        out = torch.empty(nbytes, dtype=torch.uint8, device=b.device)
    _req(out, "out", torch.uint8, (nbytes,))
    _lib.check(lib().xpa_s3_split_b(_p(b), k, n, b.stride(0), b.stride(1), _p(out), _stream(b.device)),
               "xpa_s3_split_b")
    return out


_SPLIT_PLANS = {}


def s3_split_batch(pairs, scales=None, cs=None):
    """K40's split of up to 4 matrices in one launch: pairs = [(b [k, 256] any strides, out uint8 buffer), ...].
    scales (r05, K42C): per pair None or (w f32 [k - start], a, start): rows k >= start scaled by a * w[k - start]
    before the split; cs = (out f32 [256], slope): out[j] = slope * sum_c w[c] b[start + c, j] of the first scaled
    pair."""
    if scales is not None or cs is not None:
        return _s3_split_batch_scaled(pairs, scales, cs)
    L = lib()
    key = tuple((b.data_ptr(), b.shape[0], b.stride(0), b.stride(1), o.data_ptr()) for b, o in pairs)
    plan = _SPLIT_PLANS.get(key)
    if plan is None:
        for b, o in pairs:
            _req(b, "b", torch.float32, contiguous=False)
            if b.shape[1] != 256:
                raise ValueError("s3_split_batch: b must be [k, 256]")
            _req(o, "out", torch.uint8, (int(L.xpa_s3_split_bytes(b.shape[0], 256)),))
        n = len(pairs)
        arrs = ((ctypes.c_void_p * n)(*[k[0] for k in key]), (ctypes.c_int64 * n)(*[k[1] for k in key]),
                (ctypes.c_int64 * n)(*[k[2] for k in key]), (ctypes.c_int64 * n)(*[k[3] for k in key]),
                (ctypes.c_void_p * n)(*[k[4] for k in key]))
        if len(_SPLIT_PLANS) > 256:
            _SPLIT_PLANS.clear()
        plan = _SPLIT_PLANS[key] = (n, arrs, [ctypes.cast(a, ctypes.c_void_p) for a in arrs])
    n, _keep, args = plan
    _lib.check(L.xpa_s3_split_batch(n, *args, _stream(pairs[0][0].device)), "xpa_s3_split_batch")


def _s3_split_batch_scaled(pairs, scales, cs):
    L = lib()
    scales = scales or [None] * len(pairs)
    key = ("scaled",) + tuple((b.data_ptr(), b.shape[0], b.stride(0), b.stride(1), o.data_ptr(),
                               sc[0].data_ptr() if sc else 0, float(sc[1]) if sc else 1.0, int(sc[2]) if sc else 0)
                              for (b, o), sc in zip(pairs, scales)) + ((cs[0].data_ptr(), float(cs[1])) if cs else (0,))
    plan = _SPLIT_PLANS.get(key)
    if plan is None:
        for (b, o), sc in zip(pairs, scales):
            _req(b, "b", torch.float32, contiguous=False)
            if b.shape[1] != 256:
                raise ValueError("s3_split_batch: b must be [k, 256]")
            _req(o, "out", torch.uint8, (int(L.xpa_s3_split_bytes(b.shape[0], 256)),))
            if sc is not None:
                _req(sc[0], "scale", torch.float32, (b.shape[0] - int(sc[2]),))
        if cs is not None:
            _req(cs[0], "cs", torch.float32, (256,))
            if not any(sc is not None for sc in scales):
                raise ValueError("s3_split_batch: cs needs a scaled matrix")
        n = len(pairs)
        rows = [k[:5] for k in key[1:1 + n]]
        arrs = ((ctypes.c_void_p * n)(*[r[0] for r in rows]), (ctypes.c_int64 * n)(*[r[1] for r in rows]),
                (ctypes.c_int64 * n)(*[r[2] for r in rows]), (ctypes.c_int64 * n)(*[r[3] for r in rows]),
                (ctypes.c_void_p * n)(*[r[4] for r in rows]),
                (ctypes.c_void_p * n)(*[sc[0].data_ptr() if sc else None for sc in scales]),
                (ctypes.c_float * n)(*[float(sc[1]) if sc else 1.0 for sc in scales]),
                (ctypes.c_int64 * n)(*[int(sc[2]) if sc else 0 for sc in scales]))
        if len(_SPLIT_PLANS) > 256:
            _SPLIT_PLANS.clear()
        plan = _SPLIT_PLANS[key] = (n, arrs, [ctypes.cast(a, ctypes.c_void_p) for a in arrs])
    n, _keep, args = plan
    _lib.check(L.xpa_s3_split_batch_scaled(n, *args, _p(cs[0]) if cs else None, float(cs[1]) if cs else 0.0,
                                           _stream(pairs[0][0].device)), "xpa_s3_split_batch_scaled")


def s3_gemm_trunk_bwd_crit(dz_a, b_split, k_a, k_c, mask, dv, cs, h_sign, x, act, slope, partial_dw=None,
                           partial_db=None):
    """K42C (r05): K42S with the critic's half of g = dz_pair . Wh_pair factored (csrc/sgemm3.hip): dz_a [rows, k_a]
    (the actor's half), b_split = s3_split_batch of [Wh_a; Wh_c] with the critic rows scaled by (1 - slope_c) wc,
    mask int32 [rows, 8] / dv [rows] from the critic head (fused_heads crit_mask), cs [256] = slope_c wc . Wh_c."""
    L = lib()
    _req(dz_a, "dz_a", torch.float32, contiguous=False)
    ldz = _row_stride(dz_a, "dz_a", k_a)
    rows = dz_a.shape[0]
    d_in = x.shape[1]
    ldx = _row_stride(x, "x", d_in)
    _req(mask, "mask", torch.int32, (rows, 8))
    _req(dv, "dv", torch.float32, (rows,))
    _req(cs, "cs", torch.float32, (256,))
    _req(h_sign, "h_sign", torch.int32, (rows, 8))
    G = int(L.xpa_s3_gemm_trunk_bwd_num_partials(rows))
    if partial_dw is None:
        partial_dw = torch.empty(G, 256 * d_in, dtype=torch.float32, device=dz_a.device)
    if partial_db is None:
        partial_db = torch.empty(G, 256, dtype=torch.float32, device=dz_a.device)
    _req(partial_dw, "partial_dw", torch.float32, (G, 256 * d_in))
    _req(partial_db, "partial_db", torch.float32, (G, 256))
    _lib.check(L.xpa_s3_gemm_trunk_bwd_crit(_p(dz_a), ldz, _p(b_split), k_a, k_c, _p(mask), _p(dv), _p(cs), _p(h_sign),
                                            _p(x), ldx, rows, d_in, int(act), float(slope), _p(partial_dw),
                                            _p(partial_db), _stream(dz_a.device)), "xpa_s3_gemm_trunk_bwd_crit")
    return partial_dw, partial_db


def s3_wgrad_pair_slices(rows):
    """(sa, per_a, sc, per_c) of K41P for `rows`."""
    v = [ctypes.c_int64() for _ in range(4)]
    _lib.check(lib().xpa_s3_wgrad_pair_slices(rows, *[ctypes.byref(x) for x in v]), "xpa_s3_wgrad_pair_slices")
    sa, sc, per_a, per_c = (x.value for x in v)
    return sa, per_a, sc, per_c


def s3_wgrad_pair(dz_a, h, mask, dv, wc, slope, out_a=None, out_c=None):
    """K41P (r05): the paired hidden layer's weight-gradient slices — out_a [sa, 256, 256] of dz_a^T h (six-product
    split) and out_c [sc, 256, 256] of the critic's wc[c] ((1 - slope) m^T Y + slope colsum(Y)), Y = dv (.) h (three
    products: m exact in bf16).  The caller sums the slices (f64, fixed order)."""
    _req(dz_a, "dz_a", torch.float32, contiguous=False)
    _req(h, "h", torch.float32, contiguous=False)
    rows = dz_a.shape[0]
    lda, ldb = _row_stride(dz_a, "dz_a", 256), _row_stride(h, "h", 256)
    if h.shape[0] != rows:
        raise ValueError("dz_a and h must have the same rows")
    _req(mask, "mask", torch.int32, (rows, 8))
    _req(dv, "dv", torch.float32, (rows,))
    _req(wc, "wc", torch.float32, (256,))
    sa, per_a, sc, per_c = s3_wgrad_pair_slices(rows)
    if out_a is None:
        out_a = torch.empty(sa, 256, 256, dtype=torch.float32, device=dz_a.device)
    if out_c is None:
        out_c = torch.empty(sc, 256, 256, dtype=torch.float32, device=dz_a.device)
    _req(out_a, "out_a", torch.float32, (sa, 256, 256))
    _req(out_c, "out_c", torch.float32, (sc, 256, 256))
    _lib.check(lib().xpa_s3_wgrad_pair(_p(dz_a), lda, _p(h), ldb, rows, _p(mask), _p(dv), _p(wc), float(slope), sa,
                                       per_a, sc, per_c, _p(out_a), _p(out_c), _stream(dz_a.device)),
               "xpa_s3_wgrad_pair")
    return out_a, out_c


def s3_gemm(a, b_split, k, out=None):
    """K40: out [m, 256] = a [m, k] . B for B split by s3_split (f32 accuracy on the bf16 matrix cores)."""
    _req(a, "a", torch.float32, contiguous=False)
    lda = _row_stride(a, "a", k)
    m = a.shape[0]
    if out is None:
        out = torch.empty(m, 256, dtype=torch.float32, device=a.device)
    ldc = _row_stride(out, "out", 256)
    if out.shape[0] != m:
        raise ValueError("out must have %d rows" % m)
    _lib.check(lib().xpa_s3_gemm(_p(a), lda, _p(b_split), _p(out), ldc, m, k, 256, _stream(a.device)), "xpa_s3_gemm")
    return out


_GROUP_ARGS = {}


def s3_gemm_group(problems, k):
    """K40G (r05): [(a [m, k] view, b_split, out [m, 256] view), ...] (<= 32, one m / lda / ldc) in one launch; each
    out is s3_gemm(a, b_split, k)'s bit for bit."""
    n = len(problems)
    if not 1 <= n <= 32:
        raise ValueError("1..32 problems")
    a0, _, c0 = problems[0]
    m = a0.shape[0]
    lda, ldc = _row_stride(a0, "a", k), _row_stride(c0, "out", 256)
    key = tuple((a.data_ptr(), b.data_ptr(), c.data_ptr()) for a, b, c in problems) + (lda, ldc, m, k)
    arrs = _GROUP_ARGS.get(key)
    if arrs is None:
        for a, b, c in problems:
            _req(a, "a", torch.float32, contiguous=False)
            _req(c, "out", torch.float32, contiguous=False)
            if a.shape[0] != m or c.shape[0] != m or a.stride(0) != lda or c.stride(0) != ldc or a.shape[1] != k:
                raise ValueError("s3_gemm_group: every problem needs the same m / lda / ldc")
        arrs = ((ctypes.c_void_p * n)(*[a.data_ptr() for a, _, _ in problems]),
                (ctypes.c_void_p * n)(*[b.data_ptr() for _, b, _ in problems]),
                (ctypes.c_void_p * n)(*[c.data_ptr() for _, _, c in problems]))
        if len(_GROUP_ARGS) > 64:
            _GROUP_ARGS.clear()
        _GROUP_ARGS[key] = arrs
    _lib.check(lib().xpa_s3_gemm_group(n, arrs[0], arrs[1], arrs[2], lda, ldc, m, k, _stream(a0.device)),
               "xpa_s3_gemm_group")


def s3_gemm_group_act(problems, k, ys, act, slope, channels, bias_partial):
    """K40G with the previous block's activation backward (r05): problems as s3_gemm_group, ys the previous block's
    output at each out's offsets (same row stride); bias_partial [xpa_s3_gemm_group_act_num_partials, channels]."""
    n = len(problems)
    if not 1 <= n <= 32 or len(ys) != n:
        raise ValueError("1..32 problems, one y each")
    a0, _, c0 = problems[0]
    m = a0.shape[0]
    lda, ldc = _row_stride(a0, "a", k), _row_stride(c0, "out", 256)
    for (a, _, c), y in zip(problems, ys):
        _req(a, "a", torch.float32, contiguous=False)
        _req(c, "out", torch.float32, contiguous=False)
        _req(y, "y", torch.float32, contiguous=False)
        if a.shape[0] != m or c.shape[0] != m or a.stride(0) != lda or c.stride(0) != ldc or a.shape[1] != k or \
                y.shape != c.shape or y.stride() != c.stride():
            raise ValueError("s3_gemm_group_act: one m / lda / ldc, y shaped and strided as out")
    G = int(lib().xpa_s3_gemm_group_act_num_partials(n, m))
    _req(bias_partial, "bias_partial", torch.float32, (G, channels))
    arr = lambda ts: (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])   # noqa: E731
    _lib.check(lib().xpa_s3_gemm_group_act(n, arr([p[0] for p in problems]), arr([p[1] for p in problems]),
                                           arr([p[2] for p in problems]), arr(ys), lda, ldc, m, k, act, float(slope),
                                           channels, _p(bias_partial), _stream(a0.device)), "xpa_s3_gemm_group_act")


def s3_gemm_trunk_bwd(dz, b_split, k, h, x, act, slope, partial_dw=None, partial_db=None, h_sign=None):
    """K42: g = dz [rows, k] . B (split) kept in registers; the first representation layer's backward on it (dz1 =
    g * act'(h), its bias / weight gradients) as per-block partials ([G, 256 * d_in], [G, 256]); g is not stored.
    h_sign (int32 [rows, 8], K16R's sign bits; act 0 / 1): K42S, act' from the bits (h is not read, may be None)."""
    L = lib()
    _req(dz, "dz", torch.float32, contiguous=False)
    ldz = _row_stride(dz, "dz", k)
    rows = dz.shape[0]
    ldh = _row_stride(h, "h", 256) if h_sign is None else 0
    d_in = x.shape[1]
    ldx = _row_stride(x, "x", d_in)
    G = int(L.xpa_s3_gemm_trunk_bwd_num_partials(rows))
    if partial_dw is None:
        partial_dw = torch.empty(G, 256 * d_in, dtype=torch.float32, device=dz.device)
    if partial_db is None:
        partial_db = torch.empty(G, 256, dtype=torch.float32, device=dz.device)
    _req(partial_dw, "partial_dw", torch.float32, (G, 256 * d_in))
    _req(partial_db, "partial_db", torch.float32, (G, 256))
    if h_sign is not None:
        _req(h_sign, "h_sign", torch.int32, (rows, 8))
        _lib.check(L.xpa_s3_gemm_trunk_bwd_sign(_p(dz), ldz, _p(b_split), k, _p(h_sign), _p(x), ldx, rows, d_in,
                                                int(act), float(slope), _p(partial_dw), _p(partial_db),
                                                _stream(dz.device)), "xpa_s3_gemm_trunk_bwd_sign")
        return partial_dw, partial_db
    _lib.check(L.xpa_s3_gemm_trunk_bwd(_p(dz), ldz, _p(b_split), k, _p(h), ldh, _p(x), ldx, rows, d_in, int(act),
                                       float(slope), _p(partial_dw), _p(partial_db), _stream(dz.device)),
               "xpa_s3_gemm_trunk_bwd")
    return partial_dw, partial_db


def s3_gemm_rows_pair(a, b0_split, b1_split, bias, out=None):
    """K40R (r05): out [m, 512] = a [m, 256] . [B0 | B1] + bias (B0 / B1 split by s3_split / s3_split_batch, k = 256):
    the rollout's paired hidden layer; each output is s3_gemm's + bias bit for bit."""
    _req(a, "a", torch.float32, contiguous=False)
    lda = _row_stride(a, "a", 256)
    m = a.shape[0]
    _req(bias, "bias", torch.float32, (512,))
    if out is None:
        out = torch.empty(m, 512, dtype=torch.float32, device=a.device)
    ldc = _row_stride(out, "out", 512)
    if out.shape[0] != m:
        raise ValueError("out must have %d rows" % m)
    nb = int(lib().xpa_s3_split_bytes(256, 256))
    for b in (b0_split, b1_split):
        _req(b, "b_split", torch.uint8, (nb,))
    _lib.check(lib().xpa_s3_gemm_rows_pair(_p(a), lda, _p(b0_split), _p(b1_split), _p(bias), _p(out), ldc, m,
                                           _stream(a.device)), "xpa_s3_gemm_rows_pair")
    return out


def s3_gemm_rows_pair_trunk(x, w, b, act, slope, mean, var, clip, xn, col, col_ld, cursor, b0_split, b1_split, bias,
                            out=None):
    """K40T (r06): the rollout's trunk (obs normalisation + Linear(d_in, 256) + act, d_in <= 18; xn and the buffer column
    col (nullable) get the normalised rows as xpa_thin_linear_act_fwd_norm writes them) and K40R on its h in one launch;
    h stays in LDS.  out [m, 512] equals the two-launch form's bit for bit."""
    _req(x, "x", torch.float32, contiguous=False)
    m, d_in = x.shape
    if x.stride(1) != 1 or not 1 <= d_in <= 18:
        raise ValueError("x must be [m, d_in <= 18] with unit column stride")
    _req(w, "w", torch.float32, (256, d_in))
    _req(b, "b", torch.float32, (256,))
    _req(mean, "mean", torch.float32, (d_in,))
    _req(var, "var", torch.float32, (d_in,))
    _req(bias, "bias", torch.float32, (512,))
    if xn.dtype != torch.float32 or xn.shape[0] != m or xn.shape[1] != d_in or xn.stride(1) != 1:
        raise ValueError("xn must be float32 [m, d_in] with unit column stride")
    if out is None:
        out = torch.empty(m, 512, dtype=torch.float32, device=x.device)
    ldc = _row_stride(out, "out", 512)
    if out.shape[0] != m:
        raise ValueError("out must have %d rows" % m)
    nb = int(lib().xpa_s3_split_bytes(256, 256))
    for bb in (b0_split, b1_split):
        _req(bb, "b_split", torch.uint8, (nb,))
    _lib.check(lib().xpa_s3_gemm_rows_pair_trunk(
        int(act), _p(x), x.stride(0), d_in, _p(w), _p(b), float(slope), _p(mean), _p(var), float(clip), _p(xn),
        xn.stride(0), _p(col) if col is not None else None, int(col_ld), _p(cursor) if col is not None else None,
        _p(b0_split), _p(b1_split), _p(bias), _p(out), ldc, m, _stream(x.device)), "xpa_s3_gemm_rows_pair_trunk")
    return out


def s3_split_padded(b, k_pad, out=None):
    """The split of b [kv, 256] (any strides) padded with zero rows to k_pad (a multiple of 16): K40F's operand for a
    layer width that is not a multiple of 16 (xpa_s3_split_batch_padded)."""
    _req(b, "b", torch.float32, contiguous=False)
    kv, n = b.shape
    if n != 256 or k_pad % 16 or k_pad < kv:
        raise ValueError("s3_split_padded: b must be [kv, 256], kv <= k_pad, k_pad % 16 == 0")
    L = lib()
    nbytes = int(L.xpa_s3_split_bytes(k_pad, 256))
    if out is None:
        out = torch.empty(nbytes, dtype=torch.uint8, device=b.device)
    _req(out, "out", torch.uint8, (nbytes,))
    arr = lambda t, v: (t * 1)(v)   # noqa: E731
    _lib.check(L.xpa_s3_split_batch_padded(1, arr(ctypes.c_void_p, b.data_ptr()), arr(ctypes.c_int64, k_pad),
                                           arr(ctypes.c_int64, kv), arr(ctypes.c_int64, b.stride(0)),
                                           arr(ctypes.c_int64, b.stride(1)), arr(ctypes.c_void_p, out.data_ptr()),
                                           _stream(b.device)), "xpa_s3_split_batch_padded")
    return out


def s3_gemm_value(a, b_split, k, bias, act, slope, w_out, b_out, out=None):
    """K40V (r06): v [m] = act(a [m, k] . B + bias) . w_out + b_out (act = code 0 identity / 1 LeakyReLU / 2 tanh; B =
    s3_split(W^T) of the critic's last hidden layer, 256 columns; w_out [256] or [1, 256], b_out [1])."""
    _req(a, "a", torch.float32, contiguous=False)
    if a.dim() != 2 or a.stride(1) != 1 or a.shape[1] < k or k % 16:
        raise ValueError("a must be [m, >= k] with unit column stride, k % 16 == 0")
    m = a.shape[0]
    _req(bias, "bias", torch.float32, (HEAD_HIDDEN,))
    if w_out.numel() != HEAD_HIDDEN or not w_out.is_contiguous() or w_out.dtype != torch.float32:
        raise ValueError("w_out must be 256 contiguous float32 values")
    _req(b_out, "b_out", torch.float32, (1,))
    if out is None:
        out = torch.empty(m, dtype=torch.float32, device=a.device)
    _req(out, "out", torch.float32, (m,))
    _lib.check(lib().xpa_s3_gemm_value(_p(a), a.stride(0), _p(b_split), _p(out), m, k, _p(bias), int(act), float(slope),
                                       _p(w_out), _p(b_out), _stream(a.device)), "xpa_s3_gemm_value")
    return out


def s3_gemm_bias_act(a, b_split, k, bias, act, slope, out=None, sign=None, ridx=None):
    """K40F (r05): out [m, 256] = act(a [m, k] . B + bias) (act 0 identity / 1 LeakyReLU / 2 tanh); sign (int32 [m, 8],
    act 0 / 1): the output's sign bits for K42W.  a's columns past the layer width must be zero (padded rows).
    ridx (int64 [m]): the row-index form — row r is a[ridx[r]] of a [n_rows, width], k <= width + 16 with readable,
    finite slack after a's last row (xpa_s3_gemm_bias_act_rows)."""
    _req(a, "a", torch.float32, contiguous=False)
    if ridx is not None:
        _req(ridx, "ridx", torch.int64)
        if a.dim() != 2 or a.stride(1) != 1 or k > a.stride(0) + 16:
            raise ValueError("a must be [n_rows, width] with unit column stride and k <= width + 16")
        m = ridx.shape[0]
        _req(bias, "bias", torch.float32, (256,))
        if out is None:
            out = torch.empty(m, 256, dtype=torch.float32, device=a.device)
        ldc = _row_stride(out, "out", 256)
        if sign is not None:
            _req(sign, "sign", torch.int32, (m, 8))
        _lib.check(lib().xpa_s3_gemm_bias_act_rows(_p(a), a.stride(0), _p(ridx), _p(b_split), _p(out), ldc, m, k,
                                                   _p(bias), int(act), float(slope),
                                                   _p(sign) if sign is not None else None, _stream(a.device)),
                   "xpa_s3_gemm_bias_act_rows")
        return out
    lda = _row_stride(a, "a", k)
    m = a.shape[0]
    _req(bias, "bias", torch.float32, (256,))
    if out is None:
        out = torch.empty(m, 256, dtype=torch.float32, device=a.device)
    ldc = _row_stride(out, "out", 256)
    if out.shape[0] != m:
        raise ValueError("out must have %d rows" % m)
    if sign is not None:
        _req(sign, "sign", torch.int32, (m, 8))
    _lib.check(lib().xpa_s3_gemm_bias_act(_p(a), lda, _p(b_split), _p(out), ldc, m, k, _p(bias), int(act),
                                          float(slope), _p(sign) if sign is not None else None, _stream(a.device)),
               "xpa_s3_gemm_bias_act")
    return out


def s3_gemm_trunk_bwd_dz(dz, b_split, k, h_sign, act, slope, dz_out, partial_db, crit=None):
    """K42W (r05): g = dz [rows, k] . B (split); dz_out [rows, 256] = g act'(h) from h's sign bits, partial_db [G, 256]
    (the wide trunk layer's; its dW from s3_wgrad on the layer input and dz_out).  crit = (k_a, k_c, mask, dv, cs):
    K42C's factored critic half (dz = the actor's half, [rows, k_a])."""
    L = lib()
    _req(dz, "dz", torch.float32, contiguous=False)
    rows = dz.shape[0]
    ld_out = _row_stride(dz_out, "dz_out", 256)
    _req(h_sign, "h_sign", torch.int32, (rows, 8))
    G = int(L.xpa_s3_gemm_trunk_bwd_num_partials(rows))
    _req(partial_db, "partial_db", torch.float32, (G, 256))
    if dz_out.shape[0] != rows:
        raise ValueError("dz_out must have %d rows" % rows)
    if crit is not None:
        k_a, k_c, mask, dv, cs = crit
        ldz = _row_stride(dz, "dz_a", k_a)
        _req(mask, "mask", torch.int32, (rows, 8))
        _req(dv, "dv", torch.float32, (rows,))
        _req(cs, "cs", torch.float32, (256,))
        _lib.check(L.xpa_s3_gemm_trunk_bwd_crit_dz(_p(dz), ldz, _p(b_split), k_a, k_c, _p(mask), _p(dv), _p(cs),
                                                   _p(h_sign), rows, int(act), float(slope), _p(dz_out), ld_out,
                                                   _p(partial_db), _stream(dz.device)), "xpa_s3_gemm_trunk_bwd_crit_dz")
        return dz_out, partial_db
    ldz = _row_stride(dz, "dz", k)
    _lib.check(L.xpa_s3_gemm_trunk_bwd_dz(_p(dz), ldz, _p(b_split), k, _p(h_sign), rows, int(act), float(slope),
                                          _p(dz_out), ld_out, _p(partial_db), _stream(dz.device)),
               "xpa_s3_gemm_trunk_bwd_dz")
    return dz_out, partial_db


def gather_minibatch_pitched(idx, obs, obs_out, adv=None, adv_partials=None):
    """K4 into rows of obs_out [B, pitch] (pitch >= the row width; columns past it untouched, so a zero pad stays
    zero): the wide trunk's K40F operand.  obs [n_rows, d] f32 contiguous, d % 4 == 0."""
    _req(idx, "idx", torch.int64)
    B = idx.shape[0]
    if obs.dim() != 2 or not obs.is_contiguous():
        raise ValueError("obs must be a contiguous [n_rows, d] tensor")
    _req(obs_out, "obs_out", torch.float32, contiguous=False)
    d = obs.shape[1]
    if obs_out.dim() != 2 or obs_out.shape[0] != B or obs_out.stride(1) != 1 or obs_out.stride(0) < d:
        raise ValueError("obs_out must be [B, >= %d] with unit column stride" % d)
    if adv is not None:
        _req(adv, "adv", torch.float32)
        _req(adv_partials, "adv_partials", torch.float64, (gather_num_partials(B), 2))
    _lib.check(lib().xpa_gather_minibatch_pitched(_p(idx), B, obs.shape[0], _p(obs), d * 4, _p(obs_out),
                                                  obs_out.stride(0) * 4, _p(adv) if adv is not None else None,
                                                  _p(adv_partials) if adv is not None else None, None,
                                                  _stream(obs.device)), "xpa_gather_minibatch_pitched")
    return obs_out


def s3_wgrad_slices(rows, m):
    return int(lib().xpa_s3_wgrad_num_slices(rows, m))


def s3_wgrad(a, b, out=None, slices=None, aidx=None, m=None):
    """K41: per-slice partials out [S, m, 256] of a^T b over the rows (a [rows, m] = dz, b [rows, 256] = the layer
    input; unit column strides), on the bf16 matrix cores by the three-way split.  The caller sums the S slices.
    aidx (int64 [rows], r05): a's row r is a[aidx[r]] of a [n_rows, width] (m given, m <= width + 127: output rows past
    the width are garbage for the caller to drop; a needs readable slack after its last row; xpa_s3_wgrad_rows).
    m > a.shape[1] without aidx (r06): the rows in place, the same padding rule (xpa_s3_wgrad_padded)."""
    if aidx is not None:
        _req(a, "a", torch.float32, contiguous=False)
        _req(b, "b", torch.float32, contiguous=False)
        _req(aidx, "aidx", torch.int64)
        rows = aidx.shape[0]
        ldb = _row_stride(b, "b", 256)
        if b.shape[0] != rows or a.dim() != 2 or a.stride(1) != 1 or m is None:
            raise ValueError("aidx form: b [rows, 256], a [n_rows, width], m given")
        S = slices or s3_wgrad_slices(rows, m)
        if out is None:
            out = torch.empty(S, m, 256, dtype=torch.float32, device=a.device)
        _req(out, "out", torch.float32, (S, m, 256))
        _lib.check(lib().xpa_s3_wgrad_rows(_p(a), a.stride(0), _p(aidx), _p(b), ldb, rows, m, 256, S, _p(out),
                                           _stream(a.device)), "xpa_s3_wgrad_rows")
        return out
    _req(a, "a", torch.float32, contiguous=False)
    _req(b, "b", torch.float32, contiguous=False)
    if m is not None and m != a.shape[1]:
        # r06 (xpa_s3_wgrad_padded): m output rows over a's narrower rows (m <= width + 127); the rows past the width
        # read on into the next row and, after the last row, into slack of a's own storage, which must be readable
        rows, width = a.shape
        if a.dim() != 2 or a.stride(1) != 1 or not width < m <= width + 127:
            raise ValueError("padded form: a [rows, width] with width < m <= width + 127")
        lda, ldb = a.stride(0), _row_stride(b, "b", 256)
        need = a.storage_offset() + (rows - 1) * lda + m
        if a.untyped_storage().nbytes() // 4 < need:
            raise ValueError("padded form: a needs %d floats of slack after its last row" % (m - width))
        if b.shape[0] != rows:
            raise ValueError("a and b must have the same rows")
        S = slices or s3_wgrad_slices(rows, m)
        if out is None:
            out = torch.empty(S, m, 256, dtype=torch.float32, device=a.device)
        _req(out, "out", torch.float32, (S, m, 256))
        _lib.check(lib().xpa_s3_wgrad_padded(_p(a), lda, _p(b), ldb, rows, m, 256, S, _p(out), _stream(a.device)),
                   "xpa_s3_wgrad_padded")
        return out
    rows, m = a.shape
    lda, ldb = _row_stride(a, "a", m), _row_stride(b, "b", 256)
    if b.shape[0] != rows:
        raise ValueError("a and b must have the same rows")
    S = slices or s3_wgrad_slices(rows, m)
    if out is None:
        out = torch.empty(S, m, 256, dtype=torch.float32, device=a.device)
    _req(out, "out", torch.float32, (S, m, 256))
    _lib.check(lib().xpa_s3_wgrad(_p(a), lda, _p(b), ldb, rows, m, 256, S, _p(out), _stream(a.device)), "xpa_s3_wgrad")
    return out


# ------------------------------------------------------------------------------------------------
def gae_scan(rew, val, term, closed, boot, gamma, gae_lambda, use_gae=True, adv=None, ret=None):
    """K1.  All [n_envs, horizon]; closed uint8, the rest float32.  Returns (adv, ret)."""
    N, T = rew.shape
    for name, t, dt in (("rew", rew, torch.float32), ("val", val, torch.float32), ("term", term, torch.float32),
                        ("closed", closed, torch.uint8), ("boot", boot, torch.float32)):
        _req(t, name, dt, (N, T))
    adv = torch.empty_like(rew) if adv is None else _req(adv, "adv", torch.float32, (N, T))
    ret = torch.empty_like(rew) if ret is None else _req(ret, "ret", torch.float32, (N, T))
    ev = TIMER.kernel_events("gae")
    if ev is None:
        rc = lib().xpa_gae_scan(_p(rew), _p(val), _p(term), _p(closed), _p(boot), N, T, float(gamma), float(gae_lambda),
                                int(bool(use_gae)), _p(adv), _p(ret), _stream(rew.device))
    else:
        rc = lib().xpa_gae_scan_timed(_p(rew), _p(val), _p(term), _p(closed), _p(boot), N, T, float(gamma),
                                      float(gae_lambda), int(bool(use_gae)), _p(adv), _p(ret), ev[0], ev[1],
                                      _stream(rew.device))
    _lib.check(rc, "xpa_gae_scan")
    return adv, ret


def gae_scan_compact(rew, val, term, slot_t, vboot, gamma, gae_lambda, use_gae=True, adv=None, ret=None, boot=None):
    """K1, compact closures (xpa_gae_scan_compact): rows close at terminals, at slot_t[n] (one deferred
    truncation per env, -1 = none) and at the last step, bootstrapped by vboot = [V(truncation slots);
    V(last obs)] ([2 n_envs]).  Writes the two bootstraps into `boot` and resets slot_t (the state
    xpa_rollout_bootstrap_fixup + xpa_gae_scan leave).  Returns (adv, ret)."""
    N, T = rew.shape
    for name, t, dt in (("rew", rew, torch.float32), ("val", val, torch.float32), ("term", term, torch.float32),
                        ("boot", boot, torch.float32)):
        _req(t, name, dt, (N, T))
    _req(slot_t, "slot_t", torch.int32, (N,))
    _req(vboot, "vboot", torch.float32, (2 * N,))
    adv = torch.empty_like(rew) if adv is None else _req(adv, "adv", torch.float32, (N, T))
    ret = torch.empty_like(rew) if ret is None else _req(ret, "ret", torch.float32, (N, T))
    ev = TIMER.kernel_events("gae")
    e0, e1 = (None, None) if ev is None else ev
    rc = lib().xpa_gae_scan_compact(_p(rew), _p(val), _p(term), _p(slot_t), _p(vboot), N, T, float(gamma),
                                    float(gae_lambda), int(bool(use_gae)), _p(adv), _p(ret), _p(boot), e0, e1,
                                    _stream(rew.device))
    _lib.check(rc, "xpa_gae_scan_compact")
    return adv, ret


def gae_value_ok(T, z_critic=None):
    """True when xpa_gae_scan_value covers horizon T (DPP row segments of 16-64 lanes)."""
    return T % 4 == 0 and T >= 36 and (z_critic is None or z_critic.shape[1] == HEAD_HIDDEN)


def gae_scan_value(rew, val, term, slot_t, z_critic, act, w_critic, b_critic, gamma, gae_lambda, use_gae=True,
                   adv=None, ret=None, boot=None):
    """K1V (xpa_gae_scan_value): gae_scan_compact with the deferred bootstrap values formed inside the scan from
    the critic's hidden pre-activations z_critic [2 n_envs, 256] (rows: truncation slots, then last-step obs),
    act = (code, slope) and the critic's output layer (w_critic [1, 256], b_critic [1]).  Returns (adv, ret)."""
    N, T = rew.shape
    for name, t, dt in (("rew", rew, torch.float32), ("val", val, torch.float32), ("term", term, torch.float32),
                        ("boot", boot, torch.float32)):
        _req(t, name, dt, (N, T))
    _req(slot_t, "slot_t", torch.int32, (N,))
    if z_critic.dtype != torch.float32 or z_critic.device.type != "cuda" or z_critic.shape[0] != 2 * N:
        raise ValueError("z_critic must be a float32 ROCm tensor [2 n_envs, %d]" % HEAD_HIDDEN)
    ld = _row_stride(z_critic, "z_critic", HEAD_HIDDEN)
    _req(w_critic, "w_critic", torch.float32)
    _req(b_critic, "b_critic", torch.float32)
    if w_critic.numel() != HEAD_HIDDEN or b_critic.numel() != 1:
        raise ValueError("the critic's output layer must be Linear(%d, 1)" % HEAD_HIDDEN)
    if not gae_value_ok(T, z_critic):
        raise ValueError("xpa_gae_scan_value needs horizon % 4 == 0 and >= 36 (got %d)" % T)
    adv = torch.empty_like(rew) if adv is None else _req(adv, "adv", torch.float32, (N, T))
    ret = torch.empty_like(rew) if ret is None else _req(ret, "ret", torch.float32, (N, T))
    ev = TIMER.kernel_events("gae")
    e0, e1 = (None, None) if ev is None else ev
    rc = lib().xpa_gae_scan_value(_p(rew), _p(val), _p(term), _p(slot_t), int(act[0]), _p(z_critic), ld,
                                  float(act[1]), _p(w_critic), _p(b_critic), N, T, HEAD_HIDDEN, float(gamma),
                                  float(gae_lambda), int(bool(use_gae)), _p(adv), _p(ret), _p(boot), e0, e1,
                                  _stream(rew.device))
    _lib.check(rc, "xpa_gae_scan_value")
    return adv, ret


def _event_timed_median_us(launch, reps):
    """Median duration (us) of `launch(ev_start, ev_stop)` over `reps` synchronised launches, each timed by
    dispatch-attached events (the clock xpa_gae_scan_timed uses)."""
    rt = TIMER._hip()
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    for ev in (e0, e1):
        if rt.hipEventCreate(ctypes.byref(ev)) != 0:
            raise RuntimeError("hipEventCreate failed")
    times = []
    try:
        for i in range(reps + 3):
            launch(e0, e1)
            rt.hipEventSynchronize(e1)
            ms = ctypes.c_float()
            if rt.hipEventElapsedTime(ctypes.byref(ms), e0, e1) != 0:
                raise RuntimeError("hipEventElapsedTime failed")
            if i >= 3:
                times.append(ms.value * 1e3)
    finally:
        rt.hipEventDestroy(e0)
        rt.hipEventDestroy(e1)
    times.sort()
    return times[len(times) // 2]


def dispatch_floor_us(device, reps=50):
    """Median duration (us) of an empty one-wave launch timed by dispatch-attached events, the clock
    xpa_gae_scan_timed uses: the fixed cost every launch carries on it (bench.py reports it beside K1)."""
    st = _stream(device)
    return _event_timed_median_us(
        lambda e0, e1: _lib.check(lib().xpa_dispatch_floor_timed(e0, e1, st), "xpa_dispatch_floor_timed"), reps)


def stream_copy_us(rew, val, term, reps=50):
    """Median duration (us) of a plain streaming copy of K1's algorithmic bytes (read rew/val/term, write
    two arrays of the same shape; 20 B per element) on the same clock: the floor K1 is held to."""
    n = rew.numel()
    a, o = torch.empty_like(rew), torch.empty_like(rew)
    st = _stream(rew.device)

    def launch(e0, e1):
        _lib.check(lib().xpa_stream_copy_timed(_p(rew), _p(val), _p(term), _p(a), _p(o), n, e0, e1, st),
                   "xpa_stream_copy_timed")
    return _event_timed_median_us(launch, reps)


def random_permutation(n, seed, counter, out=None, device=None):
    """Pseudo-random permutation of [0, n) keyed by (seed, counter) on device (int64 [n])."""
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=device if device is not None else "cuda")
    _req(out, "out", torch.int64, (n,))
    _lib.check(lib().xpa_random_permutation(n, int(seed) & 0xFFFFFFFF, int(counter) & 0xFFFFFFFF, _p(out),
                                            _stream(out.device)), "xpa_random_permutation")
    return out


def gather_num_partials(batch):
    return int(lib().xpa_gather_num_partials(batch))


def gather_minibatch(idx, obs, adv=None, obs_out=None, adv_partials=None, err=None):
    """K4.  idx int64 [B] flat indices into obs rows ([n_rows, ...] any dtype, contiguous).  err (int32 [1], optional):
    counts indices outside [0, n_rows) (their rows are zero-filled).
    Returns (obs_out [B, ...], adv_partials float64 [n_partials, 2] or None)."""
    _req(idx, "idx", torch.int64)
    if idx.dim() != 1:
        raise ValueError("idx must be 1-D")
    B = idx.shape[0]
    if not obs.is_contiguous() or obs.device.type != "cuda":
        raise ValueError("obs must be a contiguous device tensor")
    row_shape = tuple(obs.shape[1:])
    row_bytes = obs[0].numel() * obs.element_size() if obs.shape[0] > 0 else 0
    if obs_out is None:
        obs_out = torch.empty((B,) + row_shape, dtype=obs.dtype, device=obs.device)
    elif tuple(obs_out.shape) != (B,) + row_shape or obs_out.dtype != obs.dtype or not obs_out.is_contiguous():
        raise ValueError("obs_out must be contiguous %s %s" % ((B,) + row_shape, obs.dtype))
    if adv is not None:
        _req(adv, "adv", torch.float32)
        if adv.numel() != obs.shape[0]:
            raise ValueError("adv must have one entry per obs row")
        if adv_partials is None:
            adv_partials = torch.empty((gather_num_partials(B), 2), dtype=torch.float64, device=obs.device)
        else:
            _req(adv_partials, "adv_partials", torch.float64, (gather_num_partials(B), 2))
    rc = lib().xpa_gather_minibatch(_p(idx), B, obs.shape[0], _p(obs), row_bytes, _p(obs_out), _p(adv) if adv is not None else None,
                                    _p(adv_partials) if adv is not None else None,
                                    _p(_req(err, "err", torch.int32, (1,))) if err is not None else None, _stream(obs.device))
    _lib.check(rc, "xpa_gather_minibatch")
    return obs_out, (adv_partials if adv is not None else None)


class LossWorkspace:
    """Reusable outputs of K2 for a fixed (batch, act_dim) (keeps the update step allocation-free)."""

    def __init__(self, batch, act_dim, device, dist):
        n = int(lib().xpa_loss_num_partials(batch))
        w = int(lib().xpa_loss_partial_width(act_dim))
        self.batch, self.act_dim = batch, act_dim
        self.partials = torch.empty((n, w), dtype=torch.float32, device=device)
        self.d_head = torch.empty((batch, act_dim), dtype=torch.float32, device=device)
        self.d_v = torch.empty((batch,), dtype=torch.float32, device=device)
        self.scalars = torch.empty((N_OUT,), dtype=torch.float32, device=device)
        self.d_logstd = torch.empty((act_dim,), dtype=torch.float32, device=device) if dist == "gaussian" else None


def policy_loss(algo, dist, head, logstd, v, act, adv, ret, old_logp=None, idx=None, adv_partials=None,
                clip_range=0.2, vf_coef=0.25, ent_coef=0.0, ws=None, d_logstd_out=None):
    """K2 + finalize.  Returns (scalars[6] device tensor, d_head, d_logstd or None, d_v).

    head [B, A] float32; logstd [A] (gaussian); v [B].  act/old_logp/adv/ret are read at idx[b]
    (idx int64 [B]) or at b when idx is None.  adv_partials (float64 [*, 2]) => per-minibatch adv-norm."""
    if algo not in ALGO or dist not in DIST:
        raise ValueError("algo must be ppo|a2c and dist gaussian|categorical")
    _req(head, "head", torch.float32)
    if head.dim() != 2:
        raise ValueError("head must be [B, A]")
    B, A = head.shape
    _req(v, "v", torch.float32, (B,))
    if dist == "gaussian":
        _req(logstd, "logstd", torch.float32, (A,))
    if idx is not None:
        _req(idx, "idx", torch.int64, (B,))
    rows = adv.numel()
    _req(adv, "adv", torch.float32)
    _req(ret, "ret", torch.float32)
    if ret.numel() != rows:
        raise ValueError("ret and adv must have the same number of rows")
    if idx is None and rows != B:
        raise ValueError("without idx, adv/ret must have B rows")
    _req(act, "act", torch.float32)
    if act.numel() != rows * (A if dist == "gaussian" else 1):
        raise ValueError("act has %d elements, expected %d" % (act.numel(), rows * (A if dist == "gaussian" else 1)))
    if algo == "ppo":
        if old_logp is None:
            raise ValueError("PPO needs old_logp")
        _req(old_logp, "old_logp", torch.float32)
        if old_logp.numel() != rows:
            raise ValueError("old_logp must have one entry per row")
    if adv_partials is not None:
        _req(adv_partials, "adv_partials", torch.float64)
    if ws is None or ws.batch != B or ws.act_dim != A:
        ws = LossWorkspace(B, A, head.device, dist)
    s = _stream(head.device)
    L = lib()
    ev = TIMER.start("loss")
    rc = L.xpa_policy_loss_fwd_bwd(ALGO[algo], DIST[dist], B, A, _p(head), _p(logstd) if dist == "gaussian" else None,
                                   _p(v), _p(idx), rows, _p(act), _p(old_logp) if algo == "ppo" else None, _p(adv), _p(ret),
                                   _p(adv_partials), adv_partials.shape[0] if adv_partials is not None else 0,
                                   float(clip_range), float(vf_coef), float(ent_coef), _p(ws.d_head), _p(ws.d_v),
                                   _p(ws.partials), s)
    TIMER.stop("loss", ev)
    _lib.check(rc, "xpa_policy_loss_fwd_bwd")
    d_logstd = ws.d_logstd
    if d_logstd_out is not None and dist == "gaussian":
        _req(d_logstd_out, "d_logstd_out", torch.float32, (A,))
        d_logstd = d_logstd_out
    rc = L.xpa_policy_loss_finalize(ALGO[algo], DIST[dist], B, A, _p(ws.partials), ws.partials.shape[0],
                                    float(vf_coef), float(ent_coef), _p(ws.scalars), _p(d_logstd), s)
    _lib.check(rc, "xpa_policy_loss_finalize")
    return ws.scalars, ws.d_head, d_logstd, ws.d_v


# ------------------------------------------------------------------------------------------------
HEAD_HIDDEN = 256  # hidden width K12 handles (64 lanes x 4 columns)
HEAD_KMAX = 18   # widest head of the fused head kernels K12 / K16 (and K14's rollout head)
TRUNK_DMAX = 20  # widest trunk input K16X forms in its prologue (xpa_head_gemm_trunk_*)


class HeadWorkspace:
    """Outputs and per-block partials of K12 for a fixed (batch, K)."""

    def __init__(self, batch, k, device, paired=False):
        H = HEAD_HIDDEN
        G = int(lib().xpa_head_fused_num_partials(batch))
        self.batch, self.k, self.G, self.paired = batch, k, G, paired
        f32 = dict(dtype=torch.float32, device=device)
        if paired:   # actor | critic halves of one [batch, 512] gradient (one dX / dW GEMM downstream)
            self.dz_pair = torch.empty((batch, 2 * H), **f32)
            self.dz_actor, self.dz_critic = self.dz_pair[:, :H], self.dz_pair[:, H:]
        else:
            self.dz_pair = None
            self.dz_actor = torch.empty((batch, H), **f32)
            self.dz_critic = torch.empty((batch, H), **f32)
        self.p_dw_actor = torch.empty((G, k * H), **f32)
        self.p_dbh_actor = torch.empty((G, H), **f32)
        self.p_dbo_actor = torch.empty((G, k), **f32)
        self.p_dw_critic = torch.empty((G, H), **f32)
        self.p_dbh_critic = torch.empty((G, H), **f32)
        self.p_dbo_critic = torch.empty((G, 1), **f32)
        self.loss_partials = torch.zeros((G, int(lib().xpa_loss_partial_width(k))), **f32)
        self.scalars = torch.empty((N_OUT,), **f32)


def _colsum(part, out, s):
    _lib.check(lib().xpa_colsum_finalize(_p(part), part.shape[0], part.shape[1], _p(out), s), "xpa_colsum_finalize")


class ColsumQueue:
    """Collects column-sum finalizes (partials [G, C] -> out [C]) and launches them together with
    xpa_colsum_finalize_batch (16 segments per launch).  The ctypes argument arrays are cached per
    set of buffers, so a steady-state update re-uses them."""

    MAX_SEGS = 16

    def __init__(self):
        self.items = []
        self._plans = {}
        self._ticket = None
        self.loss = None   # deferred loss finalize (defer_loss): run as one extra block of the flush

    def reset(self):
        """Drop queued finalizes (e.g. those of an aborted graph capture) without launching them."""
        self.items = []
        self.loss = None

    def defer_loss(self, algo, dist, batch, act_dim, loss_partials, vf_coef, ent_coef, scalars, d_logstd):
        """Queue xpa_policy_loss_finalize_sq for the flush (its d logstd share of the clip norm lands in sq[0])."""
        self.loss = (int(algo), int(dist), int(batch), int(act_dim), loss_partials, float(vf_coef), float(ent_coef),
                     scalars, d_logstd)

    def add(self, part, out, tmap=None):
        """tmap (r05) = (inner, valid, ld): column r inner + i of the partials goes to out[i ld + r] for r < valid
        (xpa_colsum_finalize_batch_map; e.g. K41V's padded dW^T slices into W [256, d_in]); out then holds
        inner * valid elements."""
        _req(part, "partials", torch.float32)
        _req(out, "out", torch.float32)
        if tmap is None:
            if part.dim() != 2 or out.numel() != part.shape[1]:
                raise ValueError("partials must be [G, C] and out must have C elements")
        else:
            inner, valid, ld = (int(v) for v in tmap)
            if (part.dim() != 2 or part.shape[1] % inner or valid > part.shape[1] // inner or out.numel() != inner * valid
                    or not out.is_contiguous() or ld != valid):
                raise ValueError("tmap: partials [G, rows * inner], out contiguous [inner, valid], ld == valid")
        self.items.append((part, out, tmap))

    def flush(self, device=None, sq=None):
        """Launch the queued finalizes.  sq (float64 tensor, >= tiles + 2 entries, sq[0] written beforehand):
        when the queue fits one launch, also the clip norm of the outputs + sq[0], left at sq[1 + tiles]
        (xpa_colsum_finalize_batch_sq).  Returns (that total's view or None, output elements written)."""
        if not self.items:
            loss, self.loss = self.loss, None
            if loss is not None:   # a deferred loss finalize with no column tiles to ride on: run it alone
                a, d, B, K, lp, vf, ent, sc, dls = loss
                dev = device if device is not None else lp.device
                _lib.check(lib().xpa_policy_loss_finalize_sq(a, d, B, K, _p(lp), lp.shape[0], vf, ent, _p(sc), _p(dls),
                                                             _p(sq) if sq is not None else None, _stream(dev)),
                           "xpa_policy_loss_finalize")
            return None, 0
        key = tuple((p.data_ptr(), p.shape[0], p.shape[1], o.data_ptr(), tm) for p, o, tm in self.items)
        plan = self._plans.get(key)
        if plan is None:
            plan = []
            for i in range(0, len(key), self.MAX_SEGS):
                chunk = key[i:i + self.MAX_SEGS]
                n = len(chunk)
                arrs = ((ctypes.c_void_p * n)(*[c[0] for c in chunk]), (ctypes.c_int64 * n)(*[c[1] for c in chunk]),
                        (ctypes.c_int64 * n)(*[c[2] for c in chunk]), (ctypes.c_void_p * n)(*[c[3] for c in chunk]))
                tiles = int(lib().xpa_colsum_batch_tiles(n, ctypes.cast(arrs[1], ctypes.c_void_p),
                                                         ctypes.cast(arrs[2], ctypes.c_void_p)))
                tmap = None
                if any(c[4] is not None for c in chunk):   # the map entry (r05): (inner, valid, ld) per segment
                    tmap = (ctypes.c_int64 * (3 * n))(*[v for c in chunk for v in (c[4] or (0, 0, 0))])
                plan.append((n, arrs, [ctypes.cast(a, ctypes.c_void_p) for a in arrs], tiles, tmap))
            self._plans[key] = plan
        dev = device if device is not None else self.items[0][0].device
        s = _stream(dev)
        L = lib()
        total = None
        loss, self.loss = self.loss, None
        one = sq is not None and len(plan) == 1 and plan[0][3] + 2 <= sq.numel()
        if loss is not None and not one:   # the loss finalize on its own (d logstd share into sq[0] if any)
            a, d, B, K, lp, vf, ent, sc, dls = loss
            _lib.check(L.xpa_policy_loss_finalize_sq(a, d, B, K, _p(lp), lp.shape[0], vf, ent, _p(sc), _p(dls),
                                                     _p(sq) if sq is not None else None, s),
                       "xpa_policy_loss_finalize")
            loss = None
        if one:
            if self._ticket is None:
                self._ticket = torch.zeros((_lib.COLSUM_TICKET_INTS,), dtype=torch.int32, device=dev)
            n, _keep, args, tiles, tmap = plan[0]
            if tmap is not None:
                la = loss if loss is not None else (0, 0, 0, 0, None, 0.0, 0.0, None, None)
                a, d, B, K, lp, vf, ent, sc, dls = la
                _lib.check(L.xpa_colsum_finalize_batch_map(n, *args, ctypes.cast(tmap, ctypes.c_void_p), _p(sq),
                                                           _p(self._ticket), a, d, B, K,
                                                           _p(lp) if lp is not None else None,
                                                           lp.shape[0] if lp is not None else 0, vf, ent,
                                                           _p(sc) if sc is not None else None,
                                                           _p(dls) if dls is not None else None, s),
                           "xpa_colsum_finalize_batch_map")
            elif loss is not None:   # one launch: the column tiles + the loss finalize block
                a, d, B, K, lp, vf, ent, sc, dls = loss
                _lib.check(L.xpa_colsum_finalize_batch_sq_loss(n, *args, _p(sq), _p(self._ticket), a, d, B, K, _p(lp),
                                                               lp.shape[0], vf, ent, _p(sc), _p(dls), s),
                           "xpa_colsum_finalize_batch_sq_loss")
            else:
                _lib.check(L.xpa_colsum_finalize_batch_sq(n, *args, _p(sq), _p(self._ticket), s),
                           "xpa_colsum_finalize_batch_sq")
            total = sq[1 + tiles:2 + tiles]
        else:
            for n, _keep, args, _tiles, tmap in plan:
                if tmap is not None:
                    _lib.check(L.xpa_colsum_finalize_batch_map(n, *args, ctypes.cast(tmap, ctypes.c_void_p), None, None,
                                                               0, 0, 0, 0, None, 0, 0.0, 0.0, None, None, s),
                               "xpa_colsum_finalize_batch_map")
                else:
                    _lib.check(L.xpa_colsum_finalize_batch(n, *args, s), "xpa_colsum_finalize_batch")
        written = sum(o.numel() for _, o, _ in self.items)
        self.items = []
        return total, written


K16W_ENABLED = False  # fused_heads' gemm form: K16W (xpa_head_gemm_ws_*) where it applies, else K16
# The update's hidden-layer GEMMs on the bf16 matrix cores by the three-way split (K16S heads, K40 dX, K41 dW):
# the f32 GEMM's accuracy, not the f32 MFMA's bits.  Read when a learner's update is built / captured.
S3_GEMMS = True
S3_HEADS = "s3q"   # with S3_GEMMS: "s3" K16S (both fragments split in the k loop), "s3p" K16P (Wh's planes split once),
                   # "s3q" K16Q (K16P's bits, 32 x 128 wave tiles)


def fused_heads(algo, dist, ws, z_actor, w_actor, b_actor, act_actor, z_critic, w_critic, b_critic, act_critic,
                logstd, act, adv, ret, old_logp=None, idx=None, adv_partials=None, clip_range=0.2, vf_coef=0.25,
                ent_coef=0.0, grads=None, colsum_queue=None, gemm=None, sq_logstd=None, defer_loss=False, trunk=None,
                wh_split=None, crit_mask=None):
    """K12 actor + critic heads, loss finalize and the column-sum finalizes.

    z_*: hidden pre-activations [B, 256] (unit column stride; row stride = the workspace dz row stride,
    e.g. the halves of a [B, 512] actor|critic pre-activation with a paired workspace); w_*/b_*: output layer
    gemm = (x [B, 256], (w_h_actor, b_h_actor), (w_h_critic, b_h_critic)): K16 — the hidden layers' GEMMs
    run inside the head kernels on the matrix cores and z_actor / z_critic are not used (pass None).
    trunk = (x_rows [B, d_in], w_in [256, d_in], b_in, slope_in, h_out[, h_sign]) with gemm: K16X — the trunk layer
    Linear(d_in <= TRUNK_DMAX, 256) + the heads' activation is formed inside the launches too; gemm's x must be h_out,
    which the actor launch writes.  wh_split = (planes of w_h_actor^T, planes of w_h_critic^T) (s3_split): K16P; with
    trunk as well K16R (h formed in both launches' k loops, the actor writes h and, given h_sign int32 [B, 8], its
    sign bits for K42S).  crit_mask = (mask int32 [B, 8], dv f32 [B]) with the K16Q heads (r05): the critic writes its
    hidden activations' sign bits and d loss / d v per row instead of dz_critic (K41P / K42C's factored critic).
    (K x 256 / 1 x 256); act_*: (code, slope)
    of the hidden activation.  colsum_queue: an ops.ColsumQueue to defer the column-sum finalizes into
    (flushed by the caller), else they run here.  grads: dict with the gradient views to write — 'w_actor', 'b_actor',
    'bh_actor', 'w_critic', 'b_critic', 'bh_critic', 'logstd' (gaussian).  Returns (scalars, dz_actor,
    dz_critic)."""
    if algo not in ALGO or dist not in DIST:
        raise ValueError("algo must be ppo|a2c and dist gaussian|categorical")
    H = HEAD_HIDDEN
    B = gemm[0].shape[0] if gemm is not None else z_actor.shape[0]
    K = w_actor.shape[0]
    if ws.batch != B or ws.k != K:
        raise ValueError("fused heads need a matching workspace")
    ld = ws.dz_actor.stride(0)
    if gemm is not None:
        x, (wha, bha), (whc, bhc) = gemm
        _req(x, "x", torch.float32, contiguous=False)
        if tuple(x.shape) != (B, H) or x.stride(1) != 1:
            raise ValueError("x must be [%d, %d] with unit column stride" % (B, H))
        for name, w_ in (("w_h_actor", wha), ("w_h_critic", whc)):
            _req(w_, name, torch.float32, (H, H))
    else:
        for name, zz in (("z_actor", z_actor), ("z_critic", z_critic)):
            _req(zz, name, torch.float32, contiguous=False)
            if tuple(zz.shape) != (B, H) or zz.stride() != (ld, 1):
                raise ValueError("%s must be [%d, %d] with row stride %d" % (name, B, H, ld))
    _req(w_actor, "w_actor", torch.float32, (K, H))
    _req(w_critic, "w_critic", torch.float32, (1, H))
    if idx is not None:
        _req(idx, "idx", torch.int64, (B,))
    rows = adv.numel()
    _req(adv, "adv", torch.float32)
    _req(ret, "ret", torch.float32, (rows,))
    _req(act, "act", torch.float32)
    if act.numel() != rows * (K if dist == "gaussian" else 1):
        raise ValueError("act has %d elements, expected %d" % (act.numel(), rows * (K if dist == "gaussian" else 1)))
    if algo == "ppo":
        _req(old_logp, "old_logp", torch.float32, (rows,))
    if adv_partials is not None:
        _req(adv_partials, "adv_partials", torch.float64)
    dev = w_actor.device
    s = _stream(dev)
    L = lib()
    W = ws.loss_partials.shape[1]
    ev = TIMER.start("heads")
    n_adv = adv_partials.shape[0] if adv_partials is not None else 0
    p_logstd = _p(logstd) if dist == "gaussian" else None
    p_old = _p(old_logp) if algo == "ppo" else None
    if trunk is not None:
        if gemm is None or trunk[4] is not x:
            raise ValueError("trunk needs gemm with x = the trunk's h output")
        xr, w0, b0, slope0, h_out = trunk[:5]
        h_sign = trunk[5] if len(trunk) > 5 else None
        _req(xr, "x_rows", torch.float32)
        din = xr.shape[1]
        if xr.dim() != 2 or xr.shape[0] != B or din > TRUNK_DMAX or tuple(w0.shape) != (H, din):
            raise ValueError("trunk rows must be [%d, <= %d] with w_in [%d, d_in]" % (B, TRUNK_DMAX, H))
    if trunk is not None and wh_split is not None:
        # K16R: h formed from the gathered rows inside both launches (Wh as its bf16 planes); the actor writes h
        # and its sign bits
        if h_sign is not None:
            _req(h_sign, "h_sign", torch.int32, (B, 8))
        wsa, wsc = wh_split
        _lib.check(L.xpa_head_gemm_s3r_actor(ALGO[algo], DIST[dist], act_actor[0], B, K, H, _p(xr), xr.stride(0), din,
                                             _p(w0), _p(b0), float(slope0), _p(h_out), h_out.stride(0),
                                             _p(h_sign) if h_sign is not None else None, _p(wsa), _p(bha), ld,
                                             _p(w_actor), _p(b_actor), float(act_actor[1]), p_logstd, _p(idx), rows,
                                             _p(act), p_old, _p(adv), _p(adv_partials), n_adv, float(clip_range),
                                             float(ent_coef), _p(ws.dz_actor), _p(ws.p_dw_actor), _p(ws.p_dbh_actor),
                                             _p(ws.p_dbo_actor), _p(ws.loss_partials), W, s), "xpa_head_gemm_s3r_actor")
        _lib.check(L.xpa_head_gemm_s3r_critic(act_critic[0], B, H, _p(xr), xr.stride(0), din, _p(w0), _p(b0),
                                              float(slope0), _p(wsc), _p(bhc), ld, _p(w_critic), _p(b_critic),
                                              float(act_critic[1]), _p(idx), rows, _p(ret), float(vf_coef),
                                              _p(ws.dz_critic), _p(ws.p_dw_critic), _p(ws.p_dbh_critic),
                                              _p(ws.p_dbo_critic), _p(ws.loss_partials), W, s),
                   "xpa_head_gemm_s3r_critic")
    elif trunk is not None:
        _lib.check(L.xpa_head_gemm_trunk_actor(ALGO[algo], DIST[dist], act_actor[0], B, K, H, _p(xr), xr.stride(0), din,
                                               _p(w0), _p(b0), float(slope0), _p(h_out), h_out.stride(0), _p(wha),
                                               _p(bha), ld, _p(w_actor), _p(b_actor), float(act_actor[1]), p_logstd,
                                               _p(idx), rows, _p(act), p_old, _p(adv), _p(adv_partials), n_adv,
                                               float(clip_range), float(ent_coef), _p(ws.dz_actor), _p(ws.p_dw_actor),
                                               _p(ws.p_dbh_actor), _p(ws.p_dbo_actor), _p(ws.loss_partials), W, s),
                   "xpa_head_gemm_trunk_actor")
        # the critic reads the h the actor launch wrote (plain K16)
        _lib.check(L.xpa_head_gemm_critic(act_critic[0], B, H, _p(h_out), h_out.stride(0), _p(whc), _p(bhc), ld,
                                          _p(w_critic), _p(b_critic), float(act_critic[1]), _p(idx), rows, _p(ret),
                                          float(vf_coef), _p(ws.dz_critic), _p(ws.p_dw_critic), _p(ws.p_dbh_critic),
                                          _p(ws.p_dbo_critic), _p(ws.loss_partials), W, s), "xpa_head_gemm_critic")
    elif gemm is not None:
        # K16W (wave-specialised, the epilogue overlapped with the GEMM) for heads up to 8 wide; K16 otherwise
        wsa = K16W_ENABLED and K <= 8
        fa = L.xpa_head_gemm_ws_actor if wsa else L.xpa_head_gemm_s3_actor if S3_GEMMS else L.xpa_head_gemm_actor
        fc = (L.xpa_head_gemm_ws_critic if K16W_ENABLED else L.xpa_head_gemm_s3_critic if S3_GEMMS
              else L.xpa_head_gemm_critic)
        if wh_split is not None and not wsa and not K16W_ENABLED:   # K16P / K16Q: the hidden weights as bf16 planes
            if S3_HEADS == "s3q":
                fa, fc = L.xpa_head_gemm_s3q_actor, L.xpa_head_gemm_s3q_critic
            else:
                fa, fc = L.xpa_head_gemm_s3p_actor, L.xpa_head_gemm_s3p_critic
            wha, whc = wh_split
        _lib.check(fa(ALGO[algo], DIST[dist], act_actor[0], B, K, H, _p(x), x.stride(0), _p(wha),
                      _p(bha), ld, _p(w_actor), _p(b_actor), float(act_actor[1]), p_logstd, _p(idx),
                      rows, _p(act), p_old, _p(adv), _p(adv_partials), n_adv, float(clip_range),
                      float(ent_coef), _p(ws.dz_actor), _p(ws.p_dw_actor), _p(ws.p_dbh_actor),
                      _p(ws.p_dbo_actor), _p(ws.loss_partials), W, s), "xpa_head_gemm_actor")
        if crit_mask is not None:
            if not (wh_split is not None and S3_HEADS == "s3q" and not K16W_ENABLED):
                raise ValueError("crit_mask needs the K16Q heads")
            cm, cdv = crit_mask
            _req(cm, "crit mask", torch.int32, (B, 8))
            _req(cdv, "crit dv", torch.float32, (B,))
            _lib.check(L.xpa_head_gemm_s3q_critic_mask(act_critic[0], B, H, _p(x), x.stride(0), _p(whc), _p(bhc), ld,
                                                       _p(w_critic), _p(b_critic), float(act_critic[1]), _p(idx), rows,
                                                       _p(ret), float(vf_coef), None, _p(ws.p_dw_critic),
                                                       _p(ws.p_dbh_critic), _p(ws.p_dbo_critic), _p(ws.loss_partials),
                                                       W, s, _p(cm), _p(cdv)), "xpa_head_gemm_s3q_critic_mask")
        else:
            _lib.check(fc(act_critic[0], B, H, _p(x), x.stride(0), _p(whc), _p(bhc), ld, _p(w_critic),
                          _p(b_critic), float(act_critic[1]), _p(idx), rows, _p(ret), float(vf_coef),
                          _p(ws.dz_critic), _p(ws.p_dw_critic), _p(ws.p_dbh_critic),
                          _p(ws.p_dbo_critic), _p(ws.loss_partials), W, s), "xpa_head_gemm_critic")
    else:
        _lib.check(L.xpa_head_fused_actor(ALGO[algo], DIST[dist], act_actor[0], B, K, H, ld, _p(z_actor), _p(w_actor),
                                          _p(b_actor), float(act_actor[1]), p_logstd, _p(idx), rows, _p(act), p_old,
                                          _p(adv), _p(adv_partials), n_adv, float(clip_range), float(ent_coef),
                                          _p(ws.dz_actor), _p(ws.p_dw_actor), _p(ws.p_dbh_actor), _p(ws.p_dbo_actor),
                                          _p(ws.loss_partials), W, s), "xpa_head_fused_actor")
        _lib.check(L.xpa_head_fused_critic(act_critic[0], B, H, ld, _p(z_critic), _p(w_critic), _p(b_critic),
                                           float(act_critic[1]), _p(idx), rows, _p(ret), float(vf_coef),
                                           _p(ws.dz_critic), _p(ws.p_dw_critic), _p(ws.p_dbh_critic),
                                           _p(ws.p_dbo_critic), _p(ws.loss_partials), W, s), "xpa_head_fused_critic")
    TIMER.stop("heads", ev)
    g = grads or {}
    d_logstd = g.get("logstd")
    if dist == "gaussian" and d_logstd is None:
        d_logstd = torch.empty((K,), dtype=torch.float32, device=dev)
    queue = colsum_queue if colsum_queue is not None else ColsumQueue()
    if defer_loss and colsum_queue is not None:
        # run by the queue's flush (one extra block of the batched finalize launch; writes sq[0] there)
        queue.defer_loss(ALGO[algo], DIST[dist], B, K, ws.loss_partials, vf_coef, ent_coef, ws.scalars, d_logstd)
    else:
        # sq_logstd: device address of one double receiving sum(d_logstd^2) (the clip norm's share of logstd)
        _lib.check(L.xpa_policy_loss_finalize_sq(ALGO[algo], DIST[dist], B, K, _p(ws.loss_partials), ws.G,
                                                 float(vf_coef), float(ent_coef), _p(ws.scalars), _p(d_logstd),
                                                 sq_logstd, s), "xpa_policy_loss_finalize")
    for key, part in (("w_actor", ws.p_dw_actor), ("b_actor", ws.p_dbo_actor), ("bh_actor", ws.p_dbh_actor),
                      ("w_critic", ws.p_dw_critic), ("b_critic", ws.p_dbo_critic), ("bh_critic", ws.p_dbh_critic)):
        if key in g:
            queue.add(part, g[key])
    if colsum_queue is None:
        queue.flush(dev)
    return ws.scalars, ws.dz_actor, ws.dz_critic


# ------------------------------------------------------------------------------------------------
def rms_num_partials(n):
    return int(lib().xpa_rms_num_partials(n))


def rms_update(x, mean, var, count, partials=None, reduce_partials=None, world=1, ticket=None):
    """K5a+b: RunningMeanStd.update(x) on device.  x [n, dim] float32 (row stride may exceed dim);
    mean/var float32 [dim], count float64 [1] — all updated in place.
    reduce_partials(partials): optional in-place SUM across ranks of the f64 partials (the
    mpi_moments-style synchronised statistics, statistic_tools.py:20-32); the merge then counts
    n * world rows.  All ranks must hold the same running mean (it is the partials' shift).
    ticket (int32 [1], zeroed once): single-launch form (xpa_rms_update: the last block merges)."""
    n, dim = x.shape
    ld = _row_stride(x, "x", dim)
    _req(mean, "mean", torch.float32, (dim,))
    _req(var, "var", torch.float32, (dim,))
    _req(count, "count", torch.float64, (1,))
    np_ = rms_num_partials(n)
    if partials is None:
        partials = torch.empty((2 * np_, dim), dtype=torch.float64, device=x.device)
    else:
        _req(partials, "partials", torch.float64, (2 * np_, dim))
    s = _stream(x.device)
    if ticket is not None and reduce_partials is None:
        _req(ticket, "ticket", torch.int32, (1,))
        _lib.check(lib().xpa_rms_update(_p(x), n, dim, ld, _p(mean), _p(var), _p(count), _p(partials), _p(ticket), s),
                   "xpa_rms_update")
        return
    _lib.check(lib().xpa_rms_partials(_p(x), n, dim, ld, _p(mean), _p(partials), s), "xpa_rms_partials")
    if reduce_partials is not None:
        reduce_partials(partials)
        n = n * int(world)
    _lib.check(lib().xpa_rms_merge(_p(partials), np_, n, dim, _p(mean), _p(var), _p(count), s), "xpa_rms_merge")


def store_column(x, buf, cursor):
    """Raw observation rows x [N, ...] into buf [N, T, ...] at column cursor.ptr (graph-capturable)."""
    N = x.shape[0]
    if not x.is_contiguous() or not buf.is_contiguous() or x.device.type != "cuda" or buf.dtype != x.dtype:
        raise ValueError("store_column: contiguous device tensors of one dtype")
    if buf.shape[0] != N or tuple(buf.shape[2:]) != tuple(x.shape[1:]):
        raise ValueError("store_column: buf must be [N, T] + x.shape[1:]")
    _req(cursor, "cursor", torch.int32, (4,))
    row_bytes = x[0].numel() * x.element_size()
    _lib.check(lib().xpa_store_column(_p(x), N, row_bytes, _p(buf), buf.shape[1], _p(cursor), _stream(x.device)),
               "xpa_store_column")


def obs_normalize(x, mean, var, clip_range, out, col_out=None, col_ld=0, cursor=None):
    """K5c: out = clip((x - mean)/(sqrt(var)+1e-8)); optionally also into a buffer column."""
    n, dim = x.shape
    ldx = _row_stride(x, "x", dim)
    ldo = _row_stride(out, "out", dim)
    _req(mean, "mean", torch.float32, (dim,))
    _req(var, "var", torch.float32, (dim,))
    if col_out is not None:
        _req(col_out, "col_out", torch.float32)
        _req(cursor, "cursor", torch.int32, (4,))
    rc = lib().xpa_obs_normalize(_p(x), n, dim, ldx, _p(mean), _p(var), float(clip_range), _p(out), ldo, _p(col_out),
                                 int(col_ld), _p(cursor), _stream(x.device))
    _lib.check(rc, "xpa_obs_normalize")
    return out


# ------------------------------------------------------------------------------------------------
def new_cursor(device):
    """xpa_cursor_t {ptr, step, reserved[2]} as an int32[4] device tensor."""
    return torch.zeros((4,), dtype=torch.int32, device=device)


def rollout_sample(dist, head, logstd, v, cursor, seed, buf_act, buf_logp, buf_val, env_in, act_clip=1.0):
    """K3: sample actions for every env, store act/logp/val at column cursor.ptr, write env input."""
    _req(head, "head", torch.float32)
    N, A = head.shape
    _req(v, "v", torch.float32, (N,))
    _req(cursor, "cursor", torch.int32, (4,))
    _req(buf_logp, "buf_logp", torch.float32)
    _req(buf_val, "buf_val", torch.float32)
    if buf_logp.dim() != 2 or buf_logp.shape[0] != N or tuple(buf_val.shape) != tuple(buf_logp.shape):
        raise ValueError("buf_logp/buf_val must be [n_envs, horizon]")
    T = buf_logp.shape[1]
    _req(buf_act, "buf_act", torch.float32, (N, T, A) if dist == "gaussian" else (N, T))
    ld_env = _row_stride(env_in, "env_in", A)
    if env_in.dtype != torch.float32 or env_in.shape[0] != N:
        raise ValueError("env_in must be float32 [n_envs, act_dim]")
    if dist == "gaussian":
        _req(logstd, "logstd", torch.float32, (A,))
    rc = lib().xpa_rollout_sample(DIST[dist], N, A, T, _p(head), _p(logstd) if dist == "gaussian" else None, _p(v),
                                  _p(cursor), int(seed) & 0xFFFFFFFF, float(act_clip), _p(buf_act), _p(buf_logp),
                                  _p(buf_val), _p(env_in), ld_env, _stream(head.device))
    _lib.check(rc, "xpa_rollout_sample")


def rollout_policy_head(dist, z_actor, z_critic, act, w_actor, b_actor, w_critic, b_critic, logstd, cursor, seed,
                        buf_act, buf_logp, buf_val, env_in, act_clip=1.0):
    """K14: hidden activation + output layers + K3 sampling/store in one launch.  z_* [N, 256] hidden
    pre-activations with unit column stride and a common row stride; act = (code, slope)."""
    N, H = z_actor.shape
    ld = z_actor.stride(0)
    for name, z in (("z_actor", z_actor), ("z_critic", z_critic)):
        _req(z, name, torch.float32, contiguous=False)
        if tuple(z.shape) != (N, HEAD_HIDDEN) or z.stride() != (ld, 1):
            raise ValueError("%s must be [N, %d] with the same row stride" % (name, HEAD_HIDDEN))
    A = w_actor.shape[0]
    _req(w_actor, "w_actor", torch.float32, (A, H))
    _req(w_critic, "w_critic", torch.float32, (1, H))
    _req(cursor, "cursor", torch.int32, (4,))
    _req(buf_logp, "buf_logp", torch.float32)
    _req(buf_val, "buf_val", torch.float32)
    if buf_logp.dim() != 2 or buf_logp.shape[0] != N or tuple(buf_val.shape) != tuple(buf_logp.shape):
        raise ValueError("buf_logp/buf_val must be [n_envs, horizon]")
    T = buf_logp.shape[1]
    _req(buf_act, "buf_act", torch.float32, (N, T, A) if dist == "gaussian" else (N, T))
    ld_env = _row_stride(env_in, "env_in", A)
    if dist == "gaussian":
        _req(logstd, "logstd", torch.float32, (A,))
    rc = lib().xpa_rollout_policy_head(DIST[dist], act[0], N, A, T, H, ld, _p(z_actor), _p(z_critic), float(act[1]),
                                       _p(w_actor), _p(b_actor), _p(w_critic), _p(b_critic),
                                       _p(logstd) if dist == "gaussian" else None, _p(cursor), int(seed) & 0xFFFFFFFF,
                                       float(act_clip), _p(buf_act), _p(buf_logp), _p(buf_val), _p(env_in), ld_env,
                                       _stream(z_actor.device))
    _lib.check(rc, "xpa_rollout_policy_head")


def rollout_step_workspace(n_envs, obs_dim, rms, device):
    """K14F workspace (xpa_rollout_step_workspace): (partials f64, tickets int32 zeroed once; launches leave them 0)."""
    nt = ctypes.c_int64()
    nd = int(lib().xpa_rollout_step_workspace(int(n_envs), int(obs_dim), int(bool(rms)), ctypes.byref(nt)))
    if nd <= 0:
        raise ValueError("K14F needs 1 <= obs_dim <= 64")
    return (torch.empty(nd, dtype=torch.float64, device=device), torch.zeros(nt.value, dtype=torch.int32, device=device))


def _rollout_step_post(post, N, T, D, device):
    """The post-step argument tail of xpa_rollout_step_synthbox from `post` (a dict, see rollout_policy_head_synthbox)."""
    p = dict(post)
    S = _n_slots(p["slot_t"], N)
    _req(p["slot_obs"], "slot_obs", torch.float32, (S * N, D))
    _req(p["overflow"], "overflow", torch.int32, (1,))
    _req(p["obs_mean"], "obs_mean", torch.float32, (D,))
    _req(p["obs_var"], "obs_var", torch.float32, (D,))
    if p.get("obs_count") is not None:
        _req(p["obs_count"], "obs_count", torch.float64, (1,))
    ldn = _row_stride(p["boot_norm"], "boot_norm", D)
    for name in ("ret_mean", "ret_var"):
        _req(p[name], name, torch.float32, (1,))
    _req(p["ret_count"], "ret_count", torch.float64, (1,))
    _req(p["returns"], "returns", torch.float32, (N,))
    for name in ("buf_rew", "buf_term", "buf_boot"):
        _req(p[name], name, torch.float32, (N, T))
    _req(p["buf_closed"], "buf_closed", torch.uint8, (N, T))
    part, tickets = p["workspace"]
    nt = ctypes.c_int64()
    nd = int(lib().xpa_rollout_step_workspace(N, D, int(p.get("obs_count") is not None), ctypes.byref(nt)))
    _req(part, "part", torch.float64, (nd,))
    _req(tickets, "tickets", torch.int32, (nt.value,))
    return [_p(p["slot_obs"]), _p(p["slot_t"]), S, _p(p["overflow"]), int(bool(p.get("slot_from_next", False))),
            _p(p["obs_mean"]), _p(p["obs_var"]), _p(p.get("obs_count")), float(p["obs_clip"]), _p(p["boot_norm"]), ldn,
            _p(p["ret_mean"]), _p(p["ret_var"]), _p(p["ret_count"]), _p(p["returns"]), _p(p["buf_rew"]),
            _p(p["buf_term"]), _p(p["buf_closed"]), _p(p["buf_boot"]), float(p["gamma"]),
            int(bool(p.get("mask_returns", True))), int(bool(p.get("use_rewnorm", True))), float(p.get("rew_range", 5.0)),
            int(bool(p.get("atari_lifeloss", False))), _p(part), _p(tickets)]


def rollout_policy_head_synthbox(z_actor, z_critic, act, w_actor, b_actor, w_critic, b_critic, logstd, cursor, seed,
                                 buf_act, buf_logp, buf_val, env, act_clip=1.0, post=None):
    """K14 (Gaussian) + the SynthBox env step of envs.SynthBoxVecEnv `env` in one launch
    (xpa_rollout_policy_head_synthbox): same buffers as rollout_policy_head, then the env's state, final
    obs, reward, flags and episode counters exactly as env.step_device() after K14 would write them (the
    env pre-activation as a fixed-order chain instead of the GEMM: ulp-level differences).
    post (r06, K14F: xpa_rollout_step_synthbox): also K8's deferred, normalised post step in the same launch — a dict of
    rollout_post's deferred-norm arguments (slot_obs, slot_t, overflow, obs_mean, obs_var, obs_clip, boot_norm, ret_mean,
    ret_var, ret_count, returns, buf_rew, buf_term, buf_closed, buf_boot, gamma, mask_returns, use_rewnorm, rew_range,
    atari_lifeloss), slot_from_next (A2C: kept rows from the next observation), obs_count (or None: with it the next
    step's obs_rms.update as rollout_post(rms=...)), workspace = rollout_step_workspace(N, D, obs_count is not None)."""
    N, H = z_actor.shape
    ld = z_actor.stride(0)
    for name, z in (("z_actor", z_actor), ("z_critic", z_critic)):
        _req(z, name, torch.float32, contiguous=False)
        if tuple(z.shape) != (N, HEAD_HIDDEN) or z.stride() != (ld, 1):
            raise ValueError("%s must be [N, %d] with the same row stride" % (name, HEAD_HIDDEN))
    A = w_actor.shape[0]
    _req(w_actor, "w_actor", torch.float32, (A, H))
    _req(w_critic, "w_critic", torch.float32, (1, H))
    _req(cursor, "cursor", torch.int32, (4,))
    _req(logstd, "logstd", torch.float32, (A,))
    T = buf_logp.shape[1]
    _req(buf_act, "buf_act", torch.float32, (N, T, A))
    if env.num_envs != N or env.A != A or env.discrete:
        raise ValueError("the fused env step needs a continuous-action env of matching shape")
    from .envs import NOISE, TERM_THRESH, RESET_SCALE
    if post is not None:
        rc = lib().xpa_rollout_step_synthbox(
            act[0], N, A, T, H, ld, _p(z_actor), _p(z_critic), float(act[1]), _p(w_actor), _p(b_actor), _p(w_critic),
            _p(b_critic), _p(logstd), _p(cursor), int(seed) & 0xFFFFFFFF, float(act_clip), _p(buf_act), _p(buf_logp),
            _p(buf_val), env.D, _p(env.Wcat_t), env.noise_seed, env.max_episode_steps, NOISE, TERM_THRESH,
            RESET_SCALE, _p(env.X), env.X.stride(0), _p(env.final_obs), _p(env.rew), _p(env.term), _p(env.trunc),
            _p(env.ep_step), _p(env.ep_index), _p(env.ep_score), _p(env.ep_last_score), _p(env.ep_last_len),
            *_rollout_step_post(post, N, T, env.D, z_actor.device), _stream(z_actor.device))
        _lib.check(rc, "xpa_rollout_step_synthbox")
        return
    rc = lib().xpa_rollout_policy_head_synthbox(
        act[0], N, A, T, H, ld, _p(z_actor), _p(z_critic), float(act[1]), _p(w_actor), _p(b_actor), _p(w_critic),
        _p(b_critic), _p(logstd), _p(cursor), int(seed) & 0xFFFFFFFF, float(act_clip), _p(buf_act), _p(buf_logp),
        _p(buf_val), env.D, _p(env.Wcat_t), env.noise_seed, env.max_episode_steps, NOISE, TERM_THRESH,
        RESET_SCALE, _p(env.X), env.X.stride(0), _p(env.final_obs), _p(env.rew), _p(env.term), _p(env.trunc),
        _p(env.ep_step), _p(env.ep_index), _p(env.ep_score), _p(env.ep_last_score), _p(env.ep_last_len),
        _stream(z_actor.device))
    _lib.check(rc, "xpa_rollout_policy_head_synthbox")


def value_head(z_critic, act, w_critic, b_critic, out=None):
    """K14 value-only: v = act(z_critic) . w + b for every row."""
    N, H = z_critic.shape
    _req(z_critic, "z_critic", torch.float32, contiguous=False)
    if H != HEAD_HIDDEN or z_critic.stride(1) != 1:
        raise ValueError("z_critic must be [N, %d] with unit column stride" % HEAD_HIDDEN)
    _req(w_critic, "w_critic", torch.float32, (1, H))
    out = torch.empty((N,), dtype=torch.float32, device=z_critic.device) if out is None else out
    _req(out, "out", torch.float32, (N,))
    _lib.check(lib().xpa_value_head(act[0], N, H, z_critic.stride(0), _p(z_critic), float(act[1]), _p(w_critic),
                                    _p(b_critic), _p(out), _stream(z_critic.device)), "xpa_value_head")
    return out


def post_workspace(n_envs, device):
    """K8 workspace: (partials f64 [3 * blocks], ticket int32 [1] = 0)."""
    g = int(lib().xpa_rollout_post_num_blocks(n_envs))
    return (torch.zeros(3 * g, dtype=torch.float64, device=device), torch.zeros(1, dtype=torch.int32, device=device))


def rollout_post(rew, term, trunc, v_boot, cursor, ret_mean, ret_var, ret_count, returns, buf_rew, buf_term,
                 buf_closed, buf_boot, gamma, mask_returns=True, use_rewnorm=True, rew_range=5.0, atari_lifeloss=False,
                 deferred=None, workspace=None, v_boot_mid=None, rms=None):
    """K8: reward normalisation, return tracker + ret_rms, rewards/terminals/closures into the buffer
    column cursor.ptr, then cursor.ptr = (ptr + 1) % horizon, cursor.step += 1.
    deferred = (boot_obs [N, D] (row stride may exceed D), slot_obs [S N, D], slot_t int32 [S N], overflow
    int32 [1]): no v_boot; truncation rows are kept (up to S per env) for bootstrap_fixup after the rollout.
    workspace = post_workspace(N) (kept by the caller across steps; allocated here when None).
    v_boot_mid [N] (not deferred): the bootstrap values of closures before the rollout's last step (A2C's
    V(norm(reset_obs)), a2c_agent.py:88-95); v_boot is used at the last step (and everywhere when None).
    rms = (x [N, D] the observation the env step produced, obs_count f64 [1], rms_part f64 [2 * blocks, D]) with the
    8 / 9-element deferred form (r05, D <= 64): the next step's obs_rms.update folded in (obs_mean / obs_var of
    `deferred` and obs_count updated in place after the normalisation used the old statistics)."""
    N = rew.shape[0]
    _req(rew, "rew", torch.float32, (N,))
    _req(term, "term", torch.uint8, (N,))
    _req(trunc, "trunc", torch.uint8, (N,))
    if deferred is None:
        _req(v_boot, "v_boot", torch.float32, (N,))
    _req(cursor, "cursor", torch.int32, (4,))
    for name, t in (("ret_mean", ret_mean), ("ret_var", ret_var)):
        _req(t, name, torch.float32, (1,))
    _req(ret_count, "ret_count", torch.float64, (1,))
    _req(returns, "returns", torch.float32, (N,))
    T = buf_rew.shape[1]
    for name, t in (("buf_rew", buf_rew), ("buf_term", buf_term), ("buf_boot", buf_boot)):
        _req(t, name, torch.float32, (N, T))
    _req(buf_closed, "buf_closed", torch.uint8, (N, T))
    part, ticket = workspace if workspace is not None else post_workspace(N, rew.device)
    if deferred is not None and len(deferred) in (8, 9):
        # (final_obs RAW, slot_obs, slot_t, overflow, obs_mean, obs_var, obs_clip, boot_norm[, slot_src RAW]):
        # normalisation of the final observations folded into K8 (xpa_rollout_post_deferred_norm); slot_src (A2C:
        # the env's next observations) replaces final_obs as the source of kept truncation rows
        final_obs, slot_obs, slot_t, overflow, obs_mean, obs_var, obs_clip, boot_norm = deferred[:8]
        slot_src = deferred[8] if len(deferred) == 9 else None
        D = slot_obs.shape[1]
        S = _n_slots(slot_t, N)
        ldf = _row_stride(final_obs, "final_obs", D)
        ldn = _row_stride(boot_norm, "boot_norm", D)
        lds = _row_stride(slot_src, "slot_src", D) if slot_src is not None else 0
        _req(slot_obs, "slot_obs", torch.float32, (S * N, D))
        _req(overflow, "overflow", torch.int32, (1,))
        _req(obs_mean, "obs_mean", torch.float32, (D,))
        _req(obs_var, "obs_var", torch.float32, (D,))
        if rms is not None:
            rx, rcount, rpart = rms
            rld = _row_stride(rx, "rms_x", D)
            if rx.shape[0] != N:
                raise ValueError("rms_x must have one row per env")
            _req(rcount, "obs_count", torch.float64, (1,))
            _req(rpart, "rms_part", torch.float64, (2 * int(lib().xpa_rollout_post_num_blocks(N)), D))
            rc = lib().xpa_rollout_post_deferred_norm_rms(
                N, T, _p(rew), _p(term), _p(trunc), _p(final_obs), ldf, _p(slot_src), lds, D, _p(obs_mean),
                _p(obs_var), _p(rcount), float(obs_clip), _p(boot_norm), ldn, _p(slot_obs), _p(slot_t), S,
                _p(overflow), _p(cursor), _p(ret_mean), _p(ret_var), _p(ret_count), _p(returns), _p(buf_rew),
                _p(buf_term), _p(buf_closed), _p(buf_boot), float(gamma), int(bool(mask_returns)),
                int(bool(use_rewnorm)), float(rew_range), int(bool(atari_lifeloss)), _p(part), _p(ticket), _p(rx), rld,
                _p(rpart), _stream(rew.device))
            _lib.check(rc, "xpa_rollout_post_deferred_norm_rms")
            return
        rc = lib().xpa_rollout_post_deferred_norm(
            N, T, _p(rew), _p(term), _p(trunc), _p(final_obs), ldf, _p(slot_src), lds,
            D, _p(obs_mean), _p(obs_var), float(obs_clip),
            _p(boot_norm), ldn, _p(slot_obs), _p(slot_t), S, _p(overflow), _p(cursor), _p(ret_mean), _p(ret_var),
            _p(ret_count), _p(returns), _p(buf_rew), _p(buf_term), _p(buf_closed), _p(buf_boot), float(gamma),
            int(bool(mask_returns)), int(bool(use_rewnorm)), float(rew_range), int(bool(atari_lifeloss)), _p(part),
            _p(ticket), _stream(rew.device))
        _lib.check(rc, "xpa_rollout_post_deferred_norm")
        return
    if deferred is not None:
        boot_obs, slot_obs, slot_t, overflow = deferred
        D = slot_obs.shape[1]
        S = _n_slots(slot_t, N)
        ld = _row_stride(boot_obs, "boot_obs", D)
        _req(slot_obs, "slot_obs", torch.float32, (S * N, D))
        _req(overflow, "overflow", torch.int32, (1,))
        rc = lib().xpa_rollout_post_deferred(N, T, _p(rew), _p(term), _p(trunc), _p(boot_obs), ld, D, _p(slot_obs),
                                             _p(slot_t), S, _p(overflow), _p(cursor), _p(ret_mean), _p(ret_var),
                                             _p(ret_count), _p(returns), _p(buf_rew), _p(buf_term), _p(buf_closed),
                                             _p(buf_boot), float(gamma), int(bool(mask_returns)),
                                             int(bool(use_rewnorm)), float(rew_range), int(bool(atari_lifeloss)),
                                             _p(part), _p(ticket), _stream(rew.device))
        _lib.check(rc, "xpa_rollout_post_deferred")
        return
    if v_boot_mid is not None:
        _req(v_boot_mid, "v_boot_mid", torch.float32, (N,))
    rc = lib().xpa_rollout_post(N, T, _p(rew), _p(term), _p(trunc), _p(v_boot), _p(v_boot_mid), _p(cursor),
                                _p(ret_mean), _p(ret_var),
                                _p(ret_count), _p(returns), _p(buf_rew), _p(buf_term), _p(buf_closed), _p(buf_boot),
                                float(gamma), int(bool(mask_returns)), int(bool(use_rewnorm)), float(rew_range),
                                int(bool(atari_lifeloss)), _p(part), _p(ticket), _stream(rew.device))
    _lib.check(rc, "xpa_rollout_post")


def _n_slots(slot_t, N):
    """Deferred truncation slots per env of a slot_t buffer ([S N] or [S, N] int32, contiguous)."""
    _req(slot_t, "slot_t", torch.int32)
    if slot_t.numel() == 0 or slot_t.numel() % N:
        raise ValueError("slot_t must hold n_slots x n_envs entries")
    return slot_t.numel() // N


def bootstrap_fixup(values, slot_t, buf_term, buf_boot):
    """After a deferred rollout: values [(S + 1) N] = V(slot rows, slot-major) then V(last-step final obs);
    slot_t [S N] (S = slots per env)."""
    N, T = buf_boot.shape
    S = _n_slots(slot_t, N)
    _req(values, "values", torch.float32, ((S + 1) * N,))
    _req(buf_term, "buf_term", torch.float32, (N, T))
    _req(buf_boot, "buf_boot", torch.float32, (N, T))
    _lib.check(lib().xpa_rollout_bootstrap_fixup(N, T, _p(values), _p(slot_t), S, _p(buf_term), _p(buf_boot),
                                                 _stream(values.device)), "xpa_rollout_bootstrap_fixup")


def dqn_td_loss(evalQ, targetQ, act, rew, term, gamma, dQ=None, td_abs=None, scalars=None, err=None):
    """K19 (xpa_dqn_td_loss): the PER-DQN TD target / MSE loss / d loss d evalQ / |TD| of one batch
    (perdqn_learner.py:23-30).  evalQ / targetQ [B, A] f32 (row-strided allowed), act / rew / term [B] f32.
    Returns (dQ [B, A], td_abs [B], scalars [2] = (Qloss, predictQ mean)), all on device."""
    B, A = evalQ.shape
    ld_e = _row_stride(evalQ, "evalQ", A)
    ld_t = _row_stride(targetQ, "targetQ", A)
    for name, t in (("act", act), ("rew", rew), ("term", term)):
        _req(t, name, torch.float32, (B,))
    dQ = torch.empty((B, A), dtype=torch.float32, device=evalQ.device) if dQ is None else _req(dQ, "dQ",
                                                                                               torch.float32, (B, A))
    td_abs = torch.empty(B, dtype=torch.float32, device=evalQ.device) if td_abs is None else \
        _req(td_abs, "td_abs", torch.float32, (B,))
    scalars = torch.empty(2, dtype=torch.float32, device=evalQ.device) if scalars is None else \
        _req(scalars, "scalars", torch.float32, (2,))
    rc = lib().xpa_dqn_td_loss(B, A, _p(evalQ), ld_e, _p(targetQ), ld_t, _p(act), _p(rew), _p(term), float(gamma),
                               _p(dQ), A, _p(td_abs), _p(scalars), _p(err), _stream(evalQ.device))
    _lib.check(rc, "xpa_dqn_td_loss")
    return dQ, td_abs, scalars
