"""Timing probe of K40T's phases at C2 (4096 rows, d_in 17): the fused launch, its prologue alone, it without the trunk
FMAs, and the two-launch form (thin_fwd_norm + K40R in its 2x4 and 3x2 forms); HIP events around 200 launches each."""
import torch

from xuanpolicy_amd import ops


def timed(fn, n=200):
    for _ in range(10):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    dev = torch.device("cuda:0")
    M, din = 4096, 17
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, din, device=dev, generator=g)
    mean, var = torch.zeros(din, device=dev), torch.ones(din, device=dev)
    W, b = torch.randn(256, din, device=dev, generator=g) * 0.2, torch.zeros(256, device=dev)
    sa = ops.s3_split(torch.randn(256, 256, device=dev, generator=g))
    sc = ops.s3_split(torch.randn(256, 256, device=dev, generator=g))
    bias = torch.zeros(512, device=dev)
    xn = torch.empty(M, din, device=dev)
    h = torch.empty(M, 256, device=dev)
    z = torch.empty(M, 512, device=dev)
    L = ops.lib()
    res = {}

    def fused():
        ops.s3_gemm_rows_pair_trunk(x, W, b, 1, 0.01, mean, var, 5.0, xn, None, 0, None, sa, sc, bias, out=z)

    def trunk():
        L.xpa_thin_linear_act_fwd_norm(1, ops._p(x), din, M, din, 256, ops._p(W), ops._p(b), 0.01, ops._p(h), 256,
                                       ops._p(mean), ops._p(var), 5.0, ops._p(xn), din, None, 0, None, ops._stream())

    def pair():
        ops.s3_gemm_rows_pair(h, sa, sc, bias, out=z)
    for name, bits, fn in (("k40t", 0, fused), ("k40t_no_trunk_fma", 4096, fused), ("k40t_prologue_only", 8192, fused),
                           ("thin_fwd_norm", 0, trunk), ("k40r_2x4", 0, pair), ("k40r_3x2", 1024, pair)):
        L.xpa_s3_probe(bits)
        res[name] = round(timed(fn), 2)
        L.xpa_s3_probe(0)
    print(res)


if __name__ == "__main__":
    main()
