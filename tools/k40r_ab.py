"""A/B of the rollout's paired hidden GEMM at C2's rollout shape ([4096, 256] x [256, 512]): K40R 2 stages x 4 chunks (default),
3 x 1 (xpa_s3_probe bit 512), 3 x 2 (bit 1024) and the f32 library GEMM (F.linear), alternating in one process, event-timed."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.nn.functional as F
    from xuanpolicy_amd import ops
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    x = torch.randn(M, 256, device=dev, generator=g)
    w = torch.randn(512, 256, device=dev, generator=g) / 16
    b = torch.randn(512, device=dev, generator=g)
    sa, sc = ops.s3_split(w[:256].t()), ops.s3_split(w[256:].t())
    out = torch.empty(M, 512, device=dev)
    L = ops.lib()

    def t(fn, reps=200):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) * 1e3 / reps, 2)

    res = {"k40r_2x4": [], "k40r_3x1": [], "k40r_3x2": [], "f_linear": []}
    for _ in range(5):
        for name, pr in (("k40r_2x4", 0), ("k40r_3x1", 512), ("k40r_3x2", 1024)):
            L.xpa_s3_probe(pr)
            res[name].append(t(lambda: ops.s3_gemm_rows_pair(x, sa, sc, b, out=out)))
        L.xpa_s3_probe(0)
        res["f_linear"].append(t(lambda: F.linear(x, w, b)))
    print(json.dumps({"M": M, **res}))


if __name__ == "__main__":
    main()
