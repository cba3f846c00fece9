"""Probe the K28 / K29 conv kernels alone at the C3 update shapes (B = 16384): for rocprofv3 --kernel-trace / --pmc.
python tools/conv_probe.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    import torch
    from xuanpolicy_amd import _lib, ops
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda:0")
    L, s = ops.lib(), ops._stream(dev)
    B = 16384
    for (H, Cin, Cout, k, st) in ((21, 32, 64, 4, 2), (10, 64, 64, 3, 1)):
        p = (k - st) // 2
        OH = (H + 2 * p - k) // st + 1
        x = torch.rand(B, H, H, Cin, device=dev)
        w = torch.randn(Cout, Cin, k, k, device=dev) * 0.05
        b = torch.zeros(Cout, device=dev)
        y = torch.empty(B, OH, OH, Cout, device=dev)
        g = torch.randn(B, OH, OH, Cout, device=dev)
        G = int(L.xpa_conv_wgrad_num_partials())
        part = torch.empty(G, Cout * Cin * k * k, device=dev)
        dx = torch.empty(B, H, H, Cin, device=dev)
        Gd = int(L.xpa_conv_dgrad_num_partials(B, H, H))
        bp = torch.empty(Gd, Cin, device=dev)
        for _ in range(reps):
            _lib.check(L.xpa_conv_fwd(1, ops._p(x), B, H, H, Cin, ops._p(w), ops._p(b), Cout, k, st, p, 0.0, ops._p(y), s),
                       "fwd")
            # production: conv3 (stride 1) folds its own ReLU backward (act 1 + bias partials), conv2 gets dz from K28
            act = 1 if st == 1 else -1
            bpart = torch.empty(G, Cout, device=dev)
            _lib.check(L.xpa_conv_wgrad(act, ops._p(g), ops._p(y) if act >= 0 else None, 0.0, ops._p(x), B, H, H, Cin,
                                        Cout, k, st, p, ops._p(part), ops._p(bpart) if act >= 0 else None, s), "wgrad")
            if st == 1:
                _lib.check(L.xpa_conv_dgrad(ops._p(g), B, OH, OH, Cout, ops._p(w), Cin, k, st, p, H, H, 1, ops._p(x), 0.0,
                                            ops._p(dx), ops._p(bp), s), "dgrad")
        torch.cuda.synchronize()
    print("ok")
