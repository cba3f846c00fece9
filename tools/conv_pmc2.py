"""Launch K28 (conv2 / conv3 forward) and K29 (conv2 / conv3 weight gradient) a few times at the C3 update's shapes
(B = 16384: conv2 32 -> 64, 4x4 s2 p1 on 21x21; conv3 64 -> 64, 3x3 s1 p1 on 10x10), for rocprofv3 --pmc passes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    import torch
    from xuanpolicy_amd import _lib, ops
    dev = torch.device("cuda:0")
    L, st = ops.lib(), ops._stream(dev)
    B = 16384
    x2 = torch.randn(B, 21, 21, 32, device=dev)
    w2, b2 = torch.randn(64, 32, 4, 4, device=dev) * 0.05, torch.zeros(64, device=dev)
    y2 = torch.empty(B, 10, 10, 64, device=dev)
    w3, b3 = torch.randn(64, 64, 3, 3, device=dev) * 0.05, torch.zeros(64, device=dev)
    y3 = torch.empty(B, 10, 10, 64, device=dev)
    g3 = torch.randn(B, 10, 10, 64, device=dev)
    G = int(L.xpa_conv_wgrad_num_partials())
    part2 = torch.empty(G, 64 * 32 * 16, device=dev)
    part3 = torch.empty(G, 64 * 64 * 9, device=dev)
    form = os.environ.get("XPA_IG_FORM")
    if form is not None:
        L.xpa_conv_igemm_form(int(form))
    for _ in range(3):
        _lib.check(L.xpa_conv_fwd(1, ops._p(x2), B, 21, 21, 32, ops._p(w2), ops._p(b2), 64, 4, 2, 1, 0.0, ops._p(y2), st),
                   "k28 conv2")
        _lib.check(L.xpa_conv_fwd(1, ops._p(y2), B, 10, 10, 64, ops._p(w3), ops._p(b3), 64, 3, 1, 1, 0.0, ops._p(y3), st),
                   "k28 conv3")
        _lib.check(L.xpa_conv_wgrad(-1, ops._p(g3), None, 0.0, ops._p(y2), B, 10, 10, 64, 64, 3, 1, 1, ops._p(part3), None,
                                    st), "k29 conv3")
        _lib.check(L.xpa_conv_wgrad(-1, ops._p(y2), None, 0.0, ops._p(x2), B, 21, 21, 32, 64, 4, 2, 1, ops._p(part2), None,
                                    st), "k29 conv2")
    torch.cuda.synchronize()
    print("ok")
