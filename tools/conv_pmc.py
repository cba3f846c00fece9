"""Launch K25 / K26 / K27 a few times at the C3 update's shapes, for rocprofv3 --pmc passes:
    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES \
        SQ_INSTS_VALU SQ_INSTS_MFMA -- python tools/conv_pmc.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    import torch
    from xuanpolicy_amd import _lib, ops
    dev = torch.device("cuda:0")
    L, st = ops.lib(), ops._stream(dev)
    B = 16384
    x = torch.randint(0, 256, (B, 84, 84, 4), dtype=torch.uint8, device=dev)
    w1, b1 = torch.randn(32, 4, 8, 8, device=dev) * 0.05, torch.zeros(32, device=dev)
    y1 = torch.empty((B, 21, 21, 32), device=dev)
    g = torch.randn(B * 441, 32, device=dev)
    wpart = torch.empty(int(L.xpa_conv1_u8_wgrad_num_partials()), 8192, device=dev)
    dy2 = torch.randn(B, 10, 10, 64, device=dev)
    w2 = torch.randn(64, 32, 4, 4, device=dev) * 0.05
    dx2 = torch.empty((B, 21, 21, 32), device=dev)
    for _ in range(3):
        _lib.check(L.xpa_conv1_u8_fwd(1, ops._p(x), B, 84, 84, 4, 8, 4, 2, ops._p(w1), ops._p(b1), 32, 0.0, ops._p(y1),
                                      st), "k25")
        _lib.check(L.xpa_conv1_u8_wgrad(ops._p(g), ops._p(x), B, 84, 84, 4, 8, 4, 2, 32, ops._p(wpart), st), "k26")
        _lib.check(L.xpa_conv_dgrad_s2k(ops._p(dy2), B, 10, 10, 64, ops._p(w2), 32, 4, 2, 1, 21, 21, ops._p(dx2), st),
                   "k27")
    torch.cuda.synchronize()
    print("ok")
