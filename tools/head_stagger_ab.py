"""r06: the K16Q heads (C2 minibatch, K = 6 actor, critic) timed with their second-slot blocks started late by
n x ~0.85 us (xpa_head_stagger), n swept, arms alternated; events around `reps` back-to-back launches.
python tools/head_stagger_ab.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    import torch
    from xuanpolicy_amd import _lib, ops
    dev = torch.device("cuda:0")
    B, H, K = 65536, 256, 6
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, H, device=dev, generator=g)
    wha, whc = (torch.randn(H, H, device=dev, generator=g) * 0.06 for _ in range(2))
    bha, bhc = (torch.randn(H, device=dev, generator=g) * 0.1 for _ in range(2))
    wa, ba = torch.randn(K, H, device=dev, generator=g) * 0.06, torch.zeros(K, device=dev)
    wc, bc = torch.randn(1, H, device=dev, generator=g) * 0.06, torch.zeros(1, device=dev)
    R = 4 * B
    act = torch.randn(R, K, device=dev, generator=g)
    adv, ret, old = (torch.randn(R, device=dev, generator=g) for _ in range(3))
    idx = torch.randperm(R, device=dev)[:B]
    logstd = torch.zeros(K, device=dev)
    ws = ops.HeadWorkspace(B, K, dev, paired=True)
    _, part = ops.gather_minibatch(idx, torch.zeros(R, 4, device=dev), adv=adv)
    L, s = ops.lib(), ops._stream(dev)
    W = ws.loss_partials.shape[1]
    spa, spc = ops.s3_split(wha.t()), ops.s3_split(whc.t())

    def actor():
        _lib.check(L.xpa_head_gemm_s3q_actor(0, 0, 1, B, K, H, ops._p(x), H, ops._p(spa), ops._p(bha), 2 * H, ops._p(wa),
                                             ops._p(ba), 0.01, ops._p(logstd), ops._p(idx), R, ops._p(act), ops._p(old),
                                             ops._p(adv), ops._p(part), part.shape[0], 0.2, 0.0, ops._p(ws.dz_actor),
                                             ops._p(ws.p_dw_actor), ops._p(ws.p_dbh_actor), ops._p(ws.p_dbo_actor),
                                             ops._p(ws.loss_partials), W, s), "actor")

    def critic():
        _lib.check(L.xpa_head_gemm_s3q_critic(1, B, H, ops._p(x), H, ops._p(spc), ops._p(bhc), 2 * H, ops._p(wc),
                                              ops._p(bc), 0.01, ops._p(idx), R, ops._p(ret), 0.25, ops._p(ws.dz_critic),
                                              ops._p(ws.p_dw_critic), ops._p(ws.p_dbh_critic), ops._p(ws.p_dbo_critic),
                                              ops._p(ws.loss_partials), W, s), "critic")

    def timed(fn, reps=40):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return round(e0.elapsed_time(e1) / reps * 1e3, 2)
    res = {}
    for rnd in range(2):
        for n in (0, 4, 8, 12, 16, 24):
            assert L.xpa_head_stagger(n) == 0
            res.setdefault(n, []).append((timed(actor), timed(critic)))
    L.xpa_head_stagger(0)
    print(json.dumps({"stagger_units_0.85us": res}), flush=True)
