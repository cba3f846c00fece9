"""Do the actor and critic head launches (K16Q) overlap when co-resident?  Times, at the C2 minibatch, the two
launches back to back on one stream vs on two streams (so their blocks can share CUs), and each alone.

    python tools/head_conc.py [--reps 30]"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    import torch
    from xuanpolicy_amd import ops
    L = ops.lib()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    B, H, K = 65536, 256, 6
    R = 4 * B
    x = torch.randn(B, H, device=dev, generator=g)
    wha, whc = (torch.randn(H, H, device=dev, generator=g) * 0.06 for _ in range(2))
    bha, bhc = (torch.randn(H, device=dev, generator=g) * 0.1 for _ in range(2))
    wa, ba = torch.randn(K, H, device=dev, generator=g) * 0.06, torch.zeros(K, device=dev)
    wc, bc = torch.randn(1, H, device=dev, generator=g) * 0.06, torch.zeros(1, device=dev)
    act = torch.randn(R, K, device=dev, generator=g)
    adv, ret, old = (torch.randn(R, device=dev, generator=g) for _ in range(3))
    idx = torch.randperm(R, device=dev)[:B]
    logstd = torch.zeros(K, device=dev)
    ws = ops.HeadWorkspace(B, K, dev, paired=True)
    _, part = ops.gather_minibatch(idx, torch.zeros(R, 4, device=dev), adv=adv)
    W = ws.loss_partials.shape[1]
    wsa, wsc = ops.s3_split(wha.t()), ops.s3_split(whc.t())
    mask = torch.empty((B, 8), dtype=torch.int32, device=dev)
    dv = torch.empty((B,), device=dev)
    p = ops._p
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def actor(st):
        sp = ctypes_stream(st)
        assert L.xpa_head_gemm_s3q_actor(0, 0, 1, B, K, H, p(x), H, p(wsa), p(bha), 2 * H, p(wa), p(ba), 0.01,
                                         p(logstd), p(idx), R, p(act), p(old), p(adv), p(part), part.shape[0], 0.2,
                                         0.0, p(ws.dz_actor), p(ws.p_dw_actor), p(ws.p_dbh_actor), p(ws.p_dbo_actor),
                                         p(ws.loss_partials), W, sp) == 0

    def critic(st):
        sp = ctypes_stream(st)
        assert L.xpa_head_gemm_s3q_critic_mask(1, B, H, p(x), H, p(wsc), p(bhc), 2 * H, p(wc), p(bc), 0.01, p(idx), R,
                                               p(ret), 0.25, None, p(ws.p_dw_critic), p(ws.p_dbh_critic),
                                               p(ws.p_dbo_critic), p(ws.loss_partials), W, sp, p(mask), p(dv)) == 0

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        import time
        t0 = time.perf_counter()
        for _ in range(a.reps):
            fn()
        torch.cuda.synchronize()
        return round((time.perf_counter() - t0) / a.reps * 1e6, 2)

    cur = torch.cuda.current_stream()

    def both_one():
        actor(cur)
        critic(cur)

    def both_two():
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        actor(s1)
        critic(s2)
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    res = {}
    for _ in range(3):
        for name, fn in (("actor", lambda: actor(cur)), ("critic", lambda: critic(cur)), ("both_one_stream", both_one),
                         ("both_two_streams", both_two)):
            res.setdefault(name, []).append(timed(fn))
    print(json.dumps(res), flush=True)


def ctypes_stream(st):
    import ctypes
    return ctypes.c_void_p(st.cuda_stream)


if __name__ == "__main__":
    main()
