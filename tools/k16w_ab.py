"""K16 vs K16W vs K16S at the C2 minibatch shape (65 536 rows, hidden 256, Gaussian actor K = 6, PPO; critic), one process.

    python tools/k16w_ab.py [--reps 30] [--out gpurun_out/k16w_ab.json]

Per-launch device time from events around `reps` back-to-back launches of each kernel (actor, critic), alternating
the variants so that both see the same box state; under `rocprofv3 --kernel-trace --stats` the per-kernel rows give
the same numbers without the event timer's dispatch floor.  fp32 MFMA floor per head: 2 x 65 536 x 256 x 256 FLOP /
157.3 TFLOP/s = 54.6 us."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--out", default=None)
    ap.add_argument("--probe", action="store_true", help="also time K16W with parts switched off")
    ap.add_argument("--forms", default="k16,k16w,k16s,k16p,k16q")
    a = ap.parse_args()
    import torch
    from xuanpolicy_amd import ops
    dev = torch.device("cuda:0")
    L, s = ops.lib(), ops._stream(dev)
    B, H, K = a.batch, 256, 6
    R = 4096 * 128
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(B, H, device=dev, generator=g)
    wh_a, wh_c = (torch.randn(H, H, device=dev, generator=g) / 16 for _ in range(2))
    bh_a, bh_c = (torch.randn(H, device=dev, generator=g) * 0.1 for _ in range(2))
    w_a, b_a = torch.randn(K, H, device=dev, generator=g) / 16, torch.randn(K, device=dev, generator=g) * 0.1
    w_c, b_c = torch.randn(1, H, device=dev, generator=g) / 16, torch.randn(1, device=dev, generator=g) * 0.1
    logstd = -torch.ones(K, device=dev)
    idx = torch.randperm(R, device=dev, generator=g)[:B].contiguous()
    adv, ret = torch.randn(R, device=dev, generator=g), torch.randn(R, device=dev, generator=g)
    act = torch.randn(R, K, device=dev, generator=g) * 0.5
    old = -1.5 + 0.3 * torch.randn(R, device=dev, generator=g)
    G = int(L.xpa_head_fused_num_partials(B))
    Wd = int(L.xpa_loss_partial_width(K))
    dz = torch.empty(B, 2 * H, device=dev)
    parts = [torch.empty(G, n, device=dev) for n in (K * H, H, K, H, H, 1)]
    lp = torch.zeros(G, Wd, device=dev)
    p = ops._p

    pre = {False: "xpa_head_gemm_", True: "xpa_head_gemm_ws_", "s3": "xpa_head_gemm_s3_", "s3p": "xpa_head_gemm_s3p_", "s3q": "xpa_head_gemm_s3q_"}
    sp_a, sp_c = ops.s3_split(wh_a.t()), ops.s3_split(wh_c.t())   # K16P: Wh^T's planes

    def actor(ws):
        f = getattr(L, pre[ws] + "actor")
        return f(0, 0, 1, B, K, H, p(x), H, p(sp_a) if ws in ("s3p", "s3q") else p(wh_a), p(bh_a), 2 * H, p(w_a), p(b_a), 0.01, p(logstd), p(idx), R,
                 p(act), p(old), p(adv), None, 0, 0.2, 0.0, p(dz), p(parts[0]), p(parts[1]), p(parts[2]), p(lp), Wd, s)

    def critic(ws):
        f = getattr(L, pre[ws] + "critic")
        return f(1, B, H, p(x), H, p(sp_c) if ws in ("s3p", "s3q") else p(wh_c), p(bh_c), 2 * H, p(w_c), p(b_c), 0.01, p(idx), R, p(ret), 0.25,
                 p(dz[:, H:]), p(parts[3]), p(parts[4]), p(parts[5]), p(lp), Wd, s)

    res = {}
    for _ in range(a.rounds):
        fmap = {"k16": False, "k16w": True, "k16s": "s3", "k16p": "s3p", "k16q": "s3q"}
        for ws in [fmap[f] for f in a.forms.split(",")]:
            for name, fn in (("actor", actor), ("critic", critic)):
                assert fn(ws) == 0
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    fn(ws)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / a.reps
                res.setdefault("%s_%s" % ({False: "k16", True: "k16w", "s3": "k16s", "s3p": "k16p", "s3q": "k16q"}[ws], name), []).append(round(us, 2))
    if a.probe:   # K16W with parts switched off (xpa_head_gemm_ws_probe): 1 no epilogue, 2 no MFMA, 4 no DMA
        for mask in (1, 2, 4, 5, 3, 6, 7):
            assert L.xpa_head_gemm_ws_probe(mask) == 0
            for name, fn in (("actor", actor), ("critic", critic)):
                fn(True)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    fn(True)
                e1.record()
                torch.cuda.synchronize()
                res["k16w_%s_probe%d" % (name, mask)] = [round(e0.elapsed_time(e1) * 1e3 / a.reps, 2)]
        assert L.xpa_head_gemm_ws_probe(0) == 0
    floor = 2.0 * B * H * H / 157.3e12 * 1e6
    out = {"batch": B, "floor_us_per_head": round(floor, 2), "us_per_launch": res,
           "frac_of_fp32_mfma_peak": {k: round(floor / min(v), 3) for k, v in res.items()}}
    print(json.dumps(out))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
