"""Diagnostics for the head-kernel NaN seen in test_head_gemm_kernels_vs_fp64_autograd (K16W at 4133 / 777, K16S at
20037): runs each form on the test's inputs and prints which dz rows are non-finite (tile, row in tile, idx validity).

    python tools/nan_probe.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def case(algo, dist, K, B, code, form, reps=3):
    import torch
    from xuanpolicy_amd import ops
    DEV = torch.device("cuda:0")
    L, s = ops.lib(), ops._stream()
    g = torch.Generator(device=DEV).manual_seed(B + K)
    H, R = 256, B + 300
    x = torch.randn(B, H, device=DEV, generator=g)
    wh_a, wh_c = (torch.randn(H, H, device=DEV, generator=g) / 16 for _ in range(2))
    bh_a, bh_c = (torch.randn(H, device=DEV, generator=g) * 0.1 for _ in range(2))
    w_a = torch.randn(K, H, device=DEV, generator=g) / 16
    b_a = torch.randn(K, device=DEV, generator=g) * 0.1
    w_c = torch.randn(1, H, device=DEV, generator=g) / 16
    b_c = torch.randn(1, device=DEV, generator=g) * 0.1
    logstd = (-1 + 0.1 * torch.randn(K, device=DEV, generator=g)) if dist == "gaussian" else None
    idx = torch.randperm(R, device=DEV, generator=g)[:B].contiguous()
    idx[B // 2] = -1
    idx[B - 1] = R + 5
    adv = torch.randn(R, device=DEV, generator=g)
    ret = torch.randn(R, device=DEV, generator=g)
    act = (torch.randn(R, K, device=DEV, generator=g) * 0.5 if dist == "gaussian"
           else torch.randint(0, K, (R,), device=DEV, generator=g).float())
    old = -1.5 + 0.3 * torch.randn(R, device=DEV, generator=g) if algo == "ppo" else None
    G = int(L.xpa_head_fused_num_partials(B))
    W = int(L.xpa_loss_partial_width(K))
    pre = {"k16": "xpa_head_gemm_", "ws": "xpa_head_gemm_ws_", "s3": "xpa_head_gemm_s3_", "s3p": "xpa_head_gemm_s3p_"}[form]
    fa, fc = getattr(L, pre + "actor"), getattr(L, pre + "critic")
    wa, wc = (ops.s3_split(wh_a.t()), ops.s3_split(wh_c.t())) if form == "s3p" else (wh_a, wh_c)
    for rep in range(reps):
        dz = torch.full((B, 2 * H), 777.0, device=DEV)
        parts = [torch.full((G, n), 555.0, device=DEV) for n in (K * H, H, K, H, H, 1)]
        lp = torch.zeros(G, W, device=DEV)
        p = ops._p
        assert fa(ops.ALGO[algo], ops.DIST[dist], code, B, K, H, p(x), H, p(wa), p(bh_a), 2 * H, p(w_a), p(b_a), 0.01,
                  p(logstd), p(idx), R, p(act), p(old), p(adv), None, 0, 0.2, 0.01, p(dz), p(parts[0]), p(parts[1]),
                  p(parts[2]), p(lp), W, s) == 0
        assert fc(code, B, H, p(x), H, p(wc), p(bh_c), 2 * H, p(w_c), p(b_c), 0.01, p(idx), R, p(ret), 0.25,
                  p(dz[:, H:]), p(parts[3]), p(parts[4]), p(parts[5]), p(lp), W, s) == 0
        torch.cuda.synchronize()
        for half, name in ((slice(0, H), "actor"), (slice(H, 2 * H), "critic")):
            d = dz[:, half]
            bad = (~torch.isfinite(d)).any(1).nonzero().flatten().cpu()
            left = (d == 777.0).all(1).nonzero().flatten().cpu()
            if len(bad) or len(left):
                rows = bad.tolist()[:12]
                print("%s %s B=%d rep %d: %d non-finite rows %s (tiles %s, in-tile %s, idx %s), %d unwritten rows %s" % (
                    form, name, B, rep, len(bad), rows, [r // 64 for r in rows], [r % 64 for r in rows],
                    [int(idx[r]) for r in rows], len(left), left.tolist()[:8]), flush=True)
        for i, t in enumerate(parts + [lp]):
            if not torch.isfinite(t).all():
                print("%s B=%d rep %d: partial %d non-finite rows %s" % (
                    form, B, rep, i, (~torch.isfinite(t)).any(1).nonzero().flatten().tolist()[:8]), flush=True)
    print("done", form, B, flush=True)


def main():
    for args in [("ppo", "gaussian", 6, 4133, 1, "ws"), ("a2c", "categorical", 8, 777, 0, "ws"),
                 ("ppo", "gaussian", 6, 20037, 1, "s3"), ("ppo", "gaussian", 6, 20037, 1, "k16"),
                 ("ppo", "gaussian", 6, 20037, 1, "s3p"), ("ppo", "gaussian", 6, 4133, 1, "k16"),
                 ("ppo", "gaussian", 6, 4133, 1, "s3")]:
        case(*args)


if __name__ == "__main__":
    main()
