"""A/B of the split GEMMs' k-loop forms at the C2 update shapes, alternating in one process (event-timed per launch).

    python tools/pp_ab.py [--reps 30] [--rounds 4] [--out gpurun_out/pp_ab.json] [--forms 0,256]

K40 (plain dX GEMM, dz_pair [65 536, 512] . Wh_pair) and K42S (the dX GEMM + the trunk backward from sign bits) under
xpa_s3_probe masks (0 = the production form; 256 = the ping-pong k loop; 128 = K42S's lookahead), and K41V (dW)."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def _time(fn, reps):
    import torch
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--forms", default="0,256")
    ap.add_argument("--wgrad-forms", default="0,256")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from xuanpolicy_amd import ops
    L = ops.lib()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    M, K, din = 65536, 512, 17
    dz = torch.randn(M, K, device=dev, generator=g)
    w = torch.randn(K, 256, device=dev, generator=g) / 16
    sp = ops.s3_split(w)
    out = torch.empty(M, 256, device=dev)
    xr = torch.randn(M, din, device=dev, generator=g)
    h = torch.randn(M, 256, device=dev, generator=g)
    bits = (h > 0).view(M, 8, 32).to(torch.int32)
    sign = (bits << torch.arange(8, device=dev, dtype=torch.int32).view(1, 8, 1)).sum(1).to(torch.uint8)
    sign = sign.contiguous().view(torch.int32).view(M, 8)
    S = ops.s3_wgrad_slices(M, K)
    part = torch.empty(S, K, 256, device=dev)
    forms = [int(f) for f in a.forms.split(",")]
    wforms = [int(f) for f in a.wgrad_forms.split(",")]
    res = {"k40": {f: [] for f in forms}, "k42s": {f: [] for f in forms}, "k41v": {f: [] for f in wforms}}
    for _ in range(a.rounds):
        for f in forms:
            assert L.xpa_s3_probe(f) == 0
            res["k40"][f].append(round(_time(lambda: ops.s3_gemm(dz, sp, K, out=out), a.reps), 2))
            res["k42s"][f].append(round(_time(lambda: ops.s3_gemm_trunk_bwd(dz, sp, K, None, xr, 1, 0.01, h_sign=sign),
                                              a.reps), 2))
        for f in wforms:
            assert L.xpa_s3_probe(f) == 0
            res["k41v"][f].append(round(_time(lambda: ops.s3_wgrad(dz, h, out=part), a.reps), 2))
    assert L.xpa_s3_probe(0) == 0
    flop6 = 6 * 2.0 * M * K * 256
    res["bf16x6_floor_us_at_2p5PF"] = round(flop6 / 2.5e15 * 1e6, 2)
    res = {k: ({str(f): v for f, v in d.items()} if isinstance(d, dict) else d) for k, d in res.items()}
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
