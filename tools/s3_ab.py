"""K40 (f32 GEMM by a bf16 three-way split) vs torch's f32 GEMM (hipBLASLt) at the update's dX shape.

    python tools/s3_ab.py [--reps 30] [--out gpurun_out/s3_ab.json]

g = dz_pair [65 536, 512] . Wh_pair [512, 256] (C2 minibatch, paired hidden layer), plus K = 256.  Event-timed
per-launch device time over `reps` back-to-back launches, alternating the forms; under `rocprofv3 --kernel-trace
--stats` the per-kernel rows give the same numbers.  f32 MFMA floor: 2 M K N / 157.3 TFLOP/s; the split's bf16
floor: 6 x 2 M K N / 2.5 PFLOP/s."""
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--probe", action="store_true", help="also time K40 / K41 with parts switched off (xpa_s3_probe)")
    a = ap.parse_args()
    import torch
    from xuanpolicy_amd import ops
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    for (M, K) in ((65536, 512), (65536, 256)):
        x = torch.randn(M, K, device=dev, generator=g)
        w = torch.randn(K, 256, device=dev, generator=g) / 16
        out = torch.empty(M, 256, device=dev)
        sp = ops.s3_split(w)
        key = "M%d_K%d" % (M, K)
        r = res.setdefault(key, {"s3_us": [], "torch_us": [], "split_us": []})
        for _ in range(a.rounds):
            r["s3_us"].append(round(_time(lambda: ops.s3_gemm(x, sp, K, out=out), a.reps), 2))
            r["torch_us"].append(round(_time(lambda: torch.mm(x, w, out=out), a.reps), 2))
            r["split_us"].append(round(_time(lambda: ops.s3_split(w, out=sp), a.reps), 2))
        flop = 2.0 * M * K * 256
        r["f32_floor_us"] = round(flop / 157.3e12 * 1e6, 2)
        r["bf16x6_floor_us"] = round(6 * flop / 2.5e15 * 1e6, 2)
        r["s3_frac_of_f32_floor"] = round(r["f32_floor_us"] / min(r["s3_us"]), 3)
        r["torch_frac_of_f32_floor"] = round(r["f32_floor_us"] / min(r["torch_us"]), 3)
    # K41: dW = dz^T x (the paired hidden layer's weight gradient) vs the learner's split-K batched f32 GEMM (8 slices)
    B = 65536
    dz = torch.randn(B, 512, device=dev, generator=g)
    x_in = torch.randn(B, 256, device=dev, generator=g)
    x = x_in
    S = ops.s3_wgrad_slices(B, 512)
    part = torch.empty(S, 512, 256, device=dev)
    ws8 = torch.empty(8, 512, 256, device=dev)
    r = res.setdefault("wgrad_B%d_M512" % B, {"s3_us": [], "torch_bmm8_us": [], "slices": S})
    for _ in range(a.rounds):
        r["s3_us"].append(round(_time(lambda: ops.s3_wgrad(dz, x, out=part), a.reps), 2))
        r["torch_bmm8_us"].append(round(_time(lambda: torch.bmm(dz.view(8, B // 8, 512).transpose(1, 2),
                                                                  x.view(8, B // 8, 256), out=ws8), a.reps), 2))
    flop = 2.0 * B * 512 * 256
    r["f32_floor_us"] = round(flop / 157.3e12 * 1e6, 2)
    r["s3_frac_of_f32_floor"] = round(r["f32_floor_us"] / min(r["s3_us"]), 3)
    r["torch_frac_of_f32_floor"] = round(r["f32_floor_us"] / min(r["torch_bmm8_us"]), 3)
    if a.probe:   # 1 no MFMA, 2 no operand loads, 4 one MFMA instead of six; + 8: K40's two-block form / K41W; 16: K40W;
        # 64: K41V's interleaved schedule
        L = ops.lib()
        M, K = 65536, 512
        x = torch.randn(M, K, device=dev, generator=g)
        sp = ops.s3_split(torch.randn(K, 256, device=dev, generator=g) / 16)
        out = torch.empty(M, 256, device=dev)
        pr = res.setdefault("probe_us", {})
        for mask in (0, 1, 2, 3, 4, 6, 8, 9, 10, 11, 12, 16, 32, 64):
            assert L.xpa_s3_probe(mask) == 0
            pr["k40_%d" % mask] = round(_time(lambda: ops.s3_gemm(x, sp, K, out=out), a.reps), 2)
            if mask < 8 or mask in (8, 16, 64):
                pr["k41_%d" % mask] = round(_time(lambda: ops.s3_wgrad(dz, x_in, out=part), a.reps), 2)
        assert L.xpa_s3_probe(0) == 0
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
