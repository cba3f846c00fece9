"""Where K16's time goes: the fused hidden-GEMM + head kernels timed whole and with parts compiled out.

    python tools/head_probe.py build        # here (no GPU): tools/_probe/libxpa_probe{0..6}.so
    python tools/head_probe.py run          # on the GPU box: one child process per variant

Variants (head.hip, XPA_HEAD_PROBE): 0 the product kernel, 1 the GEMM alone (staging + MFMA, result
kept live), 2 the epilogue alone (no GEMM), 3 operand staging alone (no MFMA), 4 the epilogue without its
dz stores, 5 the epilogue without phase 2, 6 the GEMM without its operand DMAs (MFMA stream on stale LDS).

r01 findings (65 536 rows, fp32 MFMA floor 54.6 us per head at 2.4 GHz): register-staged K16 actor 134 /
critic 99 us = GEMM 92 (staging 37, not overlapped with the MFMAs) + epilogue 40 / 16 (not overlapped
either).  A register-direct variant (no LDS staging) ran its GEMM in 110-122 us: SQ_WAIT_INST_ANY 88 % of
wave cycles — in-loop VGPR-destination loads stall MFMA issue.
LDS-DMA 3-stage ring (current): actor 121-124 / critic 92-94; GEMM alone 89-92 / 84-88; MFMA stream without
the DMAs 68-74 (so the loop itself reaches ~80 % of the floor and the DMAs add ~17 us); staging alone
26-31; epilogue alone 39 / 15 (phase 1 + loss 20 / 9 after batching the head-weight scalar loads, which
had been one branch + load + wait per output).  Rejected: per-wave private operand rings (each wave
DMAs its own A copy + its B rows, no k-loop barrier): GEMM 100 / 92, worse — the 4x A re-reads cost more
than the barriers (MFMA stream alone only 70 / 66 without them).
r03: fragment prefetch (chunk c + 1's ds_reads in flight during chunk c's MFMAs, DMAs two chunks ahead,
measured as an A/B variant and dropped): GEMM alone 88.5 / 88.2 vs 89.0 / 86.1, full 115.9 / 97.3 vs 113.8 / 98.0
— the fragment reads' latency was not what bounds the loop.  hipBLASLt's own F.linear of the same
[65 536 x 256] x [256 x 256] shape: 82.6 us (0.66 of the floor) — K16's GEMM is within 7 % of it.
Shape: the C2
minibatch (65 536 rows, hidden 256, Gaussian actor K = 6, PPO); per-launch device time from events
around `reps` back-to-back launches."""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
OUT = os.path.join(HERE, "_probe")
VARIANTS = {0: "full", 1: "gemm only", 2: "epilogue only", 3: "staging only", 4: "epilogue without dz stores",
            5: "epilogue without phase 2", 6: "gemm without operand DMAs", 7: "K16P without its B-plane DMAs",
            8: "K16P without the A split (f32 bits as bf16)", 9: "K16P without the A split and without DMAs",
            10: "epilogue without phase 1", 11: "epilogue without the loss",
            12: "gemm only without the A split (f32 bits as bf16)"}
# XPA_PROBE_FORM=s3p times the K16P entries (Wh as its bf16 planes, r04) instead of the f32 K16 ones
FORM = os.environ.get("XPA_PROBE_FORM", "k16")
FLAGS = {}   # variant -> hipcc defines, when not just -DXPA_HEAD_PROBE=<variant>
# variant subset: XPA_PROBE_VARIANTS=0,1,7 (default all)
_sel = os.environ.get("XPA_PROBE_VARIANTS")
if _sel:
    VARIANTS = {int(v): VARIANTS[int(v)] for v in _sel.split(",")}


def build():
    from xuanpolicy_amd import _lib
    os.makedirs(OUT, exist_ok=True)
    procs = []
    for v in VARIANTS:
        cmd = ([os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")] + _lib.HIPCC_FLAGS + ["-shared"] + FLAGS.get(v, ["-DXPA_HEAD_PROBE=%d" % v]) + ["-o",
               os.path.join(OUT, "libxpa_probe%d.so" % v)] + [os.path.join(_lib.CSRC, s) for s in _lib.SOURCES])
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        if p.wait() != 0:
            raise SystemExit("probe build failed")


def child(v, reps=30):
    import torch
    from xuanpolicy_amd import _lib, ops
    _lib.load(os.path.join(OUT, "libxpa_probe%d.so" % v))
    dev = torch.device("cuda:0")
    B, H, K = 65536, 256, int(os.environ.get("XPA_PROBE_K", "6"))   # XPA_PROBE_K=17: C4's actor head
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
    L, s = _lib.load(), ops._stream(dev)
    W = ws.loss_partials.shape[1]

    pre = "xpa_head_gemm_%s_" % FORM if FORM in ("s3p", "s3q") else "xpa_head_gemm_"
    fa, fc = getattr(L, pre + "actor"), getattr(L, pre + "critic")
    if FORM in ("s3p", "s3q"):
        wha, whc = ops.s3_split(wha.t()), ops.s3_split(whc.t())

    def actor():
        _lib.check(fa(0, 0, 1, B, K, H, ops._p(x), H, ops._p(wha), ops._p(bha), 2 * H, ops._p(wa),
                                         ops._p(ba), 0.01, ops._p(logstd), ops._p(idx), R, ops._p(act), ops._p(old),
                                         ops._p(adv), ops._p(part), part.shape[0], 0.2, 0.0, ops._p(ws.dz_actor),
                                         ops._p(ws.p_dw_actor), ops._p(ws.p_dbh_actor), ops._p(ws.p_dbo_actor),
                                         ops._p(ws.loss_partials), W, s), "actor")

    def critic():
        _lib.check(fc(1, B, H, ops._p(x), H, ops._p(whc), ops._p(bhc), 2 * H, ops._p(wc),
                                          ops._p(bc), 0.01, ops._p(idx), R, ops._p(ret), 0.25, ops._p(ws.dz_critic),
                                          ops._p(ws.p_dw_critic), ops._p(ws.p_dbh_critic), ops._p(ws.p_dbo_critic),
                                          ops._p(ws.loss_partials), W, s), "critic")

    res = {}
    fns = [("actor", actor), ("critic", critic)]
    if v == 0 and FORM not in ("s3p", "s3q"):   # the library GEMM of the same shape, for reference
        import torch.nn.functional as F
        fns.append(("hipblaslt_linear_256x256", lambda: F.linear(x, wha, bha)))
    for name, fn in fns:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        res[name] = round(e0.elapsed_time(e1) / reps * 1e3, 2)
    flops = 2.0 * B * H * H
    res["gemm_floor_us_at_peak"] = round(flops / 157.3e6, 2)
    print(json.dumps({"variant": VARIANTS[v], "form": FORM, "K": K, **res}), flush=True)


def run():
    for v in VARIANTS:
        subprocess.run([sys.executable, __file__, "child", str(v)], check=True, timeout=300)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    elif sys.argv[1] == "child":
        child(int(sys.argv[2]))
    else:
        run()
