#!/usr/bin/env python
"""Benchmark: end-to-end PPO-Clip env-steps/s at num_envs=4096, horizon=128 (BASELINE.json config C2:
SynthBox(obs=17, act=6), ppo/mujoco.yaml hyper-parameters: n_epoch 16, n_minibatch 8, [256] nets,
LeakyReLU, Adam eps=1e-5, LinearLR) plus the GAE kernel's HBM roofline.

A "step" is one PPO iteration on every rank: 128 env steps of the 4096-env device-resident rollout
(obs-RMS + normalise, policy forward, action sample, env step, bootstrap critic, bookkeeping), the GAE
scan over [4096, 128], then 16 epochs x 8 minibatches of 65 536 (gather, heads forward, fused loss
fwd+bwd kernel, MLP backward, [RCCL all-reduce], grad-clip, Adam, LinearLR).  Inputs start resident in
HBM (the env lives on the GPU).  value = env-steps processed by all ranks / max-over-ranks wall time.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N ... bench.py --gpus N ...     (one process per GPU, RCCL)
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (MI355X_MICROARCH.md; the 2:1-sparsity figure is not used)
FP32_MFMA_PEAK_TFLOPS = 157.3  # dense f32-input MFMA (= f32 vector rate; no xf32 on gfx950), same table
# r06 (tools/clock_probe.hip, profiles/r06/clock/): the clock a dense v_mfma_f32_32x32x16_bf16 loop on random data holds
# (in-kernel s_memtime / s_memrealtime, known-cycle and GRBM_GUI_ACTIVE methods agree on >= 20 ms dispatches) against the
# 2.4 GHz the peak assumes; reported beside `frac` as the bf16 peak the split kernels can reach on this part
BF16_MFMA_LOOP_CLOCK_GHZ, PEAK_CLOCK_GHZ = 1.86, 2.4


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=8)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--n-envs", type=int, default=4096)
    p.add_argument("--horizon", type=int, default=128)
    p.add_argument("--obs-dim", type=int, default=17)
    p.add_argument("--act-dim", type=int, default=6)
    p.add_argument("--hidden", type=int, default=256)
    p.add_argument("--n-epoch", type=int, default=16)
    p.add_argument("--n-minibatch", type=int, default=8)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-updates", type=int, default=24, help="updates timed in the bounded CPU sample")
    p.add_argument("--no-sweep", action="store_true")
    p.add_argument("--no-per", action="store_true", help="skip the C5 PER (K6) measurement")
    p.add_argument("--no-c1", action="store_true", help="skip the C1 CartPole measurement")
    p.add_argument("--no-c3", action="store_true", help="skip the C3 Atari A2C measurement")
    p.add_argument("--no-c4", action="store_true", help="skip the C4 Box(376,17) measurement")
    p.add_argument("--no-kernel-timing", action="store_true")
    p.add_argument("--out", default=None, help="also write the JSON line to this file")
    p.add_argument("--gae-form", choices=("k40v", "value", "split"), default="value",
                   help="k40v (r06, opt-in: the scan faster, the K40V launch before it slower than value's GEMM): the deferred bootstraps' critic to the value on the split GEMM (K40V, the value "
                        "head in its epilogue), then the compact GAE scan (K1) on exactly the §8(d) bytes; value: the "
                        "value head fused into the GAE scan (K1V, one launch); split: hipBLASLt + value head (K14) "
                        "then the compact GAE scan")
    p.add_argument("--trunk-heads", choices=("on", "off"), default="off",
                   help="K16X (trunk layer inside the head GEMM launches) or r03's K13 forward + K16 (A/B)")
    p.add_argument("--gemm", choices=("f32", "split3"), default="split3",
                   help="the update's hidden-layer GEMMs: f32 MFMA (K16 + hipBLASLt) or the bf16 three-way split "
                        "(K16S + K40 + K41, the f32 GEMM's accuracy on the bf16 matrix cores)")
    p.add_argument("--s3-heads", choices=("s3", "s3p", "s3q"), default="s3q",
                   help="with --gemm split3: K16S (both fragments split in the k loop), K16P (Wh's planes split once) or "
                        "K16Q (K16P with 32 x 128 wave tiles, bit-identical)")
    p.add_argument("--thin-store", choices=("nt", "plain"), default="nt",
                   help="K13's h stores: non-temporal (default) or plain (A/B; xpa_thin_probe)")
    p.add_argument("--dz-store", choices=("nt", "plain"), default="nt",
                   help="the head kernels' dz stores: non-temporal (default) or plain (A/B; xpa_head_store_probe)")
    p.add_argument("--s3-probe", type=int, default=0, help="xpa_s3_probe mask for A/B runs (0: the production forms)")
    p.add_argument("--pair-sa", type=int, default=0, help="K41P's actor share of 128 slices (0: the default)")
    p.add_argument("--crit-factored", choices=("on", "off"), default="on",
                   help="the critic's factored backward (K41P / K42C, r05) or its dz_critic through K41V / K42S")
    p.add_argument("--sync-obs-rms", choices=("off", "step", "rollout"), default="off",
                   help="world > 1: obs_rms synchronised across ranks per env step (outside the graphs) or per rollout")
    p.add_argument("--global-advnorm", choices=("on", "off"), default="off",
                   help="world > 1: each minibatch's advantage moments averaged across ranks (a second collective)")
    p.add_argument("--fuse-post", choices=("on", "off"), default="on",
                   help="K14F: K8's post step + the next obs_rms.update inside the env-fused K14 launch (r06)")
    p.add_argument("--fold-rms", choices=("on", "off"), default="off",
                   help="the next step's obs-RMS update folded into K8 (r05 opt-in, measured neutral) or its own launch")
    p.add_argument("--rollout-h-store", choices=("plain", "nt"), default="nt",
                   help="the rollout trunk's h stores: non-temporal (default) or plain (A/B; xpa_thin_probe bit 2)")
    p.add_argument("--rollout-split", choices=("on", "off"), default="on",
                   help="the rollout's paired hidden GEMM on the split (K40R, r05) or the f32 library GEMM")
    p.add_argument("--wide-trunk", choices=("on", "off"), default="on",
                   help="C4's 376-wide trunk layer on the split GEMMs (K40F / K42W / K41V, r05) or the f32 library GEMMs")
    p.add_argument("--dp-path", choices=("on", "off"), default="on",
                   help="at world 1: also time C2 with the data-parallel update path attached (distributed.LocalGradSync: "
                        "its own clip-norm pass, eager K9; no collective) -> dp_update_path")
    p.add_argument("--no-pmc", action="store_true", help="skip the live rocprofv3 --pmc HBM-traffic passes")
    p.add_argument("--no-rocprof", action="store_true",
                   help="skip the child rocprofv3 --kernel-trace run that times the in-loop GAE launches")
    return p.parse_args()


def gae_bytes(n_envs, horizon, mid_truncations):
    """20 B per (env, step) + 4 B per env (last bootstrap) + 4 B per mid-buffer
    truncation bootstrap."""
    return 20.0 * n_envs * horizon + 4.0 * n_envs + 4.0 * mid_truncations


def loss_bytes_gauss(batch, act_dim):
    """Gaussian loss fwd+bwd = 4 (3A + 5) B per sample."""
    return 4.0 * (3 * act_dim + 5) * batch


def heads_bytes(batch, act_dim, hidden=256):
    """K12 actor + critic launches per minibatch: each reads its hidden
    pre-activations and writes dz (2 x 4 x hidden B per row); the actor reads act (4A), old_logp,
    adv and idx (4 + 4 + 8), the critic ret and idx (4 + 8)."""
    return batch * (2 * 2 * 4 * hidden + 4 * act_dim + 16 + 12)


def pair_gemm_flops(batch, d_in, hidden=256):
    """Paired actor|critic hidden-layer forward GEMM: [B, d_in] x [d_in, 2 hidden]."""
    return 2.0 * batch * d_in * 2 * hidden


def gae_value_bytes(n_envs, horizon, mid_truncations, hidden=256):
    """K1V (xpa_gae_scan_value): K1's bytes + the critic hidden pre-activations of the deferred pass it reads to
    form the bootstrap values, 2 n_envs rows x hidden f32 (every env's truncation-slot row and last-step row:
    the critic pass runs at a fixed [2N, D] shape) + the output layer."""
    return gae_bytes(n_envs, horizon, mid_truncations) + 4.0 * (2 * n_envs * hidden + hidden + 1)


def gae_graph_replay_us(agent, reps=50):
    """The in-loop GAE launch alone (the form the agent ran), `reps` launches on the agent's live buffers captured
    back to back in one hipGraph (no host dispatch gaps between launches), timed with events on the replay
    stream."""
    import torch
    from xuanpolicy_amd import ops
    mem = agent.memory
    adv, ret = torch.empty_like(mem.rewards), torch.empty_like(mem.rewards)
    slot = torch.full((mem.n_envs,), -1, dtype=torch.int32, device=mem.rewards.device)
    vboot = torch.zeros(2 * mem.n_envs, device=mem.rewards.device)
    boot = torch.empty_like(mem.rewards)
    form = getattr(agent, "gae_form", "compact")
    if form == "value":
        fm = agent.learner._fused_mlp()
        zc = fm.rollout_value_hidden(agent._boot_pair)
        lin_co = fm.critic[-1][0]
        act = fm.critic[-2][1:]

        def launch():  # slots empty after the rollout's GAE
            ops.gae_scan_value(mem.rewards, mem.values, mem.terminals, slot, zc, act, lin_co.weight, lin_co.bias,
                               mem.gamma, mem.gae_lam, mem.use_gae, adv=adv, ret=ret, boot=boot)
    else:
        def launch():  # the compact-closure form; slots empty after the rollout's GAE
            ops.gae_scan_compact(mem.rewards, mem.values, mem.terminals, slot, vboot, mem.gamma, mem.gae_lam,
                                 mem.use_gae, adv=adv, ret=ret, boot=boot)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        launch()        # warm
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            for _ in range(reps):
                launch()
        g.replay()
        side.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(200000)
        e0.record(side)
        g.replay()
        e1.record(side)
        e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def live_gae_traffic(form, timeout_s=150):
    """roofline.traffic measured in this run: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE: separate passes,
    the TCC block cannot hold both) over tools/gae_pmc.py --quick (the GAE launch at the bench size, 4096 x 128,
    caches evicted by a 512 MiB read before each launch), each in a child process under `timeout -s KILL`; the
    gfx950 corrections of MI355X_MICROARCH.md §HBM (FETCH_SIZE in KiB, half of a wide streaming read -> x2;
    WRITE_SIZE exact for 16-B stores) applied by tools/pmc_summary.py.  Returns (per-launch HBM bytes or None,
    note)."""
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None, "rocprofv3 not found"
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import pmc_summary
    tmp = tempfile.mkdtemp(prefix="xpa_pmc_")
    dirs = {}
    env = dict(os.environ, TMPDIR="/tmp")
    for ctr, tag in (("FETCH_SIZE", "f"), ("WRITE_SIZE", "w")):
        d = os.path.join(tmp, tag)
        cmd = ["timeout", "-s", "KILL", str(timeout_s), exe, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o",
               tag, "--", sys.executable, os.path.join(REPO, "tools", "gae_pmc.py"), "--quick"]
        try:
            r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=timeout_s + 30)
        except Exception as e:   # noqa: BLE001 - reported, never fatal to the bench line
            return None, "pmc pass %s failed: %r" % (ctr, e)
        if r.returncode != 0:
            return None, "pmc pass %s exited %d: %s" % (ctr, r.returncode, r.stderr[-300:])
        dirs[ctr] = d
    out = os.path.join(tmp, "pmc.json")
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        pmc_summary.main(dirs["FETCH_SIZE"], dirs["WRITE_SIZE"], out)
    with open(out) as f:
        res = json.load(f)
    key = "hbm_bytes_per_launch_" + ("value" if form == "value" else "compact")
    return res.get(key), "live rocprofv3 --pmc passes over tools/gae_pmc.py --quick (%s form, 4096 x 128)" % form


def live_gae_rocprof(args, timeout_s=300, form=None):
    """The in-loop GAE launch timed by the profiler: a child `rocprofv3 --kernel-trace` run of this bench (same
    workload and GAE form, 2 warmup + 8 timed iterations, no side measurements); the average kernel-trace duration of
    the 8 timed in-loop GAE launches (r05: 8, from 3).  Returns (avg us, [us, ...], note) or (None, None, note)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None, None, "rocprofv3 not found"
    tmp = tempfile.mkdtemp(prefix="xpa_kt_")
    cmd = ["timeout", "-s", "KILL", str(timeout_s), exe, "--kernel-trace", "--output-format", "csv", "-d", tmp, "-o",
           "run", "--", sys.executable, os.path.abspath(__file__), "--steps", "8", "--warmup", "2", "--gae-form",
           form or args.gae_form, "--n-envs", str(args.n_envs), "--horizon", str(args.horizon), "--obs-dim", str(args.obs_dim),
           "--act-dim", str(args.act_dim), "--hidden", str(args.hidden), "--n-epoch", str(args.n_epoch),
           "--n-minibatch", str(args.n_minibatch), "--no-pmc", "--no-rocprof", "--no-cpu-baseline", "--no-sweep",
           "--no-per", "--no-c1", "--no-c3", "--no-c4", "--no-kernel-timing"]
    try:
        r = subprocess.run(cmd, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), capture_output=True, text=True,
                           timeout=timeout_s + 30)
    except Exception as e:   # noqa: BLE001 - reported, never fatal to the bench line
        return None, None, "rocprofv3 child run failed: %r" % (e,)
    files = glob.glob(os.path.join(tmp, "**", "*kernel_trace.csv"), recursive=True)
    if r.returncode != 0 or not files:
        return None, None, "rocprofv3 child run exited %d: %s" % (r.returncode, r.stderr[-300:])
    rows = [x for x in csv.DictReader(open(files[0])) if "gae_dpp_kernel" in x["Kernel_Name"]]
    rows.sort(key=lambda x: int(x["Start_Timestamp"]))
    dur = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3 for x in rows[:10]]
    if len(dur) < 10:
        return None, None, "expected 10 in-loop GAE launches in the trace, found %d" % len(dur)
    timed = dur[2:10]
    return sum(timed) / len(timed), [round(d, 3) for d in timed], (
        "rocprofv3 --kernel-trace of a child run of this bench (same workload, --gae-form %s; 2 warmup + 8 timed "
        "iterations): the 8 timed in-loop GAE launches" % (form or args.gae_form))


def cache_flush(flush, mode):
    """Evict the caches before a timed launch.  "read": sum a 512 MiB buffer (other data replaces ours in L2 and
    the Infinity Cache and leaves nothing dirty); "write": fill it (the evicting lines are dirty, so the timed
    kernel's own misses also pay their write-back to HBM); "none": nothing."""
    if mode == "read":
        flush.sum()
    elif mode == "write":
        flush.fill_(1.0)


def loss_sweep(device, sizes=(65536, 262144, 1048576, 4194304), act_dim=6, reps=7, flush_mode="read"):
    """K2 alone (xpa_policy_loss_fwd_bwd, Gaussian PPO, rows in order: the drop-in learners' form; the C2
    fast path fuses the loss into K16's epilogue instead), caches flushed (cache_flush: 512 MiB read) before each
    timed launch.
    Inputs as SURVEY.md §8(d): mu ~ N(0, 0.5), logstd = -1 + N(0, 0.1), actions drawn around mu, adv / ret / v
    ~ N(0, 1)."""
    import torch
    from xuanpolicy_amd import _lib, ops
    flush = torch.ones(512 * 1024 * 1024 // 4, dtype=torch.float32, device=device)
    for _ in range(2):
        flush.sum()   # written once; read passes leave it clean
    L = ops.lib()
    s = ops._stream(device)
    out = []
    A = act_dim
    for B in sizes:
        g = torch.Generator(device=device).manual_seed(B + 1)
        mu = torch.randn(B, A, device=device, generator=g) * 0.5
        logstd = -1.0 + 0.1 * torch.randn(A, device=device, generator=g)
        act = mu + torch.exp(logstd) * torch.randn(B, A, device=device, generator=g)
        old = torch.randn(B, device=device, generator=g) * 0.3 - 2.0
        adv, ret, v = (torch.randn(B, device=device, generator=g) for _ in range(3))
        ws = ops.LossWorkspace(B, A, device, "gaussian")
        times = []
        for _ in range(reps):
            cache_flush(flush, flush_mode)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = L.xpa_policy_loss_fwd_bwd(ops.ALGO["ppo"], ops.DIST["gaussian"], B, A, ops._p(mu), ops._p(logstd),
                                           ops._p(v), None, B, ops._p(act), ops._p(old), ops._p(adv), ops._p(ret),
                                           None, 0, 0.2, 0.25, 0.0, ops._p(ws.d_head), ops._p(ws.d_v),
                                           ops._p(ws.partials), s)
            e1.record()
            _lib.check(rc, "xpa_policy_loss_fwd_bwd")
            e1.synchronize()
            times.append(e0.elapsed_time(e1))
        times.sort()
        ms = times[len(times) // 2]
        b = loss_bytes_gauss(B, A)
        out.append({"batch": B, "act_dim": A, "ms": round(ms, 5), "GB/s": round(b / ms / 1e6, 1),
                    "frac": round(b / ms / 1e6 / HBM_PEAK_GBS, 3), "algorithmic_bytes": int(b)})
        del mu, logstd, act, old, adv, ret, v, ws
    del flush
    torch.cuda.empty_cache()
    return out


def gae_sweep(device, sizes=(4096, 65536, 262144, 1048576), horizon=128, reps=7, flush_mode="read"):
    """GAE kernel alone (the in-loop compact form, ~1/8 of the rows with a mid-buffer truncation),
    caches flushed (cache_flush: 512 MiB read) before each timed launch."""
    import torch
    from xuanpolicy_amd import ops
    flush = torch.ones(512 * 1024 * 1024 // 4, dtype=torch.float32, device=device)
    for _ in range(2):
        flush.sum()   # written once; read passes leave it clean
    out = []
    for N in sizes:
        g = torch.Generator(device=device).manual_seed(N)
        rew = torch.randn(N, horizon, device=device, generator=g)
        val = torch.randn(N, horizon, device=device, generator=g)
        term = (torch.rand(N, horizon, device=device, generator=g) < 0.01).float()
        vboot = torch.randn(2 * N, device=device, generator=g)
        slot0 = torch.where(torch.rand(N, device=device, generator=g) < 0.125,
                            torch.randint(0, horizon - 1, (N,), device=device, generator=g), -1).to(torch.int32)
        slot = torch.empty_like(slot0)
        adv = torch.empty_like(rew)
        ret = torch.empty_like(rew)
        boot = torch.empty_like(rew)
        mid = int((slot0 >= 0).sum())
        times = []
        for _ in range(reps):
            slot.copy_(slot0)
            cache_flush(flush, flush_mode)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.gae_scan_compact(rew, val, term, slot, vboot, 0.99, 0.95, True, adv=adv, ret=ret, boot=boot)
            e1.record()
            e1.synchronize()
            times.append(e0.elapsed_time(e1))
        times.sort()
        ms = times[len(times) // 2]
        b = gae_bytes(N, horizon, mid)
        out.append({"n_envs": N, "horizon": horizon, "ms": round(ms, 5), "GB/s": round(b / ms / 1e6, 1),
                    "frac": round(b / ms / 1e6 / HBM_PEAK_GBS, 3), "algorithmic_bytes": int(b)})
        del rew, val, term, vboot, slot0, slot, adv, ret, boot
    del flush
    torch.cuda.empty_cache()
    return out


def per_bench(device, n_envs=8, n_size=131072, batch=2048, frames=True, reps=50):
    """C5 (BASELINE.json configs[4]): K6 on 8 x 131 072 = 1 M transitions, batch 2048, f64 trees.
    Times xpa_per_sample and xpa_per_update_priorities (HIP events over `reps` back-to-back calls on
    the launch stream), the K4 gather of 2048 uint8 4x84x84 frame pairs (obs + next obs) out of the
    1 M-transition replay, and the restated reference (oracle/per_ref.py, the reference's Python trees)
    on one host core for the same sample + update."""
    import torch
    from xuanpolicy_amd import ops
    from xuanpolicy_amd.per import PerOffPolicyBuffer

    class _Space:
        def __init__(self, shape):
            self.shape = shape
    buf = PerOffPolicyBuffer(_Space((4, 84, 84) if frames else (1,)), _Space(()), {}, n_envs, n_size, batch, 0.6,
                             device=device, obs_dtype=torch.uint8)
    cap = buf.capacity
    g = torch.Generator(device=device).manual_seed(0)
    buf.sum_tree[:, cap:] = torch.rand((n_envs, cap), generator=g, device=device, dtype=torch.float64) + 0.05
    buf.min_tree[:, cap:] = buf.sum_tree[:, cap:]
    lvl = cap
    while lvl > 1:
        half = lvl // 2
        buf.sum_tree[:, half:lvl] = buf.sum_tree[:, lvl:2 * lvl:2] + buf.sum_tree[:, lvl + 1:2 * lvl:2]
        buf.min_tree[:, half:lvl] = torch.minimum(buf.min_tree[:, lvl:2 * lvl:2], buf.min_tree[:, lvl + 1:2 * lvl:2])
        lvl = half
    buf.size, buf.ptr = n_size, 0
    prio = torch.rand(batch, generator=g, device=device) * 4
    steps, flat, _ = buf.sample_indices(0.4)
    torch.cuda.synchronize()

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3
    t_sample = timed(lambda: buf.sample_indices(0.4))
    t_update = timed(lambda: buf.update_priorities(steps, prio, check=False))
    res = {"config": "C5: %d envs x %d slots (%d transitions, capacity 2^%d per env), batch %d, f64 trees" %
                     (n_envs, n_size, n_envs * n_size, cap.bit_length() - 1, batch),
           "sample_us": round(t_sample, 2), "update_priorities_us": round(t_update, 2),
           "bound": "latency (log2(capacity) dependent tree levels per draw / update)"}
    if frames:
        obs_rows = buf.observations.reshape(n_envs * n_size, -1)
        out = torch.empty((batch, obs_rows.shape[1]), dtype=torch.uint8, device=device)
        t_gather = timed(lambda: (ops.gather_minibatch(flat, obs_rows, obs_out=out),
                                  ops.gather_minibatch(flat, buf.next_observations.reshape(n_envs * n_size, -1),
                                                       obs_out=out)))
        gb = 2 * 2 * batch * obs_rows.shape[1]
        res.update({"gather_frames_us": round(t_gather, 2), "gather_bytes": gb,
                    "gather_GBps": round(gb / t_gather / 1e3, 1), "gather_frac_of_hbm_peak":
                    round(gb / t_gather / 1e3 / HBM_PEAK_GBS, 4)})
    del buf
    torch.cuda.empty_cache()
    # restated reference on the host (one core, the reference is single-threaded Python)
    sys.path.insert(0, REPO)
    import numpy as np
    from oracle.per_ref import PerBufferRef
    ref = PerBufferRef(n_envs, n_size, batch, 0.6, obs_shape=(1,))
    rng = np.random.default_rng(0)
    for i in range(n_envs):
        vals = list(rng.random(cap) + 0.05)
        ref.it_sum[i].value[cap:] = vals
        ref.it_min[i].value[cap:] = vals
        for node in range(cap - 1, 0, -1):
            ref.it_sum[i].value[node] = ref.it_sum[i].value[2 * node] + ref.it_sum[i].value[2 * node + 1]
            ref.it_min[i].value[node] = min(ref.it_min[i].value[2 * node], ref.it_min[i].value[2 * node + 1])
    ref.size = n_size
    t0 = time.perf_counter()
    st, _ = ref.sample_indices(0.4, rng.random(batch))
    t1 = time.perf_counter()
    ref.update_priorities(st.astype(np.int64), rng.random(batch).astype(np.float32) * 4)
    t2 = time.perf_counter()
    res["cpu_reference_restated"] = {"sample_us": round((t1 - t0) * 1e6, 1), "update_priorities_us":
                                     round((t2 - t1) * 1e6, 1), "cores": 1, "kind": "port"}
    res["speedup_sample_update"] = round(((t2 - t0) * 1e6) / (t_sample + t_update), 1)
    return res


def c1_bench(device, n_envs=8, n_steps=128, hidden=64, steps=5, warmup=3, cpu=True):
    """C1 (BASELINE.json configs[0]): PPO-Clip on CartPole-v1, 8 envs x 128 steps, ppo/classic_control/
    CartPole-v1.yaml (8 epochs x 8 minibatches of 128), [64] nets, on device (K18 env, K3 sampling, K1 GAE,
    K2 / K9 updates) — and the same loop on the host as the reference runs it (oracle/cpu_ref.AgentLoopRef over
    per-env CartPoleEnv objects, torch-CPU learner): the reference's own CPU-runnable configuration.  Three untimed
    iterations first: the rollout chunk graph and the per-slot update graphs are captured there, not in the timed
    region."""
    import numpy as np
    import torch
    from xuanpolicy_amd.runner import build_cartpole_ppo
    agent = build_cartpole_ppo(n_envs=n_envs, n_steps=n_steps, hidden=hidden, device=device)
    cfg = agent.config
    for _ in range(warmup):
        agent.train(n_steps, log=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        agent.train(n_steps, log=False)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    res = {"workload": "PPO-Clip CartPole-v1 num_envs=%d horizon=%d, ppo/classic_control/CartPole-v1.yaml (n_epoch %d, "
                       "n_minibatch %d), nets [%d] LeakyReLU" % (n_envs, n_steps, cfg.n_epoch, cfg.n_minibatch,
                                                               hidden),
           "metric": "env-steps/s", "value": round(n_envs * n_steps * steps / el, 1),
           "ms_per_iteration": round(el / steps * 1e3, 2), "iterations": steps, "dtype": "f32 (f64 env state)"}
    del agent
    if cpu:
        from oracle import cpu_ref, synth_env
        torch.manual_seed(1)
        np.random.seed(1)
        nthreads = torch.get_num_threads()
        torch.set_num_threads(1)     # 128-row minibatches: one thread is the reference's fastest setting here
        envs = [synth_env.CartPoleEnv(i, seed=1) for i in range(n_envs)]
        pol = cpu_ref.build_actor_critic_ref(4, 2, [hidden], [hidden], [hidden], discrete=True)
        opt = torch.optim.Adam(pol.parameters(), cfg.learning_rate, eps=1e-5)
        sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.0, total_iters=cfg.running_steps)
        lrn = cpu_ref.LearnerRef(pol, opt, sch, "ppo", cfg.vf_coef, cfg.ent_coef, cfg.clip_range, cfg.clip_grad_norm,
                                 True)
        loop = cpu_ref.AgentLoopRef(envs, pol, lrn, n_steps, cfg.n_epoch, cfg.n_minibatch, cfg.gamma, cfg.gae_lambda)
        loop.run_steps(n_steps)          # warm-up iteration
        t0 = time.perf_counter()
        loop.run_steps(2 * n_steps)
        el_cpu = time.perf_counter() - t0
        torch.set_num_threads(nthreads)
        res["cpu_reference_loop"] = {"value": round(n_envs * n_steps * 2 / el_cpu, 1), "unit": "env-steps/s",
                                     "cores": 1, "kind": "port", "sample": "2 full iterations (%d updates) of the "
                                     "restated reference loop after one warm-up iteration" % (2 * cfg.n_epoch *
                                                                                            cfg.n_minibatch)}
        res["speedup_vs_cpu"] = round(res["value"] / res["cpu_reference_loop"]["value"], 2)
    torch.cuda.empty_cache()
    return res


def c5_bench(device, n_envs=8, n_size=131072, batch=2048, steps=20, warmup=3, cpu_updates=3, tree_cpu_us=None):
    """C5 (BASELINE.json configs[4]): the PER-DQN training step at full size — replay 8 x 131 072 = 1 M uint8
    4x84x84 transitions (obs + next: 56 GB in HBM), batch 2048, 18 actions, BasicQnetwork over Basic_CNN
    [32, 64, 64] / q_hidden [512] (perdqn/atari.yaml).  One step = one env step of the 8 envs + store (K6 store)
    + sample (K6) + K4 frame gathers + eval / target Q forwards + K19 + backward + Adam + K6 priority update, the
    agent loop with start_training = 0 and train_frequency 1 over a replay pre-filled to capacity (frames and
    leaf priorities synthetic).  CPU leg: the restated reference learner (oracle PerDQNLearnerRef, torch CPU)
    on `cpu_updates` batches of 2048 plus the reference's Python trees (oracle/per_ref) for the same calls."""
    import numpy as np
    import torch
    from xuanpolicy_amd.runner import build_perdqn
    agent = build_perdqn(n_envs=n_envs, n_size=n_size, batch_size=batch, device=device, start_training=0,
                         sync_frequency=500)
    mem = agent.memory
    cap = mem.capacity
    g = torch.Generator(device=device).manual_seed(0)
    mem.sum_tree[:, cap:cap + n_size] = torch.rand((n_envs, n_size), generator=g, device=device,
                                                   dtype=torch.float64) + 0.05
    mem.min_tree[:, cap:cap + n_size] = mem.sum_tree[:, cap:cap + n_size]
    lvl = cap
    while lvl > 1:
        half = lvl // 2
        mem.sum_tree[:, half:lvl] = mem.sum_tree[:, lvl:2 * lvl:2] + mem.sum_tree[:, lvl + 1:2 * lvl:2]
        mem.min_tree[:, half:lvl] = torch.minimum(mem.min_tree[:, lvl:2 * lvl:2], mem.min_tree[:, lvl + 1:2 * lvl:2])
        lvl = half
    mem.size, mem.ptr = n_size, 0
    agent.train(warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    agent.train(steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    res = {"workload": "PER-DQN SynthAtari(4x84x84 uint8, 18 actions), replay %d x %d = %d transitions, batch %d, "
                       "BasicQnetwork Basic_CNN [32,64,64]/[8,4,3]/[4,2,1] + q [512], perdqn/atari.yaml" %
                       (n_envs, n_size, n_envs * n_size, batch),
           "metric": "learner steps/s (one env step of %d envs + one batch-%d update each)" % (n_envs, batch),
           "value": round(steps / el, 2), "ms_per_step": round(el / steps * 1e3, 3),
           "env_steps_per_s": round(steps * n_envs / el, 1), "steps": steps, "dtype": "f32 (uint8 frames)",
           "replay_bytes_in_hbm": int(2 * mem.observations.numel())}
    del agent, mem
    torch.cuda.empty_cache()
    if cpu_updates:
        from oracle import cpu_ref
        torch.manual_seed(0)
        pol = cpu_ref.build_qnetwork_ref(18, [32, 64, 64], [8, 4, 3], [4, 2, 1], [512])
        opt = torch.optim.Adam(pol.parameters(), 1e-4, eps=1e-5)
        lrn = cpu_ref.PerDQNLearnerRef(pol, opt, None, 0.99, 500)
        rng = np.random.default_rng(0)
        obs = rng.integers(0, 256, (batch, 84, 84, 4), dtype=np.uint8)
        nxt = rng.integers(0, 256, (batch, 84, 84, 4), dtype=np.uint8)
        act = rng.integers(0, 18, batch).astype(np.float32)
        rew = rng.normal(0, 1, batch).astype(np.float32)
        term = np.zeros(batch, np.float32)
        lrn.update(obs, act, rew, nxt, term)      # warm-up
        t0 = time.perf_counter()
        for _ in range(cpu_updates):
            lrn.update(obs, act, rew, nxt, term)
        t_upd = (time.perf_counter() - t0) / cpu_updates
        t_tree = (tree_cpu_us or 0.0) * 1e-6
        res["cpu_reference_step"] = {"value": round(1.0 / (t_upd + t_tree), 3), "unit": "learner steps/s",
                                     "cores": torch.get_num_threads(), "kind": "port",
                                     "sample": "%d batch-%d PerDQN_Learner updates (restated, torch CPU) %.3f s each "
                                               "+ one PER sample + priority update of the reference's Python trees "
                                               "%.3f s (per_kernels.cpu_reference_restated; the frame gather and "
                                               "env step not counted)"
                                               % (cpu_updates, batch, t_upd, t_tree)}
        res["speedup_vs_cpu"] = round(res["value"] / res["cpu_reference_step"]["value"], 1)
    return res


def c3_bench(device, n_envs=1024, n_steps=128, steps=2, warmup=1, cpu=True, kernels=True):
    """C3 (BASELINE.json configs[2]): A2C, SynthAtari uint8 4x84x84 frames, AC_CNN_Atari, 1024 envs x
    128 steps (a2c/atari.yaml: 4 epochs x 8 minibatches of 16 384), everything resident on the GPU."""
    import torch
    from xuanpolicy_amd.runner import build_atari_a2c
    agent = build_atari_a2c(n_envs=n_envs, n_steps=n_steps, device=device)
    for _ in range(warmup):
        agent.train(n_steps)
    torch.cuda.synchronize()
    agent.timers = {"rollout": 0.0, "update": 0.0}
    t0 = time.perf_counter()
    for _ in range(steps):
        agent.train(n_steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    res = {"workload": "A2C SynthAtari(4x84x84 uint8, 6 actions) num_envs=%d horizon=%d, a2c/atari.yaml (n_epoch 4, "
                       "n_minibatch 8), AC_CNN_Atari [32,64,64]/[8,4,3]/[4,2,1] + fc 512" % (n_envs, n_steps),
           "metric": "env-steps/s", "value": round(n_envs * n_steps * steps / el, 1),
           "ms_per_iteration": round(el / steps * 1e3, 2), "iterations": steps, "dtype": "f32 (uint8 frames)",
           "host_timer_split_ms": {k: round(v / steps * 1e3, 2) for k, v in agent.timers.items()}}
    del agent
    torch.cuda.empty_cache()
    if kernels:
        res["roofline"] = c3_kernels(device)
    if cpu:
        res["cpu_baseline"] = c3_cpu_baseline(n_envs, n_steps)
        res["speedup_vs_cpu"] = round(res["value"] / res["cpu_baseline"]["value"], 1)
    return res


def c3_cpu_baseline(n_envs=1024, n_steps=128, n_epoch=4, n_minibatch=8, steps_timed=3, updates_timed=2):
    """The C3 loop as the reference runs it on the host (a2c_agent.py:57-107): per-env SynthAtari stepping
    (DummyVecEnv_Atari), the AC_CNN_Atari policy forward on NumPy frames / 255.0 (cnn.py:89-92), the buffer column
    store and fancy-index sample (memory_tools.py:526-560), and A2C_Learner.update (autograd, clip_grad_norm_,
    Adam) on torch CPU — restated in oracle/cpu_ref (build_atari_ac_ref, LearnerRef).  Bounded sample:
    `steps_timed` env steps of all envs and `updates_timed` minibatch updates (B = N T / n_minibatch), extrapolated
    to one iteration (n_steps steps + n_epoch n_minibatch updates)."""
    import numpy as np
    import torch
    from oracle import cpu_ref, synth_env
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    K = 6
    pol = cpu_ref.build_atari_ac_ref(K)
    opt = torch.optim.Adam(pol.parameters(), 7e-4, eps=1e-5)
    lrn = cpu_ref.LearnerRef(pol, opt, None, "a2c", 0.25, 0.01, 0.0, 0.2, True)
    envs = [synth_env.SynthAtariEnv(i, seed=1, n_actions=K, max_episode_steps=27000) for i in range(n_envs)]
    obs = np.stack([e.reset()[0] for e in envs])
    col = np.zeros_like(obs)
    t_act = t_env = t_store = 0.0
    for _ in range(steps_timed):
        t0 = time.perf_counter()
        with torch.no_grad():
            logits, _, v = pol.heads(obs)
            a = torch.distributions.Categorical(logits=logits).sample().numpy()
        t1 = time.perf_counter()
        nxt = []
        for i, e in enumerate(envs):
            o, r, te, tr, info = e.step(int(a[i]))
            if tr:
                o = e.reset()[0]
            nxt.append(o)
        nxt = np.stack(nxt)
        t2 = time.perf_counter()
        col[:] = obs
        t3 = time.perf_counter()
        obs = nxt
        t_act, t_env, t_store = t_act + t1 - t0, t_env + t2 - t1, t_store + t3 - t2
    B = n_envs * n_steps // n_minibatch
    rng = np.random.default_rng(0)
    pool = rng.integers(0, 256, (2 * B,) + obs.shape[1:], dtype=np.uint8)
    t_upd = []
    for _ in range(updates_timed):
        t0 = time.perf_counter()
        idx = rng.permutation(2 * B)[:B]
        ob = pool[idx]
        act, ret, adv = rng.integers(0, K, B), rng.normal(0, 1, B).astype(np.float32), rng.normal(0, 1, B)
        adv = ((adv - adv.mean()) / (adv.std() + 1e-8)).astype(np.float32)
        lrn.update(ob, act, ret, adv)
        t_upd.append(time.perf_counter() - t0)
    step_s = (t_act + t_env + t_store) / steps_timed
    upd_s = sum(t_upd) / len(t_upd)
    it_s = n_steps * step_s + n_epoch * n_minibatch * upd_s
    return {"value": round(n_envs * n_steps / it_s, 1), "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": "%d env steps of %d envs (policy forward %.3f s, per-env SynthAtari step %.3f s, store %.3f s per "
                      "step) + %d A2C updates at B=%d (%.2f s each, incl. the fancy-index sample) -> iteration = %d x "
                      "%.3f s + %d x %.2f s = %.1f s" % (steps_timed, n_envs, t_act / steps_timed, t_env / steps_timed,
                                                         t_store / steps_timed, updates_timed, B, upd_s, n_steps,
                                                         step_s, n_epoch * n_minibatch, upd_s, it_s)}


def c3_kernels(device, batch=16384):
    """The C3 update's hand-written kernels at its shapes (minibatch of `batch` frames): K25 conv1 forward from uint8,
    K26 conv1 weight gradient from uint8, K27 conv2 data gradient (fp32 MFMA: FLOP / time vs the fp32 matrix peak) and
    K22 (ReLU backward + bias sums over conv1's [B*21*21, 32]; HBM).  HIP events around single launches on the launch
    stream, median of 7 (the buffers exceed every cache)."""
    import torch
    from xuanpolicy_amd import _lib, ops
    L = ops.lib()
    st = ops._stream(device)
    x = torch.randint(0, 256, (batch, 84, 84, 4), dtype=torch.uint8, device=device)
    rows, C = batch * 21 * 21, 32
    w1, b1 = torch.randn(32, 4, 8, 8, device=device) * 0.05, torch.zeros(32, device=device)
    y1 = torch.empty((batch, 21, 21, 32), device=device)
    g = torch.randn(rows, C, device=device)
    h = torch.relu(torch.randn(rows, C, device=device))
    part = torch.empty(int(L.xpa_act_bwd_bias_num_partials(rows, C)), C, device=device)
    wpart = torch.empty(int(L.xpa_conv1_u8_wgrad_num_partials()), 8192, device=device)
    dy2 = torch.randn(batch, 10, 10, 64, device=device)
    w2 = torch.randn(64, 32, 4, 4, device=device) * 0.05
    dx2 = torch.empty((batch, 21, 21, 32), device=device)

    def timed(fn, reps=7):
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        return ts[len(ts) // 2]
    form0 = int(L.xpa_conv1_form(-1))
    f_us, w_us = {}, {}
    try:
        for bit, tag in ((1, "bf16"), (0, "f32")):   # r05: K25B / K26B (bf16 matrix cores) and the fp32-MFMA forms
            L.xpa_conv1_form((form0 & ~3) | (3 if bit else 0))
            f_us[tag] = timed(lambda: _lib.check(L.xpa_conv1_u8_fwd(1, ops._p(x), batch, 84, 84, 4, 8, 4, 2, ops._p(w1),
                                                                    ops._p(b1), 32, 0.0, ops._p(y1), st), "conv1_u8_fwd"))
            w_us[tag] = timed(lambda: _lib.check(L.xpa_conv1_u8_wgrad(ops._p(g), ops._p(x), batch, 84, 84, 4, 8, 4, 2, 32,
                                                                      ops._p(wpart), st), "conv1_u8_wgrad"))
    finally:
        L.xpa_conv1_form(form0)
    d_us = {}
    try:
        for bit, tag in ((4, "bf16"), (0, "f32")):   # r05: K27B and the fp32-MFMA K27
            L.xpa_conv1_form((form0 & ~4) | bit)
            d_us[tag] = timed(lambda: _lib.check(L.xpa_conv_dgrad_s2k(ops._p(dy2), batch, 10, 10, 64, ops._p(w2), 32, 4,
                                                                      2, 1, 21, 21, ops._p(dx2), st), "conv_dgrad_s2k"))
    finally:
        L.xpa_conv1_form(form0)
    b_us = timed(lambda: _lib.check(L.xpa_act_bwd_bias(1, ops._p(g), ops._p(h), rows, C, 0.0, ops._p(g), ops._p(part),
                                                       st), "act_bwd_bias"))
    c1_flops = 2.0 * rows * 256 * 32            # [rows, 8*8*4] x [256, 32]
    c2_flops = 2.0 * batch * 21 * 21 * 32 * 256  # every input pixel: 4 taps x 64 channels
    bb = 12.0 * rows * C

    def mfma(name, us, flops, shape):
        return {"kernel": name, "bound": "mfma", "avg_launch_us": round(us, 2), "flops_per_launch": flops,
                "achieved": round(flops / us / 1e6, 1), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(flops / us / 1e6 / FP32_MFMA_PEAK_TFLOPS, 4), "shape": shape}
    def bf16(name, us, flops, shape, planes=3):
        # `planes` bf16 products per f32 product (3: the frames are exact in bf16; 6: both operands split), priced on
        # the bf16 matrix peak
        r = {"kernel": name, "bound": "mfma", "avg_launch_us": round(us, 2), "flops_per_launch": flops * planes,
             "achieved": round(flops * planes / us / 1e6, 1), "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
             "frac": round(flops * planes / us / 1e6 / BF16_MFMA_PEAK_TFLOPS, 4), "shape": shape,
             "f32_equivalent_tflops": round(flops / us / 1e6, 1)}
        return r

    c1s = "%d frames 84x84x4 uint8 -> [B, 21, 21, 32] (8x8 s4 p2, bias + ReLU)" % batch
    c1w = "dW [32, 4, 8, 8] over %d x 441 rows" % batch
    return {"conv1_u8_fwd": bf16("xpa_conv1_u8_fwd (K25B: 3 bf16 products, the weight split)", f_us["bf16"],
                                 c1_flops, c1s),
            "conv1_u8_fwd_f32": mfma("xpa_conv1_u8_fwd (K25, fp32 MFMA form)", f_us["f32"], c1_flops, c1s),
            "conv1_u8_wgrad": bf16("xpa_conv1_u8_wgrad (K26B: 3 bf16 products, the dz split; partials + f64 "
                                   "finalize)", w_us["bf16"], c1_flops, c1w),
            "conv1_u8_wgrad_f32": mfma("xpa_conv1_u8_wgrad (K26, fp32 MFMA form)", w_us["f32"], c1_flops, c1w),
            "conv_dgrad_s2k": bf16("xpa_conv_dgrad_s2k (K27B: 6 bf16 products, both operands split)", d_us["bf16"],
                                   c2_flops, "dX [B, 21, 21, 32] from dY [B, 10, 10, 64], 4x4 s2 p1", planes=6),
            "conv_dgrad_s2k_f32": mfma("xpa_conv_dgrad_s2k (K27, fp32 MFMA form)", d_us["f32"], c2_flops,
                                       "dX [B, 21, 21, 32] from dY [B, 10, 10, 64], 4x4 s2 p1"),
            "act_bwd_bias": {"kernel": "xpa_act_bwd_bias (K22, ReLU)", "bound": "hbm", "avg_launch_us": round(b_us, 2),
                             "algorithmic_bytes_per_launch": int(bb), "achieved": round(bb / b_us / 1e3, 1),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(bb / b_us / 1e3 / HBM_PEAK_GBS, 4),
                             "shape": "conv1 output [%d x 21 x 21, 32] (dh, h read, dz written: 12 B per element)"
                                      % batch}}


def c4_bench(device, rank, world, n_envs=4096, n_steps=128, steps=2, warmup=1):
    """C4 (BASELINE.json configs[3]): PPO-Clip SynthBox(obs=376, act=17), 4096 envs per GPU, the env shards
    of all ranks trained together with one all-reduce of the flat gradient per minibatch (every rank runs
    this; max-over-ranks wall time).  At world = 1 it is one GPU's shard of the 8-GPU configuration."""
    import torch
    import torch.distributed as dist
    from xuanpolicy_amd.distributed import broadcast_parameters
    from xuanpolicy_amd.runner import build_synthbox_ppo
    agent = build_synthbox_ppo(n_envs=n_envs, n_steps=n_steps, obs_dim=376, act_dim=17, hidden=256, seed=2,
                               device=device, shard=rank)
    agent.learner.enable_fast_path()
    if world > 1:
        broadcast_parameters(agent.policy)
    for _ in range(warmup):
        agent.train(n_steps)
    torch.cuda.synchronize()
    gs = agent.learner.grad_sync
    c0 = gs.collectives if gs is not None else 0
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        agent.train(n_steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    n_upd = steps * agent.n_epoch * agent.n_minibatch
    if world > 1:
        e = torch.tensor([el], dtype=torch.float64, device=device)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        el = float(e)
    res = {"workload": "PPO-Clip SynthBox(obs=376,act=17) num_envs=%d/GPU x %d GPU horizon=%d, ppo/mujoco.yaml, "
                       "nets [256] LeakyReLU" % (n_envs, world, n_steps),
           "metric": "env-steps/s", "value": round(world * n_envs * n_steps * steps / el, 1),
           "ms_per_iteration": round(el / steps * 1e3, 2), "iterations": steps, "n_gpus": world,
           "fused_heads": bool(getattr(agent.learner._fused_mlp(), "fused_heads", False)),
           "collectives_per_minibatch": (gs.collectives - c0) / n_upd if gs is not None else 0}
    del agent
    torch.cuda.empty_cache()
    return res


def dp_path_bench(device, args, steps=3, warmup=2):
    """C2 on one GPU with the data-parallel update path attached (distributed.LocalGradSync in place of the
    all-reduce) and, in the same call, without it: the per-rank cost of world > 1 apart from the collective itself —
    the clip norm from its own pass (the producers' partials are not the averaged gradient's), K9 launched from the
    host per minibatch.  The two arms alternate (A B A B) so box drift hits both alike."""
    import torch
    from xuanpolicy_amd.distributed import LocalGradSync
    from xuanpolicy_amd.runner import build_synthbox_ppo
    N, T = args.n_envs, args.horizon

    def arm(hooked):
        agent = build_synthbox_ppo(n_envs=N, n_steps=T, obs_dim=args.obs_dim, act_dim=args.act_dim,
                                   hidden=args.hidden, n_epoch=args.n_epoch, n_minibatch=args.n_minibatch, seed=1,
                                   device=device)
        agent.learner.enable_fast_path()
        agent.fuse_value_gae = args.gae_form in ("k40v", "value")
        agent.value_gemm = args.gae_form == "k40v"
        hook = None
        if hooked:
            hook = agent.learner.grad_sync = LocalGradSync(agent.learner.flat_grads)
        for _ in range(warmup):
            agent.train(T)
        torch.cuda.synchronize()
        c0 = hook.calls if hook else 0
        t0 = time.perf_counter()
        for _ in range(steps):
            agent.train(T)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        calls = (hook.calls - c0) if hook else 0
        del agent
        torch.cuda.empty_cache()
        return el / steps * 1e3, calls
    ms = {True: [], False: []}
    calls = 0
    for hooked in (False, True, False, True):
        m, c = arm(hooked)
        ms[hooked].append(m)
        calls = max(calls, c)
    on, off = min(ms[True]), min(ms[False])
    return {"what": "C2 with the world > 1 update path on one GPU (grad_sync hook without a collective: own clip-norm "
                    "pass, host-launched K9 per minibatch) against the world-1 path, arms alternated, best of 2 x %d "
                    "iterations each" % steps,
            "value": round(N * T / (on * 1e-3), 1), "unit": "env-steps/s", "ms_per_iteration": round(on, 3),
            "world1_ms_per_iteration": round(off, 3), "delta_ms_per_iteration": round(on - off, 3),
            "delta_us_per_minibatch": round((on - off) * 1e3 / (args.n_epoch * args.n_minibatch), 2),
            "arms_ms": {"dp_path": [round(x, 3) for x in ms[True]], "world1": [round(x, 3) for x in ms[False]]},
            "hook_calls_per_minibatch": calls / (steps * args.n_epoch * args.n_minibatch)}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(args, cores):
    """The oracle's restatement of the reference loop (oracle/cpu_ref.AgentLoopRef: per-env
    DummyVecEnv stepping, per-env finish_path, numpy fancy-index sampling, torch-CPU learner with
    Adam(eps=1e-5) + LinearLR) on a bounded sample of the same workload."""
    import numpy as np
    import torch
    from oracle import cpu_ref, synth_env
    N, T, D, A, H = args.n_envs, args.horizon, args.obs_dim, args.act_dim, args.hidden
    torch.manual_seed(1)
    np.random.seed(1)
    envs = [synth_env.SynthBoxEnv(D, A, seed=1, env_index=i) for i in range(N)]
    pol = cpu_ref.build_actor_critic_ref(D, A, [H], [H], [H])
    opt = torch.optim.Adam(pol.parameters(), 4e-4, eps=1e-5)
    sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.0, total_iters=100000000)
    lrn = cpu_ref.LearnerRef(pol, opt, sch, "ppo", 0.25, 0.0, 0.2, 0.5, True)
    # torch intra-op threads: the fastest of a few counts up to the box's CPU share for the learner update (the
    # baseline's dominant phase), so the baseline is not slowed by an oversubscribed or cross-socket thread pool
    B = N * T // args.n_minibatch
    rng = np.random.default_rng(0)
    probe = (rng.normal(0, 1, (B, D)).astype(np.float32), rng.normal(0, 0.5, (B, A)).astype(np.float32),
             rng.normal(0, 1, B).astype(np.float32), rng.normal(0, 1, B).astype(np.float32),
             (-1.5 + 0.3 * rng.normal(0, 1, B)).astype(np.float32))
    saved = {k: v.clone() for k, v in pol.state_dict().items()}
    thread_probe = {}
    for th in sorted({c for c in (4, 8, 16, 32, cores) if c <= cores}):
        torch.set_num_threads(th)
        lrn.update(*probe)
        t0 = time.perf_counter()
        for _ in range(2):
            lrn.update(*probe)
        thread_probe[th] = round((time.perf_counter() - t0) / 2, 4)
    cores = min(thread_probe, key=thread_probe.get)
    torch.set_num_threads(cores)
    pol.load_state_dict(saved)   # the probe's steps undone: a fresh optimizer below
    opt = torch.optim.Adam(pol.parameters(), 4e-4, eps=1e-5)
    sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.0, total_iters=100000000)
    lrn = cpu_ref.LearnerRef(pol, opt, sch, "ppo", 0.25, 0.0, 0.2, 0.5, True)
    loop = cpu_ref.AgentLoopRef(envs, pol, lrn, T, args.n_epoch, args.n_minibatch, 0.99, 0.95)
    t0 = time.perf_counter()
    loop.run_steps(T, max_updates=args.cpu_updates)
    wall = time.perf_counter() - t0
    tm = loop.timers
    per_update = (tm["sample"] + tm["update"]) / max(loop.n_updates, 1)
    ut = np.asarray(loop.update_times)
    n_updates_full = args.n_epoch * ((N * T + (N * T // args.n_minibatch) - 1) // (N * T // args.n_minibatch))
    rollout = tm["act"] + tm["env"] + tm["store"]
    iteration = rollout + tm["gae"] + n_updates_full * per_update
    res = {"value": round(N * T / iteration, 1), "unit": "env-steps/s", "cores": cores, "kind": "port",
           "sample": ("one %dx%d rollout (per-env SynthBoxEnv stepping as DummyVecEnv_Gym) + per-env finish_path "
                      "GAE + %d of the %d minibatch updates (B=%d) timed in %.1f s; iteration time = rollout %.2f s "
                      "+ GAE %.2f s + %d x %.3f s per update (sample + learner.update) = %.2f s"
                      % (N, T, loop.n_updates, n_updates_full, N * T // args.n_minibatch, wall, rollout, tm["gae"],
                         n_updates_full, per_update, iteration)),
           "per_update_s": {"mean": round(float(ut.mean()), 4), "std": round(float(ut.std()), 4),
                            "min": round(float(ut.min()), 4), "max": round(float(ut.max()), 4), "n": int(ut.size)},
           "cpu_model": _cpu_model(), "affinity_cpus": len(os.sched_getaffinity(0)),
           "update_s_by_threads": thread_probe,
           "threads_note": "torch intra-op threads: the fastest learner update among the counts probed up to the box's "
                           "CPU share (OMP_NUM_THREADS, 16 on the GPU box; the affinity mask spans the whole host)"}
    cal = os.path.join(REPO, "tests", "golden", "cpu_calibration.json")
    if os.path.exists(cal):   # tools/cpu_calibrate.py: the restated phases against the real reference, same host
        with open(cal) as f:
            c = json.load(f)
        res["calibration"] = {"host": c.get("host"), "threads": c.get("threads"),
                              "port_over_reference": c.get("port_over_reference"), "loop": c.get("loop"),
                              "note": "measured in the build container (the reference is importable only there): per "
                                      "phase and for one whole iteration of the reference's own PPOCLIP_Agent.train"}
    # the same loop with the env vectorised in numpy (synth_env.SynthBoxVec), so the
    # speedup is not credited only to removing the per-env Python stepping; the updates cost the same.
    venv = synth_env.SynthBoxVec(N, D, A, seed=1)
    loop2 = cpu_ref.AgentLoopRef(None, pol, lrn, T, args.n_epoch, args.n_minibatch, 0.99, 0.95, vectorized_env=venv)
    loop2.run_steps(T, max_updates=0)
    tm2 = loop2.timers
    rollout2 = tm2["act"] + tm2["env"] + tm2["store"]
    iteration2 = rollout2 + tm2["gae"] + n_updates_full * per_update
    res["vectorized_env_variant"] = {
        "value": round(N * T / iteration2, 1), "unit": "env-steps/s", "cores": cores,
        "sample": "rollout with the numpy-vectorised env %.2f s (act %.2f, env %.2f, store %.2f) + GAE %.2f s + the "
                  "same %d x %.3f s updates = %.2f s" % (rollout2, tm2["act"], tm2["env"], tm2["store"], tm2["gae"],
                                                          n_updates_full, per_update, iteration2)}
    return res


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_cmd(gpus, argv, port):
    """The child command of a self-launched multi-rank run: torch.distributed.run, one process per GPU of this node,
    rendezvous on 127.0.0.1, this script with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(gpus),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def check_world(gpus, env=None):
    """--gpus N is the number of ranks: under a launcher (WORLD_SIZE in the environment) it must equal WORLD_SIZE.
    Returns the launcher's world size, or None when no launcher started this process."""
    env = os.environ if env is None else env
    if "WORLD_SIZE" not in env:
        return None
    world = int(env["WORLD_SIZE"])
    if world != gpus:
        raise SystemExit("bench.py: --gpus %d but the launcher started WORLD_SIZE=%d ranks; they must agree"
                         % (gpus, world))
    return world


def self_launch(args, argv):
    """`python bench.py --gpus N` (N > 1) with no launcher environment: start the N ranks as children through
    torch.distributed.run — before this process touches torch.cuda or HIP, and as a child process, never an exec —
    relay their output (stderr and every non-JSON stdout line to stderr, as it arrives), print rank 0's JSON line
    and exit with the launcher's status.  Every rank then asserts WORLD_SIZE == --gpus (check_world)."""
    import subprocess
    cmd = launch_cmd(args.gpus, argv, _free_port())
    print("bench.py: launching %d ranks: %s" % (args.gpus, " ".join(cmd)), file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, cwd=REPO)
    line = None
    for ln in p.stdout:
        if ln.startswith("{") and '"metric"' in ln:
            line = ln.strip()
        else:
            sys.stderr.write(ln)
            sys.stderr.flush()
    rc = p.wait()
    if line is not None:
        print(line, flush=True)
    if rc == 0 and line is None:
        print("bench.py: the ranks exited 0 without a JSON line", file=sys.stderr)
        rc = 1
    return rc


def allreduce_probe(learner, device, reps=20):
    """world > 1: one all-reduce of a buffer of the flat gradient's size (not the gradient itself) on this process
    group, timed over `reps` back-to-back calls (host clock, synchronised): the per-minibatch collective's cost."""
    import torch
    import torch.distributed as dist
    gs = getattr(learner, "grad_sync", None)
    if gs is None:
        return None
    buf = torch.zeros_like(gs.fg.flat)
    op = dist.ReduceOp.AVG if gs.avg else dist.ReduceOp.SUM
    for _ in range(3):
        dist.all_reduce(buf, op=op)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        dist.all_reduce(buf, op=op)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / reps * 1e6
    t = torch.tensor([us], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return {"bytes": int(buf.numel() * buf.element_size()), "avg_us": round(float(t), 2), "reps": reps,
            "backend": dist.get_backend()}


def main():
    args = parse()
    if args.gpus > 1 and check_world(args.gpus) is None:
        sys.exit(self_launch(args, sys.argv[1:]))
    check_world(args.gpus)
    import torch
    import torch.distributed as dist
    from xuanpolicy_amd import ops
    from xuanpolicy_amd.distributed import broadcast_parameters, init_from_env, local_device
    from xuanpolicy_amd.runner import build_synthbox_ppo

    ops.S3_GEMMS = args.gemm == "split3"
    ops.S3_HEADS = args.s3_heads
    from xuanpolicy_amd.fused_mlp import FusedActorCritic
    FusedActorCritic.CRIT_FACTORED = args.crit_factored == "on"
    FusedActorCritic.WIDE_TRUNK = args.wide_trunk == "on"
    FusedActorCritic.ROLLOUT_SPLIT = args.rollout_split == "on"
    import xuanpolicy_amd.agents as _agents
    _agents.FOLD_RMS = args.fold_rms == "on"
    _agents.FUSE_POST = args.fuse_post == "on"
    if args.pair_sa:
        ops.lib().xpa_s3_wgrad_pair_tune(args.pair_sa)
    thin_probe = (1 if args.thin_store == "plain" else 0) | (2 if args.rollout_h_store == "plain" else 0)
    if thin_probe:
        ops.lib().xpa_thin_probe(thin_probe)
    if args.s3_probe:
        ops.lib().xpa_s3_probe(args.s3_probe)
    rank, local, world = init_from_env()
    device = local_device(local)
    torch.cuda.set_device(device)
    if args.dz_store == "plain":
        assert ops.lib().xpa_head_store_probe(1) == 0
    N, T = args.n_envs, args.horizon
    dp_variants = {}   # SURVEY.md §8(e)'s global-statistics variants (world > 1 only; default: per-shard statistics)
    if args.sync_obs_rms != "off":
        dp_variants["sync_obs_rms"] = "rollout" if args.sync_obs_rms == "rollout" else True
    if args.global_advnorm == "on":
        dp_variants["global_advnorm"] = True
    agent = build_synthbox_ppo(n_envs=N, n_steps=T, obs_dim=args.obs_dim, act_dim=args.act_dim, hidden=args.hidden,
                               n_epoch=args.n_epoch, n_minibatch=args.n_minibatch, seed=1, device=device,
                               shard=rank, **dp_variants)
    agent.learner.enable_fast_path()  # flat params/grads, fused clip+Adam, RCCL hook when world > 1
    agent.fuse_value_gae = args.gae_form in ("k40v", "value")
    agent.value_gemm = args.gae_form == "k40v"
    fm0 = agent.learner._fused_mlp()
    if fm0 is not None:
        fm0.use_trunk_heads = args.trunk_heads == "on"
    if world > 1:
        broadcast_parameters(agent.policy)

    for _ in range(args.warmup):
        agent.train(T)
    torch.cuda.synchronize()
    # In the timed region only the GAE launches carry timing events, and those are recorded by the
    # dispatches themselves (hipExtLaunchKernel): no extra packets in the stream.
    ops.TIMER.enabled = not args.no_kernel_timing
    ops.TIMER.only = {"gae"}
    ops.TIMER.reset()
    gs = agent.learner.grad_sync
    coll0 = gs.collectives if gs is not None else 0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        agent.train(T)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e)
    n_updates = args.steps * args.n_epoch * args.n_minibatch
    dp = None
    if world > 1:
        probe = allreduce_probe(agent.learner, device)
        ms_step = elapsed / args.steps * 1e3
        dp = {"collectives_per_minibatch": (gs.collectives - coll0) / n_updates if gs is not None else None,
              "allreduce": probe,
              "allreduce_time_share": (round(probe["avg_us"] * 1e-3 * args.n_epoch * args.n_minibatch / ms_step, 4)
                                       if probe else None),
              "note": "allreduce: one all-reduce of a buffer of the flat gradient's size, timed alone after the timed "
                      "region (max over ranks); time share = its time x updates per iteration / ms_per_step"}
    gae_ms_timed = ops.TIMER.mean_ms("gae")
    gae_launches = ops.TIMER.count("gae")
    # One more (untimed) iteration with event pairs around the K12 launches and the paired GEMM, and
    # events at the iteration's rollout | update boundary.
    phase_ms = None
    if not args.no_kernel_timing:
        ops.TIMER.reset()
        ops.TIMER.only = {"heads", "gemm_pair"}
        e_start = torch.cuda.Event(enable_timing=True)
        agent.phase_events = []
        e_start.record()
        agent.train(T)
        torch.cuda.synchronize()
        ev = dict(agent.phase_events)
        agent.phase_events = None
        if "rollout_end" in ev and "update_end" in ev:
            phase_ms = {"rollout": round(e_start.elapsed_time(ev["rollout_end"]), 3),
                        "update_incl_gae": round(ev["rollout_end"].elapsed_time(ev["update_end"]), 3),
                        "note": "device events at the iteration's phase boundaries, one extra iteration after the "
                                "timed region (the heads/GEMM event pairs of that iteration included)"}
    ops.TIMER.enabled = False
    ops.TIMER.only = None

    gae_ms = gae_ms_timed
    loss_ms = ops.TIMER.mean_ms("loss")
    heads_ms = ops.TIMER.mean_ms("heads")
    gemm_ms = ops.TIMER.mean_ms("gemm_pair")
    mem = agent.memory
    # Back-to-back replay of the same GAE launch on the agent's live buffers (after the timed region):
    # per-launch time without the event/dispatch overhead a single bracketed launch carries.
    replay_us = None if args.no_kernel_timing else gae_graph_replay_us(agent)
    floor_us = None if args.no_kernel_timing else ops.dispatch_floor_us(device)
    copy_us = None if args.no_kernel_timing else ops.stream_copy_us(mem.rewards, mem.values, mem.terminals)
    mid_trunc = int(((mem.closed[:, :-1] > 0) & (mem.terminals[:, :-1] == 0)).sum())
    B = N * T // args.n_minibatch
    c4 = None if args.no_c4 else c4_bench(device, rank, world)   # collective: every rank
    result = None
    if rank == 0:
        value = world * N * T * args.steps / elapsed
        roofline = None
        if gae_ms:
            form = getattr(agent, "gae_form", "compact")
            gb = gae_value_bytes(N, T, mid_trunc, args.hidden) if form == "value" else gae_bytes(N, T, mid_trunc)
            gb_k1 = gae_bytes(N, T, mid_trunc)
            # achieved / frac: SURVEY.md §8(d)'s algorithmic bytes (20 B per (env, step) + the bootstraps) over the
            # launch's duration, as the bench contract defines them; the value-fused launch also reads the critic's
            # hidden pre-activations (its extra bytes are reported beside, as launch_bytes_*)
            # the PMC child passes run at N = 1 only (at world > 1 the other ranks would wait on rank 0's children)
            traffic, traffic_note = ((None, "skipped (--no-pmc)") if args.no_pmc else
                                     (None, "skipped (world > 1: measured at N = 1)") if world > 1 else
                                     live_gae_traffic(form))
            rp_us, rp_list, rp_note = (None, None, "skipped") if args.no_rocprof or world > 1 else \
                live_gae_rocprof(args)
            # the other GAE form's in-loop launch under the profiler (split: the compact scan alone, exactly the §8(d)
            # bytes; value: the value-fused scan)
            other = "split" if form == "value" else "value"
            rs_us, rs_list, rs_note = (None, None, "skipped") if args.no_rocprof or world > 1 else \
                live_gae_rocprof(args, form=other)
            # headline: the profiler's in-loop duration (the event timer's dispatch-attached events carry a floor of
            # several us: dispatch_floor_us); the event-timed figure stays beside it
            launch_us = rp_us if rp_us else gae_ms * 1e3
            ach = gb_k1 / launch_us / 1e3
            # a plain copy of the launch's own bytes (3 reads + 2 writes of 16 B per 4 elements) on the event clock
            launch_copy_us = None
            if not args.no_kernel_timing:
                nl = int(gb) // 20 // 4 * 4   # the copy kernel moves float4s
                bufs = [torch.empty(nl, device=device) for _ in range(3)]
                launch_copy_us = ops.stream_copy_us(*bufs)
                del bufs
            if form == "value":
                act_code = agent.learner._fused_mlp().critic[-2][1]
                kname = "xpa_gae_scan_value: critic output layer + bootstrap fixup + GAE (gae_dpp_kernel<5, 1, %d>)" \
                    % act_code
            else:
                kname = "xpa_gae_scan_compact (gae_dpp_kernel<5, 1>)" + (
                    "; the deferred bootstrap values from K40V (xpa_s3_gemm_value) in the launch before"
                    if args.gae_form == "k40v" else "")
            roofline = {"kernel": kname, "bound": "hbm", "achieved": round(ach, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "traffic_note": traffic_note,
                        "traffic_over_algorithmic": round(traffic / gb_k1, 3) if traffic else None,
                        "traffic_over_launch_bytes": round(traffic / gb, 3) if traffic else None,
                        "avg_launch_us": round(launch_us, 3),
                        "avg_launch_source": ("rocprofv3 kernel trace of the in-loop launches (child run, rocprof_*)"
                                              if rp_us else "HIP events (no rocprofv3 child run)"),
                        "algorithmic_bytes_per_launch": int(gb_k1),
                        "launch_bytes": int(gb),
                        "launch_bytes_achieved": round(gb / launch_us / 1e3, 1),
                        "launch_bytes_frac": round(gb / launch_us / 1e3 / HBM_PEAK_GBS, 4),
                        "event_timed_us": round(gae_ms * 1e3, 3),
                        "event_timed_frac": round(gb_k1 / gae_ms / 1e6 / HBM_PEAK_GBS, 4),
                        "event_timed_note": ("the same launches timed by dispatch-attached HIP events inside the timed "
                                             "region; that clock reads an empty launch at dispatch_floor_us"),
                        "other_form": {
                            "form": other,
                            "rocprof_inloop_us": round(rs_us, 3) if rs_us else None,
                            "rocprof_inloop_launches_us": rs_list,
                            "frac_sec8d_bytes": round(gb_k1 / rs_us / 1e3 / HBM_PEAK_GBS, 4) if rs_us else None,
                            "note": rs_note},
                        "launch_bytes_copy_us": round(launch_copy_us, 3) if launch_copy_us else None,
                        "frac_of_launch_copy": (round(launch_copy_us / (gae_ms * 1e3), 3)
                                                if launch_copy_us else None),
                        "target_note": ("north_star's >= 0.6 of the 8 TB/s peak at 4096 x 128 needs the %.1f MB "
                                        "launch in <= %.2f us; a plain copy of the same bytes in one launch takes "
                                        "k1_bytes_copy_us on the event clock (and the empty-launch floor is "
                                        "dispatch_floor_us there), so the target is above the measured single-launch "
                                        "copy ceiling at this size; it is met from 65 536 envs (gae_sweep_flushed)"
                                        % (gb_k1 / 1e6, gb_k1 / (0.6 * HBM_PEAK_GBS) / 1e3)),
                        "bytes_note": ("algorithmic bytes: 20 B per (env, step) + 4 B per bootstrap (SURVEY.md "
                                       "§8(d)); launch_bytes adds the critic hidden pre-activations the fused value "
                                       "head reads, 2 x %d rows x %d f32 + the output layer (they replace a separate "
                                       "value-head launch; traffic_over_launch_bytes compares the PMC traffic with "
                                       "them)" % (N, args.hidden)) if form == "value" else
                                      "20 B per (env, step) + 4 B per bootstrap (SURVEY.md §8(d))",
                        # the profiler's duration of the same in-loop launch (child run): frac against the §8(d)
                        # 20 B/unit bytes and against every byte the launch reads and writes
                        "rocprof_inloop_us": round(rp_us, 3) if rp_us else None,
                        "rocprof_inloop_launches_us": rp_list,
                        "rocprof_frac_sec8d_bytes": round(gb_k1 / rp_us / 1e3 / HBM_PEAK_GBS, 4) if rp_us else None,
                        "rocprof_frac_launch_bytes": round(gb / rp_us / 1e3 / HBM_PEAK_GBS, 4) if rp_us else None,
                        "rocprof_note": rp_note,
                        "launches": gae_launches,
                        "timing": "HIP events recorded by each in-loop dispatch at the kernel's own start and end "
                                  "(hipExtLaunchKernel), on the launch stream, inside the timed region",
                        "graph_replay_us": round(replay_us, 3) if replay_us else None,
                        "graph_replay_achieved": round(gb_k1 / replay_us / 1e3, 1) if replay_us else None,
                        # An empty one-wave launch on the same clock: no kernel of this launch's bytes can
                        # measure above gb / floor (tools/gae_floor.hip).
                        "dispatch_floor_us": round(floor_us, 3) if floor_us else None,
                        "frac_ceiling_at_floor": round(gb_k1 / floor_us / 1e3 / HBM_PEAK_GBS, 4) if floor_us else None,
                        # the same bytes streamed with no scan (3 loads + 2 stores of 16 B per 4 elements), same
                        # clock, same buffers: what any kernel moving K1's bytes in one launch takes here
                        "k1_bytes_copy_us": round(copy_us, 3) if copy_us else None,
                        "frac_of_copy": round(copy_us / (gae_ms * 1e3), 3) if copy_us and form != "value" else None,
                        "frac_of_copy_note": "event clock both: k1_bytes_copy_us / event_timed_us (compact form); "
                                             "the value form: frac_of_launch_copy (a copy of its launch_bytes)"}
        loss_kernel = None
        if loss_ms:
            lb = loss_bytes_gauss(B, args.act_dim)
            loss_kernel = {"kernel": "xpa_policy_loss_fwd_bwd (gaussian, ppo)", "avg_launch_us": round(loss_ms * 1e3, 3),
                           "achieved": round(lb / loss_ms / 1e6, 1), "unit": "GB/s",
                           "frac": round(lb / loss_ms / 1e6 / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": int(lb),
                           "launches": len(ops.TIMER.events.get("loss", []))}
        update_kernels = {}
        if heads_ms and getattr(agent.learner._fused_mlp(), "gemm_heads", False):
            fl = pair_gemm_flops(B, args.hidden, args.hidden)
            fmh = agent.learner._fused_mlp()
            trunk = fmh.trunk_heads and fmh.use_trunk_heads
            update_kernels["heads"] = {
                "kernel": ("xpa_head_gemm_trunk_actor + xpa_head_gemm_trunk_critic (K16X: trunk layer + hidden-layer "
                           "GEMM on fp32 MFMA + fused head epilogue, per minibatch; FLOP counted: the hidden GEMMs)"
                           if trunk else
                           ("xpa_head_gemm_%s_actor + _critic (%s: the hidden-layer f32 GEMM as an exact three-way bf16 "
                            "split on the bf16 matrix cores, 6 bf16 products per f32 product, + fused head epilogue, "
                            "per minibatch; achieved / frac: f32-GEMM FLOP against the fp32 MFMA peak)"
                            % (ops.S3_HEADS, {"s3p": "K16P", "s3q": "K16Q"}.get(ops.S3_HEADS, "K16S"))
                            if ops.S3_GEMMS else
                            "xpa_head_gemm_actor + xpa_head_gemm_critic (K16: hidden-layer GEMM on fp32 MFMA "
                            "+ fused head epilogue, per minibatch)")), "bound": "mfma",
                "avg_us": round(heads_ms * 1e3, 3), "flops": fl, "achieved": round(fl / heads_ms / 1e9, 1),
                "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(fl / heads_ms / 1e9 / FP32_MFMA_PEAK_TFLOPS, 4), "launches": ops.TIMER.count("heads"),
                "timing": "event pairs on the launch stream in one extra iteration after the timed region"}
            if ops.S3_GEMMS and not trunk:
                # r05: the roofline of the launches is the bf16 matrix cores they run on (6 bf16 products per f32
                # product); the f32-equivalent rate against the fp32 MFMA peak stays beside it
                h = update_kernels["heads"]
                h["kernel"] = h["kernel"].replace("achieved / frac: f32-GEMM FLOP against the fp32 MFMA peak",
                                                  "achieved / frac: the bf16 MFMA FLOP against the dense bf16 peak")
                h["f32_equivalent"] = {"flops": fl, "achieved": h["achieved"], "peak": FP32_MFMA_PEAK_TFLOPS,
                                       "unit": "TFLOP/s", "frac": h["frac"]}
                h.update({"flops": 6 * fl, "achieved": round(6 * fl / heads_ms / 1e9, 1), "peak": BF16_MFMA_PEAK_TFLOPS,
                          "frac": round(6 * fl / heads_ms / 1e9 / BF16_MFMA_PEAK_TFLOPS, 4)})
                h["frac_at_measured_bf16_clock"] = round(h["frac"] * PEAK_CLOCK_GHZ / BF16_MFMA_LOOP_CLOCK_GHZ, 4)
        elif heads_ms:
            hb = heads_bytes(B, args.act_dim, args.hidden)
            update_kernels["heads"] = {
                "kernel": "xpa_head_fused_actor + xpa_head_fused_critic (K12, per minibatch)", "bound": "hbm",
                "avg_us": round(heads_ms * 1e3, 3), "algorithmic_bytes": int(hb),
                "achieved": round(hb / heads_ms / 1e6, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(hb / heads_ms / 1e6 / HBM_PEAK_GBS, 4), "launches": ops.TIMER.count("heads"),
                "timing": "event pairs on the launch stream in one extra iteration after the timed region"}
        fmu = agent.learner._fused_mlp()
        if ops.S3_GEMMS and phase_ms and getattr(fmu, "gemm_heads", False):
            # r05: the update's three paired-layer products on the split (heads' forward 6 products; dX / dW 6 for the
            # actor half and 3 for the critic half when factored) against the dense bf16 peak, and the measured update
            fl = pair_gemm_flops(B, args.hidden, args.hidden)
            per_bwd = 4.5 if FusedActorCritic.CRIT_FACTORED else 6.0
            bf = (6.0 + 2 * per_bwd) * fl
            upd_us = phase_ms["update_incl_gae"] * 1e3 / (args.n_epoch * args.n_minibatch)
            update_kernels["update_floor"] = {
                "what": "one minibatch update: its paired-layer products as bf16 MFMA FLOP (heads 6 products, dX / dW %s) "
                        "at the dense bf16 peak, vs the measured update (phase events incl. the iteration's one GAE "
                        "launch, / updates per iteration)" % ("6 actor + 3 critic" if per_bwd < 6 else "6"),
                "bf16_mfma_gflop": round(bf / 1e9, 2), "floor_us": round(bf / BF16_MFMA_PEAK_TFLOPS / 1e6, 2),
                "measured_us": round(upd_us, 2), "frac": round(bf / BF16_MFMA_PEAK_TFLOPS / 1e6 / upd_us, 4),
                "frac_at_measured_bf16_clock": round(bf / BF16_MFMA_PEAK_TFLOPS / 1e6 / upd_us * PEAK_CLOCK_GHZ
                                                     / BF16_MFMA_LOOP_CLOCK_GHZ, 4),
                "clock_note": "a dense bf16 MFMA loop holds %.2f GHz on this part (tools/clock_probe.hip), not %.1f"
                              % (BF16_MFMA_LOOP_CLOCK_GHZ, PEAK_CLOCK_GHZ)}
        if gemm_ms:
            fl = pair_gemm_flops(B, args.hidden, args.hidden)
            update_kernels["gemm_pair"] = {
                "kernel": "paired actor|critic hidden-layer forward GEMM (hipBLASLt, fp32 MFMA)", "bound": "mfma",
                "avg_us": round(gemm_ms * 1e3, 3), "flops": fl, "achieved": round(fl / gemm_ms / 1e9, 1),
                "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(fl / gemm_ms / 1e9 / FP32_MFMA_PEAK_TFLOPS, 4)}
        result = {
            "metric": "env-steps/sec at num_envs=4096, horizon=128; GAE kernel HBM GB/s vs peak",
            "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "PPO-Clip SynthBox(obs=17,act=6) num_envs=%d/GPU horizon=%d, ppo/mujoco.yaml "
                                   "(n_epoch %d, n_minibatch %d, nets [%d] LeakyReLU)" %
                                   (N, T, args.n_epoch, args.n_minibatch, args.hidden),
                       "num_envs_per_gpu": N, "horizon": T, "global_envs": N * world, "minibatch": B,
                       "update_gemms": ("f32 GEMMs as exact three-way bf16 splits on the bf16 matrix cores (%s heads, %s; "
                                        "error <= 2x the f32 GEMM's vs f64: tests/test_gpu_sgemm3.py)"
                                        % ({"s3p": "K16P", "s3q": "K16Q"}.get(ops.S3_HEADS, "K16S"),
                                           "K42C dX + trunk backward and K41P dW with the critic's half factored "
                                           "(masked GEMMs, 3 products)" if FusedActorCritic.CRIT_FACTORED else
                                           "K42S dX + trunk backward, K41V dW")
                                        if ops.S3_GEMMS else "f32 MFMA (K16 heads, hipBLASLt dX / dW)"),
                       "updates_per_step": args.n_epoch * args.n_minibatch,
                       "parallelism": ("dp1 (one env shard, no collective)" if world == 1 else
                                       "dp%d (env shards; ONE all-reduce of the flat gradient per minibatch over "
                                       "%s)" % (
                                           world, "RCCL" if dist.get_backend() == "nccl" else dist.get_backend())),
                       "dp_statistics": {"sync_obs_rms": args.sync_obs_rms if world > 1 else "n/a (world 1)",
                                         "global_advnorm": args.global_advnorm if world > 1 else "n/a (world 1)"}},
            "roofline": roofline,
            "phase_split_ms": phase_ms,
            "loss_kernel": loss_kernel,
            "update_kernels": update_kernels or None,
        }
        if c4 is not None:
            result["c4_box376"] = c4
        if dp is not None:
            result["data_parallel"] = dp
        if not args.no_sweep and world == 1:
            result["gae_sweep_flushed"] = gae_sweep(device, horizon=T)
            ls = loss_sweep(device, act_dim=args.act_dim)
            result["loss_sweep_flushed"] = ls
            if result["loss_kernel"] is None and ls:
                k2 = ls[0]   # the C2 minibatch size
                result["loss_kernel"] = {
                    "kernel": "xpa_policy_loss_fwd_bwd (K2, gaussian, ppo; standalone: the C2 fast path fuses the "
                              "loss into K16's epilogue)", "bound": "hbm", "batch": k2["batch"],
                    "avg_launch_us": round(k2["ms"] * 1e3, 3), "achieved": k2["GB/s"], "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": k2["frac"], "algorithmic_bytes_per_launch": k2["algorithmic_bytes"],
                    "timing": "host-recorded events around one launch after a 512 MiB cache-flush read (median of 7); "
                              "see loss_sweep_flushed for larger batches"}
        if args.dp_path == "on" and world == 1:
            result["dp_update_path"] = dp_path_bench(device, args)
        if not args.no_c1 and world == 1:
            result["c1_cartpole"] = c1_bench(device)
        if not args.no_c3 and world == 1:
            result["c3_atari_a2c"] = c3_bench(device, cpu=not args.no_cpu_baseline, kernels=not args.no_kernel_timing)
        if not args.no_per and world == 1:
            result["per_kernels"] = per_bench(device)
            cr = result["per_kernels"].get("cpu_reference_restated", {})
            result["c5_perdqn"] = c5_bench(device, tree_cpu_us=cr.get("sample_us", 0) + cr.get("update_priorities_us", 0))
        if not args.no_cpu_baseline and world == 1:
            aff = len(os.sched_getaffinity(0))
            cores = min(aff, int(os.environ.get("OMP_NUM_THREADS", aff)))   # the box's CPU share
            result["cpu_baseline"] = cpu_baseline(args, cores)
            result["speedup_vs_cpu_baseline"] = round(value / result["cpu_baseline"]["value"], 1)
            result["speedup_vs_cpu_vectorized_env"] = round(
                value / result["cpu_baseline"]["vectorized_env_variant"]["value"], 1)
        line = json.dumps(result)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
