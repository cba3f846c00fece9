"""CPU-baseline calibration (SURVEY.md §8(d) "CPU timing plan"): the oracle's restated learner update and loop phases
against the REAL reference code, same inputs, same host, same torch threads.  Runs in the build container only (it
imports /root/reference through tests/golden/ref_loader.py; the reference never travels to the GPU box).

    python tools/cpu_calibrate.py [--threads 8] [--reps 5] [--out tests/golden/cpu_calibration.json]

Measured per phase at the C2 shapes (N = 4096, T = 128, D = 17, A = 6, nets [256] LeakyReLU, minibatch 65 536):
  update   PPOCLIP_Learner.update (ppoclip_learner.py:24-65) vs oracle.cpu_ref.LearnerRef.update, Adam + LinearLR
  sample   DummyOnPolicyBuffer.sample (memory_tools.py:231-245) vs BufferRef.sample (same indices)
  gae      finish_path over every env (memory_tools.py:206-229) vs BufferRef.finish_path (C restatement)
  store    DummyOnPolicyBuffer.store x T (memory_tools.py:196-204) vs BufferRef.store
The ratios port / reference are committed as a fixture; bench.py reports them beside its cpu_baseline so the GPU box's
number can be read against the reference's cost on the same host class."""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def _median(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--loop-updates", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(REPO, "tests", "golden", "cpu_calibration.json"))
    a = ap.parse_args()
    import numpy as np
    import torch
    import ref_loader
    ref_loader.import_reference()
    import gym
    from xuance.common.memory_tools import DummyOnPolicyBuffer
    from xuance.torch.learners import PPOCLIP_Learner
    from xuance.torch.policies import Gaussian_AC_Policy
    from xuance.torch.representations import Basic_MLP
    from xuance.torch.utils import ActivationFunctions
    from oracle import cpu_ref
    torch.set_num_threads(a.threads)
    N, T, D, A, H = 4096, 128, 17, 6, 256
    B = N * T // 8
    rng = np.random.default_rng(0)
    # ---- the two policies with the same weights
    torch.manual_seed(0)
    rep = Basic_MLP((D,), [H], None, torch.nn.init.orthogonal_, ActivationFunctions["LeakyReLU"], "cpu")
    ref_pol = Gaussian_AC_Policy(gym.spaces.Box(-1, 1, (A,)), rep, [H], [H], None, torch.nn.init.orthogonal_,
                                 ActivationFunctions["LeakyReLU"], "cpu")
    port_pol = cpu_ref.build_actor_critic_ref(D, A, [H], [H], [H])
    port_pol.load_state_dict(ref_pol.state_dict())

    def learners():
        o1 = torch.optim.Adam(ref_pol.parameters(), 4e-4, eps=1e-5)
        s1 = torch.optim.lr_scheduler.LinearLR(o1, start_factor=1.0, end_factor=0.0, total_iters=10 ** 8)
        o2 = torch.optim.Adam(port_pol.parameters(), 4e-4, eps=1e-5)
        s2 = torch.optim.lr_scheduler.LinearLR(o2, start_factor=1.0, end_factor=0.0, total_iters=10 ** 8)
        ref = PPOCLIP_Learner(ref_pol, o1, s1, "cpu", "./", vf_coef=0.25, ent_coef=0.0, clip_range=0.2,
                              clip_grad_norm=0.5, use_grad_clip=True)
        port = cpu_ref.LearnerRef(port_pol, o2, s2, "ppo", 0.25, 0.0, 0.2, 0.5, True)
        return ref, port
    ref_l, port_l = learners()
    obs = rng.normal(0, 1, (B, D)).astype(np.float32)
    act = rng.normal(0, 0.5, (B, A)).astype(np.float32)
    ret = rng.normal(0, 1, B).astype(np.float32)
    adv = rng.normal(0, 1, B).astype(np.float32)
    val = rng.normal(0, 1, B).astype(np.float32)
    old = (-1.5 + 0.3 * rng.normal(0, 1, B)).astype(np.float32)
    res = {"threads": a.threads, "host": _cpu_model(), "shapes": "N=%d T=%d D=%d A=%d nets [%d] minibatch %d" % (
        N, T, D, A, H, B)}
    ref_l.update(obs, act, ret, val, adv, old)    # warm-up (allocator, thread pool)
    port_l.update(obs, act, ret, adv, old)
    res["update_s"] = {"reference": _median(lambda: ref_l.update(obs, act, ret, val, adv, old), a.reps),
                       "port": _median(lambda: port_l.update(obs, act, ret, adv, old), a.reps)}
    # ---- buffer phases
    space_o, space_a = gym.spaces.Box(-1, 1, (D,)), gym.spaces.Box(-1, 1, (A,))
    rbuf = DummyOnPolicyBuffer(space_o, space_a, {"old_logp": ()}, N, T, True, True, 0.99, 0.95)
    pbuf = cpu_ref.BufferRef((D,), (A,), {"old_logp": ()}, N, T, gae_impl="np")   # the baseline's GAE form
    cpu_ref.build_oracle()
    cols = [(rng.normal(0, 1, (N, D)).astype(np.float32), rng.normal(0, 0.5, (N, A)).astype(np.float32),
             rng.normal(0, 1, N).astype(np.float32), rng.normal(0, 1, N).astype(np.float32),
             (rng.random(N) < 0.01).astype(np.float32), rng.normal(0, 1, N).astype(np.float32)) for _ in range(T)]

    def fill(buf):
        buf.clear() if hasattr(buf, "clear") else None
        for (o, ac, r, v, te, lp) in cols:
            buf.store(o, ac, r, v, te, {"old_logp": lp})
    res["store_s"] = {"reference": _median(lambda: fill(rbuf), a.reps), "port": _median(lambda: fill(pbuf), a.reps)}
    boots = rng.normal(0, 1, N).astype(np.float32)

    def gae(buf):
        for i in range(N):
            buf.finish_path(float(boots[i]), i)
    fill(rbuf)
    fill(pbuf)
    res["gae_s"] = {"reference": _median(lambda: gae(rbuf), a.reps), "port": _median(lambda: gae(pbuf), a.reps)}
    idx = rng.permutation(N * T)[:B]
    res["sample_s"] = {"reference": _median(lambda: rbuf.sample(idx), a.reps),
                       "port": _median(lambda: pbuf.sample(idx), a.reps)}
    res["port_over_reference"] = {k[:-2]: round(v["port"] / v["reference"], 3) for k, v in res.items()
                                  if k.endswith("_s")}
    # ---- the whole loop: one full iteration (4096 x 128 rollout over a DummyVecEnv of per-env SynthBoxEnv objects, the
    # full-buffer finish_path calls, all 16 x 8 updates) of the REFERENCE's PPOCLIP_Agent.train (ppoclip_agent.py:59-111)
    # against the bounded baseline bench.py runs on the GPU box, same env, same host, same threads
    import types
    from xuance.environment.gym.gym_vec_env import DummyVecEnv_Gym
    from xuance.torch.agents import PPOCLIP_Agent
    from oracle.synth_env import SynthBoxEnv
    cfg = types.SimpleNamespace(render=False, n_steps=T, n_minibatch=8, n_epoch=16, gamma=0.99, gae_lambda=0.95,
                                env_name="SynthBox", use_gae=True, use_advnorm=True, device="cpu", model_dir="./models/",
                                log_dir="/tmp/xpa_cal_logs/", vf_coef=0.25, ent_coef=0.0, clip_range=0.2,
                                clip_grad_norm=0.5, use_grad_clip=True, use_obsnorm=True, use_rewnorm=True,
                                obsnorm_range=5, rewnorm_range=5, seed=1, logger="tensorboard", test_mode=False)
    envs = DummyVecEnv_Gym([(lambda i=i: SynthBoxEnv(D, A, seed=1, env_index=i, spaces=(space_o, space_a)))
                            for i in range(N)])
    o3 = torch.optim.Adam(ref_pol.parameters(), 4e-4, eps=1e-5)
    s3 = torch.optim.lr_scheduler.LinearLR(o3, start_factor=1.0, end_factor=0.0, total_iters=10 ** 8)
    agent = PPOCLIP_Agent(cfg, envs, ref_pol, o3, s3, "cpu")
    envs.reset()
    torch.set_num_threads(a.threads)   # the agent's constructor may reset it
    t0 = time.perf_counter()
    agent.train(T)
    ref_iter = time.perf_counter() - t0
    from argparse import Namespace
    sys.path.insert(0, REPO)
    import bench
    ns = Namespace(n_envs=N, horizon=T, obs_dim=D, act_dim=A, hidden=H, n_epoch=16, n_minibatch=8,
                   cpu_updates=a.loop_updates)
    cb = bench.cpu_baseline(ns, a.threads)
    ref_rate = N * T / ref_iter
    res["loop"] = {"reference_iteration_s": round(ref_iter, 2), "reference_env_steps_per_s": round(ref_rate, 1),
                   "port_env_steps_per_s": cb["value"], "port_sample": cb["sample"],
                   "port_over_reference_rate": round(cb["value"] / ref_rate, 3),
                   "survey_reference_env_steps_per_s": 15877.0,
                   "note": "the reference's own PPOCLIP_Agent.train over DummyVecEnv_Gym of SynthBoxEnv (one full "
                           "iteration, every update) vs bench.cpu_baseline's bounded sample of the restated loop; the "
                           "survey's 15 877 used a simpler synthetic env (~12 us per env step vs ~18 us here)"}
    for k, v in list(res.items()):
        if k.endswith("_s"):
            res[k] = {kk: round(vv, 4) for kk, vv in v.items()}
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
