"""Tune the GEMM shapes of the C2 PPO iteration with PyTorch TunableOp (hipBLASLt + rocBLAS solution search).

    python tools/tune_gemms.py tune    # tunes every shape met in one iteration; the table is written at exit
                                       # to xuanpolicy_amd/tuning/tunableop_results0.csv
    python tools/tune_gemms.py check   # times iterations with TunableOp off vs the tuned table (tuning off)
    python tools/tune_gemms.py add c3  # tunes the shapes of one more configuration (c3: A2C AC_CNN_Atari, c4: PPO
                                       # SynthBox(376, 17)) on top of the table; `check c3` times it as above
The runner loads the table automatically (xuanpolicy_amd.runner.enable_tuned_gemms)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

TABLE = os.path.join(REPO, "xuanpolicy_amd", "tuning", "tunableop_results0.csv")


def timed(agent, iters):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        agent.train(agent.n_steps)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def builder(which):
    from xuanpolicy_amd.runner import build_atari_a2c, build_synthbox_ppo
    if which == "c3":
        return lambda **kw: build_atari_a2c(device="cuda:0", **kw)
    if which == "c4":
        return lambda **kw: build_synthbox_ppo(obs_dim=376, act_dim=17, seed=2, device="cuda:0", **kw)
    return lambda **kw: build_synthbox_ppo(device="cuda:0", **kw)


def add(which):
    """Tune one more configuration's shapes, keeping the table's entries (written back at the end)."""
    tun = torch.cuda.tunable
    tun.enable(True)
    if os.path.exists(TABLE):
        tun.read_file(TABLE)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(50)
    tun.set_filename(TABLE, False)
    agent = builder(which)(tunableop=False)
    agent.train(agent.n_steps)
    torch.cuda.synchronize()
    print("table now", len(tun.get_results()), "shapes (written to the table at exit)", flush=True)


def check(which):
    tun = torch.cuda.tunable
    tun.enable(False)
    agent = builder(which)(tunableop=False)
    agent.train(agent.n_steps)
    base = timed(agent, 2)
    tun.enable(True)
    tun.tuning_enable(False)
    tun.read_file(TABLE)
    agent.train(agent.n_steps)
    tuned = timed(agent, 2)
    print("%s untuned ms/iter %.2f tuned ms/iter %.2f speedup %.3f" % (which, base * 1e3, tuned * 1e3, base / tuned),
          flush=True)


def main(mode):
    from xuanpolicy_amd.runner import build_synthbox_ppo
    tun = torch.cuda.tunable
    if mode == "tune":
        os.makedirs(os.path.dirname(TABLE), exist_ok=True)
        if os.path.exists(TABLE):
            os.remove(TABLE)
        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_max_tuning_duration(50)
        tun.set_filename(TABLE, False)
        agent = build_synthbox_ppo(device="cuda:0", tunableop=False)
        agent.train(agent.n_steps)   # every shape met once (rollout step outside capture, then the updates)
        torch.cuda.synchronize()
        print("tuned", len(tun.get_results()), "shapes", flush=True)
        return
    agent = build_synthbox_ppo(device="cuda:0", tunableop=False)
    tun.enable(False)
    agent.train(agent.n_steps)
    base = timed(agent, 3)
    tun.enable(True)
    tun.tuning_enable(False)
    tun.read_file(TABLE)
    agent.train(agent.n_steps)
    tuned = timed(agent, 3)
    print("untuned ms/iter %.2f tuned ms/iter %.2f speedup %.3f" % (base * 1e3, tuned * 1e3, base / tuned), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "add":
        add(sys.argv[2])
    elif len(sys.argv) > 2 and sys.argv[1] == "check":
        check(sys.argv[2])
    else:
        main(sys.argv[1] if len(sys.argv) > 1 else "check")
