"""Tune the GEMM shapes of the C2 PPO iteration with PyTorch TunableOp (hipBLASLt + rocBLAS solution search).

    python tools/tune_gemms.py tune    # tunes every shape met in one iteration; the table is written at exit
                                       # to xuanpolicy_amd/tuning/tunableop_results0.csv
    python tools/tune_gemms.py check   # times iterations with TunableOp off vs the tuned table (tuning off)
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
    main(sys.argv[1] if len(sys.argv) > 1 else "check")
