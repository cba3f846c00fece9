"""C1 (CartPole, 8 envs x 128 steps) host-overhead probe: per-iteration wall time split into the rollout and
the update phase (device-synchronised), and a cProfile of the host side of a few iterations.

    python tools/c1_probe.py > gpurun_out/c1_probe.log
"""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from xuanpolicy_amd.runner import build_cartpole_ppo  # noqa: E402


def main():
    agent = build_cartpole_ppo(device="cuda:0")
    T = agent.n_steps
    for _ in range(3):
        agent.train(T, log=False)
    torch.cuda.synchronize()
    upd = agent._update_phase
    split = {"update": 0.0}

    def timed_update():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        upd()
        torch.cuda.synchronize()
        split["update"] += time.perf_counter() - t0

    agent._update_phase = timed_update
    n = 5
    t0 = time.perf_counter()
    for _ in range(n):
        agent.train(T, log=False)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print("iteration ms %.2f  update-phase ms %.2f  rest (rollout) ms %.2f" %
          (el / n * 1e3, split["update"] / n * 1e3, (el - split["update"]) / n * 1e3))
    agent._update_phase = upd
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(3):
        agent.train(T, log=False)
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(s.getvalue())


if __name__ == "__main__":
    main()
