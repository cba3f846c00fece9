"""C1 (PPO CartPole, 8 envs x 128 steps, [64] nets) alone, for rocprofv3 --kernel-trace: python tools/c1_run.py [iters]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    import torch
    from xuanpolicy_amd.runner import build_cartpole_ppo
    it = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    agent = build_cartpole_ppo(n_envs=8, n_steps=128, hidden=64, seed=1, device="cuda:0")
    for _ in range(3):
        agent.train(128, log=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        agent.train(128, log=False)
    torch.cuda.synchronize()
    print("ms/iter", (time.perf_counter() - t0) / it * 1e3)
