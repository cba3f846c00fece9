"""A/B on the GPU box: the C2 update with K16 (hidden GEMM inside the head kernels) vs the paired hipBLASLt GEMM + K12
(fm.gemm_heads = False).  Prints ms per iteration for each, 2 warm-up + 4 timed iterations."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    import torch
    from xuanpolicy_amd.runner import build_synthbox_ppo
    for gemm_heads in (True, False, True, False):
        torch.manual_seed(1)
        agent = build_synthbox_ppo(device="cuda:0")
        agent.learner.enable_fast_path()
        fm = agent.learner._fused_mlp()
        fm.gemm_heads = gemm_heads
        for _ in range(2):
            agent.train(agent.n_steps)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(4):
            agent.train(agent.n_steps)
        torch.cuda.synchronize()
        print("gemm_heads", gemm_heads, "ms/iter %.2f" % ((time.perf_counter() - t) / 4 * 1e3), flush=True)
        del agent, fm
        torch.cuda.empty_cache()
