"""K32 phase timing (s_memtime cycles per phase, averaged over the steps of one 128-step launch) on the C1 agent:
python tools/k32_stamps.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    import torch
    from xuanpolicy_amd.runner import build_cartpole_ppo
    agent = build_cartpole_ppo(n_envs=8, n_steps=128, hidden=64, seed=1, device="cuda:0")
    st = torch.zeros(16, dtype=torch.int64, device="cuda:0")
    names = ["rms", "normalise", "-", "-", "forward", "sample+env+post", "ret_rms", "loop barrier"]
    for it in range(4):
        a = agent._small_rollout()
        a.stamps = st.data_ptr()
        agent.train(128, log=False)
        torch.cuda.synchronize()
        v = st.cpu().tolist()
        print(" ".join("%s %.0f" % (n, v[i] / 128) for i, n in enumerate(names)),
              "| per step %.0f cycles, launch %.0f" % (v[8] / 128, v[8]))
