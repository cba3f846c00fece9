"""Phase timestamps (s_memtime, thread 0) of K30 xpa_small_mlp_update at C1: python tools/k30_stamps.py [split]
(split: the split form's workgroup 0 — its partials end at dW0 / bias sums; clip + Adam run in the finalize launch)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    import torch
    from xuanpolicy_amd.runner import build_cartpole_ppo
    agent = build_cartpole_ppo(n_envs=8, n_steps=128, hidden=64, seed=1, device="cuda:0", graph_update=False)
    agent.train(128, log=False)
    st = torch.zeros(16, dtype=torch.int64, device="cuda:0")
    agent.learner.small_stamps = st
    split = len(sys.argv) > 1 and sys.argv[1] == "split"
    agent.learner.small_split = split
    names = ["start", "staged", "fwd hidden", "out layers", "loss", "dW out", "dh1 dh2", "dW hidden", "dh0", "dW0",
             "adam"]
    for _ in range(3):
        agent.train(128, log=False)
        torch.cuda.synchronize()
        v = st.cpu().tolist()
        last = 9 if split else 10
        print(" ".join("%s %d" % (names[i + 1], v[i + 1] - v[i]) for i in range(last)), "| total", v[last] - v[0])
