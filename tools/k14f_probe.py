"""K14F tail cost probe (r06): the C2 env step's last launch timed with its tail cut at each stage (xpa_k14f_probe bits:
1 = after the block partial stores, 2 = after the group tickets, 4 = after the group sums, 0 = the whole tail) against
K14E alone (no post step), HIP events around a graph of 200 back-to-back launches each; run under rocprofv3 --kernel-trace --stats
for per-kernel durations.  The cursor does not advance under a cut tail (timing only)."""
import json
import sys

import torch

sys.path.insert(0, ".")


def main():
    import xuanpolicy_amd.agents as ag
    from xuanpolicy_amd import ops
    from xuanpolicy_amd.runner import build_synthbox_ppo
    agent = build_synthbox_ppo(n_envs=4096, n_steps=128, obs_dim=17, act_dim=6, hidden=256, n_epoch=1, n_minibatch=4,
                               seed=3, device="cuda:0")
    agent.train(2, log=False)   # warm the rollout path (graphs, workspaces)
    fm = agent._rollout_mlp()
    env = agent.envs
    mem = agent.memory
    x = agent.obs_norm
    rep = fm._rep_forward(x)
    z = fm._rollout_pair(rep[-1])
    H = ops.HEAD_HIDDEN
    lin_ao, lin_co = fm.actor[-1][0], fm.critic[-1][0]
    _, code, slope = fm.actor[-2]
    post = agent._k14f_post(True)
    res = {}

    def launch(p):
        ops.rollout_policy_head_synthbox(z[:, :H], z[:, H:], (code, slope), lin_ao.weight, lin_ao.bias, lin_co.weight,
                                         lin_co.bias, fm.logstd, agent.cursor, agent.seed, mem.actions,
                                         mem.auxiliary_infos["old_logp"], mem.values, env, 1.0, post=p)

    for name, bits, p in (("k14e", 0, None), ("cut1", 1, post), ("cut2", 2, post), ("cut4", 4, post),
                          ("full", 0, post)):
        ops.lib().xpa_k14f_probe(bits)
        for _ in range(20):
            launch(p)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()   # 200 launches replayed as one graph: no host issue time in the window
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(200):
                    launch(p)
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) * 1000 / 200, 2)
    ops.lib().xpa_k14f_probe(0)
    print(json.dumps({"k14f_probe_us_per_launch": res}))


if __name__ == "__main__":
    main()
