"""Diagnostic: per-update drift of the C4-shape iteration against the f64 oracle (tests/_oracle_replay.py report mode)
for the trunk / rollout GEMM forms.  python tools/c4_drift.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(wide, rsplit, seed=17):
    import torch
    from tests._oracle_replay import replay_last_step_iteration
    from xuanpolicy_amd.fused_mlp import FusedActorCritic
    from xuanpolicy_amd.runner import build_synthbox_ppo
    FusedActorCritic.WIDE_TRUNK, FusedActorCritic.ROLLOUT_SPLIT = wide, rsplit
    N, T, D, A, H = 512, 64, 376, 17, 256
    agent = build_synthbox_ppo(n_envs=N, n_steps=T, obs_dim=D, act_dim=A, hidden=H, n_epoch=2, n_minibatch=4,
                               seed=seed, device="cuda:0", max_episode_steps=T + 17)
    agent.train(T, log=False)
    agent.train(T - 1, log=False)
    rep = []
    replay_last_step_iteration(agent, D, A, [H], False, "ppo", 0.0, 2, 4, expect_mid_truncations=True, report=rep)
    out = {"wide": wide, "rollout_split": rsplit, "seed": seed, "updates": [], "weights": {}}
    for r in rep:
        if r[0] == "update":
            got, ref = r[2], r[3]
            out["updates"].append({"u": r[1], "d_actor": got[0] - ref[0], "d_critic": got[1] - ref[1],
                                   "d_entropy": got[2] - ref[2], "actor": ref[0]})
        else:
            out["weights"][r[1]] = [r[2], r[3]]
    del agent
    torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    for wide, rs, seed in ((True, True, 17), (True, False, 17), (False, True, 17), (False, False, 17),
                           (True, True, 18), (False, False, 18)):
        print(json.dumps(run(wide, rs, seed)), flush=True)
