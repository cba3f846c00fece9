"""A/B of the C3 update's conv path: K28 / K29 (use_igemm) against MIOpen (the r02 path), same box, same process.
python tools/c3_ab.py [iterations]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    import torch
    from xuanpolicy_amd import fused_cnn
    from xuanpolicy_amd.runner import build_atari_a2c
    it = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    dev = torch.device("cuda:0")
    out = {}
    for mode in (True, False, True):
        fused_cnn._Trunk.use_igemm = mode
        agent = build_atari_a2c(n_envs=1024, n_steps=128, device=dev)
        agent.train(128)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(it):
            agent.train(128)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / it * 1e3
        out.setdefault("igemm" if mode else "miopen", []).append(round(ms, 2))
        print(mode, round(ms, 2), flush=True)
        del agent
        torch.cuda.empty_cache()
    print(json.dumps(out))
