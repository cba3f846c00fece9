"""A/B of the C3 update's first-fc weight gradient (r06): K41V on the bf16 split (fused_cnn._Trunk.fc_wsplit) against
the hipBLASLt f32 GEMM, same box, same process, arms alternated (A B A B), each 1 warm-up + `it` timed iterations of
A2C on 1024 SynthAtari envs x 128 steps.  python tools/c3_fcw_ab.py [iterations]"""
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
    for mode in (True, False, True, False):
        fused_cnn._Trunk.fc_wsplit = mode
        agent = build_atari_a2c(n_envs=1024, n_steps=128, device=dev)
        agent.train(128)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(it):
            agent.train(128)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / it * 1e3
        out.setdefault("k41v" if mode else "hipblaslt", []).append(round(ms, 2))
        print(mode, round(ms, 2), flush=True)
        del agent
        torch.cuda.empty_cache()
    print(json.dumps(out))
