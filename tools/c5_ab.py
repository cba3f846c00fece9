"""A/B of the C5 (PER-DQN, batch 2048) learner step's conv path: K28 / K29 (use_igemm) against MIOpen (the r02 path),
same box, same process.  python tools/c5_ab.py [steps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    import torch
    from xuanpolicy_amd import fused_cnn
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    out = {}
    for mode in (True, False, True):
        fused_cnn._Trunk.use_igemm = mode
        r = bench.c5_bench(torch.device("cuda:0"), steps=steps, warmup=3, cpu_updates=0)
        out.setdefault("igemm" if mode else "miopen", []).append(r["ms_per_step"])
        print(mode, r["ms_per_step"], flush=True)
        torch.cuda.empty_cache()
    print(json.dumps(out))
