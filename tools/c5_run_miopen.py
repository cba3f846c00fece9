"""tools/c5_run.py with the r02 conv path (MIOpen) for a per-kernel comparison with K28 / K29."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    import torch
    from xuanpolicy_amd import fused_cnn
    fused_cnn._Trunk.use_igemm = False
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    print(json.dumps(bench.c5_bench(torch.device("cuda:0"), steps=steps, warmup=3, cpu_updates=0)))
