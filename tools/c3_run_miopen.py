"""tools/c3_run.py with the r02 conv path (MIOpen) for a per-kernel comparison with K28 / K29."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    import torch
    from xuanpolicy_amd import fused_cnn
    fused_cnn._Trunk.use_igemm = False
    print(json.dumps(bench.c3_bench(torch.device("cuda:0"), steps=1, warmup=1, cpu=False, kernels=False)))
