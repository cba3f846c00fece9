"""Run the C4 leg of bench.py alone (for rocprofv3 --kernel-trace): python tools/c4_run.py [iterations]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    import torch
    it = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 2
    if "wide-off" in sys.argv:   # the r04 trunk (library GEMMs) for A/B
        from xuanpolicy_amd.fused_mlp import FusedActorCritic
        FusedActorCritic.WIDE_TRUNK = False
    if "gather" in sys.argv:     # the wide trunk on the pitched gather (no row-index forms) for A/B
        from xuanpolicy_amd.fused_mlp import FusedActorCritic
        FusedActorCritic.WIDE_DIRECT = False
    print(json.dumps(bench.c4_bench(torch.device("cuda:0"), 0, 1, steps=it, warmup=1)))
