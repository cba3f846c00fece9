"""Run the C5 leg of bench.py alone (for rocprofv3 --kernel-trace): python tools/c5_run.py [steps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    import torch
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    print(json.dumps(bench.c5_bench(torch.device("cuda:0"), steps=steps, warmup=3, cpu_updates=0)))
