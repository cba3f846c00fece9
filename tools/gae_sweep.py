"""Flushed GAE sweep (same as bench.py's gae_sweep_flushed) as a standalone A/B driver:
   XPA_GAE_NT=0|1 python tools/gae_sweep.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    res = bench.gae_sweep(torch.device("cuda:0"), sizes=(4096, 65536, 262144, 1048576, 2097152), reps=9)
    print(json.dumps({"XPA_GAE_NT": os.environ.get("XPA_GAE_NT", "auto"), "sweep": res}))
