"""C4 shard (SynthBox(376, 17), 4096 envs) alone for a rocprofv3 --kernel-trace --stats run:
    rocprofv3 --kernel-trace --stats -d gpurun_out/c4 -o c4 -- python tools/c4_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    t0 = time.perf_counter()
    print(bench.c4_bench(torch.device("cuda:0"), 0, 1), flush=True)
    print("wall %.1f s" % (time.perf_counter() - t0))
