"""A/B of the conv kernel forms (xpa_conv1_form masks) at the C3 update shapes: python tools/conv_ab.py 7 15 ..."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    import torch
    from xuanpolicy_amd import ops
    L = ops.lib()
    for m in sys.argv[1:]:
        L.xpa_conv1_form(int(m))
        r = bench.c3_kernels(torch.device("cuda:0"))   # restores the mask it found: this one
        print(json.dumps({"mask": int(m), **{k: v["avg_launch_us"] for k, v in r.items()}}), flush=True)
