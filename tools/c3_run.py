"""Run the C3 leg of bench.py alone (for rocprofv3 --kernel-trace): python tools/c3_run.py [iterations] [--full]
(--full adds the kernel roofline and the bounded CPU baseline)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    import torch
    it = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 1
    full = "--full" in sys.argv
    for a in sys.argv[1:]:   # r05 A/B: conv1-form=<mask> (xpa_conv1_form: bit 0 K25B, bit 1 K26B)
        if a.startswith("conv1-form="):
            from xuanpolicy_amd import ops
            ops.lib().xpa_conv1_form(int(a.split("=")[1]))
        if a.startswith("igemm-form="):   # r05 A/B: xpa_conv_igemm_form (bit 0 K28B)
            from xuanpolicy_amd import ops
            ops.lib().xpa_conv_igemm_form(int(a.split("=")[1]))
        if a.startswith("fc-act="):   # r05 A/B: the last conv's activation backward in the fc epilogue (1) or K22 (0)
            from xuanpolicy_amd import fused_cnn
            fused_cnn._Trunk.fc_fuse_act = bool(int(a.split("=")[1]))
        if a.startswith("fc-split="):   # r05 A/B: the first fc layer on K40G (1) or hipBLASLt (0)
            from xuanpolicy_amd import fused_cnn
            fused_cnn._Trunk.fc_split = bool(int(a.split("=")[1]))
    if "--kernels" in sys.argv:
        print(json.dumps(bench.c3_kernels(torch.device("cuda:0"))))
        sys.exit(0)
    print(json.dumps(bench.c3_bench(torch.device("cuda:0"), steps=it, warmup=1, cpu=full, kernels=full)))
