"""K2 / K1 flushed sweeps alone (bench.loss_sweep / bench.gae_sweep) under each cache-flush mode, for A/B runs
and rocprofv3 kernel traces.

    python tools/loss_sweep.py [act_dim] [out.json] [modes, e.g. read,write,none]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    A = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    out = {}
    modes = sys.argv[3].split(",") if len(sys.argv) > 3 else ["write", "read", "none"]
    for mode in modes:
        out["loss_" + mode] = bench.loss_sweep("cuda:0", act_dim=A, flush_mode=mode)
        out["gae_" + mode] = bench.gae_sweep("cuda:0", flush_mode=mode)
        for k in ("loss_" + mode, "gae_" + mode):
            for r in out[k]:
                print(k, json.dumps(r), flush=True)
    if len(sys.argv) > 2 and sys.argv[2] != "-":
        json.dump(out, open(sys.argv[2], "w"), indent=1)
