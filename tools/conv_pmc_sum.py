"""Per-kernel sums of the rocprofv3 --pmc passes of tools/conv_pmc.sh (mean over launches):
python tools/conv_pmc_sum.py gpurun_out/pmc_conv gpurun_out/pmc_conv2"""
import csv
import glob
import json
import sys
from collections import defaultdict

if __name__ == "__main__":
    acc = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            per = defaultdict(float)
            for r in csv.DictReader(open(f)):
                name = r.get("Kernel_Name", "")
                name = name.replace("void ", "").replace("(anonymous namespace)::", "")
                name = name[:name.index("(")] if "(" in name else name
                per[(name, r.get("Dispatch_Id"), r["Counter_Name"])] += float(r["Counter_Value"])
            for (name, _, c), v in per.items():
                acc[name][c].append(v)
    out = {}
    for name, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        if "SQ_BUSY_CYCLES" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            m["mfma_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["SQ_BUSY_CYCLES"] * 32)
        if "SQ_WAVE_CYCLES" in m:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if k in m:
                    m[k + "_frac"] = m[k] / m["SQ_WAVE_CYCLES"]
        out[name.split("::")[-1]] = {k: round(v, 4) for k, v in m.items()}
    print(json.dumps(out, indent=1))
