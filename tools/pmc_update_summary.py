"""Summarise one rocprofv3 --pmc pass of tools/r04_update_pmc.sh (8 SQ counters over a short C2 bench run) into
per-kernel averages for the update's kernels, with the MFMA-busy fraction used in profiles/r04f_k16_pmc.json:
SQ_VALU_MFMA_BUSY_CYCLES (summed over the 1024 SIMDs) / (SQ_BUSY_CYCLES (summed over the 32 shader engines) / 32 x
1024) = MFMA / (BUSY x 32).

    python tools/pmc_update_summary.py gpurun_out/r04u_pmc profiles/r04u_update_pmc.json"""
import csv
import glob
import json
import sys
from collections import defaultdict

KEYS = ("s3_wgrad", "s3_gemm_trunk_bwd", "s3_trunk_bwd", "head_gemm_kernel", "thin_fwd", "colsum_finalize", "clip_adam",
        "split_batch", "gae_dpp", "rollout_policy_head", "Cijk", "s3_gemm_r64", "rms_partials", "rollout_post")


def main(pmc_dir, out):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(pmc_dir + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if not any(k in name for k in KEYS):
                continue
            short = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            if "Cijk" in short:
                short = "hipBLASLt " + short[:40]
            acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {"source": "rocprofv3 --pmc, one pass of 8 SQ counters over `bench.py --steps 1 --warmup 1` (C2); per-dispatch "
                     "means", "mfma_busy_frac": "SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES x 32)", "kernels": {}}
    for k, cs in sorted(acc.items()):
        d = {c: round(sum(v) / len(v), 1) for c, v in sorted(cs.items())}
        d["dispatches"] = max(len(v) for v in cs.values())
        busy = d.get("SQ_BUSY_CYCLES", 0.0)
        if busy:
            d["mfma_busy_frac"] = round(d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (busy * 32), 3)
        wave = d.get("SQ_WAVE_CYCLES", 0.0)
        if wave:
            d["wait_inst_lds_per_wave_cycle"] = round(d.get("SQ_WAIT_INST_LDS", 0.0) / wave, 4)
            d["wait_any_per_wave_cycle"] = round(d.get("SQ_WAIT_ANY", 0.0) / wave, 4)
            for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC"):
                if c in d:   # issue quad-cycles of that instruction class per wave quad-cycle
                    d[c.replace("SQ_ACTIVE_INST_", "").lower() + "_issue_per_wave_cycle"] = round(d[c] / wave, 4)
        res["kernels"][k] = d
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: {x: v.get(x) for x in ("mfma_busy_frac", "dispatches", "wait_inst_lds_per_wave_cycle")}
                      for k, v in res["kernels"].items()}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
