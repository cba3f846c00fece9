#!/bin/bash
# K40T phase probe under the kernel trace: per-kernel device durations (the probe's own event clock is bound by the
# Python launch rate for these ~10 us kernels)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
export PYTHONPATH=$GRAFT_REPO_ROOT
T=${1:-k40tp}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T} -o prof -- \
    python -u tools/k40t_probe.py > gpurun_out/${T}.log 2>&1
rc=$?
find gpurun_out/${T} -type f -size +4M -delete
python - <<PY
import csv, glob
f = glob.glob("gpurun_out/${T}/**/prof_kernel_stats.csv", recursive=True) + glob.glob("gpurun_out/${T}/prof_kernel_stats.csv")
for r in csv.DictReader(open(f[0])):
    n = r["Name"]
    if any(k in n for k in ("trunk_kernel", "r64_kernel", "thin_fwd_norm")):
        print(n[:100], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), round(float(r["MinNs"]) / 1e3, 2))
PY
exit $rc
