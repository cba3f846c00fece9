#!/bin/bash
# r05: K40R (the rollout's paired hidden GEMM on the split) — tests, C2 bench A/B (ROLLOUT_SPLIT on/off), rocprof.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rollout_split.py \
  tests/test_gpu_rollout.py tests/test_gpu_fastpath_e2e.py > gpurun_out/r05r_1.log 2>&1 || { tail -40 gpurun_out/r05r_1.log; exit 1; }
tail -2 gpurun_out/r05r_1.log
B="--no-c1 --no-c3 --no-c4 --no-per --no-cpu-baseline --no-sweep --no-pmc --no-rocprof"
timeout -k 10 300 python -u bench.py $B > gpurun_out/r05r_on.json 2>/dev/null || exit 1
timeout -k 10 300 python -u bench.py $B --rollout-split off > gpurun_out/r05r_off.json 2>/dev/null || exit 1
timeout -k 10 300 python -u bench.py $B > gpurun_out/r05r_on2.json 2>/dev/null || exit 1
for f in on off on2; do python -c "
import json; d=json.loads(open('gpurun_out/r05r_$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['phase_split_ms']['rollout'], d['phase_split_ms']['update_incl_gae'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05r_prof -o run -- python -u bench.py $B --steps 3 --warmup 1 --no-kernel-timing > gpurun_out/r05r_prof.log 2>&1 || exit 1
python tools/kt_top.py "$(python -c "import glob;print(glob.glob('gpurun_out/r05r_prof/**/run_kernel_trace.csv',recursive=True)[0])")" 16
