#!/bin/bash
# r05: obs-RMS fold into K8 — tests (rollout, e2e, hostenv), C2 A/B (fold on/off), rocprof.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rollout_split.py \
  tests/test_gpu_rollout.py tests/test_gpu_fastpath_e2e.py tests/test_gpu_hostenv.py tests/test_gpu_kernels.py > gpurun_out/r05f_1.log 2>&1 || { tail -40 gpurun_out/r05f_1.log; exit 1; }
tail -2 gpurun_out/r05f_1.log
B="--no-c1 --no-c3 --no-c4 --no-per --no-cpu-baseline --no-sweep --no-pmc --no-rocprof"
for cfg in on off on off; do
  timeout -k 10 300 python -u bench.py $B --fold-rms $cfg > gpurun_out/r05fold_$cfg.json 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/r05fold_$cfg.json').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['phase_split_ms']['rollout'], d['phase_split_ms']['update_incl_gae'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05fold_prof -o run -- python -u bench.py $B --steps 3 --warmup 1 --no-kernel-timing > gpurun_out/r05fold_prof.log 2>&1 || exit 1
python tools/kt_top.py "$(python -c "import glob;print(glob.glob('gpurun_out/r05fold_prof/**/run_kernel_trace.csv',recursive=True)[0])")" 16
