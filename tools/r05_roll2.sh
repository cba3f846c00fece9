#!/bin/bash
# r05: rollout A/B — K40R on/off x the rollout trunk's h stores plain/nt; rocprof of the default.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 tests/test_gpu_rollout_split.py tests/test_gpu_rollout.py > gpurun_out/r05r2_t.log 2>&1 || { tail -30 gpurun_out/r05r2_t.log; exit 1; }
tail -1 gpurun_out/r05r2_t.log
B="--no-c1 --no-c3 --no-c4 --no-per --no-cpu-baseline --no-sweep --no-pmc --no-rocprof"
for rep in 1; do
for cfg in "on nt" "off nt" "on plain" "off plain"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py $B --rollout-split $1 --rollout-h-store $2 > gpurun_out/r05r2_$1_$2_$rep.json 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/r05r2_$1_$2_$rep.json').read().strip().splitlines()[-1]); print('$1 $2 $rep', d['value'], d['phase_split_ms']['rollout'], d['phase_split_ms']['update_incl_gae'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05r2_prof -o run -- python -u bench.py $B --steps 3 --warmup 1 --no-kernel-timing > gpurun_out/r05r2_prof.log 2>&1 || exit 1
python tools/kt_top.py "$(python -c "import glob;print(glob.glob('gpurun_out/r05r2_prof/**/run_kernel_trace.csv',recursive=True)[0])")" 16
