#!/bin/bash
# r05: C4's wide trunk straight from the rollout buffer (row-index K40F / K41V) — tests, C4 A/B, rocprof.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide_trunk.py \
  "tests/test_gpu_fastpath_e2e.py::test_c4_shape_iteration_matches_oracle" tests/test_gpu_rollout.py > gpurun_out/r05d_1.log 2>&1 || { tail -40 gpurun_out/r05d_1.log; exit 1; }
tail -2 gpurun_out/r05d_1.log
timeout -k 10 200 python -u tools/c4_run.py 3 > gpurun_out/r05d_c4_direct.json 2> gpurun_out/r05d_c4.log || exit 1
timeout -k 10 200 python -u tools/c4_run.py 3 gather > gpurun_out/r05d_c4_gather.json 2>> gpurun_out/r05d_c4.log || exit 1
timeout -k 10 200 python -u tools/c4_run.py 3 > gpurun_out/r05d_c4_direct2.json 2>> gpurun_out/r05d_c4.log || exit 1
cut -c1-250 gpurun_out/r05d_c4_direct.json gpurun_out/r05d_c4_gather.json gpurun_out/r05d_c4_direct2.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05d_prof -o run -- python -u tools/c4_run.py 2 > gpurun_out/r05d_prof.log 2>&1 || exit 1
python tools/kt_top.py "$(python -c "import glob;print(glob.glob('gpurun_out/r05d_prof/**/run_kernel_trace.csv',recursive=True)[0])")" 14
