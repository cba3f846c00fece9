#!/bin/bash
# r05: the wide trunk (C4) on the split GEMMs — parity tests, C4 A/B, rocprof of the C4 leg.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wide_trunk.py \
  "tests/test_gpu_fastpath_e2e.py::test_c4_shape_iteration_matches_oracle" > gpurun_out/r05w_1.log 2>&1 || { tail -40 gpurun_out/r05w_1.log; exit 1; }
tail -3 gpurun_out/r05w_1.log
timeout -k 10 200 python -u tools/c4_run.py 3 > gpurun_out/r05w_c4_on.json 2> gpurun_out/r05w_c4_on.log || exit 1
timeout -k 10 200 python -u tools/c4_run.py 3 wide-off > gpurun_out/r05w_c4_off.json 2> gpurun_out/r05w_c4_off.log || exit 1
cat gpurun_out/r05w_c4_on.json gpurun_out/r05w_c4_off.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05w_prof -o run -- python -u tools/c4_run.py 2 > gpurun_out/r05w_prof.log 2>&1 || exit 1
python tools/kt_top.py "$(python -c "import glob;print(glob.glob('gpurun_out/r05w_prof/**/run_kernel_trace.csv',recursive=True)[0])")" 22
