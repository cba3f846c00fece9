#!/bin/bash
# r05: the wide actor head (KMAX 18) without scratch — head parity tests, C4 leg, rocprof of the C4 leg.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused_mlp.py \
  tests/test_gpu_crit_factored.py "tests/test_gpu_fastpath_e2e.py::test_c4_shape_iteration_matches_oracle" \
  "tests/test_gpu_fastpath_e2e.py::test_fast_path_iteration_with_f32_gemms_matches_oracle" > gpurun_out/r05h18_1.log 2>&1 || { tail -40 gpurun_out/r05h18_1.log; exit 1; }
tail -3 gpurun_out/r05h18_1.log
timeout -k 10 200 python -u tools/c4_run.py 3 > gpurun_out/r05h18_c4.json 2> gpurun_out/r05h18_c4.log || exit 1
cat gpurun_out/r05h18_c4.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05h18_prof -o run -- python -u tools/c4_run.py 2 > gpurun_out/r05h18_prof.log 2>&1 || exit 1
python tools/kt_top.py "$(python -c "import glob;print(glob.glob('gpurun_out/r05h18_prof/**/run_kernel_trace.csv',recursive=True)[0])")" 14
