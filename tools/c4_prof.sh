#!/bin/bash
# C4 leg alone: wall-clock line, then rocprof kernel stats + top kernels; run on the GPU box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/c4_run.py 3 > gpurun_out/c4_run.json 2> gpurun_out/c4_run.log || exit 1
cat gpurun_out/c4_run.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4p -o run -- python -u tools/c4_run.py 2 > gpurun_out/c4p.log 2>&1 || exit 1
python tools/kt_top.py "$(python -c "import glob;print(glob.glob('gpurun_out/c4p/**/run_kernel_trace.csv',recursive=True)[0])")" 15
