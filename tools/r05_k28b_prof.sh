#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05k28b; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p1 -o run -- python -u tools/c3_run.py 1 > $O/p1.log 2>&1 || exit 1
python tools/kt_top.py $O/p1/run_kernel_trace.csv 14
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p0 -o run -- python -u tools/c3_run.py 1 igemm-form=0 > $O/p0.log 2>&1 || exit 2
python tools/kt_top.py $O/p0/run_kernel_trace.csv 14
