#!/bin/bash
# rocprof kernel traces of the C5 and C4 bench legs (GPU box).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_c5 -o run -- python -u tools/c5_run.py > $O/prof_c5.log 2>&1 || { tail -5 $O/prof_c5.log; exit 1; }
tail -1 $O/prof_c5.log
python tools/kt_top.py $O/prof_c5/run_kernel_trace.csv 18
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_c4 -o run -- python -u tools/c4_run.py > $O/prof_c4.log 2>&1 || { tail -5 $O/prof_c4.log; exit 2; }
tail -1 $O/prof_c4.log
python tools/kt_top.py $O/prof_c4/run_kernel_trace.csv 14
