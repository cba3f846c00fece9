#!/bin/bash
# K29 staging change on the GPU box: the conv kernel tests, then a rocprofv3 kernel trace of one C3 iteration.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${1:-k29}
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_igemm.py tests/test_gpu_cnn.py -m gpu > $O/${T}_pytest.log 2>&1 || { tail -30 $O/${T}_pytest.log; exit 1; }
tail -1 $O/${T}_pytest.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_c3 -o run -- python -u tools/c3_run.py 1 > $O/${T}_prof_c3.log 2>&1 || { tail -5 $O/${T}_prof_c3.log; exit 3; }
python tools/kt_top.py $(ls $O/${T}_prof_c3/*/run_kernel_trace.csv 2>/dev/null || ls $O/${T}_prof_c3/run_kernel_trace.csv) 16 > $O/${T}_top_c3.txt 2>&1; cat $O/${T}_top_c3.txt
