#!/bin/bash
# r05: C3's first fc layer on the split GEMMs (K40G) — tests, C3 A/B, rocprof.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05fc
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sgemm3.py tests/test_gpu_cnn.py > $O/t1.log 2>&1 || { tail -40 $O/t1.log; exit 1; }
tail -1 $O/t1.log
timeout -k 10 300 python -u tools/c3_run.py 2 fc-split=0 > $O/c3_lib.json 2> $O/c3.log || exit 1
timeout -k 10 300 python -u tools/c3_run.py 2 > $O/c3_split.json 2>> $O/c3.log || exit 1
timeout -k 10 300 python -u tools/c3_run.py 2 fc-split=0 > $O/c3_lib2.json 2>> $O/c3.log || exit 1
timeout -k 10 300 python -u tools/c3_run.py 2 > $O/c3_split2.json 2>> $O/c3.log || exit 1
cut -c1-330 $O/c3_lib.json $O/c3_split.json $O/c3_lib2.json $O/c3_split2.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u tools/c3_run.py 1 > $O/prof.log 2>&1 || exit 3
python tools/kt_top.py $O/prof/run_kernel_trace.csv 24 > $O/top.txt 2>&1; cat $O/top.txt
