#!/bin/bash
# Extend the TunableOp table with the C3 / C4 GEMM shapes and check the effect (GPU box).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
cp xuanpolicy_amd/tuning/tunableop_results0.csv $O/tunable_before.csv
timeout -k 10 500 python -u tools/tune_gemms.py add c3 > $O/tune_c3.log 2>&1 || { tail -20 $O/tune_c3.log; exit 1; }
tail -2 $O/tune_c3.log; wc -l xuanpolicy_amd/tuning/tunableop_results0.csv
timeout -k 10 400 python -u tools/tune_gemms.py add c4 > $O/tune_c4.log 2>&1 || { tail -20 $O/tune_c4.log; exit 2; }
tail -2 $O/tune_c4.log
cp xuanpolicy_amd/tuning/tunableop_results0.csv $O/tunable_after.csv
timeout -k 10 300 python -u tools/tune_gemms.py check c3 > $O/check_c3.log 2>&1 || { tail -20 $O/check_c3.log; exit 3; }
tail -1 $O/check_c3.log
timeout -k 10 300 python -u tools/tune_gemms.py check c4 > $O/check_c4.log 2>&1 || { tail -20 $O/check_c4.log; exit 4; }
tail -1 $O/check_c4.log
echo ok
