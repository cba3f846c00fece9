#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05fcact; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cnn.py tests/test_gpu_atari.py tests/test_gpu_sgemm3.py -k "not wgrad_matches and not gemm_matches_f32" > $O/t1.log 2>&1 || { tail -40 $O/t1.log; exit 1; }
tail -1 $O/t1.log
timeout -k 10 300 python -u tools/c3_run.py 2 > $O/c3_on.json 2> $O/c3.log || exit 2
timeout -k 10 300 python -u tools/c3_run.py 2 fc-act=0 > $O/c3_off.json 2>> $O/c3.log || exit 3
timeout -k 10 300 python -u tools/c3_run.py 2 > $O/c3_on2.json 2>> $O/c3.log || exit 4
timeout -k 10 300 python -u tools/c3_run.py 2 fc-act=0 > $O/c3_off2.json 2>> $O/c3.log || exit 5
cut -c1-330 $O/c3_on.json $O/c3_off.json $O/c3_on2.json $O/c3_off2.json
