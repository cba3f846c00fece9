#!/bin/bash
# r05: conv1 on the bf16 matrix cores (K25B / K26B) — tests, kernel timings, C3 A/B, rocprof.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05c3
O=gpurun_out/r05c3
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cnn.py tests/test_gpu_igemm.py > $O/t1.log 2>&1 || { tail -40 $O/t1.log; exit 1; }
tail -2 $O/t1.log
timeout -k 10 200 python -u tools/c3_run.py --kernels > $O/kernels.json 2> $O/k.log || { tail -20 $O/k.log; exit 1; }
cat $O/kernels.json
timeout -k 10 300 python -u tools/c3_run.py 2 conv1-form=0 > $O/c3_f32.json 2> $O/c3.log || exit 1
timeout -k 10 300 python -u tools/c3_run.py 2 > $O/c3_bf16.json 2>> $O/c3.log || exit 1
timeout -k 10 300 python -u tools/c3_run.py 2 conv1-form=0 > $O/c3_f32b.json 2>> $O/c3.log || exit 1
cut -c1-400 $O/c3_f32.json $O/c3_bf16.json $O/c3_f32b.json
