#!/bin/bash
# r05: K28B (K28 on the bf16 matrix cores) — tests, kernel timings, C3 A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05k28b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_igemm.py > $O/t1.log 2>&1 || { tail -40 $O/t1.log; exit 1; }
tail -1 $O/t1.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pt -o t -- python -u tools/conv_pmc2.py > $O/pt.log 2>&1 || exit 2
python tools/kt_top.py $O/pt/t_kernel_trace.csv 8
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cnn.py tests/test_gpu_atari.py > $O/t2.log 2>&1 || { tail -40 $O/t2.log; exit 3; }
tail -1 $O/t2.log
timeout -k 10 300 python -u tools/c3_run.py 2 > $O/c3_bf16.json 2> $O/c3.log || exit 4
timeout -k 10 300 python -u tools/c3_run.py 2 igemm-form=0 > $O/c3_f32.json 2>> $O/c3.log || exit 5
timeout -k 10 300 python -u tools/c3_run.py 2 > $O/c3_bf16b.json 2>> $O/c3.log || exit 6
cut -c1-330 $O/c3_bf16.json $O/c3_f32.json $O/c3_bf16b.json
