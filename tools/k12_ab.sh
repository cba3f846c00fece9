#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/k12_ab.py > gpurun_out/k12_ab.log 2>&1 || { tail -20 gpurun_out/k12_ab.log; exit 1; }
cat gpurun_out/k12_ab.log | grep gemm_heads
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_k12 -o run -- python -u tools/k12_ab.py > gpurun_out/prof_k12.log 2>&1 || exit 2
echo ok
