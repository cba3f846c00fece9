#!/bin/bash
# K40T (XPA_ROLLOUT_TRUNK=1) against K13-norm + K40R: the rollout tests, alternated C2 bench legs, a kernel trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rollout_split.py tests/test_gpu_fastpath_e2e.py > gpurun_out/k40t_tests.log 2>&1 || { tail -30 gpurun_out/k40t_tests.log; exit 3; }
tail -3 gpurun_out/k40t_tests.log
ARGS="--steps 8 --warmup 2 --no-sweep --no-per --no-c1 --no-c3 --no-c4 --no-pmc --no-rocprof --no-cpu-baseline"
XPA_ROLLOUT_TRUNK=1 timeout -k 10 300 python -u bench.py $ARGS --out gpurun_out/k40t_on.json > gpurun_out/k40t_on.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py $ARGS --out gpurun_out/k40t_off.json > gpurun_out/k40t_off.log 2>&1 || exit 5
XPA_ROLLOUT_TRUNK=1 timeout -k 10 300 python -u bench.py $ARGS --out gpurun_out/k40t_on2.json > gpurun_out/k40t_on2.log 2>&1 || exit 6
for f in on off on2; do python -c "import json; d=json.load(open('gpurun_out/k40t_$f.json')); print('$f', d['value'], d['phase_split_ms'])"; done
XPA_ROLLOUT_TRUNK=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k40t_prof -o prof -- python -u bench.py --steps 3 --warmup 1 --no-sweep --no-per --no-c1 --no-c3 --no-c4 --no-pmc --no-rocprof --no-cpu-baseline --no-kernel-timing > gpurun_out/k40t_prof.log 2>&1
find gpurun_out/k40t_prof -type f -size +4M -delete
