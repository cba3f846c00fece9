#!/bin/bash
# C3 / C5 CNN path on the GPU box: the CNN GPU tests, the C3 bench leg, a rocprof kernel trace of one C3 iteration.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
TAG=${1:-c3}
timeout -k 10 500 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_atari.py tests/test_gpu_perdqn.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$TAG.log 2>&1 || { tail -40 $O/pytest_$TAG.log; exit 1; }
tail -1 $O/pytest_$TAG.log
timeout -k 10 300 python -u tools/c3_run.py 2 > $O/c3run_$TAG.log 2>&1 || { tail -20 $O/c3run_$TAG.log; exit 2; }
python -c "import json;d=json.loads(open('$O/c3run_$TAG.log').read().strip().splitlines()[-1]);print('$TAG c3', d['value'], d['ms_per_iteration'], d.get('host_timer_split_ms'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python -u tools/c3_run.py 2 > $O/prof_$TAG.log 2>&1 || exit 3
echo ok
