#!/bin/bash
# Quick GPU check: the named GPU test files, one short C2 bench, a rocprof kernel-stats pass of it.
#   bash tools/quick_prof.sh TAG tests/test_a.py tests/test_b.py ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
TAG=$1; shift
if [ $# -gt 0 ]; then
  timeout -k 10 500 python -u -m pytest "$@" -x -q --timeout 200 --timeout-method thread > $O/pytest_$TAG.log 2>&1 || { tail -40 $O/pytest_$TAG.log; exit 1; }
  tail -1 $O/pytest_$TAG.log
fi
Q="--no-cpu-baseline --no-sweep --no-per --no-c1 --no-c3 --no-c4"
timeout -k 10 200 python -u bench.py --steps 6 $Q --out $O/q_$TAG.json > $O/q_$TAG.log 2>&1 || { tail -20 $O/q_$TAG.log; exit 2; }
python -c "import json;d=json.loads(open('$O/q_$TAG.json').read().strip().splitlines()[-1]);print('$TAG', d['value'], d['ms_per_step'], d['phase_split_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python -u bench.py --steps 3 $Q --out $O/qp_$TAG.json > $O/prof_$TAG.log 2>&1 || exit 3
python tools/kt_top.py $O/prof_$TAG/run_kernel_trace.csv 16 > $O/top_$TAG.txt 2>&1; cat $O/top_$TAG.txt
echo ok
