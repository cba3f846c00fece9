#!/bin/bash
# rocprofv3 kernel trace + stats of a short C2 bench run (the per-kernel table of the update / rollout).
# usage: bash tools/r04_prof.sh <tag> [bench args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${1:-r04}
shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o prof -- \
    python -u bench.py --steps 3 --warmup 1 --no-sweep --no-per --no-c1 --no-c3 --no-c4 --no-pmc --no-rocprof \
    --no-cpu-baseline --no-kernel-timing "$@" > $O/${T}_prof.log 2>&1 || { tail -5 $O/${T}_prof.log; exit 3; }
echo prof ok
