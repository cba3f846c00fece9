#!/bin/bash
# One gpurun call's worth of GPU steps: each step under its own time limit; a step that ends in a fault, abort,
# segfault or time limit (exit >= 124, or 134 / 139) ends the script; a plain test failure (1) does not.
#   bash tools/gpu_round.sh TAG "step command" ["step command" ...]
# Each step's output goes to gpurun_out/TAG_<n>.log; the tail of each is printed.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
TAG=$1
shift
mkdir -p gpurun_out
n=0
worst=0
for step in "$@"; do
    n=$((n + 1))
    log=gpurun_out/${TAG}_${n}.log
    echo "== step $n: $step"
    bash -c "$step" > "$log" 2>&1
    rc=$?
    tail -6 "$log"
    echo "== step $n rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "== stopping after step $n (rc=$rc)"
        exit $rc
    fi
    [ $rc -gt $worst ] && worst=$rc
done
exit $worst
