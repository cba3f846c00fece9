#!/bin/bash
# rocprof kernel stats of the C2 bench for each K16 form (XPA_K16); run on the GPU box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for f in "$@"; do
  XPA_K16=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k16p_$f -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-sweep --no-per --no-c1 --no-c3 --no-c4 --no-kernel-timing > gpurun_out/k16p_$f.log 2>&1 || exit 1
done
