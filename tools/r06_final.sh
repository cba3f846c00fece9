#!/bin/bash
# The round's closing measurement set, one gpurun call: the whole GPU suite, smoke(), the default bench line and the
# C2 kernel table (rocprofv3 --kernel-trace --stats; trace files over 4 MB dropped so gpurun_out stays small).
#   bash tools/r06_final.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
T=${1:-r06z}
bash tools/gpu_round.sh "$T" \
    "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
    "timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
    "timeout -k 10 900 python -u bench.py --out gpurun_out/${T}_bench.json" \
    "bash tools/r04_prof.sh $T; rc=\$?; find gpurun_out/${T}_prof -type f -size +4M -delete; exit \$rc"
