#!/bin/bash
# The round's closing measurement set, one gpurun call: the whole GPU suite, smoke(), the default bench line (PMC
# traffic, CPU baseline, sweeps, the C1 / C3 / C4 / C5 legs) and the C2 kernel table.  Each step has its own time
# limit; a fault / abort / time limit ends the script (tools/gpu_round.sh).
#   bash tools/r04_final.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
T=${1:-r04x}
exec_round() { bash tools/gpu_round.sh "$@"; }
exec_round "$T" \
    "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
    "timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
    "timeout -k 10 900 python -u bench.py --out gpurun_out/${T}_bench.json" \
    "bash tools/r04_prof.sh $T"
