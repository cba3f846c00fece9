#!/bin/bash
# One rocprofv3 --pmc pass (8 SQ counters) over a short C2 bench run: the update kernels' MFMA-busy / LDS-wait
# counters (summarised by tools/pmc_update_summary.py).  usage: bash tools/r04_update_pmc.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${1:-r04u}
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/${T}_pmc -o pmc -- \
    python -u bench.py --steps 1 --warmup 1 --no-sweep --no-per --no-c1 --no-c3 --no-c4 --no-pmc --no-rocprof \
    --no-cpu-baseline --no-kernel-timing > $O/${T}_pmc.log 2>&1 || { tail -5 $O/${T}_pmc.log; exit 3; }
echo pmc ok
