#!/bin/bash
# rocprofv3 --pmc passes over tools/k16w_ab.py (K16 and K16W actor / critic at the C2 shape), one pass per counter group
# (the SQ block holds 8 counters per pass).  usage: bash tools/r04_pmc.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${1:-r04}
timeout -s KILL 60 rocprofv3 -L > $O/${T}_pmc_avail.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/${T}_pmc1 -o pmc1 -- \
    python -u tools/k16w_ab.py --rounds 1 --reps 3 > $O/${T}_pmc1.log 2>&1 || { tail -5 $O/${T}_pmc1.log; exit 3; }
echo pmc ok
