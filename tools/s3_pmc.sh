#!/bin/bash
# rocprofv3 --pmc pass over tools/s3_ab.py (K40 / K41 at the C2 shapes): MFMA busy, LDS activity / stalls.
# usage: bash tools/s3_pmc.sh <tag>   (one pass, 8 SQ counters, its own time limit)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${1:-r04}
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS \
    SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_INSTS_LDS SQ_WAVE_CYCLES --output-format csv -d $O/${T}_s3pmc \
    -o s3pmc -- python -u tools/s3_ab.py --rounds 1 --reps 3 > $O/${T}_s3pmc.log 2>&1 || { tail -5 $O/${T}_s3pmc.log; exit 3; }
echo s3 pmc ok
