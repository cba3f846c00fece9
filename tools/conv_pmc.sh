#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $O/pmc_conv -o c -- python tools/conv_pmc.py > $O/pmc_conv.log 2>&1 || { tail -5 $O/pmc_conv.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc_conv2 -o c -- python tools/conv_pmc.py > $O/pmc_conv2.log 2>&1 || { tail -5 $O/pmc_conv2.log; exit 2; }
python tools/conv_pmc_sum.py $O/pmc_conv $O/pmc_conv2 > $O/pmc_conv_sum.json && cat $O/pmc_conv_sum.json
