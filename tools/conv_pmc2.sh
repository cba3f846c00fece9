#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 120 python -u tools/conv_pmc2.py > $O/pmc2_dry.log 2>&1 || { tail -5 $O/pmc2_dry.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $O/pmc2a -o c -- python tools/conv_pmc2.py > $O/pmc2a.log 2>&1 || { tail -5 $O/pmc2a.log; exit 2; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc2b -o c -- python tools/conv_pmc2.py > $O/pmc2b.log 2>&1 || { tail -5 $O/pmc2b.log; exit 3; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pmc2t -o t -- python tools/conv_pmc2.py > $O/pmc2t.log 2>&1 || exit 4
python tools/conv_pmc_sum.py $O/pmc2a $O/pmc2b > $O/pmc2_sum.json && python -c "
import json; d=json.load(open('$O/pmc2_sum.json'))
for k,v in d.items():
    if 'conv' in k: print(k, {x: v.get(x) for x in ('mfma_busy','SQ_WAIT_ANY_frac','SQ_WAIT_INST_ANY_frac','SQ_ACTIVE_INST_ANY_frac','SQ_INSTS_VALU','SQ_INSTS_MFMA','SQ_INSTS_VMEM_RD','SQ_INSTS_LDS','SQ_LDS_BANK_CONFLICT','SQ_WAIT_INST_LDS_frac')})
"
python tools/kt_top.py $O/pmc2t/t_kernel_trace.csv 8
