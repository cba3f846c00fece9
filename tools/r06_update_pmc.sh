#!/bin/bash
# Round 6: PMC passes over a short C2 bench run (the round-6 defaults: K16Q heads with the quad phase 2, K41P / K42C),
# one rocprofv3 --pmc pass per counter set (a pass holds at most 8 SQ counters), summarised per kernel by
# tools/pmc_update_summary.py.  usage: bash tools/r06_update_pmc.sh <tag> [pass ...]   (passes: mfma valu fetch write; default mfma valu)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${1:-r06u}
shift
PASSES=${@:-mfma valu}
for P in $PASSES; do
  case $P in
    mfma) C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT";;
    valu) C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE";;
    fetch) C="FETCH_SIZE";;   # TCC: FETCH_SIZE (3 counters) and WRITE_SIZE (2) need passes of their own
    write) C="WRITE_SIZE";;
    *) echo "unknown pass $P"; exit 2;;
  esac
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/${T}_$P -o pmc -- \
      python -u bench.py --steps 1 --warmup 1 --no-sweep --no-per --no-c1 --no-c3 --no-c4 --no-pmc --no-rocprof \
      --no-cpu-baseline --no-kernel-timing --dp-path off > $O/${T}_$P.log 2>&1 || { tail -5 $O/${T}_$P.log; exit 3; }
  python tools/pmc_update_summary.py $O/${T}_$P $O/${T}_$P.json > /dev/null || exit 4
  echo "pmc $P ok"
done
