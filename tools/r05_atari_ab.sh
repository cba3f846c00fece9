#!/bin/bash
# r05: the G8P A2C replay (prod nets) under the conv / fc forms, to see which one moves the update drift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ab; mkdir -p $O
T="tests/test_gpu_atari.py::test_a2c_atari_replays_reference_agent"
for cfg in "7 1" "7 0" "0 1" "0 0"; do
  set -- $cfg
  XPA_AB_CONV_FORM=$1 XPA_AB_FC_SPLIT=$2 PYTHONPATH=tools timeout -k 10 300 python -u -m pytest -p ab_plugin -q --timeout 200 --timeout-method thread "$T" > $O/ab_$1_$2.log 2>&1
  rc=$?
  echo "form=$1 fc=$2 rc=$rc $(tail -1 $O/ab_$1_$2.log)"
  grep -o "update [0-9]*: got \[[^]]*\] ref \[[^]]*\]" $O/ab_$1_$2.log | head -3
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
