#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ab; mkdir -p $O
T="tests/test_gpu_atari.py::test_a2c_atari_replays_reference_agent"
for fc in 1 0; do
  XPA_REPORT_ENVELOPE=1 XPA_AB_FC_SPLIT=$fc PYTHONPATH=tools timeout -k 10 300 python -u -m pytest -p ab_plugin -q -s --timeout 200 --timeout-method thread "$T" -k "prod" > $O/env_$fc.log 2>&1
  echo "fc=$fc rc=$? $(tail -1 $O/env_$fc.log)"
  grep ENVELOPE $O/env_$fc.log
done
