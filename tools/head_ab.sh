#!/bin/bash
# A/B of two builds of the library on one box, alternated: the current one (A) and ab/lib_oldhead.so (B), C2 bench
# legs only.  usage: bash tools/head_ab.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
T=${1:-hab}
L=xuanpolicy_amd/libxuanpolicy_amd.so
cp $L ab/lib_cur.so || exit 2
ARGS="--steps 8 --warmup 2 --no-sweep --no-per --no-c1 --no-c3 --no-c4 --no-pmc --no-rocprof --no-cpu-baseline"
for i in 1 2 3; do
  for arm in cur oldhead; do
    cp ab/lib_$arm.so $L || exit 2
    timeout -k 10 300 python -u bench.py $ARGS --out gpurun_out/${T}_${arm}_$i.json > gpurun_out/${T}_${arm}_$i.log 2>&1 || { echo "fail $arm $i"; exit 3; }
    python -c "import json; d=json.load(open('gpurun_out/${T}_${arm}_$i.json')); print('$arm', $i, d['value'], d['update_kernels']['heads']['avg_us'], d['phase_split_ms']['update_incl_gae'])"
  done
done
cp ab/lib_cur.so $L
