#!/bin/bash
# A/B of the K16 forms (XPA_K16, csrc/head.hip) on the C2 bench's heads timing; run on the GPU box.
set -o pipefail
for f in "$@"; do
  XPA_K16=$f timeout -k 10 200 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-sweep --no-per --no-c1 --no-c3 --no-c4 --out gpurun_out/k16_ab_$f.json > gpurun_out/k16_ab_$f.log 2>&1 || exit 1
  python -c "import json;d=json.load(open('gpurun_out/k16_ab_$f.json'));print('form $f', d['value'], d['ms_per_step'], d['update_kernels']['heads']['avg_us'])"
done
