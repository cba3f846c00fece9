#!/bin/bash
# K16X (trunk layer inside the head GEMM launches) on the GPU box: its tests, the C2 bench A/B against r03's
# K13 forward + K16, and a rocprofv3 kernel-trace summary of the K16X form.  usage: bash tools/k16x_ab.sh <tag> [skip-tests]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${1:-k16x}
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fused_mlp.py tests/test_gpu_fastpath_e2e.py -m gpu > $O/${T}_pytest.log 2>&1 || { tail -30 $O/${T}_pytest.log; exit 1; }
  tail -1 $O/${T}_pytest.log
fi
Q="--no-cpu-baseline --no-sweep --no-per --no-c1 --no-c3 --no-c4 --no-pmc --no-rocprof"
for F in on off on; do
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --trunk-heads $F $Q --out $O/${T}_bench_$F.json > $O/${T}_bench_$F.log 2>&1 || { tail -5 $O/${T}_bench_$F.log; exit 5; }
  python -c "import json;d=json.load(open('$O/${T}_bench_$F.json'));print('$F', d['value'], d['ms_per_step'], d['update_kernels']['heads']['avg_us'], d['phase_split_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- python -u bench.py --steps 3 --warmup 2 $Q --no-kernel-timing --out $O/${T}_prof.json > $O/${T}_prof.log 2>&1 || { tail -5 $O/${T}_prof.log; exit 6; }
echo ok
