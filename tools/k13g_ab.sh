#!/bin/bash
# K13 gather-forward staging A/B on the GPU box: the gather tests, then the C2 bench + a rocprofv3 kernel-trace summary.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${1:-k13g}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fused_mlp.py tests/test_gpu_fastpath_e2e.py -m gpu > $O/${T}_pytest.log 2>&1 || { tail -30 $O/${T}_pytest.log; exit 1; }
tail -1 $O/${T}_pytest.log
Q="--no-cpu-baseline --no-sweep --no-per --no-c1 --no-c3 --no-c4 --no-pmc --no-rocprof"
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 $Q --out $O/${T}_bench.json > $O/${T}_bench.log 2>&1 || { tail -5 $O/${T}_bench.log; exit 5; }
python -c "import json;d=json.load(open('$O/${T}_bench.json'));print(d['value'], d['ms_per_step'], d['update_kernels']['heads']['avg_us'], d['phase_split_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- python -u bench.py --steps 3 --warmup 2 $Q --no-kernel-timing --out $O/${T}_prof.json > $O/${T}_prof.log 2>&1 || { tail -5 $O/${T}_prof.log; exit 6; }
T=$T python - <<'PY'
import csv,glob,os
f=glob.glob('gpurun_out/%s_prof/**/run_kernel_stats.csv' % os.environ['T'],recursive=True)[0]
for r in sorted(csv.DictReader(open(f)),key=lambda r:-float(r['TotalDurationNs']))[:12]:
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1))
PY
echo ok
