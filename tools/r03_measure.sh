#!/bin/bash
# Round-3 measurement set on the GPU box: GPU tests + smoke, the full bench (live PMC traffic), and rocprofv3 kernel
# traces of the C2 bench with both GAE forms (value-fused K1V vs value head + compact K1) for the A/B.
# usage: bash tools/r03_measure.sh <tag> [skip-tests]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${1:-r03}
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/${T}_pytest.log 2>&1 || { tail -15 $O/${T}_pytest.log; exit 1; }
  tail -1 $O/${T}_pytest.log
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { tail -5 $O/${T}_smoke.log; exit 7; }
  tail -1 $O/${T}_smoke.log
fi
timeout -k 10 700 python -u bench.py --out $O/${T}_bench.json > $O/${T}_bench.log 2>&1 || { tail -5 $O/${T}_bench.log; exit 5; }
echo bench ok
for F in value split; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_$F -o run -- python -u bench.py --steps 5 --gae-form $F --no-pmc --no-cpu-baseline --no-sweep --no-per --no-c1 --no-c3 --no-c4 --out $O/${T}_prof_$F.json > $O/${T}_prof_$F.log 2>&1 || { tail -5 $O/${T}_prof_$F.log; exit 6; }
  python tools/trace_summary.py $(ls $O/${T}_prof_$F/*/run_kernel_trace.csv 2>/dev/null || ls $O/${T}_prof_$F/run_kernel_trace.csv) $O/${T}_prof_$F.json $O/${T}_trace_$F.json > /dev/null || exit 8
done
echo ok
