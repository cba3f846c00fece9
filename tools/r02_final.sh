#!/bin/bash
# Round-2 measurement set on the GPU box: GPU tests, GAE PMC passes, the full bench, a rocprof kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_final.log 2>&1 || { tail -5 $O/pytest_final.log; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")" > $O/smoke_final.log 2>&1 || { tail -5 $O/smoke_final.log; exit 7; }
tail -1 $O/smoke_final.log
tail -1 $O/pytest_final.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o f -- python tools/gae_pmc.py > $O/pmc_fetch.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o w -- python tools/gae_pmc.py > $O/pmc_write.log 2>&1 || exit 3
python tools/pmc_summary.py $O/pmc_fetch $O/pmc_write $O/pmc_gae_r02.json > /dev/null || exit 4
cp $O/pmc_gae_r02.json profiles/pmc_gae_r02.json
timeout -k 10 600 python -u bench.py --out $O/bench_r02_final.json > $O/bench_r02_final.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_final -o run -- python -u bench.py --steps 5 --no-cpu-baseline --no-sweep --no-per --no-c1 --no-c3 --no-c4 --out $O/bench_r02_prof.json > $O/prof_final.log 2>&1 || exit 6
echo ok
