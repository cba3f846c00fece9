set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python -u tools/c3_run.py 1 > gpurun_out/prof_c3.log 2>&1 || exit 3
python tools/kt_top.py gpurun_out/prof_c3/run_kernel_trace.csv 30 > gpurun_out/top_c3.txt 2>&1; cat gpurun_out/top_c3.txt
