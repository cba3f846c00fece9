set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_rollout.py tests/test_gpu_fastpath_e2e.py tests/test_gpu_dropin.py tests/test_gpu_distributed.py -x -q --timeout 200 --timeout-method thread > $O/pytest_rms.log 2>&1 || { tail -30 $O/pytest_rms.log; exit 1; }
tail -1 $O/pytest_rms.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_c4b -o run -- python -u tools/c4_run.py > $O/prof_c4b.log 2>&1 || exit 2
tail -1 $O/prof_c4b.log
python tools/kt_top.py $O/prof_c4b/run_kernel_trace.csv 8
