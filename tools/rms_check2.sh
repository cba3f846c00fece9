set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_rollout.py tests/test_gpu_fastpath_e2e.py tests/test_gpu_dropin.py -x -q --timeout 200 --timeout-method thread > $O/pytest_rms2.log 2>&1 || { tail -30 $O/pytest_rms2.log; exit 1; }
tail -1 $O/pytest_rms2.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-sweep --no-per --no-c3 --out $O/bench_rms2.json > $O/bench_rms2.log 2>&1 || { tail -20 $O/bench_rms2.log; exit 2; }
python - <<'PY'
import json; d=json.load(open("gpurun_out/bench_rms2.json"))
print("c2", d["value"], d["ms_per_step"])
for k in ("c1_cartpole","c4_box376"):
    v=d.get(k) or {}
    print(k, {kk: v.get(kk) for kk in ("value","ms_per_iter","ms_per_step")})
PY
