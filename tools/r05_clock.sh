#!/bin/bash
# r05: per-kernel clock estimate = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (one --pmc pass with the kernel trace)
# over a C2 bench step and the C3 conv kernels.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05clk; mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/c2 -o c -- \
    python -u bench.py --steps 1 --warmup 1 --no-sweep --no-per --no-c1 --no-c3 --no-c4 --no-pmc --no-rocprof \
    --no-cpu-baseline --no-kernel-timing > $O/c2.log 2>&1 || { tail -5 $O/c2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/cv -o c -- \
    python -u tools/conv_pmc.py > $O/cv.log 2>&1 || { tail -5 $O/cv.log; exit 2; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/cv2 -o c -- \
    python -u tools/conv_pmc2.py > $O/cv2.log 2>&1 || { tail -5 $O/cv2.log; exit 3; }
python tools/clock_sum.py $O/c2 $O/cv $O/cv2 | tee $O/clock.txt
