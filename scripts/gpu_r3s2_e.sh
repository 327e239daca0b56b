#!/bin/bash
# round 3 (session 2): BEV band kernel on the compact table — rasteriser parity tests, then the form
# sweep (HIP-event time per 32-frame launch) with the compact table and without it (BEV_CTAB=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ctab
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capture_dist.py -k "bev or laserscan or pipeline or captured" -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/ctab/tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/ctab/tests.log; exit 1; }
tail -2 gpurun_out/ctab/tests.log
timeout -k 10 200 python scripts/bev_sweep.py 20 > gpurun_out/ctab/sweep_ctab.txt 2>&1 || { echo "sweep failed"; tail gpurun_out/ctab/sweep_ctab.txt; exit 1; }
BUGSEG_LIB=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_noctab.so timeout -k 10 200 python scripts/bev_sweep.py 20 > gpurun_out/ctab/sweep_noctab.txt 2>&1 || { echo "sweep2 failed"; tail gpurun_out/ctab/sweep_noctab.txt; exit 1; }
echo "== ctab"; cat gpurun_out/ctab/sweep_ctab.txt; echo "== noctab"; cat gpurun_out/ctab/sweep_noctab.txt
