#!/bin/bash
# round 4: BEV rasteriser — the bit-exact tests and the per-form timing sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4bev}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -k "bev or occgrid or laserscan or pipeline or capture" > gpurun_out/$T/gpu_bev.log 2>&1 || { echo "bev tests failed: $?"; tail -40 gpurun_out/$T/gpu_bev.log; exit 1; }
tail -2 gpurun_out/$T/gpu_bev.log
timeout -k 10 200 python scripts/bev_sweep.py 20 2>&1 | tee gpurun_out/$T/sweep.txt
