#!/bin/bash
# round 3 session 3: the vendor GEMM on Xception's pointwise shapes; bench.py's RCCL branch as a 1-rank job
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s3d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python scripts/gemm_lib_probe.py > $O/gemm.txt 2>&1 || { echo "gemm probe failed"; tail -20 $O/gemm.txt; exit 1; }
cat $O/gemm.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_capture_dist.py -k "rccl or distributed_branch" -m gpu -x -q -rA --timeout 240 --timeout-method thread > $O/dist.log 2>&1 || { echo "dist tests failed"; tail -40 $O/dist.log; exit 1; }
grep -E "passed|value" $O/dist.log | tail -4
