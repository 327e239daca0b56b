#!/bin/bash
# round 3 session 3: the touched kernels' parity (fp32 C64 half staging, class layer forms, GEMM forms),
# then the round profiles (fp16 headline + fp32 parity mode: rocprofv3 stats + FETCH/WRITE PMC passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3s3p
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fp32 or class or fused_bottlenecks_equal" -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3s3p/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3s3p/tests.log; exit 1; }
tail -1 gpurun_out/r3s3p/tests.log
TAG=r03_c bash scripts/gpu_r3_prof.sh || exit 1
