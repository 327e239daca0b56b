#!/bin/bash
# round 3 session 3: the whole -m gpu suite, smoke, and one full bench line (all sub-records)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3s3zz
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread > gpurun_out/r3s3zz/all_gpu.log 2>&1 || { echo "gpu suite failed: $?"; tail -60 gpurun_out/r3s3zz/all_gpu.log; exit 1; }
tail -3 gpurun_out/r3s3zz/all_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s3zz/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r3s3zz/smoke.log; exit 1; }
tail -3 gpurun_out/r3s3zz/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r3s3zz/bench.json 2> gpurun_out/r3s3zz/bench.err || { echo "bench failed"; tail -30 gpurun_out/r3s3zz/bench.err; exit 1; }
cat gpurun_out/r3s3zz/bench.json
