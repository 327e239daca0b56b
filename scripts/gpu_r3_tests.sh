#!/bin/bash
# Round-3 GPU test pass: the new tests first (named files as args), then the whole -m gpu suite and smoke.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
first="${*:-tests/test_gpu_capture_dist.py tests/test_gpu_timed_config.py}"
timeout -k 10 600 python -u -m pytest $first -m gpu -x -v -s --timeout 240 --timeout-method thread \
    > gpurun_out/r3_new_tests.log 2>&1 || { echo "new tests failed: $?"; tail -40 gpurun_out/r3_new_tests.log; exit 1; }
tail -5 gpurun_out/r3_new_tests.log
if [ -n "$NEW_ONLY" ]; then exit 0; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread \
    > gpurun_out/r3_all_gpu.log 2>&1 || { echo "gpu suite failed: $?"; tail -40 gpurun_out/r3_all_gpu.log; exit 1; }
tail -3 gpurun_out/r3_all_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r3_smoke.log; exit 1; }
cat gpurun_out/r3_smoke.log
