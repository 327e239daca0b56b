#!/bin/bash
# round 4: the whole -m gpu suite, smoke, and one full bench line (all sub-records)
# usage: gpu_r4_full.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread > gpurun_out/$T/all_gpu.log 2>&1 || { echo "gpu suite failed: $?"; tail -60 gpurun_out/$T/all_gpu.log; exit 1; }
tail -3 gpurun_out/$T/all_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -3 gpurun_out/$T/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo "bench failed"; tail -30 gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json
