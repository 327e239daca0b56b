#!/bin/bash
# round 4: the fp32 parity mode on split-f16 products — its parity tests, smoke, and the fp32 bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4fp32}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -k "fp32 or class_layer or config1 or graphdef or up_block or forward_bgr" > gpurun_out/$T/gpu_fp32.log 2>&1 || { echo "gpu fp32 tests failed: $?"; grep -E "^E |Error|assert|max\|d" gpurun_out/$T/gpu_fp32.log | head -40; tail -30 gpurun_out/$T/gpu_fp32.log; exit 1; }
tail -3 gpurun_out/$T/gpu_fp32.log
grep -h "max|dlogit|" gpurun_out/$T/gpu_fp32.log | head -20
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -3 gpurun_out/$T/smoke.log
timeout -k 10 300 python bench.py --precision fp32 --extras 0 --no-cpu-baseline --steps 10 > gpurun_out/$T/bench_fp32.json 2> gpurun_out/$T/bench_fp32.err || { echo "bench failed"; tail -30 gpurun_out/$T/bench_fp32.err; exit 1; }
python -c "import json; r=json.load(open('gpurun_out/$T/bench_fp32.json')); print(r['value'], r['ms_per_step'], r['roofline']['forward']); print(json.dumps(r['kernels']))"
