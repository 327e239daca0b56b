#!/bin/bash
# round 4: fp32 split-f16 parity tests, then the fp32 bench at 1 / 2 / 4 shard streams
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4fp32b}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -k "fp32 or class_layer or config1 or up_block or forward_bgr" > gpurun_out/$T/gpu_fp32.log 2>&1 || { echo "gpu fp32 tests failed: $?"; tail -30 gpurun_out/$T/gpu_fp32.log; exit 1; }
tail -2 gpurun_out/$T/gpu_fp32.log
grep -h "fp32 480x640 max|dlogit|\|pipeline fp32" gpurun_out/$T/gpu_fp32.log | head
for S in 2 1 4; do
timeout -k 10 300 python bench.py --precision fp32 --extras 0 --no-cpu-baseline --steps 10 --streams $S > gpurun_out/$T/bench_fp32_s$S.json 2> gpurun_out/$T/bench_fp32_s$S.err || { echo "bench failed"; tail -30 gpurun_out/$T/bench_fp32_s$S.err; exit 1; }
python -c "import json; r=json.load(open('gpurun_out/$T/bench_fp32_s$S.json')); print('streams $S', r['value'], r['ms_per_step'], r['roofline']['forward']['ms'])"
done
python -c "import json; r=json.load(open('gpurun_out/$T/bench_fp32_s2.json')); print(json.dumps(r['kernels']))"
