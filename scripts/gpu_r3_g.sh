#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_timed_config.py -k "forward_bgr or fp32 or fp16 or bf16 or config1 or pipeline or timed or multi_tile or full_size" -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3_g_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3_g_tests.log; exit 1; }
tail -2 gpurun_out/r3_g_tests.log
timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/r3g_probe.txt 2>&1 || exit 1
cat gpurun_out/r3g_probe.txt
timeout -k 10 200 python bench.py --no-cpu-baseline --extras 0 > gpurun_out/r3g_bench.json 2> gpurun_out/r3g_bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r3g_bench.json')); print(d['value'], d['ms_per_step'], d['stages_ms'], d['shard_overlap_ms']); print(d['kernels'])"
