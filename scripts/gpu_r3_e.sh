#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capture_dist.py -k "bev or laserscan or pipeline or capture" -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3_bev_tests.log 2>&1 || { echo "bev tests failed"; tail -40 gpurun_out/r3_bev_tests.log; exit 1; }
tail -2 gpurun_out/r3_bev_tests.log
timeout -k 10 120 python scripts/bev_sweep.py 20 > gpurun_out/bev_sweep.txt 2>&1; cat gpurun_out/bev_sweep.txt
timeout -k 10 200 python bench.py --no-cpu-baseline --extras 0 > gpurun_out/r3e_bench.json 2> gpurun_out/r3e_bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r3e_bench.json')); print(d['value'], d['ms_per_step'], d['stages_ms'], d['shard_overlap_ms'], d['kernels']['classes'])"
