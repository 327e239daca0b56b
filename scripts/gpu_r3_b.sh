#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./scripts/capture_probe > gpurun_out/capture_probe.txt 2>&1; echo "probe rc $?"; cat gpurun_out/capture_probe.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_timed_config.py tests/test_gpu_capture_dist.py -k "not capture" -m gpu -x -v -s --timeout 240 --timeout-method thread \
    > gpurun_out/r3_new_tests.log 2>&1 || { echo "new tests failed: $?"; tail -60 gpurun_out/r3_new_tests.log; exit 1; }
grep -E "PASS|FAIL|agreement|excused|value" gpurun_out/r3_new_tests.log | tail -30
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -k "not capture_first_bev and not first_call" \
    > gpurun_out/r3_all_gpu.log 2>&1 || { echo "gpu suite failed: $?"; tail -60 gpurun_out/r3_all_gpu.log; exit 1; }
tail -3 gpurun_out/r3_all_gpu.log
grep -E "excused" gpurun_out/r3_all_gpu.log | head -20
bash scripts/gpu_envab.sh BUGSEG_BNECK_GRID '' '-2' '' '-2' || exit 1
for i in 0 1 2 3; do echo "$(cat gpurun_out/envab/$i/setting.txt) $(python -c "import json,sys; d=json.load(open('gpurun_out/envab/$i/bench.json')); print(d['value'], d['ms_per_step'], d['stages_ms'], d.get('shard_overlap_ms'), d['kernels'].get('classes'))")"; done
timeout -k 10 120 python scripts/bev_sweep.py 20 > gpurun_out/bev_sweep.txt 2>&1; cat gpurun_out/bev_sweep.txt
