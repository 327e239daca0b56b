#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_envab.sh BUGSEG_BNECK_GRID '' '-2' '' '-2' || exit 1
for i in 0 1 2 3; do echo "$(cat gpurun_out/envab/$i/setting.txt) $(python -c "import json,sys; d=json.load(open('gpurun_out/envab/$i/bench.json')); print(d['value'], d['ms_per_step'], d['stages_ms'], d.get('shard_overlap_ms'), d['kernels'].get('classes'))")"; done
timeout -k 10 120 python scripts/bev_sweep.py 20 > gpurun_out/bev_sweep.txt 2>&1; cat gpurun_out/bev_sweep.txt
NEW_ONLY= bash scripts/gpu_r3_tests.sh || exit 1
grep -E "excused|agreement" gpurun_out/r3_all_gpu.log | head -20
