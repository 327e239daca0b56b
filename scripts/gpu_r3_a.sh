#!/bin/bash
# round 3, call A: new + full GPU tests and smoke, then the half-slot grid A/B under the 2-stream bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_r3_tests.sh || exit 1
bash scripts/gpu_envab.sh BUGSEG_BNECK_GRID '' '-2' '' '-2' || exit 1
for i in 0 1 2 3; do echo "$(cat gpurun_out/envab/$i/setting.txt) $(python -c "import json,sys; d=json.load(open('gpurun_out/envab/$i/bench.json')); print(d['value'], d['ms_per_step'], d['stages_ms']['enet_forward'], d.get('shard_overlap_ms'))")"; done
