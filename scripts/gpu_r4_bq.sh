#!/bin/bash
# round 4: BEV quad box — bit-exact tests + graph-timed sweep, then the default bench line with its
# graph-timed precision sub-records
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4bq}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
bash scripts/gpu_r4_bev.sh $T || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo "bench failed"; tail -30 gpurun_out/$T/bench.err; exit 1; }
python -c "
import json
r = json.load(open('gpurun_out/$T/bench.json'))
print('fp16', r['value'], 'bev', r['stages_ms'], 'fp32', r['fp32']['value'], r['fp32'].get('hip_graph'), 'bf16', r['bf16']['value'])
"
