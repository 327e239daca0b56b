#!/bin/bash
# round 4: BNECK_CH1_K2 = 4 as the default — bit-identity tests (forced variants, multi-tile walks, down
# forms) and the default bench line (incl. the batch-1 latency records, where the C64 8x16 form runs)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4ch4b}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -k "fused_bottlenecks or down or timed_config or small or batch" > gpurun_out/$T/gpu.log 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/$T/gpu.log; exit 1; }
tail -1 gpurun_out/$T/gpu.log
timeout -k 10 400 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo "bench failed"; tail -30 gpurun_out/$T/bench.err; exit 1; }
python -c "import json; r=json.load(open('gpurun_out/$T/bench.json')); print('fp16', r['value'], r['ms_per_step'], r['kernels']['down C64 16x16'], r['latency_b1_ms']['graph_ms'], r['latency_b1_ms_bf16']['graph_ms'], r['fp32']['value'])"
