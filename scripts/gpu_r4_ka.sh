#!/bin/bash
# round 4: asymmetric C128 with the kept residual as default — bit-identity tests, then the fp16 round
# profile (bench line, rocprofv3 stats, FETCH / WRITE passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4ka}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -k "fused or multi_tile or timed_config or bf16 or fp16 or asym" > gpurun_out/$T/gpu.log 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/$T/gpu.log; exit 1; }
tail -1 gpurun_out/$T/gpu.log
bash scripts/gpu_profile.sh ${T}_fp16 || { echo "profile failed"; exit 1; }
python -c "import json; r=[l for l in open('gpurun_out/${T}_fp16/bench.json') if l.startswith('{')][-1]; r=json.loads(r); print('fp16', r['value'], r['ms_per_step'], r['stages_ms'], r['kernels']['bneck C128 asym 20x16'])"
