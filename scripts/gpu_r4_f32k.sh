#!/bin/bash
# round 4: fp32 C128 forms with the kept residual — fp32 parity + fused/unfused identity, the fp32 forward
# table, a FETCH/WRITE PMC pass pair of the fp32 bench, and the bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4f32k}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -k "fp32 or fused or multi_tile or timed_config or config1 or pipeline" > gpurun_out/$T/gpu.log 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/$T/gpu.log; exit 1; }
tail -1 gpurun_out/$T/gpu.log
PREC=fp32 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/p32.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/p32.txt; exit 1; }
echo "== fp32"; grep -v amdgpu.ids gpurun_out/$T/p32.txt | head -8
bash scripts/gpu_profile.sh ${T}_fp32 --precision fp32 || { echo "profile failed"; exit 1; }
python -c "import json; r=[l for l in open('gpurun_out/${T}_fp32/bench.json') if l.startswith('{')][-1]; r=json.loads(r); print('fp32', r['value'], r['ms_per_step'], r['stages_ms']['enet_forward'])"
