#!/bin/bash
# round 4: fp32 probe, then the driver's sequence — the whole -m gpu suite, smoke, the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4final}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
PREC=fp32 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/p32.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/p32.txt; exit 1; }
echo "== fp32"; grep -v amdgpu.ids gpurun_out/$T/p32.txt | head -5
bash scripts/gpu_r4_full.sh $T
