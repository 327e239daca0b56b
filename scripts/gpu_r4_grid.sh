#!/bin/bash
# round 4: fused-bottleneck grid A/B — one resident round of persistent workgroups (default) against one
# tile per workgroup (BUGSEG_BNECK_GRID=100000: hardware dispatch fills the slots as workgroups finish)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4grid}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for rep in 1 2; do
  for g in 0 100000; do
    BUGSEG_BNECK_GRID=$g PREC=fp16 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/p_${g}_$rep.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/p_${g}_$rep.txt; exit 1; }
    echo "== grid $g rep $rep"; grep -E "forward|bneck|down" gpurun_out/$T/p_${g}_$rep.txt
  done
done
