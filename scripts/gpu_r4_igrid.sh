#!/bin/bash
# round 4: initial-block grid A/B (BUGSEG_INIT_GRID caps the workgroups: 9,600 tiles at 32 frames on
# 1,536 resident slots is 6.25 tiles each; 1,376 and 1,200 even the walks out at 7 and 8)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4igrid}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for rep in 1 2; do
  for g in 0 1376 1200; do
    BUGSEG_INIT_GRID=$g PREC=fp16 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/p_${g}_$rep.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/p_${g}_$rep.txt; exit 1; }
    echo "== grid $g rep $rep $(grep -E ' init ' gpurun_out/$T/p_${g}_$rep.txt)"
  done
done
