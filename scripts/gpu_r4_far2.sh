#!/bin/bash
# round 4: band BEV work-item order — far bands first (default) against nearest first
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4far2}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -k "bev or occ or band or laserscan or binary or ros or timed_config" > gpurun_out/$T/gpu.log 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/$T/gpu.log; exit 1; }
tail -1 gpurun_out/$T/gpu.log
for rep in 1 2 3; do
  for f in 0 1; do
    BUGSEG_BEV_NEAR_FIRST=$f timeout -k 10 120 python scripts/abl_probe.py 20 > gpurun_out/$T/a_${f}_$rep.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/a_${f}_$rep.txt; exit 1; }
    echo "== near_first $f rep $rep $(grep -E 'bev' gpurun_out/$T/a_${f}_$rep.txt)"
  done
done
