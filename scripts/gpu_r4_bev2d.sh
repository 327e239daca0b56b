#!/bin/bash
# round 4: band BEV kernel on a 2-D grid (item-major order without the index division and its 3 spilled
# VGPRs) — bit-exact BEV tests, A/B against the previous build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4bev2d}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -k "bev or occ or laserscan or binary or grid or band or ros or timed_config" > gpurun_out/$T/gpu.log 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/$T/gpu.log; exit 1; }
tail -1 gpurun_out/$T/gpu.log
for rep in 1 2 3; do
  for v in base new; do
    if [ $v = new ]; then unset BUGSEG_LIB; else export BUGSEG_LIB=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_$v.so; fi
    timeout -k 10 120 python scripts/abl_probe.py 20 > gpurun_out/$T/a_${v}_$rep.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/a_${v}_$rep.txt; exit 1; }
    echo "== $v $rep $(grep -E 'bev' gpurun_out/$T/a_${v}_$rep.txt)"
  done
done
