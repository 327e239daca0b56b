#!/bin/bash
# round 4: band BEV knobs re-measured on the item-major, far-first kernel: 7 waves per SIMD, 2-row parts
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4bevk}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for rep in 1 2; do
  for v in new occ7 minp2; do
    if [ $v = new ]; then unset BUGSEG_LIB; else export BUGSEG_LIB=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_$v.so; fi
    timeout -k 10 120 python scripts/abl_probe.py 20 > gpurun_out/$T/a_${v}_$rep.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/a_${v}_$rep.txt; exit 1; }
    echo "== $v $rep $(grep -E 'bev' gpurun_out/$T/a_${v}_$rep.txt)"
  done
done
