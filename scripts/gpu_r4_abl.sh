#!/bin/bash
# round 4: ablation variants of the BEV rasteriser and the class layer (timing only; wrong results)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4abl}; shift
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 120 python scripts/abl_probe.py 20 > gpurun_out/$T/default.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/default.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/default.txt
for n in "$@"; do
  BUGSEG_LIB=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_$n.so timeout -k 10 120 python scripts/abl_probe.py 20 > gpurun_out/$T/$n.txt 2>&1 || { echo "probe $n failed"; tail gpurun_out/$T/$n.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/$T/$n.txt
done
