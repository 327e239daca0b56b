#!/bin/bash
# round 4: ablation variants (BEV floor, initial block) + tile-variant env sweeps (fp16 / fp32, B = 32)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4explore}; shift
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for n in "$@"; do
  BUGSEG_LIB=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_$n.so timeout -k 10 120 python scripts/abl_probe.py 20 > gpurun_out/$T/$n.txt 2>&1 || { echo "probe $n failed"; tail gpurun_out/$T/$n.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/$T/$n.txt
done
for v in 0 1 4; do
  echo "== fp16 C128 variant $v"
  BUGSEG_BNECK_VARIANT_C128=$v PREC=fp16 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/c128_$v.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/c128_$v.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/$T/c128_$v.txt | head -6
done
for v in 0 1 2; do
  echo "== fp32 C64 variant $v"
  BUGSEG_BNECK_VARIANT_C64=$v PREC=fp32 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/f32c64_$v.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/f32c64_$v.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/$T/f32c64_$v.txt | head -4
done
for v in 0 4; do
  echo "== fp32 C128 variant $v"
  BUGSEG_BNECK_VARIANT_C128=$v PREC=fp32 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/f32c128_$v.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/f32c128_$v.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/$T/f32c128_$v.txt | head -6
done
