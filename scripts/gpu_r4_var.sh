#!/bin/bash
# round 4: cheap A/B probes at the bench shard (fp16, B = 32): C64 tile variants by env, the
# asymmetric C128 form with its residual kept (variant library)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4var}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for v in default 1 2; do
  if [ $v != default ]; then export BUGSEG_BNECK_VARIANT_C64=$v; fi
  PREC=fp16 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/c64_$v.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/c64_$v.txt; exit 1; }
  echo "== C64 variant $v"; grep -v amdgpu.ids gpurun_out/$T/c64_$v.txt | head -5
  unset BUGSEG_BNECK_VARIANT_C64
done
BUGSEG_LIB=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_keepasym.so PREC=fp16 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/keepasym.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/keepasym.txt; exit 1; }
echo "== keepasym"; grep -v amdgpu.ids gpurun_out/$T/keepasym.txt | head -5
bash scripts/gpu_r4_bev.sh $T
