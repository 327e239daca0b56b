#!/bin/bash
# round 4: bench A/B of the C64 8-wave kept-residual variant held to 8 waves per SIMD (k8 build, forced)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4c64k8}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for rep in 1 2; do
  for v in def k8; do
    unset BUGSEG_LIB BUGSEG_BNECK_VARIANT_C64
    if [ $v = k8 ]; then export BUGSEG_BNECK_VARIANT_C64=3 BUGSEG_LIB=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_k8.so; fi
    timeout -k 10 300 python bench.py --extras 0 --no-cpu-baseline > gpurun_out/$T/b_${v}_$rep.json 2> gpurun_out/$T/b_${v}_$rep.err || { echo "bench failed"; tail -30 gpurun_out/$T/b_${v}_$rep.err; exit 1; }
    python -c "import json; r=json.load(open('gpurun_out/$T/b_${v}_$rep.json')); print('bench $v $rep', r['value'], r['ms_per_step'], r['roofline']['us_per_launch'], r['stages_ms']['enet_forward'])"
  done
done
