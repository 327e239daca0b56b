#!/bin/bash
# round 3 session 3: dl_gemm128 ablations (abl1: no MFMAs, abl2: no operand loads; wrong results,
# timing only) vs the default on the Xception-65 bench (B = 32)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s3c
mkdir -p $O
export TMPDIR=/tmp
V=$PWD/bugcar_image_segmentation_amd/_variants
for lib in default abl1 abl2; do
  envs=""; [ $lib != default ] && envs="BUGSEG_LIB=$V/libbugseg_$lib.so"
  env $envs timeout -k 10 200 python3 bench_deeplab.py --backbone xception_65 --batch 32 --steps 6 --warmup 2 --no-cpu-baseline > $O/xc_$lib.json 2> $O/xc_$lib.err || { echo "xc bench $lib failed"; tail $O/xc_$lib.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/xc_$lib.json')); k=d['kernels']['conv pointwise']; print('$lib', d['value'], k['us'], k['TFLOPs'])"
done
