#!/bin/bash
# round 3 session 3: dl_gemm128 A/B — read-pipelined k-steps (rpipe) and two ablations (abl1: no MFMAs,
# abl2: no operand loads; wrong results, timing only) on the Xception-65 bench (B = 32)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s3b
mkdir -p $O
export TMPDIR=/tmp
V=$PWD/bugcar_image_segmentation_amd/_variants
BUGSEG_LIB=$V/libbugseg_rpipe.so timeout -k 10 300 python -u -m pytest tests/test_gpu_deeplab.py -k "gemm128_bit_identical and g128_vs_g64" -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lib in default rpipe abl1 abl2; do
  envs=""; [ $lib != default ] && envs="BUGSEG_LIB=$V/libbugseg_$lib.so"
  env $envs timeout -k 10 200 python3 bench_deeplab.py --backbone xception_65 --batch 32 --steps 6 --warmup 2 --no-cpu-baseline > $O/xc_$lib.json 2> $O/xc_$lib.err || { echo "xc bench $lib failed"; tail $O/xc_$lib.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/xc_$lib.json')); k=d['kernels']['conv pointwise']; print('$lib', d['value'], k['us'], k['TFLOPs'])"
done
