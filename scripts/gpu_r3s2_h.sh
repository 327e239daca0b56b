#!/bin/bash
# round 3 (session 2): fp32 parity mode with interleaved sub-MFMA chains (mma2) vs the committed HEAD
# library — parity tests of the touched kernels, per-kernel probe + fp32 bench per library; then the
# DeepLab GEMM bit-identity test and the Xception-65 profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/mma2
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "fp32 or fused_bottlenecks_equal or up_block or class_layer or forward_bgr_equals or multi_tile" -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/mma2/tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/mma2/tests.log; exit 1; }
tail -2 gpurun_out/mma2/tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_deeplab.py -k "gemm128" -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/mma2/dl_tests.log 2>&1 || { echo "dl tests failed"; tail -60 gpurun_out/mma2/dl_tests.log; exit 1; }
tail -2 gpurun_out/mma2/dl_tests.log
for lib in new head new2; do
  L=""
  [ $lib = head ] && L=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_head.so
  o=gpurun_out/mma2/$lib
  env ${L:+BUGSEG_LIB=$L} PREC=fp32 timeout -k 10 150 python scripts/batch_probe.py 32 > $o.probe 2>&1 || { echo "probe $lib failed"; tail $o.probe; exit 1; }
  env ${L:+BUGSEG_LIB=$L} timeout -k 10 200 python bench.py --precision fp32 --no-cpu-baseline --extras 0 > $o.json 2> $o.err || { echo "bench $lib failed"; tail $o.err; exit 1; }
  python -c "import json; d=json.load(open('$o.json')); r=d['roofline']; print('$lib', d['value'], d['ms_per_step'], r['forward']['ms'], r['forward']['mfma_frac'], r['kernel_mfma_frac'])"
  grep -E "forward|C64|C128|up|init|classes|C16" $o.probe | head -14
done
bash scripts/gpu_xc_profile.sh r03_b_xc || exit 1
echo xc profile done
# the bench's BEV stage on the compact table vs the uint4-slot form (same box)
for lib in ctab noctab; do
  L=""
  [ $lib = noctab ] && L=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_noctab.so
  env ${L:+BUGSEG_LIB=$L} timeout -k 10 200 python bench.py --no-cpu-baseline --extras 0 > gpurun_out/mma2/bev_$lib.json 2> gpurun_out/mma2/bev_$lib.err || { echo "bev bench $lib failed"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/mma2/bev_$lib.json')); print('$lib', d['value'], d['stages_ms'])"
done
# C = 16 tile variants (stage-5 block): 16x16 (the pick) vs 32x16 / 16x32, fused-vs-unfused parity first
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fused_bottlenecks_equal" -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/mma2/c16_tests.log 2>&1 || { echo "c16 tests failed"; tail -40 gpurun_out/mma2/c16_tests.log; exit 1; }
tail -1 gpurun_out/mma2/c16_tests.log
for v in 0 1 2 0; do
  BUGSEG_BNECK_VARIANT_C16=$v PREC=fp16 timeout -k 10 150 python scripts/batch_probe.py 32 > gpurun_out/mma2/c16_v$v.probe 2>&1 || { echo "c16 probe $v failed"; exit 1; }
  echo "C16 variant $v"; grep -E "forward|C16" gpurun_out/mma2/c16_v$v.probe
done
# up kernel with its weight reads kept in the loop (96 instead of 226 VGPRs) vs the default
for lib in default upnh; do
  L=""
  [ $lib = upnh ] && L=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_upnh.so
  env ${L:+BUGSEG_LIB=$L} PREC=fp16 timeout -k 10 150 python scripts/batch_probe.py 32 > gpurun_out/mma2/up_$lib.probe 2>&1 || { echo "up probe $lib failed"; exit 1; }
  echo "up $lib"; grep -E "forward|up C" gpurun_out/mma2/up_$lib.probe
done
