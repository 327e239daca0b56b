#!/bin/bash
# round 3 session 3: (1) the deep-pipeline Xception GEMM (BUGSEG_DL_GP = 3/4/5) bit-identity + timing,
# (2) the fp32 C64 register-epilogue variant (libbugseg_r3f32: 4 workgroups per CU) parity + timing
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s3a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_deeplab.py -k "gemm128_bit_identical" -m gpu -x -q --timeout 240 --timeout-method thread > $O/gp_tests.log 2>&1 || { echo "gp tests failed"; tail -40 $O/gp_tests.log; exit 1; }
tail -1 $O/gp_tests.log
for gp in 0 3 4 5; do
  BUGSEG_DL_GP=$gp timeout -k 10 200 python3 bench_deeplab.py --backbone xception_65 --batch 32 --steps 6 --warmup 2 --no-cpu-baseline > $O/xc_gp$gp.json 2> $O/xc_gp$gp.err || { echo "xc bench gp$gp failed"; tail $O/xc_gp$gp.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/xc_gp$gp.json')); k=d['kernels']['conv pointwise']; print('gp$gp', d['value'], k['us'], k['TFLOPs'])"
done
L=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_r3f32.so
BUGSEG_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fp32" -m gpu -x -q --timeout 240 --timeout-method thread > $O/f32_tests.log 2>&1 || { echo "f32 tests failed"; tail -40 $O/f32_tests.log; exit 1; }
tail -1 $O/f32_tests.log
for lib in default r3f32; do
  envs=""; [ $lib = r3f32 ] && envs="BUGSEG_LIB=$L"
  env $envs PREC=fp32 timeout -k 10 120 python scripts/batch_probe.py 32 > $O/probe_$lib.txt 2>&1 || { echo "probe $lib failed"; tail $O/probe_$lib.txt; exit 1; }
  head -4 $O/probe_$lib.txt
  env $envs timeout -k 10 200 python bench.py --precision fp32 --no-cpu-baseline --extras 0 > $O/bench_$lib.json 2> $O/bench_$lib.err || { echo "bench $lib failed"; tail $O/bench_$lib.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$lib.json')); print('$lib', d['value'], d['ms_per_step'], d['roofline']['forward'])"
done
