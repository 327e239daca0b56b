#!/bin/bash
# round 3 (session 2): class-layer prefetch depth and initial-block patch prefetch A/B — parity tests of
# both kernels, then per-kernel-tag launch times (batch_probe, fp16, B = 32) and bench lines per variant
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/clsinit
export TMPDIR=/tmp PREC=fp16
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "class_layer or forward_bgr_equals or fp16_vs or bf16_vs or class_counts or fullconv" -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/clsinit/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/clsinit/tests.log; exit 1; }
tail -2 gpurun_out/clsinit/tests.log
for lib in base cls1 initpf0; do
  L=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_$lib.so
  o=gpurun_out/clsinit/$lib
  BUGSEG_LIB=$L timeout -k 10 120 python scripts/batch_probe.py 32 > $o.probe 2>&1 || { echo "probe $lib failed"; tail $o.probe; exit 1; }
  BUGSEG_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --extras 0 > $o.json 2> $o.err || { echo "bench $lib failed"; tail $o.err; exit 1; }
  python -c "import json; d=json.load(open('$o.json')); print('$lib', d['value'], d['ms_per_step'])"
  grep -E "forward|init|classes" $o.probe
done
