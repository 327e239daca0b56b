#!/bin/bash
# round 3 session 3: fp32 C64 half-staged epilogue (libbugseg_hstg: 4 workgroups per CU) parity + timing
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s3e
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_hstg.so
BUGSEG_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fp32" -m gpu -x -q --timeout 240 --timeout-method thread > $O/f32_tests.log 2>&1 || { echo "f32 tests failed"; tail -40 $O/f32_tests.log; exit 1; }
tail -1 $O/f32_tests.log
for lib in default hstg default hstg; do
  envs=""; [ $lib = hstg ] && envs="BUGSEG_LIB=$L"
  env $envs PREC=fp32 timeout -k 10 120 python scripts/batch_probe.py 32 > $O/probe_$lib.txt 2>&1 || { echo "probe $lib failed"; tail $O/probe_$lib.txt; exit 1; }
  head -3 $O/probe_$lib.txt | tail -2
  env $envs timeout -k 10 200 python bench.py --precision fp32 --no-cpu-baseline --extras 0 > $O/bench_$lib.json 2> $O/bench_$lib.err || { echo "bench $lib failed"; tail $O/bench_$lib.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$lib.json')); print('$lib', d['value'], d['ms_per_step'], d['roofline']['forward']['ms'], d['roofline']['forward']['mfma_frac'])"
done
