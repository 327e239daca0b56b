#!/bin/bash
# round 3 session 3: C16 20x16 tile variant (default build, cost model) and the swizzled up-kernel weights
# (libbugseg_swz: 4 workgroups per CU for up C64): parity, then per-kernel times and bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s3g
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_swz.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fused_bottlenecks_equal or multi_tile or canonical_plan or fp32" -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
BUGSEG_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fused_bottlenecks_equal or up" -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests_swz.log 2>&1 || { echo "swz tests failed"; tail -40 $O/tests_swz.log; exit 1; }
tail -1 $O/tests_swz.log
for cfg in "c16v0:BUGSEG_BNECK_VARIANT_C16=0" "default:" "swz:BUGSEG_LIB=$L" "c16v0:BUGSEG_BNECK_VARIANT_C16=0" "default:" "swz:BUGSEG_LIB=$L"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs PREC=fp16 timeout -k 10 120 python scripts/batch_probe.py 32 > $O/probe_$name.txt 2>&1 || { echo "probe $name failed"; tail $O/probe_$name.txt; exit 1; }
  grep -E "forward|C16|up C64" $O/probe_$name.txt
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --extras 0 > $O/bench_$name.json 2> $O/bench_$name.err || { echo "bench $name failed"; tail $O/bench_$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$name.json')); print('$name', d['value'], d['ms_per_step'], d['roofline']['forward']['ms'])"
done
PREC=fp32 timeout -k 10 120 python scripts/batch_probe.py 32 > $O/probe_f32.txt 2>&1 && grep -E "forward|C16" $O/probe_f32.txt
BUGSEG_BNECK_VARIANT_C16=0 PREC=fp32 timeout -k 10 120 python scripts/batch_probe.py 32 > $O/probe_f32_v0.txt 2>&1 && grep -E "forward|C16" $O/probe_f32_v0.txt
