#!/bin/bash
# round 3 (session 2): BNECK_PIPE A/B — the new multi-tile-walk parity test, then per-kernel-tag launch
# times (batch_probe, fp16, B = 32) and bench lines for {pipe, nopipe} x {full grid, half grid, 8x16 C128}
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pipe
export TMPDIR=/tmp PREC=fp16
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "multi_tile" -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pipe/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pipe/tests.log; exit 1; }
tail -2 gpurun_out/pipe/tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fused_bottlenecks_equal or multi_tile_workgroups" -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pipe/tests2.log 2>&1 || { echo "tests2 failed"; tail -40 gpurun_out/pipe/tests2.log; exit 1; }
tail -2 gpurun_out/pipe/tests2.log
for lib in pipe nopipe nodk; do
  L=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_$lib.so
  cfgs='"full:" "half:BUGSEG_BNECK_GRID=-2" "v4:BUGSEG_BNECK_VARIANT_C128=4"'
  [ $lib = nodk ] && cfgs='"full:"'
  eval "set -- $cfgs"
  for cfg in "$@"; do
    name=${cfg%%:*}; envs=${cfg#*:}
    o=gpurun_out/pipe/${lib}_$name
    env BUGSEG_LIB=$L $envs timeout -k 10 120 python scripts/batch_probe.py 32 > $o.probe 2>&1 || { echo "probe $lib $name failed"; tail $o.probe; exit 1; }
    env BUGSEG_LIB=$L $envs timeout -k 10 120 python bench.py --no-cpu-baseline --extras 0 > $o.json 2> $o.err || { echo "bench $lib $name failed"; tail $o.err; exit 1; }
    python -c "import json; d=json.load(open('$o.json')); print('$lib $name', d['value'], d['ms_per_step'])"
    grep -E "forward|C128|down" $o.probe
  done
done
