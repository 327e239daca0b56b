#!/bin/bash
# round 3 (session 2): the initial block fused into down1 — parity tests, then bench lines and
# per-kernel tables BUGSEG_INIT_FUSE=1 vs the two launches (fp16, B = 32 probe; bench default)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/initfuse
export TMPDIR=/tmp PREC=fp16
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "initial_block_fused or canonical_plan or forward_bgr_equals or multi_tile or fused_bottlenecks_equal" -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/initfuse/tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/initfuse/tests.log; exit 1; }
tail -2 gpurun_out/initfuse/tests.log
for cfg in "fused:BUGSEG_INIT_FUSE=1" "unfused:" "fused2:BUGSEG_INIT_FUSE=1" "unfused2:"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  o=gpurun_out/initfuse/$name
  env $envs timeout -k 10 120 python scripts/batch_probe.py 32 > $o.probe 2>&1 || { echo "probe $name failed"; tail $o.probe; exit 1; }
  env $envs timeout -k 10 120 python bench.py --no-cpu-baseline --extras 0 > $o.json 2> $o.err || { echo "bench $name failed"; tail $o.err; exit 1; }
  python -c "import json; d=json.load(open('$o.json')); print('$name', d['value'], d['ms_per_step'], d['roofline']['forward']['ms'])"
  grep -E "forward|init|down C64" $o.probe
done
