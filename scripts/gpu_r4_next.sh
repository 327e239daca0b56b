#!/bin/bash
# round 4: fp32 occupancy variants (forward + kernel table at B = 32) and the 2-stream bench with half
# the fused-bottleneck slots per kernel (two shards' kernels co-resident)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4next}; shift
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for n in "$@"; do
  BUGSEG_LIB=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_$n.so PREC=fp32 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/$n.txt 2>&1 || { echo "probe $n failed"; tail gpurun_out/$T/$n.txt; exit 1; }
  echo "== $n"; grep -v amdgpu.ids gpurun_out/$T/$n.txt
done
for g in 0 -2; do
  BUGSEG_BNECK_GRID=$g timeout -k 10 300 python bench.py --extras 0 --no-cpu-baseline > gpurun_out/$T/bench_g$g.json 2> gpurun_out/$T/bench_g$g.err || { echo "bench failed"; tail -30 gpurun_out/$T/bench_g$g.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/$T/bench_g$g.json')); print('grid $g', r['value'], r['ms_per_step'], r['shard_overlap_ms'])"
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -k "fp32 or bgr or init or pool or fullconv or timed_config or fp16 or bf16" > gpurun_out/$T/gpu.log 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/$T/gpu.log; exit 1; }
tail -2 gpurun_out/$T/gpu.log
PREC=fp16 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/probe16.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/probe16.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/probe16.txt
