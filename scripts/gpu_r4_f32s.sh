#!/bin/bash
# round 4: fp32 parity mode with split-f16 t0 storage + 32-B LDS pads — parity tests, per-kernel
# times against the variants (no split / old pads / C16 occupancy 4), the fp32 and fp16 bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4f32s}; shift
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -k "fp32 or timed_config or class or fused or multi or up_block or pipeline or config1" > gpurun_out/$T/gpu.log 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/$T/gpu.log; exit 1; }
tail -2 gpurun_out/$T/gpu.log
PREC=fp32 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/probe32.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/probe32.txt; exit 1; }
echo "== default"; grep -v amdgpu.ids gpurun_out/$T/probe32.txt
for n in "$@"; do
  BUGSEG_LIB=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_$n.so PREC=fp32 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/$n.txt 2>&1 || { echo "probe $n failed"; tail gpurun_out/$T/$n.txt; exit 1; }
  echo "== $n"; grep -v amdgpu.ids gpurun_out/$T/$n.txt
done
timeout -k 10 300 python bench.py --precision fp32 --extras 0 --no-cpu-baseline --steps 10 > gpurun_out/$T/bench32.json 2> gpurun_out/$T/bench32.err || { echo "bench failed"; tail -30 gpurun_out/$T/bench32.err; exit 1; }
timeout -k 10 300 python bench.py --extras 0 --no-cpu-baseline > gpurun_out/$T/bench16.json 2> gpurun_out/$T/bench16.err || { echo "bench failed"; tail -30 gpurun_out/$T/bench16.err; exit 1; }
python -c "
import json
for p in ('32', '16'):
    r = json.load(open('gpurun_out/$T/bench' + p + '.json'))
    print(p, r['value'], r['ms_per_step'], r['stages_ms'])
"
