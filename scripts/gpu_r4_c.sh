#!/bin/bash
# round 4: fp32 parity tests + forward tables (default, no-pad variant), BEV ablations (graph-timed),
# fp32 bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4c}; shift
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -k "fp32 or fused or multi or config1 or timed_config" > gpurun_out/$T/gpu.log 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/$T/gpu.log; exit 1; }
tail -1 gpurun_out/$T/gpu.log
for n in "" f32nopad; do
  if [ -n "$n" ]; then export BUGSEG_LIB=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_$n.so; fi
  PREC=fp32 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/p32_$n.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/p32_$n.txt; exit 1; }
  echo "== fp32 $n"; grep -v amdgpu.ids gpurun_out/$T/p32_$n.txt | head -9
  unset BUGSEG_LIB
done
for n in "$@"; do
  BUGSEG_LIB=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_$n.so timeout -k 10 120 python scripts/abl_probe.py 20 > gpurun_out/$T/$n.txt 2>&1 || { echo "probe $n failed"; tail gpurun_out/$T/$n.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/$T/$n.txt | head -1
done
timeout -k 10 300 python bench.py --precision fp32 --extras 0 --no-cpu-baseline --steps 10 > gpurun_out/$T/bench32.json 2> gpurun_out/$T/bench32.err || { echo "bench failed"; tail -30 gpurun_out/$T/bench32.err; exit 1; }
python -c "
import json
r = json.load(open('gpurun_out/$T/bench32.json'))
print('fp32', r['value'], r['ms_per_step'], r['stages_ms'])
"
