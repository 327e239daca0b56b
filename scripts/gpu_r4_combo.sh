#!/bin/bash
# round 4: the whole GPU suite, then BEV sweep, per-kernel tables (fp16 default; fp32 default + variants)
# and the bench lines (fp16, fp32)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4combo}; shift
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread > gpurun_out/$T/gpu.log 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/$T/gpu.log; exit 1; }
tail -2 gpurun_out/$T/gpu.log
timeout -k 10 200 python scripts/bev_sweep.py 20 > gpurun_out/$T/sweep.txt 2>&1 || { echo "sweep failed"; tail gpurun_out/$T/sweep.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/sweep.txt | head -8
timeout -k 10 120 python scripts/abl_probe.py 20 > gpurun_out/$T/abl_default.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/abl_default.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/abl_default.txt
PREC=fp32 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/probe32.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/probe32.txt; exit 1; }
echo "== fp32 default"; grep -v amdgpu.ids gpurun_out/$T/probe32.txt
for n in "$@"; do
  BUGSEG_LIB=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_$n.so PREC=fp32 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/$n.txt 2>&1 || { echo "probe $n failed"; tail gpurun_out/$T/$n.txt; exit 1; }
  echo "== $n"; grep -v amdgpu.ids gpurun_out/$T/$n.txt | head -8
done
timeout -k 10 300 python bench.py --precision fp32 --extras 0 --no-cpu-baseline --steps 10 > gpurun_out/$T/bench32.json 2> gpurun_out/$T/bench32.err || { echo "bench failed"; tail -30 gpurun_out/$T/bench32.err; exit 1; }
timeout -k 10 300 python bench.py --extras 0 --no-cpu-baseline > gpurun_out/$T/bench16.json 2> gpurun_out/$T/bench16.err || { echo "bench failed"; tail -30 gpurun_out/$T/bench16.err; exit 1; }
python -c "
import json
for p in ('32', '16'):
    r = json.load(open('gpurun_out/$T/bench' + p + '.json'))
    print(p, r['value'], r['ms_per_step'], r['stages_ms'], {k: v['us_per_launch'] for k, v in r['kernels'].items()})
"
