#!/bin/bash
# round 4: C128 8x16 tiles with the next tile's loads in flight (XPF) — the multi-tile-walk parity tests,
# then forward tables and the bench line with the symmetric C128 layers on 8x16 (BUGSEG_BNECK_C128_SMALL)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4xpf}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -k "multi_tile or fused_bottlenecks or fp32 or timed_config or config1" > gpurun_out/$T/gpu.log 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/$T/gpu.log; exit 1; }
tail -1 gpurun_out/$T/gpu.log
for s in 0 1; do
  if [ $s = 1 ]; then export BUGSEG_BNECK_C128_SMALL=1; fi
  PREC=fp16 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/p16_$s.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/p16_$s.txt; exit 1; }
  echo "== small=$s"; grep -v amdgpu.ids gpurun_out/$T/p16_$s.txt | head -7
  timeout -k 10 300 python bench.py --extras 0 --no-cpu-baseline > gpurun_out/$T/bench_$s.json 2> gpurun_out/$T/bench_$s.err || { echo "bench failed"; tail -30 gpurun_out/$T/bench_$s.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/$T/bench_$s.json')); print('small=$s', r['value'], r['ms_per_step'], r['stages_ms']['enet_forward'])"
done
unset BUGSEG_BNECK_C128_SMALL
PREC=fp32 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/p32.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/p32.txt; exit 1; }
echo "== fp32"; grep -v amdgpu.ids gpurun_out/$T/p32.txt | head -7
timeout -k 10 300 python bench.py --precision fp32 --extras 0 --no-cpu-baseline --steps 10 > gpurun_out/$T/bench32.json 2> gpurun_out/$T/bench32.err || { echo "bench failed"; tail -30 gpurun_out/$T/bench32.err; exit 1; }
python -c "import json; r=json.load(open('gpurun_out/$T/bench32.json')); print('fp32', r['value'], r['ms_per_step'], r['stages_ms']['enet_forward'])"
