#!/bin/bash
# Round 6: the class layer fused into the last bottleneck — parity, then the fp32 / fp16 bench lines
#   bash scripts/gpu_r6_cls.sh TAG [pytest -k expression]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-cls}; K=${2:-"class_fusion or class_layer or canonical or launch_spans or fused_bottlenecks_equal"}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_capture_dist.py -k "$K" -s > gpurun_out/$T/parity.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/$T/parity.log; exit 1; }
tail -3 gpurun_out/$T/parity.log
for p in fp32 fp16; do
  timeout -k 10 240 python -u bench.py --extras 0 --no-cpu-baseline --precision $p > gpurun_out/$T/bench_$p.json 2> gpurun_out/$T/bench_$p.err || { echo "bench $p failed"; tail -20 gpurun_out/$T/bench_$p.err; exit 1; }
  python - $p gpurun_out/$T/bench_$p.json <<'PY'
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:6s} {r['value']:9.1f} fps {r['ms_per_step']:.3f} ms  " + "  ".join(f"{k}:{v['us_per_launch']}" for k, v in r["kernels"].items()), flush=True)
PY
done
