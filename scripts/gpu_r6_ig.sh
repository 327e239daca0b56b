#!/bin/bash
# round 6: implicit-GEMM dense conv (DeepLab bf16) — deeplab GPU tests, then the ResNet-101 bench with
# IG on and off (BUGSEG_DL_IG=0), then the per-kernel profile of the default
#   bash scripts/gpu_r6_ig.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r6ig}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_deeplab.py \
  > gpurun_out/$T/tests.log 2>&1 || { tail -40 gpurun_out/$T/tests.log; exit 1; }
grep -E "passed|failed|implicit GEMM" gpurun_out/$T/tests.log | tail -4
for ig in 1 0; do
  BUGSEG_DL_IG=$ig timeout -k 10 300 python -u bench_deeplab.py --backbone resnet_v1_101_beta --batch 16 --steps 10 \
    --no-cpu-baseline > gpurun_out/$T/bench_ig$ig.json 2> gpurun_out/$T/bench_ig$ig.err || { tail -20 gpurun_out/$T/bench_ig$ig.err; exit 1; }
  python - gpurun_out/$T/bench_ig$ig.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], d["ms_per_step"], {k: round(v["us"], 1) for k, v in d["roofline"].get("kernels", d.get("kernels", {})).items()} if "kernels" in d["roofline"] else {k: round(v["us"], 1) for k, v in d.get("kernels", {}).items()})
PY
done
exit 0
