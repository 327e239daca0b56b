#!/bin/bash
# round 3 (session 2): 256 x 256 glds GEMM for the deep 1x1s — bit-identity tests, then the DeepLab
# benches (Xception-65 B = 32, MobileNetV2 B = 64) with it and without it (BUGSEG_DL_G256=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/g256
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 500 python -u -m pytest tests/test_gpu_deeplab.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/g256/tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/g256/tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 gpurun_out/g256/tests.log
for cfg in "on:" "off:BUGSEG_DL_G256=0" "on2:"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 200 python bench_deeplab.py --backbone xception_65 --batch 32 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/g256/xc_$name.json 2> gpurun_out/g256/xc_$name.err || { echo "xc $name failed"; tail gpurun_out/g256/xc_$name.err; exit 1; }
  env $envs timeout -k 10 200 python bench_deeplab.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/g256/mb_$name.json 2> gpurun_out/g256/mb_$name.err || { echo "mb $name failed"; tail gpurun_out/g256/mb_$name.err; exit 1; }
  python - <<PY
import json
for k in ("xc", "mb"):
    d = json.load(open("gpurun_out/g256/%s_$name.json" % k))
    r = d["roofline"]
    print("$name", k, d["value"], d["ms_per_step"], r["bound"], r["achieved"], r["frac"], r["kernel"][:90])
PY
done
