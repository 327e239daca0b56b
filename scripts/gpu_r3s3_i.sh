#!/bin/bash
# round 3 session 3: the 256 x 128 two-per-CU DeepLab GEMM tile (BUGSEG_DL_P2) bit-identity + Xception timing;
# then the step as one HIP graph vs eager and 1 / 3 shard streams (bench lines)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s3i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_deeplab.py -k "gemm128_bit_identical and p2" -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "p2 tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for p2 in 0 1 0 1; do
  BUGSEG_DL_P2=$p2 timeout -k 10 200 python3 bench_deeplab.py --backbone xception_65 --batch 32 --steps 6 --warmup 2 --no-cpu-baseline > $O/xc_p2$p2.json 2> $O/xc_p2$p2.err || { echo "xc bench p2=$p2 failed"; tail $O/xc_p2$p2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/xc_p2$p2.json')); k=d['kernels']['conv pointwise']; print('p2=$p2', d['value'], k['us'], k['TFLOPs'])"
done
bash scripts/gpu_r3s3_h.sh || exit 1
