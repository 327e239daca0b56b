#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/offs
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "multistream or captured" -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3_h_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3_h_tests.log; exit 1; }
tail -2 gpurun_out/r3_h_tests.log
for k in 0 4 10 16 0 4 10 16; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --extras 0 --shard-offset $k > gpurun_out/offs/b$k.json 2> gpurun_out/offs/b$k.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/offs/b$k.json')); print('offset $k', d['value'], d['ms_per_step'])"
done
