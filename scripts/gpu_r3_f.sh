#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capture_dist.py -k "bev or laserscan or pipeline or capture or fused or multi_tile or forward_bgr or fp32 or fp16 or bf16 or config1" -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3_f_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3_f_tests.log; exit 1; }
tail -2 gpurun_out/r3_f_tests.log
timeout -k 10 120 python scripts/bev_sweep.py 20 > gpurun_out/bev_sweep.txt 2>&1; cat gpurun_out/bev_sweep.txt
bash scripts/gpu_ab.sh ak0 ak1s0 ak1s1 || exit 1
for n in ak0 ak1s0 ak1s1; do echo "== $n"; grep -E "asym|forward" gpurun_out/ab/$n/probe.txt; python -c "import json; d=json.load(open('gpurun_out/ab/$n/bench.json')); print(d['value'], d['ms_per_step'])"; python scripts/pmc_summary.py gpurun_out/ab/$n /tmp/x.md /tmp/x.json > /dev/null 2>&1; grep -i asym /tmp/x.md; done
