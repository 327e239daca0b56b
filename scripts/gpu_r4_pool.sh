#!/bin/bash
# round 4: packed-f16 pool in the initial block — parity (pool forms equal, BGR == preprocess + forward,
# storage oracles), the fp16 kernel table and bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4pool}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -k "init or bgr or fp16 or bf16 or pool or timed_config or preprocess" > gpurun_out/$T/gpu.log 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/$T/gpu.log; exit 1; }
tail -1 gpurun_out/$T/gpu.log
for sc in 0 1; do
  if [ $sc = 1 ]; then export BUGSEG_INIT_POOL_SCAN=1; fi
  PREC=fp16 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/p16_$sc.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/p16_$sc.txt; exit 1; }
  echo "== scan=$sc"; grep -E "forward|init" gpurun_out/$T/p16_$sc.txt
done
unset BUGSEG_INIT_POOL_SCAN
timeout -k 10 300 python bench.py --extras 0 --no-cpu-baseline > gpurun_out/$T/bench16.json 2> gpurun_out/$T/bench16.err || { echo "bench failed"; tail -30 gpurun_out/$T/bench16.err; exit 1; }
python -c "import json; r=json.load(open('gpurun_out/$T/bench16.json')); print('fp16', r['value'], r['ms_per_step'], r['kernels']['init'])"
