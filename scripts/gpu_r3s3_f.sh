#!/bin/bash
# round 3 session 3: the fp32 16x16 class layer (cls16_kernel) — parity, then timing vs the 32x32 form
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s3f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fp32 or class" -m gpu -x -q -rA --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -60 $O/tests.log; exit 1; }
grep -E "passed|failed|class layer 16x16" $O/tests.log | tail -6
for form in 16 0 16 0; do
  BUGSEG_CLS16=$form PREC=fp32 timeout -k 10 120 python scripts/batch_probe.py 32 > $O/probe_$form.txt 2>&1 || { echo "probe $form failed"; tail $O/probe_$form.txt; exit 1; }
  grep -E "forward|classes" $O/probe_$form.txt
  BUGSEG_CLS16=$form timeout -k 10 200 python bench.py --precision fp32 --no-cpu-baseline --extras 0 > $O/bench_$form.json 2> $O/bench_$form.err || { echo "bench $form failed"; tail $O/bench_$form.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$form.json')); print('cls16=$form', d['value'], d['ms_per_step'], d['roofline']['forward']['ms'], d['roofline']['forward']['mfma_frac'], d['kernels']['classes'])"
done
