#!/bin/bash
# round 3 session 3: bench.py with the graph-replay default — its distributed-branch tests, then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s3j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_capture_dist.py -m gpu -x -q -rA --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
grep -E "passed|hip_graph" $O/tests.log | tail -3
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['config']['hip_graph'], d['roofline']['frac'], d['fp32']['roofline']['forward']['mfma_frac'])"
