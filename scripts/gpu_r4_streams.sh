#!/bin/bash
# round 4: shard streams A/B in the bench (2 shards of 32 frames vs 4 of 16 vs 1 of 64)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4streams}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for rep in 1 2; do
  for st in 2 4 1; do
    timeout -k 10 300 python bench.py --extras 0 --no-cpu-baseline --streams $st > gpurun_out/$T/b_${st}_$rep.json 2> gpurun_out/$T/b_${st}_$rep.err || { echo "bench failed"; tail -30 gpurun_out/$T/b_${st}_$rep.err; exit 1; }
    python -c "import json; r=json.load(open('gpurun_out/$T/b_${st}_$rep.json')); print('streams $st rep $rep', r['value'], r['ms_per_step'])"
  done
done
