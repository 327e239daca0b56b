#!/bin/bash
# round 4: 2-stream bench A/B — fused bottlenecks on all resident slots (default) against half of them
# (BUGSEG_BNECK_GRID=-2: the two shards' launches can be co-resident and desynchronise)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4half}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for rep in 1 2; do
  for g in 0 -2; do
    BUGSEG_BNECK_GRID=$g timeout -k 10 300 python bench.py --extras 0 --no-cpu-baseline > gpurun_out/$T/b_${g}_$rep.json 2> gpurun_out/$T/b_${g}_$rep.err || { echo "bench failed"; tail -30 gpurun_out/$T/b_${g}_$rep.err; exit 1; }
    python -c "import json; r=json.load(open('gpurun_out/$T/b_${g}_$rep.json')); print('grid $g rep $rep', r['value'], r['ms_per_step'], r['shard_overlap_ms'])"
  done
done
