#!/bin/bash
# round 3 session 3: the step as one captured HIP graph vs eager, and 1 / 2 / 3 shard streams (bench lines only)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s3h
mkdir -p $O
export TMPDIR=/tmp
for cfg in "eager:--graph 0" "graph:--graph 1" "s1:--streams 1" "s3:--streams 3" "eager2:--graph 0" "graph2:--graph 1"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 200 python bench.py --no-cpu-baseline --extras 0 $args > $O/bench_$name.json 2> $O/bench_$name.err || { echo "bench $name failed"; tail $O/bench_$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$name.json')); print('$name', d['value'], d['ms_per_step'])"
done
