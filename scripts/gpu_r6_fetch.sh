#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per kernel tag for one bench configuration (PMC passes, each its own run)
#   bash scripts/gpu_r6_fetch.sh TAG "ENV=VAL ..." "bench args"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-fetch}; EV=${2:-}; ARGS=${3:-}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for kv in $EV; do export "$kv"; done
CMD="$GRAFT_REPO_ROOT/bench.py --extras 0 --no-cpu-baseline --steps 10 $ARGS"
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $CMD > $O/fetch.json 2> $O/fetch.err || { echo "fetch pass failed"; tail -5 $O/fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $CMD > $O/write.json 2> $O/write.err || { echo "write pass failed"; tail -5 $O/write.err; exit 1; }
cd $GRAFT_REPO_ROOT
python - $O <<'PY'
import csv, glob, sys
from collections import defaultdict
sys.path.insert(0, "scripts")
from layer_times import short
o = sys.argv[1]
res = {}
for c, d in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
    f = glob.glob(f"{o}/{d}/**/*counter_collection.csv", recursive=True)[0]
    vals = defaultdict(list)
    for row in csv.DictReader(open(f)):
        if row["Counter_Name"] == c:
            vals[short(row["Kernel_Name"])].append(float(row["Counter_Value"]) * 1024.0 * (2 if c == "FETCH_SIZE" else 1))
    res[c] = {k: sum(v) / len(v) for k, v in vals.items()}
for k in sorted(res["FETCH_SIZE"]):
    if k.startswith(("bneck", "down", "up", "init", "classes")):
        print(f"{k:32s} read {res['FETCH_SIZE'][k] / 1e6:8.1f} MB  write {res['WRITE_SIZE'].get(k, 0) / 1e6:8.1f} MB per launch")
PY
