#!/bin/bash
# round 6: up-block whole-line stores — parity (fused == unfused, up pair), then fp32 bench + WRITE_SIZE pass
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r6up}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/mixed_range_diag.py > $O/mixed.log 2>&1 || { echo "mixed diag failed"; tail -20 $O/mixed.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "(fused_bottlenecks_equal_unfused and fp32) or up_block_pair" > $O/parity.log 2>&1 || { echo "parity failed"; tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
CMD="$GRAFT_REPO_ROOT/bench.py --precision fp32 --extras 0 --no-cpu-baseline --steps 10"
timeout -k 10 300 python -u $CMD > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $CMD > $O/write.json 2> $O/write.err || { echo "write pass failed"; tail -5 $O/write.err; exit 1; }
cd $GRAFT_REPO_ROOT
python - $O <<'PY'
import csv, glob, json, sys
from collections import defaultdict
sys.path.insert(0, "scripts")
from layer_times import short
o = sys.argv[1]
r = json.loads(open(o + "/bench.json").read().strip().splitlines()[-1])
print("bench", r["value"], "fps", {k: v["us_per_launch"] for k, v in r["kernels"].items()})
f = glob.glob(o + "/write/**/*counter_collection.csv", recursive=True)[0]
vals = defaultdict(list)
for row in csv.DictReader(open(f)):
    if row["Counter_Name"] == "WRITE_SIZE":
        vals[short(row["Kernel_Name"])].append(float(row["Counter_Value"]) * 1024.0)
for k, v in sorted(vals.items()):
    print(f"WRITE {k:40s} {sum(v) / len(v) / 1e6:8.1f} MB per launch ({len(v)} launches)")
PY
