#!/bin/bash
# bench configuration sweep (one line per configuration) + a kernel trace of the default command
#   bash scripts/gpu_sweep.sh TAG "ARGSETS" [prof]    ARGSETS: ';'-separated bench argument sets
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-sweep}; SETS=${2:-"--streams 2"}; PROF=${3:-}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
IFS=';' read -ra A <<< "$SETS"
i=0
for s in "${A[@]}"; do
  timeout -k 10 240 python -u bench.py --extras 0 --no-cpu-baseline $s > gpurun_out/$T/s$i.json 2> gpurun_out/$T/s$i.err || { echo "set $i failed"; tail -5 gpurun_out/$T/s$i.err; exit 1; }
  python - "$s" gpurun_out/$T/s$i.json <<'PY'
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ro = r["roofline"]
top = list(r["kernels"].items())[:4]
print(f"{sys.argv[1]:40s} {r['value']:9.1f} fps  {r['ms_per_step']:.3f} ms  dom {ro['us_per_launch']:.1f} us (iso {ro['isolated']['us_per_launch']:.1f}) frac {ro['frac']:.3f}  " +
      "  ".join(f"{k}:{v['us_per_launch']}" for k, v in top), flush=True)
PY
  i=$((i+1))
done
if [ -n "$PROF" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$T/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --extras 0 --no-cpu-baseline $PROF > $GRAFT_REPO_ROOT/gpurun_out/$T/prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/$T/prof.err || { echo "prof failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/$T/prof.err; exit 1; }
  echo "prof ok"
fi
