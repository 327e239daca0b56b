#!/bin/bash
# round 6 GPU session step: [range tests] -> [whole -m gpu suite] -> [smoke] -> [bench line]
#   bash scripts/gpu_r6.sh TAG "STEPS"   (STEPS: any of range timed dist suite smoke bench benchx; default: range suite smoke bench)
# Each GPU step runs under its own time limit; the first failure ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r6}
STEPS=${2:-"range suite smoke bench"}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
for s in $STEPS; do
  case $s in
    range) timeout -k 10 600 $PYT tests/test_gpu_range.py > gpurun_out/$T/range.log 2>&1; rc=$? ;;
    timed) timeout -k 10 600 $PYT tests/test_gpu_timed_config.py > gpurun_out/$T/timed.log 2>&1; rc=$? ;;
    dist) timeout -k 10 600 $PYT tests/test_gpu_capture_dist.py -k "bench or two_ranks" > gpurun_out/$T/dist.log 2>&1; rc=$? ;;
    suite) timeout -k 10 900 $PYT -m gpu tests > gpurun_out/$T/suite.log 2>&1; rc=$? ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1; rc=$? ;;
    bench) timeout -k 10 600 python -u bench.py --extras 0 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err; rc=$? ;;
    benchx) timeout -k 10 900 python -u bench.py > gpurun_out/$T/benchx.json 2> gpurun_out/$T/benchx.err; rc=$? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  echo "== $s rc=$rc"
  if [ $rc -ne 0 ]; then
    for f in gpurun_out/$T/*; do echo "--- $f"; tail -25 "$f"; done
    exit $rc
  fi
done
grep -E "passed|failed" gpurun_out/$T/*.log 2>/dev/null | tail -5
grep -hE "max\|dlogit\||undamped|x 1e|fp32 B=64|batch independence|frame [0-9]: max" gpurun_out/$T/range.log gpurun_out/$T/timed.log 2>/dev/null | head -40
[ -f gpurun_out/$T/bench.json ] && cut -c1-600 gpurun_out/$T/bench.json
exit 0
