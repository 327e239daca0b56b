#!/bin/bash
# quick GPU check: the given test files, then an A/B of library builds (scripts/gpu_ab.sh)
#   bash scripts/gpu_quick.sh TAG "test files" "libs" ["bench args"]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-q}; TESTS=${2:-}; LIBS=${3:-}; ARGS=${4:-}
mkdir -p gpurun_out/$T
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > gpurun_out/$T/tests.log 2>&1
  rc=$?; tail -3 gpurun_out/$T/tests.log
  [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/$T/tests.log | head -20; exit $rc; }
fi
[ -n "$LIBS" ] && bash scripts/gpu_ab.sh $T "$LIBS" "$ARGS"
exit $?
