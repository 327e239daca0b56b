#!/bin/bash
# Profile set for one precision: the bench line, a rocprofv3 kernel trace of the same command, and the
# FETCH_SIZE / WRITE_SIZE PMC passes (each its own run, MI355X_MICROARCH.md's HBM recipe).
#   bash scripts/gpu_prof.sh TAG PRECISION [extra bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-prof}; P=${2:-fp32}; shift 2; X="$*"
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
CMD="$GRAFT_REPO_ROOT/bench.py --precision $P --extras 0 --no-cpu-baseline $X"
timeout -k 10 300 python -u $CMD > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $CMD > $O/trace.json 2> $O/trace.err || { echo "trace failed"; tail -5 $O/trace.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $CMD > $O/fetch.json 2> $O/fetch.err || { echo "fetch pass failed"; tail -5 $O/fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $CMD > $O/write.json 2> $O/write.err || { echo "write pass failed"; tail -5 $O/write.err; exit 1; }
echo "profile set ok"
