# Round profile: one bench line, the rocprofv3 kernel-trace/stats run of the same command, then HBM
# traffic counters in separate passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950).
# Usage: bash scripts/gpu_profile.sh TAG [bench args]; summarise with scripts/prof_summary.py and
# scripts/pmc_summary.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-prof}; shift
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --extras 0 $*"
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/$TAG/trace.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/$TAG/fetch -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/$TAG/fetch.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/$TAG/write -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/$TAG/write.log 2>&1 || exit 1
echo done
