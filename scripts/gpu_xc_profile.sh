#!/bin/bash
# Xception-65 / DeepLabV3+ (config 4, other export) profile: bench line, rocprofv3 kernel-trace/stats,
# FETCH_SIZE and WRITE_SIZE passes (summarise: python scripts/dl_pmc_summary.py gpurun_out/TAG
# profiles/TAG_pmc_traffic.md profiles/dl_pmc_traffic_xception.json --batch 32 --backbone xception_65)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-xcprof}
ARGS="--backbone xception_65 --batch 32 --steps 6 --warmup 2 --no-cpu-baseline"
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python3 bench_deeplab.py $ARGS > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/trace -o run --output-format csv -- python3 bench_deeplab.py $ARGS > gpurun_out/$TAG/trace.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/$TAG/fetch -o run --output-format csv -- python3 bench_deeplab.py $ARGS > gpurun_out/$TAG/fetch.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/$TAG/write -o run --output-format csv -- python3 bench_deeplab.py $ARGS > gpurun_out/$TAG/write.log 2>&1 || exit 1
echo done
