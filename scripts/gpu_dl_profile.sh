# DeepLab (config 4) round profile: bench line, rocprofv3 kernel-trace/stats of the same command,
# then FETCH_SIZE and WRITE_SIZE in separate --pmc passes (summarised by scripts/dl_pmc_summary.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-dlprof}
ARGS=${DLARGS:-"--steps 10 --warmup 3 --no-cpu-baseline"}   # e.g. DLARGS="--backbone resnet_v1_101_beta --batch 16 ..."
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python3 bench_deeplab.py $ARGS > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/trace -o run --output-format csv -- python3 bench_deeplab.py $ARGS > gpurun_out/$TAG/trace.log 2>&1 || exit 1
[ "$2" = nopmc ] && { echo done; exit 0; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/$TAG/fetch -o run --output-format csv -- python3 bench_deeplab.py $ARGS > gpurun_out/$TAG/fetch.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/$TAG/write -o run --output-format csv -- python3 bench_deeplab.py $ARGS > gpurun_out/$TAG/write.log 2>&1 || exit 1
echo done
