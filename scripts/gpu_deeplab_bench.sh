# DeepLab (config 4) bench line + rocprofv3 kernel stats of the same command.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dl
export TMPDIR=/tmp
timeout -k 10 300 python bench_deeplab.py --steps 10 --warmup 3 > gpurun_out/dl/bench.json 2> gpurun_out/dl/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dl/prof -o run --output-format csv -- python bench_deeplab.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/dl/prof.log 2>&1 || exit 1
echo done
