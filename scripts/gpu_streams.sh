set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x --timeout 500 > gpurun_out/pytest_gpu.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_gpu.log
for s in 1 2 4; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --streams $s > gpurun_out/bench_s$s.json 2> gpurun_out/bench_s$s.err || exit 1
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --streams 2 --batch 128 > gpurun_out/bench_s2_b128.json 2> gpurun_out/bench_s2_b128.err || exit 1
echo done
