# Iteration loop with per-layer timing: GPU parity tests, a kernel trace of 9 single-stream B=64
# forwards (scripts/layer_times.py reads it), one bf16 bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/layers
timeout -k 10 600 python -m pytest tests -m gpu -q -x --timeout 500 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/layers -o run --output-format csv -- python3 scripts/bneck_ablate.py 0 > gpurun_out/layers/log.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_bf16.json 2> gpurun_out/bench_bf16.err || exit 1
echo done
