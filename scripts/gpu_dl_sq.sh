# DeepLab SQ wave-cycle breakdown per op (one --pmc pass, 6 SQ counters), plus parity + bench at the defaults.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/dlsq
timeout -k 10 300 python -u -m pytest tests/test_gpu_deeplab.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dlsq/pytest.log 2>&1 || { tail -30 gpurun_out/dlsq/pytest.log; exit 1; }
tail -1 gpurun_out/dlsq/pytest.log
timeout -k 10 200 python bench_deeplab.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/dlsq/bench.json 2> gpurun_out/dlsq/bench.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/dlsq/sq -o run --output-format csv -- python3 bench_deeplab.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/dlsq/sq.log 2>&1 || exit 1
echo done
