# DeepLab parity at both conv tilings + bench A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dl
timeout -k 10 400 python -u -m pytest tests/test_gpu_deeplab.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_deeplab.log 2>&1 || { tail -30 gpurun_out/pytest_deeplab.log; exit 1; }
tail -1 gpurun_out/pytest_deeplab.log
BUGSEG_DL_NB=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_deeplab.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_deeplab4.log 2>&1 || { tail -30 gpurun_out/pytest_deeplab4.log; exit 1; }
tail -1 gpurun_out/pytest_deeplab4.log
timeout -k 10 300 python bench_deeplab.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/dl/bench_nb2.json 2> gpurun_out/dl/bench_nb2.err || exit 1
BUGSEG_DL_NB=8 timeout -k 10 300 python bench_deeplab.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/dl/bench_nb8.json 2> gpurun_out/dl/bench_nb8.err || exit 1
echo done
