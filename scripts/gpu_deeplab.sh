# DeepLab parity tests only.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_deeplab.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_deeplab.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_deeplab.log
