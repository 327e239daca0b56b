# GPU check of the kept-residual bottleneck: the bit-identity / parity tests of the fused kernels,
# then the A/B of scripts/gpu_ab.sh (keep0 = residual re-read, keep1 = kept in registers).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_keep.log 2>&1 || { tail -30 gpurun_out/pytest_keep.log; exit 1; }
tail -2 gpurun_out/pytest_keep.log
bash scripts/gpu_ab.sh "$@"
