# parity tests of the fused kernels, then library A/B (gpu_ab.sh, NOPMC) and env A/B of the grid cap
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_keep.log 2>&1 || { tail -30 gpurun_out/pytest_keep.log; exit 1; }
tail -2 gpurun_out/pytest_keep.log
NOPMC=1 bash scripts/gpu_ab.sh glds0 glds1 || exit 1
bash scripts/gpu_envab.sh BUGSEG_BNECK_GRID '' '2048'
