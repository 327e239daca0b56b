# DeepLab conv k-step prefetch depth A/B: parity at PD 2 and 3, then per-op bench at PD 1, 2, 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pd
for pd in 2 3; do
  BUGSEG_DL_PD=$pd timeout -k 10 300 python -u -m pytest tests/test_gpu_deeplab.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pd/pytest$pd.log 2>&1 || { tail -30 gpurun_out/pd/pytest$pd.log; exit 1; }
  tail -1 gpurun_out/pd/pytest$pd.log
done
for pd in 1 2 3; do
  BUGSEG_DL_PD=$pd timeout -k 10 200 python bench_deeplab.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/pd/pd$pd.json 2> gpurun_out/pd/pd$pd.err || exit 1
done
echo done
