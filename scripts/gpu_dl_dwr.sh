# DeepLab depthwise rows-per-thread A/B (stride-1 layers): parity at the default (4) and 8, bench at 2, 4, 8.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dwr
for r in 4 8; do
  BUGSEG_DL_DWR=$r timeout -k 10 300 python -u -m pytest tests/test_gpu_deeplab.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dwr/pytest$r.log 2>&1 || { tail -30 gpurun_out/dwr/pytest$r.log; exit 1; }
  tail -1 gpurun_out/dwr/pytest$r.log
done
for r in 2 4 8; do
  BUGSEG_DL_DWR=$r timeout -k 10 200 python bench_deeplab.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/dwr/r$r.json 2> gpurun_out/dwr/r$r.err || exit 1
done
echo done
