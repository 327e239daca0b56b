# A/B: depthwise-fused projections vs separate depthwise launches (per-op times), + fused parity test.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dl
timeout -k 10 300 python -u -m pytest tests/test_gpu_deeplab.py -x -q -k fused --timeout 120 --timeout-method thread > gpurun_out/pytest_deeplab_fuse.log 2>&1 || { tail -30 gpurun_out/pytest_deeplab_fuse.log; exit 1; }
tail -1 gpurun_out/pytest_deeplab_fuse.log
timeout -k 10 300 python bench_deeplab.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/dl/bench_plain.json 2>/dev/null || exit 1
for nb in 2 4; do
BUGSEG_DL_NB=$nb BUGSEG_DL_FUSE_DW=1 timeout -k 10 300 python bench_deeplab.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/dl/bench_fuse$nb.json 2>/dev/null || exit 1
done
echo done
