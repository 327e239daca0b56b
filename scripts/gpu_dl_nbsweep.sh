# DeepLab per-op A/B of the conv tiling (pixel fragments per wave) after the XCD-aware block order.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/nb
for nb in 2 4 8; do
  BUGSEG_DL_NB=$nb timeout -k 10 200 python bench_deeplab.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/nb/nb$nb.json 2> gpurun_out/nb/nb$nb.err || exit 1
done
timeout -k 10 200 python bench_deeplab.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/nb/auto.json 2> gpurun_out/nb/auto.err || exit 1
echo done
