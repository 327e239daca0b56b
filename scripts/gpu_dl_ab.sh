# A/B of whole-library variants (scripts/build_variant_all.sh) on the DeepLab benches: per variant the
# Xception (B = 32) and MobileNetV2 (B = 64) lines, with per-op-tag times.
# usage: bash scripts/gpu_dl_ab.sh NAME ...   -> gpurun_out/dlab/NAME/{x,m}.json
set -o pipefail
cd $GRAFT_REPO_ROOT
for n in "$@"; do
  lib=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_$n.so
  o=gpurun_out/dlab/$n
  mkdir -p $o
  BUGSEG_LIB=$lib timeout -k 10 200 python bench_deeplab.py --backbone xception_65 --batch 32 --steps 10 --warmup 3 --no-cpu-baseline > $o/x.json 2> $o/x.err || exit 1
  BUGSEG_LIB=$lib timeout -k 10 200 python bench_deeplab.py --batch 64 --steps 10 --warmup 3 --no-cpu-baseline > $o/m.json 2> $o/m.err || exit 1
  echo "$n done"
done
