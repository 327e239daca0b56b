# A/B: batch_probe.py under each library of bugcar_image_segmentation_amd/_variants (filter: $1 regex)
cd $GRAFT_REPO_ROOT
pat=${1:-.}
for lib in bugcar_image_segmentation_amd/_variants/libbugseg_*.so; do
  n=$(basename $lib .so); n=${n#libbugseg_}
  BUGSEG_LIB=$PWD/$lib timeout -k 10 100 python scripts/batch_probe.py 32 2>&1 | grep -E "$pat|forward" | sed "s/^/$n /" || exit 1
done > gpurun_out/variants.txt
