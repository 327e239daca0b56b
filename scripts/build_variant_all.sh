# Debug: whole-library variants differing in -D flags applied to EVERY source (A/B probes on the GPU box).
# usage: bash scripts/build_variant_all.sh NAME:FLAGS ...   -> bugcar_image_segmentation_amd/_variants/libbugseg_NAME.so
set -e
cd "$(dirname "$0")/.."
P=bugcar_image_segmentation_amd
mkdir -p $P/_variants
for v in "$@"; do
  name=${v%%:*}; flags=${v#*:}
  d=$P/_variants/obj_$name
  mkdir -p $d
  objs=""
  for s in conv_kernels.hip cls_kernels.hip init_kernels.hip bneck_kernels.hip up_kernels.hip prep_kernels.hip bev_kernels.hip deeplab_kernels.hip bugseg_runtime.cpp deeplab_runtime.cpp; do
    lang=""; case $s in *.hip) lang="-x hip";; esac
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$P/csrc $flags $lang -c $P/csrc/$s -o $d/$s.o &
    objs="$objs $d/$s.o"
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $P/_variants/libbugseg_$name.so $objs
  echo $P/_variants/libbugseg_$name.so
done
