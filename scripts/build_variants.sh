# Debug: libbugseg variants differing in one source's -D flags (for A/B probes on the GPU box).
# usage: bash scripts/build_variants.sh <source.hip> NAME:FLAGS ...   -> bugcar_image_segmentation_amd/_variants/libbugseg_NAME.so
set -e
cd "$(dirname "$0")/.."
python -m bugcar_image_segmentation_amd.build > /dev/null
src=$1; shift
P=bugcar_image_segmentation_amd
mkdir -p $P/_variants
for v in "$@"; do
  name=${v%%:*}; flags=${v#*:}
  objs=""
  for o in $P/_build/*.o; do
    if [ "$(basename $o)" = "$src.o" ]; then
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$P/csrc $flags -x hip -c $P/csrc/$src -o $P/_variants/$name.o
      objs="$objs $P/_variants/$name.o"
    else
      objs="$objs $o"
    fi
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $P/_variants/libbugseg_$name.so $objs
  echo $P/_variants/libbugseg_$name.so
done
