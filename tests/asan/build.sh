# Host-only ASan + UBSan build of the runtime's parsing paths and the driver
# that exercises them. The two runtime translation units and the driver are instrumented (host code;
# -fsanitize only after -Xarch_host: no device sanitizer); the kernel objects come from the normal
# build (bugcar_image_segmentation_amd/_build) uninstrumented. CPU only: the driver touches no device.
# usage: bash tests/asan/build.sh OUT_DIR
set -e
cd "$(dirname "$0")/../.."
OUT=${1:-tests/asan/_build}
P=bugcar_image_segmentation_amd
mkdir -p $OUT
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined"
FLAGS="--offload-arch=gfx950 -O1 -g -std=c++17 -fno-omit-frame-pointer -Iinclude -I$P/csrc"
python -m bugcar_image_segmentation_amd.build > /dev/null
for s in bugseg_runtime deeplab_runtime; do
  /opt/rocm/bin/hipcc $FLAGS $SAN -c $P/csrc/$s.cpp -o $OUT/$s.o &
done
/opt/rocm/bin/hipcc $FLAGS $SAN -c tests/asan/asan_driver.cpp -o $OUT/asan_driver.o &
wait
KOBJ=""
for s in conv_kernels cls_kernels init_kernels bneck_kernels bneck2_kernels up_kernels prep_kernels bev_kernels deeplab_kernels; do
  KOBJ="$KOBJ $P/_build/$s.hip.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 $SAN -o $OUT/asan_driver $OUT/asan_driver.o $OUT/bugseg_runtime.o $OUT/deeplab_runtime.o $KOBJ
echo $OUT/asan_driver
