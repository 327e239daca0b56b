# A/B of whole-library variants (scripts/build_variant_all.sh): per variant, per-kernel-tag launch times
# (batch_probe.py at the bench shard size), the bench line (no CPU baseline, no sub-records) and the
# HBM traffic counters of batch_probe in two separate rocprofv3 passes (FETCH_SIZE, WRITE_SIZE).
# usage: [NOPMC=1] bash scripts/gpu_ab.sh NAME ...   (summaries: python scripts/pmc_summary.py gpurun_out/ab/NAME)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for n in "$@"; do
  lib=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_$n.so
  o=gpurun_out/ab/$n
  mkdir -p $o
  BUGSEG_LIB=$lib timeout -k 10 120 python scripts/batch_probe.py 32 > $o/probe.txt 2>&1 || exit 1
  BUGSEG_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --extras 0 > $o/bench.json 2> $o/bench.err || exit 1
  if [ -n "$NOPMC" ]; then echo "$n done"; continue; fi
  BUGSEG_LIB=$lib timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $o/fetch -o run --output-format csv -- python3 scripts/batch_probe.py 32 > $o/fetch.log 2>&1 || exit 1
  BUGSEG_LIB=$lib timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $o/write -o run --output-format csv -- python3 scripts/batch_probe.py 32 > $o/write.log 2>&1 || exit 1
  echo "$n done"
done
