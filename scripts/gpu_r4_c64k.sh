#!/bin/bash
# round 4: C64 bottleneck as an 8-wave workgroup with the residual kept (variant 3) — bit-identity tests
# (every variant forced, multi-tile walks), A/B kernel tables against the default 16x16 form, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4c64k}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -k "fused_bottlenecks" > gpurun_out/$T/gpu.log 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/$T/gpu.log; exit 1; }
tail -1 gpurun_out/$T/gpu.log
for rep in 1 2; do
  for v in def k6 k8; do
    unset BUGSEG_LIB BUGSEG_BNECK_VARIANT_C64
    [ $v != def ] && export BUGSEG_BNECK_VARIANT_C64=3
    [ $v = k8 ] && export BUGSEG_LIB=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_k8.so
    PREC=fp16 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/p_${v}_$rep.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/p_${v}_$rep.txt; exit 1; }
    echo "== $v $rep $(grep -E 'forward' gpurun_out/$T/p_${v}_$rep.txt) | $(grep -E 'bneck C64' gpurun_out/$T/p_${v}_$rep.txt)"
  done
done
unset BUGSEG_LIB BUGSEG_BNECK_VARIANT_C64
for v in def k6; do
  [ $v = k6 ] && export BUGSEG_BNECK_VARIANT_C64=3
  timeout -k 10 300 python bench.py --extras 0 --no-cpu-baseline > gpurun_out/$T/b_$v.json 2> gpurun_out/$T/b_$v.err || { echo "bench failed"; tail -30 gpurun_out/$T/b_$v.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/$T/b_$v.json')); print('bench $v', r['value'], r['ms_per_step'], r['roofline']['us_per_launch'], r['roofline']['kernel'][:60])"
done
