#!/bin/bash
# round 4: class-layer addressing (flat pixel index, one pixel computation per group, 32-bit buffer
# stores) — class-map parity, A/B kernel tables against the previous build, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4cls}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -k "class or cls or binary or timed_config or forward or lut or argmax" > gpurun_out/$T/gpu.log 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/$T/gpu.log; exit 1; }
tail -1 gpurun_out/$T/gpu.log
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export BUGSEG_LIB=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_base.so; else unset BUGSEG_LIB; fi
    for p in fp16 fp32; do
      PREC=$p timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/p_${v}_${p}_$rep.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/p_${v}_${p}_$rep.txt; exit 1; }
      echo "== $v $p $rep $(grep -E 'forward' gpurun_out/$T/p_${v}_${p}_$rep.txt) $(grep -E 'classes' gpurun_out/$T/p_${v}_${p}_$rep.txt)"
    done
  done
done
unset BUGSEG_LIB
timeout -k 10 300 python bench.py --extras 0 --no-cpu-baseline > gpurun_out/$T/bench16.json 2> gpurun_out/$T/bench16.err || { echo "bench failed"; tail -30 gpurun_out/$T/bench16.err; exit 1; }
python -c "import json; r=json.load(open('gpurun_out/$T/bench16.json')); print('fp16', r['value'], r['ms_per_step'], r['kernels']['classes'])"
