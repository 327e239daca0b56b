#!/bin/bash
# round 4: band BEV kernel with at least 2 or 4 row parts per band (more, smaller work items) —
# bit-exact BEV tests, A/B against the previous build and the 256-thread form, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4minp}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -k "bev or occ or laserscan or binary or grid or band or ros or timed_config" > gpurun_out/$T/gpu.log 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/$T/gpu.log; exit 1; }
tail -1 gpurun_out/$T/gpu.log
for rep in 1 2; do
  for v in base minp2 minp4 new; do
    if [ $v = new ]; then unset BUGSEG_LIB; else export BUGSEG_LIB=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_$v.so; fi
    timeout -k 10 120 python scripts/abl_probe.py 20 > gpurun_out/$T/a_${v}_$rep.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/a_${v}_$rep.txt; exit 1; }
    echo "== $v $rep $(grep -E 'bev' gpurun_out/$T/a_${v}_$rep.txt)"
  done
done
unset BUGSEG_LIB
timeout -k 10 300 python bench.py --extras 0 --no-cpu-baseline > gpurun_out/$T/bench16.json 2> gpurun_out/$T/bench16.err || { echo "bench failed"; tail -30 gpurun_out/$T/bench16.err; exit 1; }
python -c "import json; r=json.load(open('gpurun_out/$T/bench16.json')); print('fp16', r['value'], r['ms_per_step'], r['stages_ms'], r['shard_overlap_ms'])"
