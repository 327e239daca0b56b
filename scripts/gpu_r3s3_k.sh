#!/bin/bash
# round 3 session 3: BEV band kernel early exit for waves of cells outside the camera footprint (BEV_DEAD)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s3k
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_dead.so
BUGSEG_LIB=$L timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capture_dist.py tests/test_gpu_timed_config.py -k "bev or laserscan or pipeline or capture or stream" -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in "dead:BUGSEG_LIB=$L" "nodead:" "dead:BUGSEG_LIB=$L" "nodead:"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --extras 0 > $O/bench_$name.json 2> $O/bench_$name.err || { echo "bench $name failed"; tail $O/bench_$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$name.json')); print('$name', d['value'], d['ms_per_step'], d['stages_ms'], d['shard_overlap_ms'])"
done
