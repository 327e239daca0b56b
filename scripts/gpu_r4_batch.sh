#!/bin/bash
# round 4: one box, several checks — BEV forms (tests + sweep), the class layer (tests), per-kernel
# launch times at the bench shard (fp16, fp32), and the bench lines (fp16 headline, fp32)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4batch}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -k "bev or occgrid or laserscan or pipeline or capture or class_layer or fp32 or timed_config or bgr or init" > gpurun_out/$T/gpu.log 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/$T/gpu.log; exit 1; }
tail -2 gpurun_out/$T/gpu.log
timeout -k 10 200 python scripts/bev_sweep.py 20 > gpurun_out/$T/sweep.txt 2>&1 || { echo "sweep failed"; tail gpurun_out/$T/sweep.txt; exit 1; }
cat gpurun_out/$T/sweep.txt
PREC=fp16 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/probe16.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/probe16.txt; exit 1; }
cat gpurun_out/$T/probe16.txt
PREC=fp32 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/probe32.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/probe32.txt; exit 1; }
cat gpurun_out/$T/probe32.txt
timeout -k 10 300 python bench.py --extras 0 --no-cpu-baseline > gpurun_out/$T/bench16.json 2> gpurun_out/$T/bench16.err || { echo "bench failed"; tail -30 gpurun_out/$T/bench16.err; exit 1; }
timeout -k 10 300 python bench.py --precision fp32 --extras 0 --no-cpu-baseline --steps 10 > gpurun_out/$T/bench32.json 2> gpurun_out/$T/bench32.err || { echo "bench failed"; tail -30 gpurun_out/$T/bench32.err; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o abl -- python scripts/abl_probe.py 20 > gpurun_out/$T/prof_abl.txt 2>&1 || { echo "rocprof failed"; tail gpurun_out/$T/prof_abl.txt; exit 1; }
python -c "
import json
for p in ('fp16', 'fp32'):
    r = json.load(open('gpurun_out/$T/bench' + p[2:] + '.json'))
    print(p, r['value'], r['ms_per_step'], 'roofline', r['roofline']['frac'], 'bev', r['stages_ms'], r['shard_overlap_ms'])
"
