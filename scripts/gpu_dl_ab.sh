#!/bin/bash
# A/B of library builds on bench_deeplab.py: one line per library (BUGSEG_LIB), twice each, alternating
#   bash scripts/gpu_dl_ab.sh TAG "libA.so libB.so libA.so@VAR=value" "bench_deeplab args"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-dlab}; LIBS=${2:-libbugseg.so}; ARGS=${3:-"--backbone resnet_v1_101_beta --batch 16 --steps 10"}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for rep in 1 2; do
  for spec in $LIBS; do
    l=${spec%%@*}; ev=""; [ "$spec" != "$l" ] && ev=${spec#*@}
    n=$(basename $l .so)${ev:+_$ev}
    env $ev BUGSEG_LIB=$GRAFT_REPO_ROOT/bugcar_image_segmentation_amd/$l timeout -k 10 300 python -u bench_deeplab.py --no-cpu-baseline $ARGS > gpurun_out/$T/$n.$rep.json 2> gpurun_out/$T/$n.$rep.err || { echo "$n failed"; tail -5 gpurun_out/$T/$n.$rep.err; exit 1; }
    python - "$n" gpurun_out/$T/$n.$rep.json <<'PY'
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:24s} {r['value']:9.1f} fps {r['ms_per_step']:.3f} ms  " + "  ".join(f"{k}:{v['us']:.0f}" for k, v in r["kernels"].items()), flush=True)
PY
  done
done
