#!/bin/bash
# round 4 end: the driver's sequence (pytest -m gpu, smoke, default bench) then the profile refresh
# (rocprofv3 stats + FETCH / WRITE PMC passes, fp16 and fp32)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_r4_final.sh ${1:-r4final4} || exit 1
TAG=${2:-r04_g} bash scripts/gpu_r3_prof.sh || exit 1
echo end done
