#!/bin/bash
# round-3 profiles: the fp16 headline and the fp32 parity mode (rocprofv3 stats + FETCH/WRITE PMC passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_profile.sh ${TAG:-r03_a}_fp16 || exit 1
bash scripts/gpu_profile.sh ${TAG:-r03_a}_fp32 --precision fp32 || exit 1
echo profiles done
