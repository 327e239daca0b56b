#!/bin/bash
# round 3 session 2 profiles: fp16 headline + fp32 parity mode (stats + FETCH/WRITE passes), Xception-65
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_profile.sh ${TAG:-r03_b}_fp16 || exit 1
bash scripts/gpu_profile.sh ${TAG:-r03_b}_fp32 --precision fp32 || exit 1
bash scripts/gpu_xc_profile.sh ${TAG:-r03_b}_xc || exit 1
echo profiles done
