#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_r3s2_c.sh || exit 1
bash scripts/gpu_r3s2_d.sh || exit 1
