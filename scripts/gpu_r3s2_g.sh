#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_r3s2_full.sh || exit 1
SKIP_TESTS=1 bash scripts/gpu_r3s2_f.sh || exit 1
