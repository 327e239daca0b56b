#!/bin/bash
# both round-3 session-2 A/B passes in one box call
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_r3s2_b.sh || exit 1
bash scripts/gpu_r3s2_a.sh || exit 1
