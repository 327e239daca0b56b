set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
NOPMC=1 bash scripts/gpu_ab.sh k64off k64on k64off k64on || exit 1
bash scripts/gpu_profile.sh r02_c
