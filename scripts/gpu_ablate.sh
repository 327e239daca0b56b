set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ablate
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/ablate -o run --output-format csv -- python3 scripts/bneck_ablate.py 0 1 2 4 7 > gpurun_out/ablate/log.txt 2>&1 || exit 1
echo done
