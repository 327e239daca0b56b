# Fused-bottleneck ablation: per-kernel-tag launch times with BUGSEG_BNECK_ABLATE = 0 (none), 1 (no x
# loads), 2 (no middle-conv MFMAs), 4 (no output stores), 7 (all three) at B=32.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ablate
for f in 0 1 2 4 7; do
  BUGSEG_BNECK_ABLATE=$f timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/ablate/a$f.txt 2>&1 || exit 1
done
echo done
