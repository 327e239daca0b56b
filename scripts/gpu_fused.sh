# Fused-bottleneck iteration: bit-exactness of every tile variant vs the unfused plan, then the
# batch-size probe (per-kernel-tag launch times) with the runtime's variant choice and each variant forced.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k fused --timeout 120 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1 || exit 1
timeout -k 10 200 python scripts/batch_probe.py ${PROBE_B:-32} > gpurun_out/probe.txt 2>&1 || exit 1
BUGSEG_BNECK_VARIANT=0 timeout -k 10 200 python scripts/batch_probe.py ${PROBE_B:-32} > gpurun_out/probe_v0.txt 2>&1 || exit 1
BUGSEG_BNECK_VARIANT=1 timeout -k 10 200 python scripts/batch_probe.py ${PROBE_B:-32} > gpurun_out/probe_v1.txt 2>&1 || exit 1
echo done
