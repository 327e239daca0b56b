# Performance-only loop (no parity tests): per-layer kernel trace of 9 single-stream B=64 forwards,
# then SQ counters (two passes) on the same script. Read with scripts/layer_times.py and
# scripts/sq_layers.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/layers gpurun_out/sq gpurun_out/sq2
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/layers -o run --output-format csv -- python3 scripts/bneck_ablate.py 0 > gpurun_out/layers/log.txt 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS --kernel-trace -d gpurun_out/sq -o run --output-format csv -- python3 scripts/bneck_ablate.py 0 > gpurun_out/sq/log.txt 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL --kernel-trace -d gpurun_out/sq2 -o run --output-format csv -- python3 scripts/bneck_ablate.py 0 > gpurun_out/sq/log2.txt 2>&1 || exit 1
echo done
