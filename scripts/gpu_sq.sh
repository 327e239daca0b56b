#!/bin/bash
# SQ counter passes over a few forwards (scripts/bneck_ablate.py) for scripts/sq_layers.py
#   bash scripts/gpu_sq.sh TAG PRECISION B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-sq}; export BUGSEG_PREC=${2:-fp32}; export BUGSEG_B=${3:-64}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU --output-format csv -d $O/sq1 -o run -- python3 $GRAFT_REPO_ROOT/scripts/bneck_ablate.py 0 > $O/sq1.log 2>&1 || { echo "sq1 failed"; tail -5 $O/sq1.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $O/sq2 -o run -- python3 $GRAFT_REPO_ROOT/scripts/bneck_ablate.py 0 > $O/sq2.log 2>&1 || { echo "sq2 failed"; tail -5 $O/sq2.log; exit 1; }
echo "sq ok"
