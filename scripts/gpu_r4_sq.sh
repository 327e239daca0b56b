#!/bin/bash
# round 4: SQ counter passes over one precision's forward + BEV (scripts/probe_forward.py), then the
# per-kernel table. usage: gpu_r4_sq.sh <tag> <prec>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4sq}; P=${2:-fp16}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/$T/p1 -o run --output-format csv -- python3 scripts/probe_forward.py $P 32 3 > gpurun_out/$T/p1.log 2>&1 || { echo "pass 1 failed"; tail gpurun_out/$T/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --kernel-trace -d gpurun_out/$T/p2 -o run --output-format csv -- python3 scripts/probe_forward.py $P 32 3 > gpurun_out/$T/p2.log 2>&1 || { echo "pass 2 failed"; tail gpurun_out/$T/p2.log; exit 1; }
python3 scripts/sq_summary.py gpurun_out/$T/p1 gpurun_out/$T/p2 | tee gpurun_out/$T/sq_table.txt
