# SQ counters of the BEV rasteriser (scripts/bev_probe.py under rocprofv3 --pmc)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/bevpmc
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU --kernel-trace -d gpurun_out/bevpmc -o run --output-format csv -- python3 scripts/bev_probe.py 1 > gpurun_out/bevpmc/log.txt 2>&1 || exit 1
echo done
