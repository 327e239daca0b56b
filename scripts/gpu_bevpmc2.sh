# SQ counters of the two BEV rasteriser forms (LDS-staged: BUGSEG_BEV_FG=4; gather: BUGSEG_BEV_FG=0)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/bevpmc2; mkdir -p $o
for fg in 4 0; do
  BUGSEG_BEV_FG=$fg timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d $o/sq$fg -o run --output-format csv -- python3 scripts/bev_probe.py 3 > $o/sq$fg.log 2>&1 || exit 1
done
echo done
