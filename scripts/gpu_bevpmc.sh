# Counters of the BEV rasteriser (scripts/bev_probe.py under rocprofv3 --pmc), one pass per counter
# group (gfx950 block limits: <= 8 SQ, <= 4 TCC slots per pass)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/bevpmc; mkdir -p $o
timeout -k 10 60 python3 scripts/bev_probe.py > $o/probe.txt 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU --kernel-trace -d $o/sq -o run --output-format csv -- python3 scripts/bev_probe.py 3 > $o/sq.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $o/tcc -o run --output-format csv -- python3 scripts/bev_probe.py 3 > $o/tcc.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $o/fetch -o run --output-format csv -- python3 scripts/bev_probe.py 3 > $o/fetch.log 2>&1 || exit 1
echo done
