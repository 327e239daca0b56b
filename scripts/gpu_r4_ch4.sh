#!/bin/bash
# round 4: down C64 with 4 phase-1 fragments per load round trip (BNECK_CH1_K2=4: no spilled VGPRs;
# the wave's 6 fragments still take two round trips) — A/B kernel tables
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r4ch4}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in def ch4; do
    if [ $v = def ]; then unset BUGSEG_LIB; else export BUGSEG_LIB=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_$v.so; fi
    PREC=fp16 timeout -k 10 120 python scripts/batch_probe.py 32 > gpurun_out/$T/p_${v}_$rep.txt 2>&1 || { echo "probe failed"; tail gpurun_out/$T/p_${v}_$rep.txt; exit 1; }
    echo "== $v $rep $(grep -E 'forward' gpurun_out/$T/p_${v}_$rep.txt) | $(grep -E 'down C64' gpurun_out/$T/p_${v}_$rep.txt)"
  done
done
