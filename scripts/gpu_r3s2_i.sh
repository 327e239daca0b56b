#!/bin/bash
# round 3 (session 2): BEV right after a forward (cold) vs back to back, compact table vs uint4 slots;
# up-kernel parity + per-kernel probes (fp16 / fp32)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3s2i
export TMPDIR=/tmp
for lib in ctab noctab ctab2; do
  L=""
  [ $lib = noctab ] && L=$PWD/bugcar_image_segmentation_amd/_variants/libbugseg_noctab.so
  echo "== $lib"
  env ${L:+BUGSEG_LIB=$L} timeout -k 10 150 python scripts/bev_cold_probe.py 10 > gpurun_out/r3s2i/bev_$lib.txt 2>&1 || { echo "probe $lib failed"; tail gpurun_out/r3s2i/bev_$lib.txt; exit 1; }
  grep -E "after|back" gpurun_out/r3s2i/bev_$lib.txt
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "up_block or fused_bottlenecks_equal or fp32" -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3s2i/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3s2i/tests.log; exit 1; }
tail -1 gpurun_out/r3s2i/tests.log
for p in fp16 fp32; do
  PREC=$p timeout -k 10 150 python scripts/batch_probe.py 32 > gpurun_out/r3s2i/probe_$p.txt 2>&1 || { echo "probe $p failed"; exit 1; }
  echo "== $p"; grep -E "forward|up C" gpurun_out/r3s2i/probe_$p.txt
done
