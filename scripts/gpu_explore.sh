# Exploration: bneck phase clocks, per-kernel times under alternative C64 tiling, and end-to-end
# step time over stream counts / graph replay (one bench line each, no CPU baseline, no sub-records).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/explore; mkdir -p $o
timeout -k 10 120 python scripts/stamp_probe.py 32 > $o/stamps.txt 2>&1 || exit 1
BUGSEG_BNECK_VARIANT_C64=1 timeout -k 10 120 python scripts/batch_probe.py 32 > $o/probe_c64v1.txt 2>&1 || exit 1
for s in 1 2 4; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --extras 0 --streams $s > $o/bench_s$s.json 2> $o/bench_s$s.err || exit 1
done
timeout -k 10 120 python bench.py --no-cpu-baseline --extras 0 --streams 2 --batch 128 > $o/bench_b128.json 2> $o/bench_b128.err || exit 1
timeout -k 10 120 python bench.py --no-cpu-baseline --extras 0 --streams 2 --graph 1 > $o/bench_g.json 2> $o/bench_g.err || exit 1
echo done
