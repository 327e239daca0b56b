# A/B of runtime env knobs: per setting, per-kernel-tag launch times (batch_probe.py at the bench
# shard size) and one bench line (no CPU baseline, no sub-records).
# usage: bash scripts/gpu_envab.sh VAR 'value1' 'value2' ...   ('' = unset)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
var=$1; shift
mkdir -p gpurun_out/envab
i=0
for v in "$@"; do
  o=gpurun_out/envab/$i; mkdir -p $o; echo "$var=$v" > $o/setting.txt
  if [ -n "$v" ]; then export $var="$v"; else unset $var; fi
  timeout -k 10 120 python scripts/batch_probe.py 32 > $o/probe.txt 2>&1 || exit 1
  timeout -k 10 120 python bench.py --no-cpu-baseline --extras 0 > $o/bench.json 2> $o/bench.err || exit 1
  echo "$var=$v done"; i=$((i+1))
done
