# Stream / batch sweep of the bench (no CPU baseline).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/streams
for cfg in "64 1" "64 2" "64 4" "128 4" "128 8" "96 6"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --batch $1 --streams $2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/streams/b$1_s$2.json 2>/dev/null || exit 1
done
echo done
