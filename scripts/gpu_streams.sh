# Stream / batch / stream-priority sweep of the bench (no CPU baseline, no sub-records).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/streams
for cfg in "64 2 0" "64 2 -1" "64 1 0" "64 3 0" "64 4 0" "64 4 -1" "128 4 0" "128 2 0"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --batch $1 --streams $2 --stream-priority $3 --steps 20 --warmup 5 --no-cpu-baseline --extras 0 > gpurun_out/streams/b$1_s$2_p$3.json 2>/dev/null || exit 1
done
echo done
