#!/bin/bash
# one-rank RCCL bench (torch.distributed.run) A/B of bench arguments: bash scripts/gpu_tr1.sh TAG "ARGSETS(;-separated)"
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-tr1}; SETS=${2:-""}
mkdir -p gpurun_out/$T
IFS=';' read -ra A <<< "$SETS"
for rep in 1 2; do
  i=0
  for s in "${A[@]}"; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29600 + i)) bench.py --gpus 1 --steps 20 --warmup 5 --extras 0 --no-cpu-baseline $s > gpurun_out/$T/s$i.json 2> gpurun_out/$T/s$i.err || { echo "set $i failed"; tail -5 gpurun_out/$T/s$i.err; exit 1; }
    python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], r['value'], r['ms_per_step'])" gpurun_out/$T/s$i.json "$s"
    i=$((i+1))
  done
done
