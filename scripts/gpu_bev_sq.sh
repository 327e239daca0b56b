#!/bin/bash
# SQ / TA counters of the BEV rasteriser's default (band-staged) form at the bench shard
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/bevsq; mkdir -p $o
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --kernel-trace -d $o/p1 -o run --output-format csv -- python3 scripts/bev_probe.py 3 > $o/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM --kernel-trace -d $o/p2 -o run --output-format csv -- python3 scripts/bev_probe.py 3 > $o/p2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr --kernel-trace -d $o/p3 -o run --output-format csv -- python3 scripts/bev_probe.py 3 > $o/p3.log 2>&1 || echo "p3 failed"
python3 - <<'PY'
import csv, glob, collections
for p in ("p1", "p2", "p3"):
    fs = glob.glob(f"gpurun_out/bevsq/{p}/**/*counter_collection.csv", recursive=True)
    if not fs:
        print(p, "no csv"); continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"][:40]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        if "bev" in k or "polar" in k or "laser" in k:
            print(p, k, {c: round(sum(v) / len(v), 1) for c, v in d.items()})
PY
