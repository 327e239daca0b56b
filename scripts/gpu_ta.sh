#!/bin/bash
# TA (texture addresser: vector-memory address processing) busy and SQ instruction counts per kernel of
# the bench-shard forward (batch_probe.py), one rocprofv3 pass; summary per kernel name
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/ta; mkdir -p $o
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --kernel-trace -d $o/p -o run --output-format csv -- python3 scripts/batch_probe.py 32 > $o/p.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
fs = glob.glob("gpurun_out/ta/p/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for r in csv.DictReader(open(fs[0])):
    k = r["Kernel_Name"].split("(")[0][-40:]
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if r["Counter_Name"] == "SQ_WAVES":
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, d in agg.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    w = max(m.get("SQ_WAVES", 1), 1)
    us = sum(dur[k]) / max(len(dur[k]), 1)
    print(f"{k:42s} {us:7.1f} us  TA_BUSY_avr {m.get('TA_BUSY_avr', 0):9.0f}  per wave: vmem_rd {m.get('SQ_INSTS_VMEM_RD', 0)/w:6.1f} "
          f"valu {m.get('SQ_INSTS_VALU', 0)/w:7.1f} salu {m.get('SQ_INSTS_SALU', 0)/w:7.1f} lds {m.get('SQ_INSTS_LDS', 0)/w:6.1f} "
          f"wait_inst {m.get('SQ_WAIT_INST_ANY', 0)/max(m.get('SQ_WAVE_CYCLES', 1), 1):.2f}")
PY
