"""Per-kernel SQ counter table from rocprofv3 --pmc passes (scripts/gpu_r4_sq.sh): every dispatch of
a kernel name averaged; per-wave instruction counts, wait shares of wave cycles, LDS conflict share.

usage: python scripts/sq_summary.py dir1 [dir2 ...]  (each holds run_counter_collection.csv)"""
import csv
import glob
import re
import sys
from collections import defaultdict


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = n.replace("bugseg::", "").replace("__bf16", "bf16").replace("_Float16", "f16")
    return n[:70]


per = defaultdict(lambda: defaultdict(list))
dur = defaultdict(dict)
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            did = (f, r["Dispatch_Id"])
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if "End_Timestamp" in r and r["End_Timestamp"]:
                dur[k][did] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
rows = []
for k, c in per.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    w = m.get("SQ_WAVES", 0) or 1
    us = sum(dur[k].values()) / max(1, len(dur[k]))
    cyc = m.get("SQ_WAVE_CYCLES", 0) or 1
    rows.append((us, k, m, w, cyc))
rows.sort(key=lambda r: -r[0])
print(f"{'kernel':70s} {'us':>7s} {'waves':>7s} {'VALU/w':>7s} {'MFMA/w':>7s} {'LDS/w':>6s} {'VMRD/w':>6s} {'VMWR/w':>6s} "
      f"{'wait%':>5s} {'winst%':>6s} {'act%':>5s} {'ldsbc%':>6s}")
for us, k, m, w, cyc in rows:
    g = lambda n: m.get(n, float("nan"))  # noqa: E731
    print(f"{k:70s} {us:7.1f} {w:7.0f} {g('SQ_INSTS_VALU') / w:7.0f} {g('SQ_INSTS_MFMA') / w:7.0f} {g('SQ_INSTS_LDS') / w:6.0f} "
          f"{g('SQ_INSTS_VMEM_RD') / w:6.0f} {g('SQ_INSTS_VMEM_WR') / w:6.0f} {100 * g('SQ_WAIT_ANY') / cyc:5.1f} "
          f"{100 * g('SQ_WAIT_INST_ANY') / cyc:6.1f} {100 * g('SQ_ACTIVE_INST_ANY') / cyc:5.1f} "
          f"{100 * g('SQ_LDS_BANK_CONFLICT') / max(1, g('SQ_LDS_IDX_ACTIVE')):6.1f}")
