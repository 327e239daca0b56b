"""Kernel durations and launch gaps of a single-stream rocprofv3 --kernel-trace run (batch_probe.py):
per kernel tag, the average start->end duration and the average idle gap before it (previous kernel's
end -> this kernel's start, same queue), over the forwards of the run.

usage: python scripts/gap_summary.py gpurun_out/<dir>"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from layer_times import short  # noqa: E402

rows = list(csv.DictReader(open(next(Path(sys.argv[1]).glob("*kernel_trace.csv")))))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur, gap = defaultdict(list), defaultdict(list)
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    t = short(r["Kernel_Name"])
    dur[t].append((e - s) / 1e3)
    if prev_end is not None and 0 <= s - prev_end < 100_000:
        gap[t].append((s - prev_end) / 1e3)
    prev_end = e
print(f"{'tag':28s} {'n':>5s} {'dur us':>8s} {'gap us':>8s}")
tot_d = tot_g = 0.0
for t in sorted(dur, key=lambda t: -sum(dur[t])):
    d = sum(dur[t]) / len(dur[t]); g = sum(gap[t]) / len(gap[t]) if gap[t] else 0.0
    tot_d += sum(dur[t]); tot_g += sum(gap[t])
    print(f"{t:28s} {len(dur[t]):5d} {d:8.2f} {g:8.2f}")
print(f"busy {tot_d / 1e3:.3f} ms, gaps {tot_g / 1e3:.3f} ms ({100 * tot_g / (tot_d + tot_g):.1f}% of the span)")
