"""Print one line per A/B variant (scripts/gpu_ab.sh output): bench value, ms/step, forward ms and
the per-launch microseconds of the kernel tags given (default: the dominant ENet tags).
usage: python scripts/ab_summary.py NAME ... [--tags 'bneck C64 16x16,bneck C128 20x16']"""
import json
import sys
from pathlib import Path

args = sys.argv[1:]
tags = ["bneck C64 16x16", "bneck C128 20x16", "bneck C128 4x80", "bneck C128 asym 20x16"]
if "--tags" in args:
    i = args.index("--tags")
    tags = args[i + 1].split(",")
    args = args[:i] + args[i + 2:]
for n in args:
    p = Path("gpurun_out/ab") / n / "bench.json"
    if not p.exists():
        print(n, "missing")
        continue
    d = json.loads([ln for ln in p.read_text().splitlines() if ln.startswith('{"metric"')][-1])
    ks = d["kernels"]
    print(f"{n:12s} {d['value']:9.1f} f/s  {d['ms_per_step']:.4f} ms/step  fwd {d['stages_ms']['enet_forward']:.4f} ms  " +
          "  ".join(f"[{t}] {ks[t]['us_per_launch']:.2f}" for t in tags if t in ks))
