"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py into profiles/<name>.md:
per-kernel totals per forward (the trace holds warmup + timed + event-timing forwards), and the
ENet forward's summed kernel time to compare with bench.py's event-timed `enet_forward`.

usage: python scripts/prof_summary.py gpurun_out/prof_bf16 gpurun_out/bench_bf16.json profiles/r01_bf16.md
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def main(prof_dir, bench_json, out_md):
    prof_dir = Path(prof_dir)
    stats = list(csv.DictReader(open(next(prof_dir.glob("*kernel_stats.csv")))))
    trace = list(csv.DictReader(open(next(prof_dir.glob("*kernel_trace.csv")))))
    bench = None
    if bench_json:
        js = [ln for ln in Path(bench_json).read_text().splitlines() if ln.startswith('{"metric"')]
        bench = json.loads(js[-1]) if js else None
    n_fwd = sum(1 for r in trace if "bev_occgrid_kernel" in r["Kernel_Name"])   # one per pipeline step
    conv = [r for r in trace if "conv_kernel" in r["Kernel_Name"] or "bneck_kernel" in r["Kernel_Name"]]
    per_fwd_launches = len(conv) / max(1, n_fwd)
    conv_ns = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in conv)
    lines = [f"# rocprofv3 kernel summary: {prof_dir.name}", "",
             f"forwards in trace: {n_fwd}; ENet launches (conv_kernel + bneck_kernel) per forward: {per_fwd_launches:.1f}", "",
             "| kernel | calls | avg us | total ms | per forward us | % |", "|---|---|---|---|---|---|"]
    for r in stats:
        name = r["Name"]
        calls = int(r["Calls"])
        lines.append(f"| `{name[:90]}` | {calls} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{int(r['TotalDurationNs']) / 1e6:.3f} | {int(r['TotalDurationNs']) / 1e3 / max(1, n_fwd):.1f} | "
                     f"{float(r['Percentage']):.2f} |")
    fwd_ms = conv_ns / 1e6 / max(1, n_fwd)
    lines += ["", f"**ENet forward, sum of conv_kernel + bneck_kernel durations per forward: {fwd_ms:.4f} ms**"]
    if bench:
        lines += [f"bench.py event-timed enet_forward: {bench['stages_ms']['enet_forward']:.4f} ms "
                  f"(profiled run; the profiler clocks differ slightly, MI355X_MICROARCH.md 'DVFS give-back' (2))",
                  "", "bench line of the same command:", "", "```json", json.dumps(bench), "```"]
    Path(out_md).write_text("\n".join(lines) + "\n")
    print("\n".join(lines[:6] + lines[-8:]))


if __name__ == "__main__":
    main(*sys.argv[1:4])
