"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py into profiles/<name>.md.

Two tables: rocprofv3's own per-kernel-name statistics (run_kernel_stats.csv, verbatim numbers), and
the per-launch average duration per kernel tag (the tags bench.py's `kernels` / `roofline.kernel`
use: "bneck C64", "conv NR4 E3", ...), so the bench line's per-launch microseconds can be checked
against the profiler's. Every launch of bench.py's command has one shape (it times at the shard size).

usage: python scripts/prof_summary.py gpurun_out/<tag>/trace gpurun_out/<tag>/bench.json profiles/<name>.md
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from layer_times import short  # noqa: E402


def main(prof_dir, bench_json, out_md):
    prof_dir = Path(prof_dir)
    stats = list(csv.DictReader(open(next(prof_dir.glob("*kernel_stats.csv")))))
    trace = list(csv.DictReader(open(next(prof_dir.glob("*kernel_trace.csv")))))
    bench = None
    if bench_json and Path(bench_json).exists():
        js = [ln for ln in Path(bench_json).read_text().splitlines() if ln.startswith('{"metric"')]
        bench = json.loads(js[-1]) if js else None
    lines = [f"# rocprofv3 kernel summary: {prof_dir.parent.name}", "",
             "## rocprofv3 --stats (per kernel name)", "",
             "| kernel | calls | avg us | min us | max us | total ms | % |", "|---|---|---|---|---|---|---|"]
    for r in stats:
        lines.append(f"| `{r['Name'][:100]}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                     f"{float(r['MinNs']) / 1e3:.2f} | {float(r['MaxNs']) / 1e3:.2f} | "
                     f"{int(r['TotalDurationNs']) / 1e6:.3f} | {float(r['Percentage']):.2f} |")
    by = defaultdict(list)
    for r in trace:
        by[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    lines += ["", "## per kernel tag (kernel trace; same launches)", "",
              "| tag | launches | avg us | total ms |", "|---|---|---|---|"]
    for tag, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| {tag} | {len(v)} | {sum(v) / len(v):.2f} | {sum(v) / 1e3:.3f} |")
    # the timed loop alone: bench.py fills a one-element int16 tensor right before and right after it
    marks = sorted(int(r["Start_Timestamp"]) for r in trace if "FillFunctor<short>" in r["Kernel_Name"])
    if len(marks) >= 2:
        t0, t1 = marks[0], marks[1]
        win = defaultdict(list)
        for r in trace:
            st = int(r["Start_Timestamp"])
            if t0 < st < t1:
                win[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - st) / 1e3)
        lines += ["", f"## the timed loop only (launches between bench.py's two marker fills, {(t1 - t0) / 1e6:.3f} ms)", "",
                  "| tag | launches | avg us | min us | max us | total ms |", "|---|---|---|---|---|---|"]
        for tag, v in sorted(win.items(), key=lambda kv: -sum(kv[1])):
            lines.append(f"| {tag} | {len(v)} | {sum(v) / len(v):.2f} | {min(v):.2f} | {max(v):.2f} | {sum(v) / 1e3:.3f} |")
        if bench:
            rl = bench.get("roofline", {})
            tag = rl.get("kernel", "").split("[")[-1].split("]")[0]
            if tag in win and rl.get("us_per_launch"):
                avg = sum(win[tag]) / len(win[tag])
                lines += ["", f"bench `roofline.us_per_launch` {rl['us_per_launch']:.2f} us vs the timed loop's "
                              f"{tag} average {avg:.2f} us: ratio {rl['us_per_launch'] / avg:.3f}"]
    if bench:
        rl = bench.get("roofline", {})
        lines += ["", "## bench line of the same command", "",
                  f"roofline.kernel: {rl.get('kernel', '')}", "", "```json", json.dumps(bench), "```"]
    text = "\n".join(lines) + "\n"
    Path(out_md).write_text(text)
    print(text)


if __name__ == "__main__":
    main(*sys.argv[1:4])
