"""HBM traffic per kernel launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py.

FETCH_SIZE / WRITE_SIZE are in KiB. On gfx950 FETCH_SIZE reads exactly half the bytes of a wide
coalesced streaming read (MI355X_MICROARCH.md §HBM), so reads are doubled here; the initial
block's raw-frame read checks the factor. Infinity-Cache hits are counted too (same section), so this
is traffic at the L2's memory side. Every launch of bench.py's command has one shape (bench.py times
stages and kernels at the timed region's shard size), so per-launch averages per kernel tag are
well defined.

Writes a markdown table and profiles/pmc_traffic.json ({"per_launch_bytes": {tag: bytes}}), which
bench.py reports as roofline.traffic for its dominant kernel.

usage: python scripts/pmc_summary.py gpurun_out/<tag> [out.md] [out.json] [frames per launch]
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from layer_times import short  # noqa: E402


def per_kernel(path, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    return vals


def main(tag_dir, out_md=None, out_json=None, frames=None):
    d = Path(tag_dir)
    fetch = per_kernel(next((d / "fetch").glob("*counter_collection.csv")), "FETCH_SIZE")
    write = per_kernel(next((d / "write").glob("*counter_collection.csv")), "WRITE_SIZE")
    lines = ["| kernel | launches | read MB/launch (FETCH x2) | write MB/launch | total MB/launch |",
             "|---|---|---|---|---|"]
    per = {}
    for k in sorted(fetch, key=lambda k: -sum(fetch[k])):
        if not any(t in k for t in ("conv", "bneck", "down", "init", "bev", "up C", "classes")):   # ("init+down" too)
            continue
        n = len(fetch[k])
        r = 2 * sum(fetch[k]) / n
        w = sum(write.get(k, [0.0])) / max(1, len(write.get(k, [])))
        per[k] = r + w
        lines.append(f"| `{k}` | {n} | {r / 1e6:.1f} | {w / 1e6:.1f} | {(r + w) / 1e6:.1f} |")
    text = "\n".join(lines)
    print(text)
    if out_md:
        Path(out_md).write_text(text + "\n")
    if out_json:
        Path(out_json).write_text(json.dumps({"source": str(d), "correction": "FETCH_SIZE x2 (gfx950)",
                                              "frames_per_launch": int(frames) if frames else None,
                                              "per_launch_bytes": per}, indent=1) + "\n")
    return per


if __name__ == "__main__":
    main(*sys.argv[1:5])
