"""HBM traffic per forward from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py.

FETCH_SIZE / WRITE_SIZE are in KiB. On gfx950 FETCH_SIZE reads exactly half the bytes of a wide
coalesced streaming read (MI355X_MICROARCH.md §HBM), so reads are doubled here; the initial
block's raw-frame read (64 x 480x640x3 B = 59 MB) checks the factor: it reports 29.1 MB.
Infinity-Cache hits are counted too (same section), so this is traffic at the L2's memory side.

usage: python scripts/pmc_summary.py gpurun_out/<tag> [out.md]
"""
import csv
import sys
from collections import defaultdict
from pathlib import Path


def per_kernel(path, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return vals


def main(tag_dir, out_md=None):
    d = Path(tag_dir)
    fetch = per_kernel(next((d / "fetch").glob("*counter_collection.csv")), "FETCH_SIZE")
    write = per_kernel(next((d / "write").glob("*counter_collection.csv")), "WRITE_SIZE")
    n_fwd = len(fetch.get("bugseg::bev_occgrid_kernel(bugseg::BevArgs)", [])) or 1
    lines = ["| kernel | dispatches/fwd | read MB/fwd (x2 corrected) | write MB/fwd |", "|---|---|---|---|"]
    tot_r = tot_w = 0.0
    for k in sorted(fetch, key=lambda k: -sum(fetch[k])):
        if "conv_kernel" not in k and "bneck_kernel" not in k:
            continue
        r = 2 * sum(fetch[k]) / n_fwd / 1e6
        w = sum(write.get(k, [0])) / n_fwd / 1e6
        tot_r += r
        tot_w += w
        lines.append(f"| `{k[:80]}` | {len(fetch[k]) / n_fwd:.0f} | {r:.1f} | {w:.1f} |")
    lines += ["", f"ENet forward HBM traffic (memory side of L2): read {tot_r:.1f} MB + write {tot_w:.1f} MB = "
                  f"{tot_r + tot_w:.1f} MB per forward ({n_fwd} forwards in the trace)"]
    text = "\n".join(lines)
    print(text)
    if out_md:
        Path(out_md).write_text(text + "\n")
    return tot_r + tot_w


if __name__ == "__main__":
    main(*sys.argv[1:3])
