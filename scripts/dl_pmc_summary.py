"""HBM traffic per DeepLab op from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench_deeplab.py.

Several ops share one kernel template (the 1x1 expansions, projections and ASPP convs are all
dl_conv_kernel), so the counters are attributed per op, not per kernel name: the dispatches of
each full forward (wherever the plan's whole kernel sequence matches) are walked in plan order, conv /
dw / argmax ops take one dispatch each, the pooling op takes the gap / mean / GEMV dispatches that
follow it. Only complete forwards (warmup + timed steps) are used; the per-op timing loop after
them repeats single ops and is skipped.

Same corrections as pmc_summary.py (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are KiB,
FETCH_SIZE is doubled on gfx950. Writes a markdown table (per op tag: launches, read / write MB per
launch) and profiles/dl_pmc_traffic.json ({"per_launch_bytes": {tag: bytes}}), which
bench_deeplab.py reports as roofline.traffic for its dominant op tag.

usage: python scripts/dl_pmc_summary.py gpurun_out/<tag> [out.md] [out.json] [--batch 16] [--backbone xception_65]
(Xception-65: profiles/dl_pmc_traffic_xception.json, which bench_deeplab.py reads for that backbone)
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def dispatches(path, counter):
    """[(dispatch id, kernel name, bytes)] in dispatch order."""
    rows = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        d = int(r["Dispatch_Id"])
        v = float(r["Counter_Value"]) * 1024.0
        if d in rows:
            rows[d][2] += v
        else:
            rows[d] = [d, r["Kernel_Name"], v]
    return [tuple(rows[d]) for d in sorted(rows)]


def op_kinds(B, backbone="mobilenet_v2"):
    from bugcar_image_segmentation_amd import deeplab_spec as D
    if backbone == "xception_65":
        from bugcar_image_segmentation_amd import deeplab_xception as X
        _, ops, _, info = X.lower_xception(X.build_deeplab_xception(), B, True)
    else:
        _, ops, _, info = D.lower(D.build_deeplab(), B, True)
    return [int(o[0]) for o in ops], [t for t, _, _ in info["per_op"]]


def per_op(disp, kinds):
    """Per-op byte totals of every complete forward in `disp`."""
    from bugcar_image_segmentation_amd import deeplab_spec as D
    starts = range(len(disp))          # a forward starts wherever the whole plan's kernel sequence matches
    out = []
    for s in starts:
        j, vals, ok = s, [], True
        for kind in kinds:
            if j >= len(disp):
                ok = False
                break
            name = disp[j][1]
            # (the 1x1 convs run on dl_conv_kernel or one of the two GEMM kernels)
            want = {D.OP_PREP: ("dl_prep",), D.OP_CONV: ("dl_conv", "dl_gemm"), D.OP_DW: ("dl_dw",),
                    D.OP_ARGMAX: ("argmax",), D.OP_RESIZE: ("dl_resize_kernel",)}.get(kind, ())
            if kind == D.OP_POOL:
                v, j0 = 0.0, j
                while j < len(disp) and ("gap" in disp[j][1] or "pool" in disp[j][1]):
                    v += disp[j][2]
                    j += 1
                if j == j0:
                    ok = False
                    break
                vals.append(v)
                continue
            if not any(w in name for w in want):
                ok = False
                break
            vals.append(disp[j][2])
            j += 1
        if ok:
            out.append(vals)
    return out


def sq_table(d, B=16):
    """Per-op SQ counter values (wave-cycle breakdown) of a --pmc pass over SQ counters in `d`."""
    path = next(Path(d).glob("*counter_collection.csv"))
    names = sorted({r["Counter_Name"] for r in csv.DictReader(open(path))})
    kinds, tags = op_kinds(B)
    cols = {}
    for c in names:
        f = per_op([(i, k, v / 1024.0) for i, k, v in dispatches(path, c)], kinds)
        cols[c] = [sum(x[i] for x in f) / max(1, len(f)) for i in range(len(kinds))]
    lines = ["| op | tag | " + " | ".join(names) + " |", "|---" * (len(names) + 2) + "|"]
    for i, t in enumerate(tags):
        lines.append(f"| {i} | {t} | " + " | ".join(f"{cols[c][i]:.4g}" for c in names) + " |")
    return "\n".join(lines)


def main(argv):
    if argv and argv[0] == "--sq":
        print(sq_table(argv[1]))
        return None
    B, backbone = 16, "mobilenet_v2"
    if "--batch" in argv:
        i = argv.index("--batch")
        B = int(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    if "--backbone" in argv:
        i = argv.index("--backbone")
        backbone = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    d = Path(argv[0])
    out_md = argv[1] if len(argv) > 1 else None
    out_json = argv[2] if len(argv) > 2 else None
    kinds, tags = op_kinds(B, backbone)
    rd = per_op(dispatches(next((d / "fetch").glob("*counter_collection.csv")), "FETCH_SIZE"), kinds)
    wr = per_op(dispatches(next((d / "write").glob("*counter_collection.csv")), "WRITE_SIZE"), kinds)
    if not rd or not wr:
        raise SystemExit("no complete forward found in the counter CSVs")
    n_ops = len(kinds)
    r_op = [2.0 * sum(f[i] for f in rd) / len(rd) for i in range(n_ops)]
    w_op = [sum(f[i] for f in wr) / len(wr) for i in range(n_ops)]
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    for t, r, w in zip(tags, r_op, w_op):
        agg[t][0] += 1
        agg[t][1] += r
        agg[t][2] += w
    lines = [f"{len(rd)} / {len(wr)} complete forwards (FETCH / WRITE passes), B = {B}", "",
             "| op tag | launches per forward | read MB/launch (FETCH x2) | write MB/launch | total MB/launch |",
             "|---|---|---|---|---|"]
    per = {}
    for t, (n, r, w) in sorted(agg.items(), key=lambda kv: -(kv[1][1] + kv[1][2])):
        per[t] = (r + w) / n
        lines.append(f"| {t} | {n} | {r / n / 1e6:.1f} | {w / n / 1e6:.1f} | {(r + w) / n / 1e6:.1f} |")
    lines += ["", f"whole forward: {sum(r_op) / 1e6:.1f} MB read + {sum(w_op) / 1e6:.1f} MB written "
                  f"({(sum(r_op) + sum(w_op)) / B / 1e6:.1f} MB per frame)"]
    text = "\n".join(lines)
    print(text)
    if out_md:
        Path(out_md).write_text(text + "\n")
    if out_json:
        Path(out_json).write_text(json.dumps({"source": str(d), "correction": "FETCH_SIZE x2 (gfx950)", "batch": B, "backbone": backbone,
                                              "per_launch_bytes": per,
                                              "per_op_bytes": [r + w for r, w in zip(r_op, w_op)]}, indent=1) + "\n")
    return per


if __name__ == "__main__":
    main(sys.argv[1:])
