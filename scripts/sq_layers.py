"""Per-layer SQ counter table from rocprofv3 --pmc runs of scripts/bneck_ablate.py (one variant).

Dispatches are grouped into forwards at each initial-block launch and averaged per position, like
layer_times.py. Prints per-wave instruction counts and wait fractions per layer.

usage: python scripts/sq_layers.py gpurun_out/sq gpurun_out/sq2
"""
import csv
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from layer_times import short  # noqa: E402


def load(d):
    rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
    disp = defaultdict(dict)
    meta = {}
    for r in rows:
        k = int(r["Dispatch_Id"])
        disp[k][r["Counter_Name"]] = float(r["Counter_Value"])
        meta[k] = (r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return disp, meta


def forwards(disp, meta):
    fw, cur = [], None
    for k in sorted(disp):
        name = short(meta[k][0])
        if not any(t in meta[k][0] for t in ("conv_kernel", "bneck_kernel", "init_kernel", "up_kernel", "cls_kernel")):
            continue
        if name.startswith("init") or name.endswith("E7") or name.endswith("E4"):
            cur = []
            fw.append(cur)
        if cur is not None:
            cur.append((name, meta[k][1], disp[k]))
    return fw


def avg(fw):
    n = len(fw[0])
    out = []
    for i in range(n):
        c = defaultdict(float)
        for f in fw:
            for key, v in f[i][2].items():
                c[key] += v / len(fw)
            c["_us"] += f[i][1] / len(fw)
        out.append((fw[0][i][0], c))
    return out


def main(*dirs):
    tabs = [avg(forwards(*load(d))) for d in dirs]
    merged = []
    for i in range(len(tabs[0])):
        c = {}
        for t in tabs:
            c.update(t[i][1])
        merged.append((tabs[0][i][0], c))
    keys = ["SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU"]
    print("pos kernel            us   waves  " + " ".join(f"{k[9:]:>8}" for k in keys) +
          "  wait_any wait_inst active lds_conf/lds")
    for i, (name, c) in enumerate(merged):
        w = c.get("SQ_WAVES", 1) or 1
        wc = c.get("SQ_WAVE_CYCLES", 1) or 1
        print(f"{i:3d} {name:16s} {c['_us']:6.1f} {w:7.0f}  " +
              " ".join(f"{c.get(k, 0) / w:8.1f}" for k in keys) +
              f"  {c.get('SQ_WAIT_ANY', 0) / wc:8.2f} {c.get('SQ_WAIT_INST_ANY', 0) / wc:9.2f} "
              f"{c.get('SQ_ACTIVE_INST_ANY', 0) / wc:6.2f} "
              f"{c.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, c.get('SQ_LDS_IDX_ACTIVE', 0) or 1):6.2f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
