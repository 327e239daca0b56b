"""Per-layer kernel durations from a rocprofv3 kernel trace of repeated single-stream forwards.

The trace is cut into forwards at each launch of the initial-block kernel (EPI 7 / EPI 4); every
forward of one variant has the same launch sequence, so durations are averaged per position.
Variants (e.g. the ablation script's contexts) are split every `--per-variant` forwards.

usage: python scripts/layer_times.py gpurun_out/ablate/run_kernel_trace.csv [--per-variant 9] [--labels 0,1,2]
"""
import argparse
import csv
import re
from collections import defaultdict


# tile shape of each fused-bottleneck variant (bneck_kernels.hip BShape)
BNECK_SHAPES = {(128, 0): "16x16", (128, 1): "20x16", (128, 2): "4x80", (128, 3): "4x64", (128, 4): "8x16", (64, 0): "16x16", (64, 1): "20x16", (64, 2): "8x16",
                (16, 0): "16x16"}


def short(name):
    # fp32 bneck forms come as two kernels (bneck_kernels.hip SCL): the range-scaled one is tagged apart
    # (launched beside every unscaled one, it returns at once unless an exponent is non-zero)
    scl = bool(re.search(r"bneck_kernelI(DF16b|DF16_|f)Li\d+ELb\dELi\d+ELb\dELi\d+ELb1E", name) or
               re.search(r"bneck_kernel<[^>]*, true>", name))
    sfx = " (scaled)" if scl else ""
    m = re.search(r"bneck_kernelI(DF16b|DF16_|f)Li(\d+)ELb(\d)ELi(\d+)ELb\dELi([1-9]\d*)E", name)
    if m:   # the downsampling form (non-zero input-channel template argument)
        return f"down C{m.group(2)} {BNECK_SHAPES.get((int(m.group(2)), int(m.group(4))), '?')}{sfx}"
    # (the f32 kernels appear demangled: "void bugseg::bneck_kernel<float, 64, false, 2, false, 0, false>(...)")
    m = re.search(r"bneck_kernel<(?:__bf16|_Float16|float), (\d+), (?:false|true), (\d+), (?:false|true), ([1-9]\d*)[,>]", name)
    if m:
        return f"down C{m.group(1)} {BNECK_SHAPES.get((int(m.group(1)), int(m.group(2))), '?')}{sfx}"
    m = re.search(r"bneck_kernelI(DF16b|DF16_|f)Li(\d+)ELb(\d)ELi(\d+)E", name)
    if not m:
        m = re.search(r"bneck_kernel<(__bf16|_Float16|float), (\d+), (false|true), (\d+)", name)
    if m:
        asym = m.group(3) in ("1", "true")
        return f"bneck C{m.group(2)}{' asym' if asym else ''} {BNECK_SHAPES.get((int(m.group(2)), int(m.group(4))), '?')}{sfx}"
    if "bneck_cls_kernel" in name:
        return "bneck C16+classes 16x16"
    if "bneck2_f32_kernel" in name:
        return "bneck2 C128 16x16"
    m = re.search(r"conv_kernelI(DF16b|DF16_|f)Li(\d+)ELi(\d+)E", name)
    if m:
        return f"conv NR{m.group(2)} E{m.group(3)}"
    m = re.search(r"conv_kernel<.*, (\d+)>", name)
    if m:
        return f"conv NR1 E{m.group(1)}"
    m = re.search(r"up_kernelI(DF16b|DF16_|f)Li(\d+)ELi(\d+)ELi(\d+)E", name)
    if m:
        return f"up C{m.group(4)}"
    m = re.search(r"up_kernel<(?:__bf16|_Float16|float), (\d+), (\d+), (\d+)>", name)
    if m:
        return f"up C{m.group(3)}"
    if "cls_kernel" in name:
        return "classes"
    if "init_kernel" in name:
        return "init"
    return name.split("(")[0][-40:]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--per-variant", type=int, default=0)
    p.add_argument("--labels", default="")
    a = p.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if any(k in r["Kernel_Name"] for k in ("conv_kernel", "bneck_kernel", "init_kernel", "up_kernel", "cls_kernel"))]
    fwds, cur = [], None
    for r in rows:
        s = short(r["Kernel_Name"])
        if s.endswith("E7") or s.endswith("E4") or s.startswith("init"):
            cur = []
            fwds.append(cur)
        if cur is not None:
            cur.append((s, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, int(r["Grid_Size_X"])))
    per = a.per_variant or len(fwds)
    variants = [fwds[i:i + per] for i in range(0, len(fwds), per)]
    labels = a.labels.split(",") if a.labels else [str(i) for i in range(len(variants))]
    tables = []
    for v in variants:
        n = len(v[0])
        avg = defaultdict(float)
        for f in v:
            for i, (s, d, g) in enumerate(f[:n]):
                avg[i] += d / len(v)
        tables.append((v[0], avg))
    base = tables[0][0]
    print("pos  kernel             grid  " + "  ".join(f"{lab:>8}" for lab in labels[:len(tables)]))
    for i, (s, _, g) in enumerate(base):
        print(f"{i:3d}  {s:16s} {g // 64:6d}  " + "  ".join(f"{t[1][i]:8.1f}" for t in tables))
    print("sum                       " + "  ".join(f"{sum(t[1].values()):8.1f}" for t in tables))


if __name__ == "__main__":
    main()
