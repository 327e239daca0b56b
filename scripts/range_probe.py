"""Activation ranges of the fp32 mode's split-f16 operands (CPU, oracle numerics; not product code).

For each block: the measured max |x| of its input, and for the fused blocks the rigorous bounds of
the internal tensors the kernels derive from it (t0 <= n1 * amax + c1, t1 <= n2 * B0 + c2, with n
the largest absolute row sum of the BN-folded weights and c the largest |bias|). Shows which tensors
leave the split's comfortable window ([2^-2, 2^15) measured, [2^3, 2^15) bounded) — the cases
bugseg's per-tensor power-of-two scaling handles.

    python scripts/range_probe.py [--undamped] [--H 120 --W 160]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bugcar_image_segmentation_amd import enet_spec, synthetic  # noqa: E402
from oracle import enet_oracle as eo  # noqa: E402


def fold(u):
    s = np.asarray(u.gamma, np.float64) / np.sqrt(np.asarray(u.var, np.float64) + float(u.eps))
    b = (np.asarray(u.b, np.float64) - np.asarray(u.mean, np.float64)) * s + np.asarray(u.beta, np.float64)
    w = np.asarray(u.w, np.float64) * (s[:, None, None, None] if u.kind == 0 else s[None, :, None, None])
    return w, b


def rowsum(u):
    w, b = fold(u)
    if u.kind == 1:
        w = np.swapaxes(w, 0, 1)
    return float(np.abs(w).reshape(w.shape[0], -1).sum(1).max()), float(np.abs(b).max()), float(np.abs(w).max())


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--undamped", action="store_true")
    p.add_argument("--H", type=int, default=120)
    p.add_argument("--W", type=int, default=160)
    a = p.parse_args()
    blocks = enet_spec.build_enet(res_gamma=(0.5, 1.5)) if a.undamped else enet_spec.build_enet()
    bgr = synthetic.road_frames(1, a.H, a.W, seed=3)
    x = (bgr[..., ::-1] / 256.0 - eo.IMAGE_MEAN) / eo.IMAGE_STD
    x = np.moveaxis(x, -1, 1)
    h = torch.as_tensor(x, dtype=torch.float64)
    pools = {}
    for i, b in enumerate(blocks):
        amax = float(h.abs().max())
        line = f"{i:2d} {b.type:8s} {b.name:16s} in amax {amax:10.3e}"
        if b.type in ("regular", "down"):
            n1, c1, w1 = rowsum(b.units[0])
            B0 = n1 * amax + c1
            chain = [B0]
            for u in b.units[1:-1]:
                n, c, _ = rowsum(u)
                chain.append(n * chain[-1] + c)
            # actual internal maxima
            ext, acts = h, []
            for u in b.units:
                ext = eo._unit(ext, u, torch.float64)
                acts.append(float(ext.abs().max()))
            line += "  bounds " + " ".join(f"{v:9.2e}" for v in chain) + "  actual " + " ".join(f"{v:9.2e}" for v in acts[:-1])
            line += f"  max|w1| {w1:.2e}"
        if b.type == "initial":
            u = b.units[0]
            main = F.conv2d(h, eo._t(u.w, torch.float64), eo._t(u.b, torch.float64), stride=2, padding=1)
            k = b.attrs["pool_k"]
            ext = F.max_pool2d(h, k, stride=2, padding=(k - 1) // 2)
            y = torch.cat([main, ext], 1)
            e = b.extra
            y = eo._bn(y, np.concatenate([u.mean, e["pool_mean"]]), np.concatenate([u.var, e["pool_var"]]),
                       np.concatenate([u.gamma, e["pool_gamma"]]), np.concatenate([u.beta, e["pool_beta"]]), u.eps, torch.float64)
            h = eo._prelu(y, np.concatenate([u.slope, e["pool_slope"]]), torch.float64)
        elif b.type == "down":
            main, idx = F.max_pool2d(h, 2, stride=2, return_indices=True)
            pools[i] = (idx, h.shape[2:])
            ext = h
            for u in b.units:
                ext = eo._unit(ext, u, torch.float64)
            main = torch.cat([main, main.new_zeros((1, ext.shape[1] - main.shape[1]) + main.shape[2:])], 1)
            h = eo._prelu(main + ext, b.extra["out_slope"], torch.float64)
        elif b.type == "regular":
            ext = h
            for u in b.units:
                ext = eo._unit(ext, u, torch.float64)
            h = eo._prelu(h + ext, b.extra["out_slope"], torch.float64)
        elif b.type == "up":
            idx, size = pools[b.attrs["pool_ref"]]
            main = eo._unit(h, b.units[0], torch.float64, act=False)
            main = F.max_unpool2d(main, idx, 2, stride=2, output_size=size)
            ext, acts = h, []
            for u in b.units[1:]:
                ext = eo._unit(ext, u, torch.float64)
                acts.append(float(ext.abs().max()))
            n1, c1, _ = rowsum(b.units[1])
            B0 = n1 * amax + c1
            n2, c2, _ = rowsum(b.units[2])
            line += f"  bounds {B0:9.2e} {n2 * B0 + c2:9.2e}  actual " + " ".join(f"{v:9.2e}" for v in acts[:-1])
            h = eo._prelu(main + ext, b.extra["out_slope"], torch.float64)
        elif b.type == "fullconv":
            u = b.units[0]
            h = F.conv_transpose2d(h, eo._t(u.w, torch.float64), eo._t(u.b, torch.float64), stride=2,
                                   padding=(u.pad_h, u.pad_w), output_padding=u.out_pad)
        print(line)
    print(f"logits amax {float(h.abs().max()):.3e}")


if __name__ == "__main__":
    main()
