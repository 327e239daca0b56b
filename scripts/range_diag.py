"""GPU diagnostic of the fp32 range scaling (prints, asserts nothing): max |dlogit| / max |logit| of the
engine against the fp64 oracle over inputs / weights that put different tensors outside the f16
window, fused and unfused plans.   python scripts/range_diag.py [H W]"""
import os
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bugcar_image_segmentation_amd import enet_spec, synthetic  # noqa: E402
from bugcar_image_segmentation_amd.models import ENET  # noqa: E402
from oracle import enet_oracle as eo  # noqa: E402


def frames(H, W, seed=3):
    bgr = synthetic.road_frames(1, H, W, seed=seed)
    return np.ascontiguousarray(np.moveaxis((bgr[..., ::-1] / 256.0 - eo.IMAGE_MEAN) / eo.IMAGE_STD, -1, 1)).astype(np.float32)


def run(name, bl, x):
    m = ENET(weights=bl, precision="fp32")
    got = m.logits(x)
    ref = eo.forward(bl, x.astype(np.float64), torch.float64)
    r32 = eo.forward(bl, x)
    amax = float(np.abs(ref).max())
    e = float(np.abs(got - ref).max())
    e32 = float(np.abs(r32 - ref).max())
    err = np.abs(got - ref).max(1) / max(amax, 1e-30)          # per pixel, relative to the max logit
    big = err > 5e-6
    ys, xs = np.nonzero(big.any(0))
    box = f"rows {ys.min()}-{ys.max()} cols {xs.min()}-{xs.max()}" if ys.size else "-"
    print(f"{name:40s} max|logit| {amax:10.3e}  engine {e / max(amax, 1e-30):9.2e}  f32-oracle {e32 / max(amax, 1e-30):9.2e}  "
          f"p50 {np.percentile(err, 50):8.1e} p99 {np.percentile(err, 99):8.1e} p99.9 {np.percentile(err, 99.9):8.1e} "
          f">5e-6: {int(big.sum())} px ({box}) finite {bool(np.isfinite(got).all())}", flush=True)


def main():
    H, W = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (120, 160)
    if os.environ.get("DIAG_BIG"):
        u = enet_spec.build_enet(res_gamma=(0.5, 1.5))
        run("undamped 480x640", u, frames(480, 640, seed=5))
        run("undamped 480x640 seed 6", u, frames(480, 640, seed=6))
        run("damped 480x640", enet_spec.build_enet(), frames(480, 640, seed=5))
        return
    fused = os.environ.get("BUGSEG_NO_FUSE", "0") in ("", "0")
    tag = "fused" if fused else "unfused"
    x = frames(H, W)
    d = enet_spec.build_enet()
    u = enet_spec.build_enet(res_gamma=(0.5, 1.5))
    run(f"{tag} damped", d, x)
    run(f"{tag} damped x*1e3", d, x * np.float32(1e3))
    run(f"{tag} damped x*1e5", d, x * np.float32(1e5))
    run(f"{tag} damped x*1e-4", d, x * np.float32(1e-4))
    run(f"{tag} undamped", u, x)
    for name, unit, f in (("regular1_1", 0, 1e3), ("regular1_1", 1, 1e3), ("regular1_1", 2, 1e3),
                          ("regular2_1", 0, 1e3), ("asymmetric2_3", 1, 1e3), ("asymmetric2_3", 2, 1e3),
                          ("upsample4_0", 1, 1e3), ("upsample4_0", 2, 1e3), ("downsample1_0", 0, 1e3),
                          ("transposed_conv", 0, 1e3)):
        bl = enet_spec.build_enet()
        for b in bl:
            if b.name == name:
                b.units[unit].w = (b.units[unit].w.astype(np.float64) * f).astype(np.float32)
        run(f"{tag} {name}[{unit}] w*{f:g}", bl, x)
    if fused:
        env = dict(os.environ, BUGSEG_NO_FUSE="1")
        sys.exit(subprocess.call([sys.executable, __file__, str(H), str(W)], env=env))


if __name__ == "__main__":
    main()
