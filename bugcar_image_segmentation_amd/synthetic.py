"""Synthetic inputs of the benchmark / tests: frames and a BEV calibration.

There is no dataset and no calibration JSON in the reference (`.gitignore:47` ignores *.json), so
the workload is synthetic with fixed seeds:
  * frames: uniform u8 (default_rng(0)) or a structured "road scene" (horizontal bands with
    gradients and noise) so the class maps are not degenerate;
  * calibration: input image size [480, 640] (rows, cols — the reference's assert convention,
    bev.py:169), output size [1000, 1000], cm_per_px 1.0, homography from a 4-point solve mapping a
    road trapezoid of the camera image onto the BEV image.
"""
from __future__ import annotations

import numpy as np

from .bev import bev_transform_tools, get_perspective_transform


def uniform_frames(B: int, H: int = 480, W: int = 640, seed: int = 0) -> np.ndarray:
    return np.random.default_rng(seed).integers(0, 256, size=(B, H, W, 3), dtype=np.uint8)


def road_frames(B: int, H: int = 480, W: int = 640, seed: int = 0) -> np.ndarray:
    rng = np.random.default_rng(seed)
    y = np.linspace(0.0, 1.0, H)[:, None, None]
    x = np.linspace(0.0, 1.0, W)[None, :, None]
    frames = np.empty((B, H, W, 3), np.uint8)
    for b in range(B):
        horizon = 0.35 + 0.1 * rng.random()
        sky = np.array([200, 160, 120]) * (1 - y) + 40 * x
        road = np.array([90, 90, 95]) + 60 * (y - horizon) + 30 * np.sin(12 * x + b)
        img = np.where(y < horizon, sky, road) + rng.normal(0, 12, size=(H, W, 3))
        frames[b] = np.clip(img, 0, 255).astype(np.uint8)
    return frames


def synthetic_bev(in_rows: int = 480, in_cols: int = 640, out_w: int = 1000, out_h: int = 1000,
                  cm_per_px: float = 1.0) -> bev_transform_tools:
    bev = bev_transform_tools([in_rows, in_cols], [out_w, out_h], (0.0, 100.0), 50.0, cm_per_px, 0.0, False)
    src = np.array([[0.44 * in_cols, 0.50 * in_rows], [0.56 * in_cols, 0.50 * in_rows],
                    [0.95 * in_cols, 0.98 * in_rows], [0.05 * in_cols, 0.98 * in_rows]])
    dst = np.array([[0.35 * out_w, 0.05 * out_h], [0.65 * out_w, 0.05 * out_h],
                    [0.58 * out_w, 0.99 * out_h], [0.42 * out_w, 0.99 * out_h]])
    bev._bev_matrix = get_perspective_transform(src, dst)
    return bev


# grid of the synthetic workload: 10 m x 10 m at 0.05 m (cell_px = 5 -> 200 x 200 cells)
GRID_W_M, GRID_H_M, CELL_M = 10.0, 10.0, 0.05
