"""ORACLE — TEST INFRASTRUCTURE ONLY. ctypes binding of the C restatement (ocv_ref.c) and the
full-path CPU oracle (preprocess -> ENet fp32/fp64 -> argmax/remap -> occupancy grid) that tests,
__graft_entry__.smoke() and bench.py's cpu_baseline use as the checker. Parity status: unpinned
against TF/OpenCV (see ocv_ref.c / enet_oracle.py headers)."""
from __future__ import annotations

import ctypes
from pathlib import Path

import numpy as np

from .build import build_oracle

_lib = None


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(str(build_oracle()))
        u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
        i8p = np.ctypeslib.ndpointer(np.int8, flags="C_CONTIGUOUS")
        dp = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
        i = ctypes.c_int
        L.ocv_invert3x3.argtypes = [dp, dp]
        L.ocv_warp_perspective_u8.argtypes = [u8p, i, i, u8p, i, i, dp]
        L.ocv_resize_nearest_u8.argtypes = [u8p, i, i, i, u8p, i, i]
        L.ocv_morph_open3x3_u8.argtypes = [u8p, i, i, u8p]
        L.ocv_resize_linear_u8.argtypes = [u8p, i, i, i, u8p, i, i]
        L.bev_occgrid_ref.argtypes = [u8p, i, i, dp, i, i, i, i, i, i, i, i, i8p]
        L.bev_occgrid_binary_ref.argtypes = [u8p, i, i, dp, i, i, i, i, i, i, i, i, i8p]
        L.bev_occgrid_laserscan_ref.argtypes = [u8p, i, i, dp, i, i, i, i, i, i, i, i, i8p]
        L.bev_occgrid_binary_laserscan_ref.argtypes = [u8p, i, i, dp, i, i, i, i, i, i, i, i, i8p, i8p]
        L.ocv_fast_atan_rad.argtypes = [ctypes.c_float, ctypes.c_float]
        L.ocv_fast_atan_rad.restype = ctypes.c_float
        for f in (L.ocv_invert3x3, L.ocv_warp_perspective_u8, L.ocv_resize_nearest_u8, L.ocv_morph_open3x3_u8,
                  L.ocv_resize_linear_u8, L.bev_occgrid_ref, L.bev_occgrid_binary_ref, L.bev_occgrid_laserscan_ref,
                  L.bev_occgrid_binary_laserscan_ref):
            f.restype = ctypes.c_int
        _lib = L
    return _lib


def invert3x3(M):
    o = np.zeros(9)
    lib().ocv_invert3x3(np.ascontiguousarray(M, np.float64).reshape(9), o)
    return o.reshape(3, 3)


def warp_perspective(src, M, dsize):
    src = np.ascontiguousarray(src, np.uint8)
    dw, dh = dsize
    out = np.empty((dh, dw), np.uint8)
    lib().ocv_warp_perspective_u8(src, src.shape[0], src.shape[1], out, dh, dw,
                                  np.ascontiguousarray(M, np.float64).reshape(9))
    return out


def resize_nearest(src, dsize):
    src = np.ascontiguousarray(src, np.uint8)
    dw, dh = dsize
    cn = 1 if src.ndim == 2 else src.shape[2]
    out = np.empty((dh, dw) + (() if src.ndim == 2 else (cn,)), np.uint8)
    lib().ocv_resize_nearest_u8(src, src.shape[0], src.shape[1], cn, out, dh, dw)
    return out


def morph_open3x3(src):
    src = np.ascontiguousarray(src, np.uint8)
    out = np.empty_like(src)
    lib().ocv_morph_open3x3_u8(src, src.shape[0], src.shape[1], out)
    return out


def resize_linear(src, dsize):
    src = np.ascontiguousarray(src, np.uint8)
    dw, dh = dsize
    cn = 1 if src.ndim == 2 else src.shape[2]
    out = np.empty((dh, dw) + (() if src.ndim == 2 else (cn,)), np.uint8)
    lib().ocv_resize_linear_u8(src, src.shape[0], src.shape[1], cn, out, dh, dw)
    return out


def occgrid_geometry(after_warp_w, after_warp_h, cm_per_px, grid_w_m, grid_h_m, cell_m):
    """bev.py:172-184 restated (host float arithmetic + int() truncation)."""
    cell_px = cell_m * 100 / cm_per_px
    occ_w = int(grid_w_m / cell_m)
    occ_w_px = int(occ_w * cell_px)
    occ_h = int(grid_h_m / cell_m)
    occ_h_px = int(occ_h * cell_px)
    left_x = int((after_warp_w - occ_w_px) / 2)
    top_y = after_warp_h - occ_h_px
    return dict(occ_w=occ_w, occ_h=occ_h, occ_w_px=occ_w_px, occ_h_px=occ_h_px, left_x=left_x, top_y=top_y)


def create_occupancy_grid(segmap, M, after_warp_w, after_warp_h, cm_per_px, grid_w_m, grid_h_m, cell_m):
    """bev.py:166-246 (non-laserscan) via the C restatement -> int8 (occ_h, occ_w)."""
    seg = np.ascontiguousarray(segmap, np.uint8)
    g = occgrid_geometry(after_warp_w, after_warp_h, cm_per_px, grid_w_m, grid_h_m, cell_m)
    out = np.empty((g["occ_h"], g["occ_w"]), np.int8)
    rc = lib().bev_occgrid_ref(seg, seg.shape[0], seg.shape[1], np.ascontiguousarray(M, np.float64).reshape(9),
                               after_warp_w, after_warp_h, g["occ_w_px"], g["occ_h_px"], g["occ_w"], g["occ_h"],
                               g["left_x"], g["top_y"], out)
    if rc != 0:
        raise MemoryError("bev_occgrid_ref failed")
    return out


def create_occupancy_grid_binary(segmap, M, after_warp_w, after_warp_h, cm_per_px, grid_w_m, grid_h_m, cell_m):
    """bev.py:97-165 (legacy binary variant, non-laserscan) via the C restatement -> int8 (occ_h, occ_w)."""
    seg = np.ascontiguousarray(segmap, np.uint8)
    g = occgrid_geometry(after_warp_w, after_warp_h, cm_per_px, grid_w_m, grid_h_m, cell_m)
    out = np.empty((g["occ_h"], g["occ_w"]), np.int8)
    rc = lib().bev_occgrid_binary_ref(seg, seg.shape[0], seg.shape[1], np.ascontiguousarray(M, np.float64).reshape(9),
                                      after_warp_w, after_warp_h, g["occ_w_px"], g["occ_h_px"], g["occ_w"], g["occ_h"],
                                      g["left_x"], g["top_y"], out)
    if rc != 0:
        raise MemoryError("bev_occgrid_binary_ref failed")
    return out


def create_occupancy_grid_laserscan(segmap, M, after_warp_w, after_warp_h, cm_per_px, grid_w_m, grid_h_m, cell_m):
    """bev.py:166-246 with is_laserscan (polar branch bev.py:216-240) via the C restatement."""
    seg = np.ascontiguousarray(segmap, np.uint8)
    g = occgrid_geometry(after_warp_w, after_warp_h, cm_per_px, grid_w_m, grid_h_m, cell_m)
    out = np.empty((g["occ_h"], g["occ_w"]), np.int8)
    rc = lib().bev_occgrid_laserscan_ref(seg, seg.shape[0], seg.shape[1], np.ascontiguousarray(M, np.float64).reshape(9),
                                         after_warp_w, after_warp_h, g["occ_w_px"], g["occ_h_px"], g["occ_w"], g["occ_h"],
                                         g["left_x"], g["top_y"], out)
    if rc != 0:
        raise MemoryError("bev_occgrid_laserscan_ref failed")
    return out


def create_occupancy_grid_binary_laserscan(segmap, M, after_warp_w, after_warp_h, cm_per_px, grid_w_m, grid_h_m,
                                           cell_m):
    """bev.py:97-165 with is_laserscan (bev.py:143-164) via the C restatement -> (grid, new) int8."""
    seg = np.ascontiguousarray(segmap, np.uint8)
    g = occgrid_geometry(after_warp_w, after_warp_h, cm_per_px, grid_w_m, grid_h_m, cell_m)
    out = np.empty((g["occ_h"], g["occ_w"]), np.int8)
    out2 = np.empty_like(out)
    rc = lib().bev_occgrid_binary_laserscan_ref(seg, seg.shape[0], seg.shape[1],
                                                np.ascontiguousarray(M, np.float64).reshape(9), after_warp_w,
                                                after_warp_h, g["occ_w_px"], g["occ_h_px"], g["occ_w"], g["occ_h"],
                                                g["left_x"], g["top_y"], out, out2)
    if rc != 0:
        raise MemoryError("bev_occgrid_binary_laserscan_ref failed")
    return out, out2


def pipeline(frames_bgr, blocks, M, after_warp_w, after_warp_h, cm_per_px, grid, model_hw, dtype=None):
    """Whole reference loop for a batch: ENET.preprocess -> ENET.predict -> create_occupancy_grid.
    Returns (class maps (B,H,W) u8, grids (B,h,w) int8, logits)."""
    import torch
    from . import enet_oracle as eo
    H, W = model_hw
    x = np.concatenate([eo.preprocess(f, W, H) for f in frames_bgr], 0).astype(np.float32)
    logits = eo.forward(blocks, x, dtype or torch.float32)
    cls = eo.LUT3[eo.argmax_classes(logits)]
    grids = np.stack([create_occupancy_grid(c, M, after_warp_w, after_warp_h, cm_per_px, *grid) for c in cls])
    return cls, grids, logits
