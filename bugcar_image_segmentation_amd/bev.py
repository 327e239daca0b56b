"""bev_transform_tools with the reference's API (bev.py), rasterising on the MI355X engine.

`fromJSON`, the constructor, `save_to_JSON` and `create_occupancy_grid` keep the reference's
names, argument meaning, shape assert and return dtype. The per-frame work — warpPerspective of the
lifted class map, the crop/pad into the grid template, the 3x3 opening that frees isolated occupied
pixels, the INTER_NEAREST downsample and the int8 encoding (bev.py:166-246) — is ONE fused gfx950
kernel (csrc/bev_kernels.hip). The geometry below (cell sizes, template offsets) is host arithmetic
written exactly as the reference writes it, because its float-to-int truncations are part of the
result.

The laserscan-like mode ("is_laserscan", bev.py:216-240 and the binary variant's bev.py:143-164) runs
on the engine too: the rasteriser, a per-ray nearest-obstacle kernel and a re-projection kernel over
polar tables the library builds once per geometry (csrc/bev_kernels.hip).

Additions: `create_occupancy_grid_device` (batched, device tensors in and out, optional ROS data
layout) and `occupancy_params`.
"""
from __future__ import annotations

import json

import numpy as np
import torch

from . import _native as N


def order_points_counter_clockwise(points, x_axis):
    """utils.py:10-44 (calibration helper): order 4 points left-of-axis first, each side by x.
    Like the reference it translates `x_axis` in place."""
    center = x_axis[0]
    translated_points = points - center
    x_axis -= center
    rotation = -np.arctan2(x_axis[1, 1], x_axis[1, 0])
    rot_mat = np.array([[np.cos(rotation), -np.sin(rotation)],
                        [np.sin(rotation), np.cos(rotation)]])
    rotated = np.transpose(np.matmul(rot_mat, np.transpose(translated_points)))
    left, right = [], []
    for i, pt in enumerate(rotated):
        (right if pt[1] < 0 else left).append((pt[0], i))
    left.sort(key=lambda t: t[0])
    right.sort(key=lambda t: t[0])
    order = [i for _, i in left] + [i for _, i in right]
    return points[order]


def get_perspective_transform(src, dst) -> np.ndarray:
    """The 4-point homography cv2.getPerspectiveTransform solves (8x8 linear system, M[2,2] = 1)."""
    src = np.asarray(src, np.float64).reshape(4, 2)
    dst = np.asarray(dst, np.float64).reshape(4, 2)
    A = np.zeros((8, 8))
    b = np.zeros(8)
    for i in range(4):
        x, y = src[i]
        u, v = dst[i]
        A[i] = [x, y, 1, 0, 0, 0, -x * u, -y * u]
        A[i + 4] = [0, 0, 0, x, y, 1, -x * v, -y * v]
        b[i], b[i + 4] = u, v
    m = np.linalg.solve(A, b)
    return np.append(m, 1.0).reshape(3, 3)


class bev_transform_tools:
    """bev.py:8-246."""

    def __init__(self, input_image_shape, desired_image_shape, dist2target, tile_length, cm_per_px, yaw,
                 make_laserscan_like=False):
        # bev.py:13-22 — note the reference's naming: input_image_shape is (rows, cols) of the segmap
        # (checked by the assert in create_occupancy_grid), desired_image_shape is (width, height).
        self.input_width = input_image_shape[0]
        self.input_height = input_image_shape[1]
        self.after_warp_width = desired_image_shape[0]
        self.after_warp_height = desired_image_shape[1]
        self.dist2target = dist2target
        self.tile_length = tile_length
        self.cm_per_px = cm_per_px
        self.yaw = yaw
        self.laserscan_like_occupancy_grid = make_laserscan_like
        self._bev_matrix = None

    @classmethod
    def fromJSON(cls, filepath):
        """bev.py:24-41. Missing keys raise KeyError like the reference."""
        with open(filepath, mode="r") as f:
            data = json.load(f)
        shape = data["output image size"]
        input_shape = data["input image size"]
        bev_matrix = np.reshape(np.array(data["bev matrix"]), (3, 3))
        dist2target = data["distance to target"]
        tile_length = data["tile_length"]
        cm_per_px = data["cm_per_px"]
        yaw = data["yaw"]
        is_laserscan = data["is_laserscan"]
        bev = cls(input_shape, shape, dist2target, tile_length, cm_per_px, yaw, is_laserscan)
        bev._bev_matrix = bev_matrix
        return bev

    def save_to_JSON(self, file_path):
        """bev.py:44-56, plus the "is_laserscan" key the reference omits (so the file round-trips
        through fromJSON, which requires it — bev.py:37)."""
        data = {
            "input image size": (self.input_width, self.input_height),
            "output image size": (self.after_warp_width, self.after_warp_height),
            "bev matrix": np.asarray(self._bev_matrix).tolist(),
            "distance to target": self.dist2target,
            "tile_length": self.tile_length,
            "cm_per_px": self.cm_per_px,
            "yaw": self.yaw,
            "is_laserscan": bool(self.laserscan_like_occupancy_grid),
        }
        with open(file_path, mode="w") as f:
            json.dump(data, f)

    def calculate_transform_matrix(self, tile_coords):
        """bev.py:58-92: map the calibration tile's image corners onto a tile_length square placed
        dist2target from the bottom centre of the BEV image, rotated by yaw (host, one-shot)."""
        cm_per_px, yaw = self.cm_per_px, self.yaw
        d2t = (self.dist2target[0] / cm_per_px, self.dist2target[1] / cm_per_px)
        mh = self.tile_length / cm_per_px
        original = np.array([[mh / 2, mh / 2], [mh / 2, -mh / 2], [-mh / 2, -mh / 2], [-mh / 2, mh / 2]])
        rot = np.array([[np.cos(yaw), -np.sin(yaw)], [np.sin(yaw), np.cos(yaw)]])
        target = (self.after_warp_width / 2 + d2t[0], self.after_warp_height - d2t[1])
        axis_pt = np.matmul(rot, np.array([100, 0])) + target
        fid_axis = np.stack([np.asarray(target, dtype=np.float64), axis_pt], axis=0)
        rotated = np.array([np.matmul(rot, p) for p in original]) + target
        rotated = order_points_counter_clockwise(rotated, fid_axis)
        M = get_perspective_transform(np.asarray(tile_coords, np.float32), rotated.astype(np.float32))
        self._bev_matrix = M
        return M

    # -- geometry ----------------------------------------------------------------------------
    def occupancy_params(self, occupancy_grid_width_in_m, occupancy_grid_height_in_m, cell_size_in_m,
                         ros_layout: bool = False, binary: bool = False, laserscan: bool | None = None) -> N.BevParams:
        """bev.py:172-184 (bev.py:101-114 for the binary variant: the same arithmetic), with the
        reference's float arithmetic and int() truncations."""
        cell_size_in_px = (cell_size_in_m * 100 / self.cm_per_px)
        occ_grid_width = int(occupancy_grid_width_in_m / cell_size_in_m)
        occ_width_pixel = int(occ_grid_width * cell_size_in_px)
        occ_grid_height = int(occupancy_grid_height_in_m / cell_size_in_m)
        occ_height_pixel = int(occ_grid_height * cell_size_in_px)
        left_x = int((self.after_warp_width - occ_width_pixel) / 2)
        top_y = self.after_warp_height - occ_height_pixel
        if occ_grid_width <= 0 or occ_grid_height <= 0 or occ_width_pixel <= 0 or occ_height_pixel <= 0:
            raise ValueError("occupancy grid has no cells")
        p = N.BevParams()
        M = np.asarray(self._bev_matrix, dtype=np.float64).reshape(9)
        for i in range(9):
            p.M[i] = float(M[i])
        p.in_rows, p.in_cols = int(self.input_width), int(self.input_height)
        p.warp_w, p.warp_h = int(self.after_warp_width), int(self.after_warp_height)
        p.occ_w_px, p.occ_h_px = occ_width_pixel, occ_height_pixel
        p.occ_w, p.occ_h = occ_grid_width, occ_grid_height
        p.left_x, p.top_y = left_x, top_y
        p.ros_layout = int(bool(ros_layout))
        p.variant = int(bool(binary))
        p.laserscan = int(bool(self.laserscan_like_occupancy_grid if laserscan is None else laserscan))
        return p

    def _check_shape(self, shape):
        assert tuple(shape) == (self.input_width, self.input_height), \
            "current segmap size: {},the segmap's original size must be the same as the required input shape, which is {}" \
            .format(tuple(shape), (self.input_width, self.input_height))

    # -- the hot path --------------------------------------------------------------------------
    def create_occupancy_grid_device(self, segmaps: torch.Tensor, occupancy_grid_width_in_m,
                                     occupancy_grid_height_in_m, cell_size_in_m, ros_layout: bool = False,
                                     out: torch.Tensor | None = None, binary: bool = False) -> torch.Tensor:
        """Batched create_occupancy_grid on device tensors: segmaps (B, rows, cols) uint8 class maps
        -> (B, h, w) int8 (or (B, w, h) in ROS data order when ros_layout). binary=True is
        create_occupancy_grid_binary (bev.py:97-165). The laserscan-like mode follows the object's
        is_laserscan flag; binary + laserscan returns (2, B, ...): the grid, then the polar
        re-projection of its nearest obstacles (the reference's returned pair, bev.py:162)."""
        if segmaps.dim() == 2:
            segmaps = segmaps.unsqueeze(0)
        self._check_shape(segmaps.shape[1:])
        seg = segmaps if segmaps.dtype == torch.uint8 else segmaps.to(torch.uint8)
        if not seg.is_cuda:
            seg = seg.to(torch.device("cuda", torch.cuda.current_device()))
        seg = seg.contiguous()
        p = self.occupancy_params(occupancy_grid_width_in_m, occupancy_grid_height_in_m, cell_size_in_m, ros_layout,
                                  binary)
        B = seg.shape[0]
        shape = (B, p.occ_w, p.occ_h) if ros_layout else (B, p.occ_h, p.occ_w)
        if binary and p.laserscan:
            shape = (2,) + shape
        if out is not None and tuple(out.shape) != shape:
            raise ValueError(f"out has shape {tuple(out.shape)}, expected {shape}")
        if out is None:
            out = torch.empty(shape, dtype=torch.int8, device=seg.device)
        N.shared_context(seg.device.index).bev(seg, B, p, out, torch.cuda.current_stream(seg.device))
        return out

    def create_occupancy_grid(self, segmap, occupancy_grid_width_in_m, occupancy_grid_height_in_m, cell_size_in_m):
        """bev.py:166-246 -> np.int8 (h, w) in {-1 unknown, 0 free, 100 occupied}. In laserscan-like mode
        (bev.py:216-240) only the obstacle cells nearest the vehicle along each polar ray stay
        occupied; obstacle cells behind them become unknown."""
        self._check_shape(np.shape(segmap))
        seg = segmap if isinstance(segmap, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(segmap, dtype=np.uint8))
        return self.create_occupancy_grid_device(seg, occupancy_grid_width_in_m, occupancy_grid_height_in_m,
                                                 cell_size_in_m)[0].cpu().numpy()

    def create_occupancy_grid_binary(self, segmap, occupancy_grid_width_in_m, occupancy_grid_height_in_m, cell_size_in_m):
        """bev.py:97-165 (legacy variant for ENET.predict_binary maps) -> np.int8 (h, w).
        Occupied = template value 1 only (bev.py:126); the reference's uint8 encoding gives
        {0: -1, 1: 100, 2: 0} and, for a 3-class map's class 2, -100 (bev.py:137-141 under NumPy 1.x
        casting). For {0,1} maps it equals create_occupancy_grid. In laserscan-like mode it returns the
        reference's pair (grid, re-projected nearest obstacles) (bev.py:143-162)."""
        self._check_shape(np.shape(segmap))
        seg = segmap if isinstance(segmap, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(segmap, dtype=np.uint8))
        g = self.create_occupancy_grid_device(seg, occupancy_grid_width_in_m, occupancy_grid_height_in_m,
                                              cell_size_in_m, binary=True)
        if self.laserscan_like_occupancy_grid:
            g = g.cpu().numpy()
            return g[0, 0], g[1, 0]
        return g[0].cpu().numpy()
