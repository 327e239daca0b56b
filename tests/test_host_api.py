"""Host-side logic of the drop-in API (CPU only, no kernel launches)."""
import json
import struct

import numpy as np
import pytest
from scipy.spatial.transform import Rotation as R

from bugcar_image_segmentation_amd import enet_spec, synthetic
from bugcar_image_segmentation_amd.bev import bev_transform_tools, get_perspective_transform
from bugcar_image_segmentation_amd.distributed import shard_bounds
from bugcar_image_segmentation_amd.occgrid_to_ros import convert_to_occupancy_grid_msg, ros_data_order
from oracle import ocv_c


def _calib(tmp_path, **over):
    data = {"input image size": [480, 640], "output image size": [1000, 1000],
            "bev matrix": synthetic.synthetic_bev()._bev_matrix.ravel().tolist(),
            "distance to target": [0.0, 100.0], "tile_length": 50.0, "cm_per_px": 1.0, "yaw": 0.0,
            "is_laserscan": False}
    data.update(over)
    p = tmp_path / "bev.json"
    p.write_text(json.dumps(data))
    return p


def test_fromjson_fields(tmp_path):
    bev = bev_transform_tools.fromJSON(_calib(tmp_path))
    assert (bev.input_width, bev.input_height) == (480, 640)       # (rows, cols), bev.py:13-14
    assert (bev.after_warp_width, bev.after_warp_height) == (1000, 1000)
    assert bev._bev_matrix.shape == (3, 3) and bev.cm_per_px == 1.0 and bev.laserscan_like_occupancy_grid is False


def test_fromjson_missing_key_raises_keyerror(tmp_path):
    p = _calib(tmp_path)
    d = json.loads(p.read_text())
    del d["is_laserscan"]
    p.write_text(json.dumps(d))
    with pytest.raises(KeyError):
        bev_transform_tools.fromJSON(p)


def test_save_to_json_round_trips(tmp_path):
    bev = bev_transform_tools.fromJSON(_calib(tmp_path))
    out = tmp_path / "saved.json"
    bev.save_to_JSON(out)
    again = bev_transform_tools.fromJSON(out)
    assert np.array_equal(again._bev_matrix, bev._bev_matrix)
    assert (again.input_width, again.input_height) == (bev.input_width, bev.input_height)


@pytest.mark.parametrize("ww,wh,grid", [(1000, 1000, (10.0, 10.0, 0.05)), (900, 700, (10, 8, 0.05)),
                                        (600, 1100, (7.3, 12.1, 0.07)), (1000, 1000, (12, 12, 0.05))])
def test_occupancy_geometry_matches_reference_arithmetic(ww, wh, grid):
    bev = bev_transform_tools([480, 640], [ww, wh], (0, 100), 50, 1.0, 0.0)
    bev._bev_matrix = np.eye(3)
    p = bev.occupancy_params(*grid)
    g = ocv_c.occgrid_geometry(ww, wh, 1.0, *grid)
    assert (p.occ_w, p.occ_h, p.occ_w_px, p.occ_h_px, p.left_x, p.top_y) == \
           (g["occ_w"], g["occ_h"], g["occ_w_px"], g["occ_h_px"], g["left_x"], g["top_y"])
    assert (p.in_rows, p.in_cols, p.warp_w, p.warp_h) == (480, 640, ww, wh)


def test_synthetic_calibration_geometry():
    bev = synthetic.synthetic_bev()
    p = bev.occupancy_params(synthetic.GRID_W_M, synthetic.GRID_H_M, synthetic.CELL_M)
    assert (p.occ_w, p.occ_h, p.occ_w_px, p.occ_h_px, p.left_x, p.top_y) == (200, 200, 1000, 1000, 0, 0)


def test_get_perspective_transform_maps_points():
    src = np.array([[10, 20], [200, 25], [220, 180], [5, 170]], np.float64)
    dst = np.array([[0, 0], [100, 0], [100, 100], [0, 100]], np.float64)
    M = get_perspective_transform(src, dst)
    h = np.c_[src, np.ones(4)] @ M.T
    assert np.allclose(h[:, :2] / h[:, 2:], dst, atol=1e-9)


def test_calculate_transform_matrix_runs():
    bev = bev_transform_tools([480, 640], [1000, 1000], (0.0, 150.0), 50.0, 1.0, 0.1)
    tile = np.array([[300, 400], [340, 400], [345, 430], [295, 430]], np.float64)
    M = bev.calculate_transform_matrix(tile)
    assert M.shape == (3, 3) and np.isfinite(M).all() and bev._bev_matrix is M


def test_ros_message():
    g = np.array([[-1, 0, 100], [100, 0, -1]], np.int8)
    pose = [1.0, 2.0, 0.5, 0.1, -0.2, 0.3]
    msg = convert_to_occupancy_grid_msg(g, 0.05, 10.0, 6.0, "stamp", "base_link", pose)
    assert msg.data == g[::-1, ::-1].T.flatten().tolist()
    assert msg.info.height == int(10.0 / 0.05) and msg.info.width == int(6.0 / 0.05)
    q = R.from_euler("xyz", pose[3:]).as_quat()
    assert np.allclose([msg.info.origin.orientation.x, msg.info.origin.orientation.y,
                        msg.info.origin.orientation.z, msg.info.origin.orientation.w], q)
    o = R.from_euler("xyz", pose[3:]).as_matrix() @ (np.array([0, -5.0, 0]) + pose[:3])
    assert np.allclose([msg.info.origin.position.x, msg.info.origin.position.y, msg.info.origin.position.z], o)
    assert msg.header.frame_id == "base_link" and msg.header.stamp == "stamp" and msg.info.resolution == 0.05
    # GPU-produced ROS order passes through unchanged
    msg2 = convert_to_occupancy_grid_msg(ros_data_order(g), 0.05, 10.0, 6.0, "s", "f", pose, ros_layout=True)
    assert msg2.data == msg.data


def test_blob_format_header_and_units(blocks):
    blob = enet_spec.serialize(blocks)
    assert blob[:4] == b"BSG1"
    ver, nb, nc = struct.unpack_from("<III", blob, 4)
    assert (ver, nb, nc) == (1, len(blocks), 15)
    btype, *attrs = struct.unpack_from("<I8i", blob, 16)
    assert btype == enet_spec.BLOCK_INITIAL and attrs[:3] == [3, 13, 3]


def test_canonical_topology_census(blocks):
    """89 convolutions; ~2.23 GMAC/frame at 640x480 (3x3 final deconv:
    4.64 GFLOP = 2 x 2.32 GMAC including the 166 MMAC final layer)."""
    assert sum(len(b.units) for b in blocks) == 89
    flops, byts = enet_spec.enet_flops_bytes(blocks, 480, 640)
    assert abs(flops / 1e9 - 4.643) < 0.01


@pytest.mark.parametrize("total,world", [(512, 8), (10, 3), (3, 4), (64, 1)])
def test_shard_bounds_partition(total, world):
    spans = [shard_bounds(total, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == total
    assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    sizes = [e - s for s, e in spans]
    assert max(sizes) - min(sizes) <= 1
