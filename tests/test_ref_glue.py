"""CPU: the oracle and the drop-in host code against fixtures the REFERENCE'S OWN glue produced
(tests/golden/ref_glue.npz, generator tests/golden/make_ref_glue.py: the reference's bev.py /
occgrid_to_ros.py / models.py run with oracle-backed stand-ins for cv2 / tensorflow / numpy_indexed /
ROS). Pins the glue — geometry truncations, crop / pad slicing, label lift and uint8 wraps, speckle
mask, binary encoding, laserscan flow, ROS layout / origin / quaternion, argmax + LUT, preprocess
normalisation — not OpenCV's or TF's arithmetic. The HIP rasteriser is checked against
the same fixtures in tests/test_gpu_ref_glue.py."""
import json
import os

import numpy as np
import pytest

from bugcar_image_segmentation_amd import occgrid_to_ros
from bugcar_image_segmentation_amd.bev import bev_transform_tools
from oracle import enet_oracle as eo
from oracle import ocv_c, ocv_np

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_glue.npz")
GEOMS = ("bench", "small_neg", "small_odd")


def test_fixture_is_the_committed_one():
    """The fixture file is the one the generator wrote when it was run (its SHA-256 is committed beside
    it): the generator executes the reference's own code, so it is never run by a test or CI job —
    only by hand in the build container — and its output is checked by content here."""
    import hashlib
    with open(FIX, "rb") as f:
        got = hashlib.sha256(f.read()).hexdigest()
    with open(FIX.replace(".npz", ".sha256")) as f:
        assert got == f.read().strip()


@pytest.fixture(scope="module")
def fx():
    with np.load(FIX, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def _geom(fx, g, tmp_path):
    d = json.loads(bytes(fx[f"{g}/json"]).decode())
    p = tmp_path / f"{g}.json"
    p.write_text(json.dumps(d))
    w, h, cell = (float(v) for v in fx[f"{g}/grid"])
    return d, str(p), (w, h, cell)


@pytest.mark.parametrize("g", GEOMS)
def test_fromjson_matches_reference(fx, g, tmp_path):
    _d, path, _grid = _geom(fx, g, tmp_path)
    b = bev_transform_tools.fromJSON(path)
    assert np.array_equal(np.asarray(b._bev_matrix, np.float64), fx[f"{g}/fromjson_M"])
    assert [b.input_width, b.input_height, b.after_warp_width, b.after_warp_height] == list(fx[f"{g}/fromjson_sizes"])


@pytest.mark.parametrize("g", GEOMS)
def test_oracles_equal_reference_occupancy_grids(fx, g, tmp_path):
    """bev.py:166-246 and :97-165, both branches, 4 segmaps per geometry (3- and 15-class maps, the
    whole u8 range, a structured map): both restatements (NumPy, plain C) equal the reference's
    glue bit for bit."""
    d, _path, (gw, gh, cell) = _geom(fx, g, tmp_path)
    M = np.asarray(d["bev matrix"], np.float64).reshape(3, 3)
    aw, ah = d["output image size"]
    cm = d["cm_per_px"]
    segs = fx[f"{g}/segmaps"]
    for i, seg in enumerate(segs):
        a = (seg, M, aw, ah, cm, gw, gh, cell)
        for mod in (ocv_np, ocv_c):
            assert np.array_equal(mod.create_occupancy_grid(*a), fx[f"{g}/plain/occgrid"][i]), (mod.__name__, i)
            assert np.array_equal(mod.create_occupancy_grid_binary(*a), fx[f"{g}/plain/occgrid_binary"][i]), (mod.__name__, i)
            assert np.array_equal(mod.create_occupancy_grid_laserscan(*a), fx[f"{g}/ls/occgrid"][i]), (mod.__name__, i)
            g0, g1 = mod.create_occupancy_grid_binary_laserscan(*a)
            assert np.array_equal(g0, fx[f"{g}/ls/occgrid_binary"][i]), (mod.__name__, i)
            assert np.array_equal(g1, fx[f"{g}/ls/occgrid_binary_new"][i]), (mod.__name__, i)


@pytest.mark.parametrize("g", GEOMS)
def test_ros_message_matches_reference(fx, g):
    """occgrid_to_ros.py:13-61 (real scipy): data order, info sizes, origin, quaternion, header."""
    grid = fx[f"{g}/plain/occgrid"][0]
    gw, gh, cell = (float(v) for v in fx[f"{g}/grid"])
    pose = fx[f"{g}/ros/pose"]
    msg = occgrid_to_ros.convert_to_occupancy_grid_msg(grid, cell, gw, gh, 12345, "base_link", pose)
    assert np.array_equal(np.asarray(msg.data, np.int64), fx[f"{g}/ros/data"])
    info = np.array([msg.info.height, msg.info.width, msg.info.resolution, msg.info.origin.position.x,
                     msg.info.origin.position.y, msg.info.origin.position.z, msg.info.origin.orientation.x,
                     msg.info.origin.orientation.y, msg.info.origin.orientation.z, msg.info.origin.orientation.w])
    assert np.array_equal(info, fx[f"{g}/ros/info"])
    hdr = json.loads(bytes(fx[f"{g}/ros/header"]).decode())
    assert msg.header.frame_id == hdr["frame_id"] and msg.header.stamp == hdr["stamp"]
    # the GPU rasteriser's ROS data order is the same layout
    assert np.array_equal(occgrid_to_ros.ros_data_order(grid).ravel(), fx[f"{g}/ros/data"])
    assert np.array_equal(ocv_np.ros_layout(grid).ravel(), fx[f"{g}/ros/data"])


def test_predict_postprocessing_matches_reference(fx):
    """models.py:53-58 / :76-81 on given logits (ties between LUT groups included): first-index
    argmax and the two remaps of the oracle (the HIP class layer is tested against these)."""
    lg = fx["enet/logits"]
    cls = eo.argmax_classes(lg)
    assert np.array_equal(eo.LUT3[cls], fx["enet/predict"])
    assert np.array_equal(eo.LUT_BINARY[cls], fx["enet/predict_binary"])


def test_preprocess_matches_reference(fx):
    """models.py:84-95 (the resize is the oracle's restatement; the colour order, /256, mean / std,
    moveaxis and batch axis are the reference's glue)."""
    ref = fx["enet/preprocess"]
    got = eo.preprocess(fx["enet/preprocess_in"], 512, 256)
    assert got.shape == ref.shape == (1, 3, 256, 512)
    assert np.array_equal(got, ref)
