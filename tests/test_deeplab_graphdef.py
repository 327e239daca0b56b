"""DeepLab GraphDef importer (bugcar_image_segmentation_amd/deeplab_graphdef.py, SURVEY.md §8(f) rows 1 + 3)
against graphs written by tests/deeplab_graph_writer.py in two encodings, and the NumPy GraphDef
interpreter (oracle/tf_graph.py, the sess.run stand-in) on the same graphs.

Bars: imported weights equal the written network's after batch-norm folding (rtol 1e-5, fp32
storage); the oracle forward of the imported network equals the written network's within 1e-4
(fp64); the interpreter's pre-resize logits equal the oracle's within 1e-4 and its
SemanticPredictions equal the oracle's class map wherever the top-2 margin exceeds 1e-4.
Parity against TF on the real deeplab.pb is unpinned (neither exists here).
"""
import numpy as np
import pytest
import torch

from bugcar_image_segmentation_amd import deeplab_spec as S
from bugcar_image_segmentation_amd import deeplab_xception as X
from bugcar_image_segmentation_amd.deeplab_graphdef import graphdef_to_npz, import_deeplab
from bugcar_image_segmentation_amd.graphdef import GraphImportError
from deeplab_graph_writer import write_deeplab_graph
from oracle import deeplab_oracle as O
from oracle import tf_graph

CROP = 65


def _net(rates=(2, 4), os_=8, ncls=S.NUM_CLASSES, crop=CROP):
    return S.build_deeplab(width=0.25, crop=crop, output_stride=os_, atrous_rates=rates, num_classes=ncls)


def _same_weights(a: S.DeepLab, b: S.DeepLab):
    ca, cb = list(S._convs(a)), list(S._convs(b))
    assert [n for n, _ in ca] == [n for n, _ in cb]
    for (name, x), (_, y) in zip(ca, cb):
        assert (x.act, x.stride, x.dil, x.depthwise) == (y.act, y.stride, y.dil, y.depthwise), name
        wx, bx = x.folded()
        wy, by = y.folded()
        assert wx.shape == wy.shape, name
        np.testing.assert_allclose(wy, wx, rtol=1e-5, atol=1e-6, err_msg=name)
        np.testing.assert_allclose(by, bx, rtol=1e-5, atol=1e-6, err_msg=name)
    assert [blk.residual for blk in a.blocks] == [blk.residual for blk in b.blocks]
    assert (a.num_classes, S.crop_hw(a)) == (b.num_classes, S.crop_hw(b))


@pytest.mark.parametrize("style", ["slim", "folded"])
@pytest.mark.parametrize("rates,os_", [((2, 4), 8), ((), 16)])
def test_import_recovers_the_network(style, rates, os_):
    net = _net(rates, os_)
    got = import_deeplab(write_deeplab_graph(net, style, 60, 65), crop=CROP)
    _same_weights(net, got)
    assert got.output_stride == os_
    if style == "slim":     # unfolded batch norm keeps its own statistics
        assert got.stem.gamma is not None and got.stem.eps == pytest.approx(net.stem.eps)
    x = np.random.default_rng(3).integers(0, 256, (2, 60, 65, 3), dtype=np.uint8)
    np.testing.assert_allclose(O.forward(got, x).numpy(), O.forward(net, x).numpy(), atol=1e-4)


@pytest.mark.parametrize("style,crop", [("slim", CROP), ("folded", CROP), ("slim", (57, 81))])
def test_interpreter_runs_the_written_graph_like_the_oracle(style, crop):
    net = _net((2,), 8, ncls=5, crop=crop)
    H, W = 57, 64
    pb = write_deeplab_graph(net, style, H, W, B=1)
    x = np.random.default_rng(4).integers(0, 256, (1, H, W, 3), dtype=np.uint8)
    ref = O.forward(net, x, dtype=torch.float64).numpy()
    lg = tf_graph.run(pb, {"ImageTensor": x}, "logits")
    np.testing.assert_allclose(np.transpose(lg, (0, 3, 1, 2)), ref, atol=1e-4)
    cls = tf_graph.run(pb, {"ImageTensor": x}, "SemanticPredictions")
    want = O.predict(net, x, logits=ref.astype(np.float32))
    up = O.resize_bilinear_tf(ref.astype(np.float32), *S.crop_hw(net))[:, :, :H, :W]
    s = np.sort(up, axis=1)
    decided = (s[:, -1] - s[:, -2]) > 1e-4
    assert cls.shape == (1, H, W)
    assert np.array_equal(np.asarray(cls, np.int64)[decided], want[decided])
    assert decided.mean() > 0.99


@pytest.mark.parametrize("crop", [CROP, (57, 81), (97, 41)])
def test_crop_is_read_from_the_graph(crop):
    """The export's pad-to-crop arithmetic (Maximum(Sub(crop, size), 0) per axis) gives the crop; an
    explicit crop overrides it; a graph without it (static PadV2) falls back to default_crop."""
    net = _net((2,), 8, crop=crop)
    pb = write_deeplab_graph(net, "slim", 33, 40)
    got = import_deeplab(pb)
    assert S.crop_hw(got) == S.crop_hw(net)
    _same_weights(net, got)
    assert S.crop_hw(import_deeplab(pb, crop=(129, 161))) == (129, 161)
    static = write_deeplab_graph(net, "folded", 33, 40, crop_in_graph=False)
    assert S.crop_hw(import_deeplab(static, default_crop=77)) == (77, 77)
    assert S.crop_hw(import_deeplab(static)) == (S.CROP, S.CROP)


def test_npz_round_trip(tmp_path):
    net = _net()
    p = tmp_path / "dl.npz"
    got = graphdef_to_npz(write_deeplab_graph(net, "slim", 65, 65), p, crop=CROP)
    _same_weights(got, S.load(p))
    net = _net(crop=(65, 97))
    got = graphdef_to_npz(write_deeplab_graph(net, "slim", 65, 65), p)
    assert S.crop_hw(S.load(p)) == (65, 97)
    _same_weights(got, S.load(p))


def test_rejects_graphs_that_are_not_deeplab():
    from graph_writer import GraphBuilder, F32
    g = GraphBuilder()
    x = g.node("Placeholder", [], name="ImageTensor", dtype=F32)
    for _ in range(6):
        x = g.node("Conv2D", [x, g.const(np.ones((1, 1, 4, 4), np.float32))], T=F32, strides=[1, 1, 1, 1],
                   padding="SAME", data_format="NHWC")
    with pytest.raises(GraphImportError, match="stem"):
        import_deeplab(g.bytes())
    net = _net()
    net.blocks[2].dw.act = S.ACT_RELU        # wrong activation after a depthwise conv
    with pytest.raises(GraphImportError, match="depthwise"):
        import_deeplab(write_deeplab_graph(net, "slim", 65, 65), crop=CROP)


def _same_xception(a, b):
    na, nb = list(X._named_convs(a)), list(X._named_convs(b))
    assert [n for n, _ in na] == [n for n, _ in nb]
    for (name, x), (_, y) in zip(na, nb):
        assert (x.act, x.stride, x.dil, x.depthwise) == (y.act, y.stride, y.dil, y.depthwise), name
        wx, bx = x.folded()
        wy, by = y.folded()
        np.testing.assert_allclose(wy, wx, rtol=1e-5, atol=1e-6, err_msg=name)
        np.testing.assert_allclose(by, bx, rtol=1e-5, atol=1e-6, err_msg=name)
    assert [(m.skip, [sp.pre_relu for sp in m.seps]) for m in a.modules] == \
        [(m.skip, [sp.pre_relu for sp in m.seps]) for m in b.modules]
    assert tuple(a.low_level) == tuple(b.low_level) and (a.low_proj is None) == (b.low_proj is None)
    assert (a.num_classes, a.output_stride, S.crop_hw(a)) == (b.num_classes, b.output_stride, S.crop_hw(b))


@pytest.mark.parametrize("style", ["slim", "folded"])
@pytest.mark.parametrize("kw", [dict(atrous_rates=(2, 4)), dict(atrous_rates=(), decoder=False),
                                dict(output_stride=8, atrous_rates=(2,), crop=(64, 98))])
def test_import_xception(style, kw):
    """Xception-65 / DeepLabV3+ graphs (fixed-padding strided layers, pre-activation ReLUs between
    separable convs, conv / sum / no skips, separable ASPP, decoder): the importer recovers the
    network, and the interpreter's logits on the written graph equal the oracle's."""
    net = X.build_deeplab_xception(width=0.25, middle=2, **{"crop": CROP, "num_classes": 5, **kw})
    H, W = 60, 64
    pb = write_deeplab_graph(net, style, H, W)
    got = import_deeplab(pb)
    _same_xception(net, got)
    x = np.random.default_rng(6).integers(0, 256, (1, H, W, 3), dtype=np.uint8)
    ref = O.forward(net, x).numpy()
    np.testing.assert_allclose(O.forward(got, x).numpy(), ref, atol=1e-4)
    lg = tf_graph.run(pb, {"ImageTensor": x}, "logits")
    np.testing.assert_allclose(np.transpose(lg, (0, 3, 1, 2)), ref, atol=1e-4)


def test_xception_npz_round_trip(tmp_path):
    net = X.build_deeplab_xception(width=0.25, middle=1, crop=(65, 81))
    p = tmp_path / "x.npz"
    S.save(net, p)
    _same_xception(net, S.load(p))
    got = graphdef_to_npz(write_deeplab_graph(net, "slim", 40, 40), p)
    _same_xception(got, S.load(p))


def test_xception_import_rejects_same_padded_strides():
    """A strided 3x3 with SAME padding is not the xception export's fixed padding (the two differ
    on even sizes): refused rather than mis-lowered."""
    from graph_writer import F32
    net = X.build_deeplab_xception(width=0.25, middle=1, crop=CROP)
    from deeplab_graph_writer import DeepLabWriter
    w = DeepLabWriter(net, "folded", 40, 40)
    orig = w.conv
    w.conv = lambda x, c, n, fixed=False: orig(x, c, n, fixed=False)
    with pytest.raises(GraphImportError, match="fixed_padding"):
        import_deeplab(w.build())


def _same_resnet(a, b):
    from bugcar_image_segmentation_amd import deeplab_resnet as R
    na, nb = list(R._named_convs(a)), list(R._named_convs(b))
    assert [n for n, _ in na] == [n for n, _ in nb]
    for (name, x), (_, y) in zip(na, nb):
        assert (x.act, x.stride, x.dil, x.depthwise) == (y.act, y.stride, y.dil, y.depthwise), name
        wx, bx = x.folded()
        wy, by = y.folded()
        np.testing.assert_allclose(wy, wx, rtol=1e-5, atol=1e-6, err_msg=name)
        np.testing.assert_allclose(by, bx, rtol=1e-5, atol=1e-6, err_msg=name)
    assert [u.stride for u in a.units] == [u.stride for u in b.units]
    assert (a.num_classes, a.output_stride, S.crop_hw(a)) == (b.num_classes, b.output_stride, S.crop_hw(b))


@pytest.mark.parametrize("style", ["slim", "folded"])
@pytest.mark.parametrize("kw", [dict(atrous_rates=(2, 4)), dict(output_stride=8, atrous_rates=(2,), crop=(64, 98)),
                                dict(atrous_rates=())])
def test_import_resnet(style, kw):
    """ResNet-v1-beta DeepLabV3 graphs (3-conv root with a fixed-padding strided conv, SAME max pool,
    bottleneck units with 1x1-conv / subsample / identity shortcuts and Relu(AddV2), atrous 3x3s in
    either encoding, dense ASPP): the importer recovers the network (a DeepLabResNet), and the
    interpreter's logits on the written graph equal the oracle's."""
    from bugcar_image_segmentation_amd import deeplab_resnet as R
    net = R.build_deeplab_resnet(depth=50, width=0.25, units=(1, 2, 2, 2), **{"crop": CROP, "num_classes": 5, **kw})
    H, W = 60, 64
    pb = write_deeplab_graph(net, style, H, W)
    got = import_deeplab(pb)
    assert isinstance(got, R.DeepLabResNet)
    _same_resnet(net, got)
    x = np.random.default_rng(8).integers(0, 256, (1, H, W, 3), dtype=np.uint8)
    ref = O.forward(net, x).numpy()
    np.testing.assert_allclose(O.forward(got, x).numpy(), ref, atol=1e-4)
    lg = tf_graph.run(pb, {"ImageTensor": x}, "logits")
    np.testing.assert_allclose(np.transpose(lg, (0, 3, 1, 2)), ref, atol=1e-4)


def test_resnet_npz_round_trip(tmp_path):
    from bugcar_image_segmentation_amd import deeplab_resnet as R
    net = R.build_deeplab_resnet(depth=50, width=0.25, units=(1, 1, 2, 1), crop=(65, 81))
    p = tmp_path / "r.npz"
    S.save(net, p)
    _same_resnet(net, S.load(p))
    got = graphdef_to_npz(write_deeplab_graph(net, "slim", 40, 40), p)
    _same_resnet(got, S.load(p))
