"""Frozen TF GraphDef import (models.py:21-31 loads enet.pb).

No enet.pb and no TensorFlow exist here (parity UNPINNED against TF). The importer is exercised on
GraphDefs written from the synthetic weights in two encodings (tests/graph_writer.py: a Keras-like
NHWC graph and an ONNX-to-TF-like NCHW graph). Three checks:
  * the NumPy GraphDef interpreter (oracle/tf_graph.py, the sess.run stand-in) reproduces the
    PyTorch-CPU ENet oracle on the written graph — so the writer and the interpreter agree on the
    op semantics;
  * the importer's block list reproduces the original network (oracle forward, fp64);
  * (GPU, tests/test_gpu_parity.py) ENET("x.pb") logits match the interpreter's within 1e-3 — the
    north star's TF-parity check, ready to run on the real enet.pb.
"""
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

sys.path.insert(0, str(Path(__file__).parent))
from graph_writer import GraphBuilder, with_biases, write_enet_graphdef  # noqa: E402

from bugcar_image_segmentation_amd import enet_spec, graphdef  # noqa: E402
from oracle import enet_oracle as eo  # noqa: E402
from oracle import tf_graph  # noqa: E402

H, W = 48, 64


@pytest.fixture(scope="module")
def net():
    return with_biases(enet_spec.build_enet())


@pytest.fixture(scope="module")
def x():
    return np.random.default_rng(0).normal(0, 1, (1, 3, H, W)).astype(np.float32)


def test_wire_format_round_trip():
    g = GraphBuilder()
    c = g.const(np.arange(6, dtype=np.float32).reshape(2, 3))
    g.node("Conv2D", [c, c], name="conv", strides=[1, 2, 2, 1], padding="SAME", data_format="NHWC", epsilon=1e-3,
           flag=True, T=("type", 1))
    nodes = graphdef.parse_graphdef(g.bytes())
    assert [n.op for n in nodes] == ["Const", "Conv2D"]
    assert np.array_equal(nodes[0].attr["value"], np.arange(6, dtype=np.float32).reshape(2, 3))
    a = nodes[1].attr
    assert a["strides"] == [1, 2, 2, 1] and a["padding"] == b"SAME" and abs(a["epsilon"] - 1e-3) < 1e-9
    assert a["flag"] is True and a["T"] == ("type", 1) and nodes[1].inputs == [nodes[0].name] * 2


def test_tensor_proto_value_fields():
    """TensorProto with typed *_val fields instead of tensor_content, last value repeated."""
    from graph_writer import _int, _key, _ld, _shape
    import struct
    body = _int(1, 1) + _ld(2, _shape([4])) + _ld(5, struct.pack("<2f", 1.5, -2.0))
    assert np.array_equal(graphdef.parse_tensor(body), np.array([1.5, -2, -2, -2], np.float32))
    body = _int(1, 3) + _ld(2, _shape([3])) + _key(7, 0) + bytes([7])
    assert np.array_equal(graphdef.parse_tensor(body), np.array([7, 7, 7], np.int32))


@pytest.mark.parametrize("style", ["nhwc", "nchw"])
def test_interpreter_matches_enet_oracle(net, x, style):
    pb = write_enet_graphdef(net, H, W, style)
    got = tf_graph.run(pb, {"input0": x}, "CATkrIDy/concat:0")
    ref = eo.forward(net, x, torch.float64)
    assert got.shape == (1, enet_spec.NUM_CLASSES, H, W)
    assert np.abs(got - ref).max() < 1e-9


@pytest.mark.parametrize("style", ["nhwc", "nchw"])
@pytest.mark.parametrize("fullconv_k,pool_k", [(3, 3), (2, 2)])
def test_import_reproduces_network(style, fullconv_k, pool_k, x):
    blocks = with_biases(enet_spec.build_enet(fullconv_k=fullconv_k, initial_pool_k=pool_k), seed=fullconv_k)
    pb = write_enet_graphdef(blocks, H, W, style)
    imp = graphdef.import_enet(pb)
    assert [b.type for b in imp] == [b.type for b in blocks]
    for bi, bo in zip(imp, blocks):
        assert bi.attrs == bo.attrs
        for ui, uo in zip(bi.units, bo.units):
            assert (ui.kind, ui.cout, ui.cin, ui.kh, ui.kw, ui.stride, ui.pad_h, ui.pad_w, ui.dil_h, ui.out_pad) == \
                   (uo.kind, uo.cout, uo.cin, uo.kh, uo.kw, uo.stride, uo.pad_h, uo.pad_w, uo.dil_h, uo.out_pad)
            assert np.array_equal(ui.w, uo.w)
            assert np.allclose(ui.slope, uo.slope)
    ref = eo.forward(blocks, x, torch.float64)
    got = eo.forward(imp, x, torch.float64)
    assert np.abs(got - ref).max() < 1e-5 * np.abs(ref).max()
    blob = graphdef.graphdef_to_blob(pb)
    assert blob[:4] == b"BSG1"


def test_not_a_graph_and_truncated_graph():
    with pytest.raises(graphdef.GraphImportError):
        graphdef.import_enet(b"")
    assert not graphdef.looks_like_graphdef(b"BSG1\0\0\0\0")


def test_missing_layer_is_named(net):
    """A graph that is not the canonical ENet: the first shape mismatch is reported."""
    short = [b for b in net if b.name != "regular4_1"]     # (after both downsampling blocks: pool_ref stays valid)
    pb = write_enet_graphdef(short, H, W, "nhwc")
    with pytest.raises(graphdef.GraphImportError, match="conv|convolutions"):
        graphdef.import_enet(pb)


def test_non_prelu_activation_rejected(net):
    """A closure that is not act(a x + b) with a piecewise-linear activation (here a sigmoid after
    the classifier's bias) is rejected rather than silently mis-imported."""
    g = GraphBuilder()
    x = g.node("Placeholder", [], name="input0", dtype=("type", 1), shape=("shape", [1, 1, 1, 4]))
    y = g.node("Conv2D", [x, g.const(np.ones((1, 1, 4, 4), np.float32))], strides=[1, 1, 1, 1], padding="VALID",
               data_format="NHWC", T=("type", 1))
    g.node("Sigmoid", [y], T=("type", 1))
    gr = graphdef.Graph(graphdef.parse_graphdef(g.bytes()))
    with pytest.raises(graphdef.GraphImportError):
        graphdef.probe_affine_act(gr, y, (1, 1, 1, 4), False)


def test_probe_recovers_bn_and_prelu_exactly():
    """Probing a FusedBatchNormV3 + PReLU closure returns the folded affine and the slope."""
    rng = np.random.default_rng(1)
    C = 8
    gamma, beta, mean, var = rng.uniform(0.5, 1.5, C), rng.normal(0, 0.1, C), rng.normal(0, 0.1, C), rng.uniform(0.5, 1.5, C)
    gamma[0] = -0.7                                    # a negative scale flips the kink's side
    slope = rng.uniform(0, 0.5, C)
    g = GraphBuilder()
    x = g.node("Placeholder", [], name="input0", dtype=("type", 1), shape=("shape", [1, 2, 2, C]))
    f = lambda a: g.const(np.asarray(a, np.float32))  # noqa: E731
    y = g.node("FusedBatchNormV3", [x, f(gamma), f(beta), f(mean), f(var)], epsilon=1e-3, data_format="NHWC",
               T=("type", 1))
    pos = g.node("Relu", [y])
    neg = g.node("Mul", [f(-slope), g.node("Relu", [g.node("Neg", [y])])])
    g.node("AddV2", [pos, neg])
    gr = graphdef.Graph(graphdef.parse_graphdef(g.bytes()))
    a, b, s, _ = graphdef.probe_affine_act(gr, "input0", (1, 2, 2, C), False)
    g32 = lambda v: np.asarray(v, np.float32).astype(np.float64)  # noqa: E731
    ea = g32(gamma) / np.sqrt(g32(var) + np.float32(1e-3))
    assert np.allclose(a, ea, rtol=1e-6) and np.allclose(b, g32(beta) - g32(mean) * ea, atol=1e-6)
    assert np.allclose(s, g32(slope), atol=1e-6)
