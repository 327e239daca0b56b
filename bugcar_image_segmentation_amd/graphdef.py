"""Frozen TensorFlow GraphDef (.pb) -> the engine's ENet block list.

The reference loads ``pretrained_models/enet.pb`` with ``GraphDef.ParseFromString`` +
``tf.import_graph_def`` and runs it with ``sess.run`` (models.py:21-31, 42-44). The graph is frozen
(utils.py:47-83: variables turned into Const nodes), so every weight is a Const (or a constant
sub-expression: Identity / Transpose / Reshape / arithmetic on Consts). This module reads that file
without TensorFlow and emits the canonical ENet block list of ``enet_spec`` (which the engine
serialises to BSG1), so ``ENET("enet.pb")`` works as in the reference.

How the graph is read (host, load time — nothing here is on the per-frame path):

* a minimal protobuf wire-format reader for GraphDef / NodeDef / AttrValue / TensorProto
  (``google.protobuf`` is present but TensorFlow's .proto descriptors are not);
* constant folding of any sub-graph that depends only on Consts (``Graph.const``);
* convolutions (``Conv2D``, ``Conv2DBackpropInput``) in graph order; their filters are folded and
  re-laid out to OIHW / IOHW, their geometry (strides, dilations, padding — ``SAME`` / ``VALID`` /
  ``EXPLICIT`` or an explicit ``Pad`` feeding them, and the crop that follows a ``VALID``
  transposed convolution) read from the attributes and the neighbouring ops;
* everything between a convolution and the next non-elementwise op (bias, batch norm in any
  encoding — FusedBatchNorm or explicit Sub/Mul/Rsqrt/Add — and the activation, whatever ops
  encode PReLU / ReLU) is an elementwise closure that is PROBED rather than pattern-matched: it is
  evaluated per channel at points right and left of its kink, which gives the per-channel affine
  (a, b) and the negative-side slope s of act(a x + b) — the unit's folded batch norm and PReLU
  slope. A closure that is not of that form (e.g. a sigmoid) is rejected;
* the units are assigned to the canonical ENet layout (``enet_spec.canonical_enet_layout``) in
  order, checking every shape; a graph that is not the canonical ENet raises ``GraphImportError``
  naming the first mismatch.

Unpinned: no enet.pb exists in this image (``.MISSING_LARGE_BLOBS:2``). The importer is exercised
on GraphDefs written from the synthetic weights in two encodings (tests/graph_writer.py), and its
output is checked numerically against a NumPy interpreter of the same GraphDef
(oracle/tf_graph.py) — the check to run on the real file once it is supplied.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

import numpy as np

from . import enet_spec as S


class GraphImportError(ValueError):
    pass


# ---------------------------------------------------------------------------------------------
# protobuf wire format
DT_NP = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64,
         10: np.bool_, 19: np.float16}


def _varint(b: bytes, i: int):
    r = s = 0
    while True:
        c = b[i]
        i += 1
        r |= (c & 0x7F) << s
        if c < 0x80:
            return r, i
        s += 7


def _fields(b: bytes):
    """Yield (field number, wire type, value) of one message; value is int for varint / fixed,
    bytes for length-delimited."""
    i, n = 0, len(b)
    while i < n:
        key, i = _varint(b, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(b, i)
        elif wt == 1:
            v = struct.unpack_from("<Q", b, i)[0]
            i += 8
        elif wt == 2:
            ln, i = _varint(b, i)
            v = b[i:i + ln]
            i += ln
        elif wt == 5:
            v = struct.unpack_from("<I", b, i)[0]
            i += 4
        else:
            raise GraphImportError(f"unsupported protobuf wire type {wt}")
        yield f, wt, v


def _signed(v: int) -> int:
    return v - (1 << 64) if v >= 1 << 63 else v


def _packed_varints(wt, v):
    if wt == 2:
        out, i = [], 0
        while i < len(v):
            x, i = _varint(v, i)
            out.append(_signed(x))
        return out
    return [_signed(v)]


def _packed_floats(wt, v, fmt="<f", size=4):
    if wt == 2:
        return list(struct.unpack(f"<{len(v) // size}{fmt[-1]}", v))
    return [struct.unpack(fmt, struct.pack("<I" if size == 4 else "<Q", v))[0]]


def _shape(b: bytes):
    dims = []
    for f, _, v in _fields(b):
        if f == 2:
            size = -1
            for f2, _, v2 in _fields(v):
                if f2 == 1:
                    size = _signed(v2)
            dims.append(size)
        elif f == 3 and v:
            return None
    return tuple(dims)


def parse_tensor(b: bytes) -> np.ndarray:
    """TensorProto -> ndarray (tensor_content or the typed *_val fields, broadcast as TF does)."""
    dtype, shape, content = 1, (), None
    vals: list = []
    for f, wt, v in _fields(b):
        if f == 1:
            dtype = v
        elif f == 2:
            shape = _shape(v) or ()
        elif f == 4:
            content = v
        elif f == 5:
            vals += _packed_floats(wt, v)
        elif f == 6:
            vals += _packed_floats(wt, v, "<d", 8)
        elif f in (7, 10, 11):
            vals += _packed_varints(wt, v)
        elif f == 13:
            vals += [np.frombuffer(struct.pack("<H", x & 0xFFFF), np.float16)[0] for x in _packed_varints(wt, v)]
    if dtype not in DT_NP:
        raise GraphImportError(f"unsupported tensor dtype {dtype}")
    dt = DT_NP[dtype]
    n = int(np.prod(shape)) if shape else 1
    if content is not None:
        return np.frombuffer(content, dt).reshape(shape).copy()
    a = np.asarray(vals, dtype=dt)
    if a.size == n:
        return a.reshape(shape)
    if a.size == 0:
        return np.zeros(shape, dt)
    full = np.empty(n, dt)                 # TF repeats the last value to fill the tensor
    full[:a.size] = a
    full[a.size:] = a[-1]
    return full.reshape(shape)


def _attr(b: bytes):
    for f, wt, v in _fields(b):
        if f == 1:                         # ListValue
            lst: dict = {"s": [], "i": [], "f": [], "type": [], "shape": []}
            for f2, wt2, v2 in _fields(v):
                if f2 == 2:
                    lst["s"].append(v2)
                elif f2 == 3:
                    lst["i"] += _packed_varints(wt2, v2)
                elif f2 == 4:
                    lst["f"] += _packed_floats(wt2, v2)
                elif f2 == 6:
                    lst["type"] += _packed_varints(wt2, v2)
                elif f2 == 7:
                    lst["shape"].append(_shape(v2))
            return next((x for x in lst.values() if x), [])
        if f == 2:
            return v                        # bytes
        if f == 3:
            return _signed(v)
        if f == 4:
            return struct.unpack("<f", struct.pack("<I", v))[0]
        if f == 5:
            return bool(v)
        if f == 6:
            return ("type", v)
        if f == 7:
            return _shape(v)
        if f == 8:
            return parse_tensor(v)
    return None


@dataclass
class Node:
    name: str
    op: str
    inputs: list = field(default_factory=list)
    attr: dict = field(default_factory=dict)


def parse_graphdef(data: bytes) -> list:
    """GraphDef bytes -> [Node] in file order (control inputs '^x' dropped)."""
    nodes = []
    for f, _, v in _fields(data):
        if f != 1:
            continue
        n = Node("", "")
        for f2, _, v2 in _fields(v):
            if f2 == 1:
                n.name = v2.decode()
            elif f2 == 2:
                n.op = v2.decode()
            elif f2 == 3:
                s = v2.decode()
                if not s.startswith("^"):
                    n.inputs.append(s)
            elif f2 == 5:
                key, val = None, None
                for f3, _, v3 in _fields(v2):
                    if f3 == 1:
                        key = v3.decode()
                    elif f3 == 2:
                        val = _attr(v3)
                n.attr[key] = val
        nodes.append(n)
    if not nodes:
        raise GraphImportError("not a GraphDef (no nodes)")
    return nodes


def looks_like_graphdef(data: bytes) -> bool:
    try:
        nodes = parse_graphdef(data[:1 << 20] if len(data) > 1 << 20 else data)
    except Exception:
        return False
    return all(n.op for n in nodes[:8])


# ---------------------------------------------------------------------------------------------
# the graph: lookup, constant folding, elementwise evaluation
def _src(name: str):
    """'node:1' -> ('node', 1)."""
    if ":" in name:
        a, b = name.rsplit(":", 1)
        if b.isdigit():
            return a, int(b)
    return name, 0


def _s(v):
    return v.decode() if isinstance(v, bytes) else v


def _bcast_binary(op):
    return {"Add": np.add, "AddV2": np.add, "BiasAdd": None, "Sub": np.subtract, "Mul": np.multiply,
            "RealDiv": np.divide, "Div": np.divide, "Maximum": np.maximum, "Minimum": np.minimum,
            "Less": np.less, "Greater": np.greater, "LessEqual": np.less_equal,
            "GreaterEqual": np.greater_equal, "SquaredDifference": lambda a, b: (a - b) ** 2}.get(op)


UNARY = {"Identity": lambda x: x, "Neg": np.negative, "Relu": lambda x: np.maximum(x, 0),
         "Relu6": lambda x: np.clip(x, 0, 6), "Abs": np.abs, "Rsqrt": lambda x: 1 / np.sqrt(x),
         "Sqrt": np.sqrt, "Square": np.square, "Reciprocal": lambda x: 1 / x, "Sigmoid": lambda x: 1 / (1 + np.exp(-x)),
         "StopGradient": lambda x: x, "Snapshot": lambda x: x}
BINARY_OPS = {"Add", "AddV2", "BiasAdd", "Sub", "Mul", "RealDiv", "Div", "Maximum", "Minimum", "Less", "Greater",
              "LessEqual", "GreaterEqual", "SquaredDifference"}
# ops whose output is an elementwise function of their non-constant input(s)
ELEMENTWISE = set(UNARY) | BINARY_OPS | {"Select", "SelectV2", "Cast", "LeakyRelu", "FusedBatchNorm",
                                         "FusedBatchNormV2", "FusedBatchNormV3", "ZerosLike", "OnesLike"}


def eval_op(node: Node, args: list):
    """NumPy semantics of the constant-foldable and elementwise TF ops (float64 math for floats)."""
    op = node.op
    if op in UNARY:
        return UNARY[op](args[0])
    if op == "BiasAdd":
        x, b = args
        if _s(node.attr.get("data_format", b"NHWC")) == "NCHW":
            return x + b.reshape((1, -1) + (1,) * (x.ndim - 2))
        return x + b
    f = _bcast_binary(op)
    if f is not None:
        return f(args[0], args[1])
    if op in ("Select", "SelectV2"):
        c, a, b = args
        if op == "Select" and c.ndim == 1 and a.ndim > 1:
            c = c.reshape((-1,) + (1,) * (a.ndim - 1))
        return np.where(c, a, b)
    if op == "Cast":
        dt = DT_NP.get(node.attr.get("DstT", ("type", 1))[1], np.float32)
        return args[0].astype(np.float64 if dt in (np.float32, np.float64) else dt)
    if op == "LeakyRelu":
        al = node.attr.get("alpha", 0.2)
        return np.where(args[0] >= 0, args[0], al * args[0])
    if op in ("FusedBatchNorm", "FusedBatchNormV2", "FusedBatchNormV3"):
        x, sc, of, mu, var = args[:5]
        eps = node.attr.get("epsilon", 1e-4)
        shp = (1, -1, 1, 1) if _s(node.attr.get("data_format", b"NHWC")) == "NCHW" else (1, 1, 1, -1)
        r = lambda t: np.asarray(t, np.float64).reshape(shp)  # noqa: E731
        return (x - r(mu)) / np.sqrt(r(var) + eps) * r(sc) + r(of)
    if op == "ZerosLike":
        return np.zeros_like(args[0])
    if op == "OnesLike":
        return np.ones_like(args[0])
    if op == "Transpose":
        return np.transpose(args[0], [int(i) for i in args[1]])
    if op == "Reshape":
        return np.reshape(args[0], [int(i) for i in np.atleast_1d(args[1])])
    if op == "ExpandDims":
        return np.expand_dims(args[0], int(args[1]))
    if op == "Squeeze":
        dims = node.attr.get("squeeze_dims") or []
        return np.squeeze(args[0], axis=tuple(dims) if dims else None)
    if op == "ConcatV2":
        return np.concatenate(args[:-1], axis=int(args[-1]))
    if op == "Pack":
        return np.stack(args, axis=int(node.attr.get("axis", 0)))
    if op == "Shape":
        return np.asarray(args[0].shape, np.int32)
    if op == "Fill":
        return np.full([int(i) for i in args[0]], args[1])
    if op == "Range":
        return np.arange(args[0], args[1], args[2])
    if op == "Prod":
        return np.prod(args[0], axis=tuple(np.atleast_1d(args[1]).astype(int)), keepdims=bool(node.attr.get("keep_dims")))
    if op == "FloorDiv":
        return np.floor_divide(args[0], args[1])
    if op == "FloorMod":
        return np.mod(args[0], args[1])
    raise GraphImportError(f"cannot evaluate op {op} ({node.name})")


class Graph:
    """Nodes by name, consumers, and constant folding."""

    def __init__(self, nodes: list):
        self.nodes = nodes
        self.by = {n.name: n for n in nodes}
        self.order = {n.name: i for i, n in enumerate(nodes)}
        self.consumers: dict = {n.name: [] for n in nodes}
        for n in nodes:
            for s in n.inputs:
                src = _src(s)[0]
                if src in self.consumers:
                    self.consumers[src].append(n)
        self._const: dict = {}

    def node(self, name: str) -> Node:
        n = self.by.get(_src(name)[0])
        if n is None:
            raise GraphImportError(f"graph references a missing node {name}")
        return n

    def is_const(self, name: str) -> bool:
        try:
            self.const(name)
            return True
        except GraphImportError:
            return False

    def const(self, name: str):
        """Value of tensor `name` if it depends only on Const nodes, else GraphImportError."""
        key = name if ":" in name else name + ":0"
        if key in self._const:
            v = self._const[key]
            if isinstance(v, GraphImportError):
                raise v
            return v
        n = self.node(name)
        try:
            if n.op == "Const":
                v = n.attr["value"]
                v = v.astype(np.float64) if v.dtype.kind == "f" else v
            elif n.op in ("Placeholder", "PlaceholderWithDefault", "VariableV2", "VarHandleOp"):
                raise GraphImportError(f"{n.name} is not constant")
            elif n.op in ("Split", "SplitV", "Unpack"):
                raise GraphImportError(f"{n.op} is not folded")
            else:
                v = eval_op(n, [self.const(s) for s in n.inputs])
        except GraphImportError as e:
            self._const[key] = e
            raise
        self._const[key] = v
        return v

    def producer_chain(self, name: str, ops: set):
        """Follow single-input pass-through ops (Identity, ...) back from `name`."""
        n = self.node(name)
        while n.op in ops and n.inputs:
            n = self.node(n.inputs[0])
        return n


# ---------------------------------------------------------------------------------------------
# convolutions and their elementwise closures
CONV_OPS = ("Conv2D", "Conv2DBackpropInput", "DepthwiseConv2dNative")
PASS = {"Identity", "StopGradient", "Snapshot"}


@dataclass
class ConvInfo:
    node: Node
    kind: int                 # UNIT_CONV / UNIT_TCONV
    w: np.ndarray             # OIHW (conv) / IOHW (tconv)
    stride: int
    dil: int
    pad: tuple                # (top, bottom, left, right)
    nchw: bool
    out: str                  # tensor the unit's output closure starts from
    out_pad: int = 0


def _geom_attr(node: Node, key: str, nchw: bool):
    v = node.attr.get(key) or [1, 1, 1, 1]
    v = [int(x) for x in v]
    return (v[2], v[3]) if nchw else (v[1], v[2])


def _same_pad(inp: int, k: int, s: int, d: int):
    ke = (k - 1) * d + 1
    out = -(-inp // s)
    tot = max((out - 1) * s + ke - inp, 0)
    return tot // 2, tot - tot // 2


def _conv_info(g: Graph, n: Node, shapes: dict) -> ConvInfo:
    nchw = _s(n.attr.get("data_format", b"NHWC")) == "NCHW"
    sh, sw = _geom_attr(n, "strides", nchw)
    dh, dw = _geom_attr(n, "dilations", nchw)
    if sh != sw or dh != dw:
        raise GraphImportError(f"{n.name}: anisotropic stride/dilation is not an ENet layer")
    padding = _s(n.attr.get("padding", b"VALID"))
    if n.op == "Conv2DBackpropInput":
        osz_name, filt_name, x_name = n.inputs
        w = g.const(filt_name)                          # [kh, kw, out, in]
        w = np.transpose(w, (3, 2, 0, 1))               # -> IOHW
        kind = S.UNIT_TCONV
    else:
        x_name, filt_name = n.inputs[:2]
        w = g.const(filt_name)                          # HWIO
        w = np.transpose(w, (3, 2, 0, 1))               # -> OIHW
        kind = S.UNIT_CONV
    pad = (0, 0, 0, 0)
    if padding == "EXPLICIT":
        ep = [int(x) for x in n.attr.get("explicit_paddings", [0] * 8)]
        pad = (ep[4], ep[5], ep[6], ep[7]) if nchw else (ep[2], ep[3], ep[4], ep[5])
    elif padding == "SAME" and kind == S.UNIT_CONV:
        ih, iw = shapes[x_name][2:4] if nchw else shapes[x_name][1:3]
        pad = _same_pad(ih, w.shape[2], sh, dh) + _same_pad(iw, w.shape[3], sw, dw)
    # an explicit Pad feeding the convolution (the ONNX -> TF encoding of conv padding)
    if kind == S.UNIT_CONV:
        src = g.producer_chain(x_name, PASS)
        if src.op in ("Pad", "PadV2") and g.is_const(src.inputs[1]):
            pv = g.const(src.inputs[1]).astype(int)
            if len(src.inputs) == 3 and float(g.const(src.inputs[2])) != 0.0:
                raise GraphImportError(f"{src.name}: non-zero constant padding")
            ph, pw = (pv[2], pv[3]) if nchw else (pv[1], pv[2])
            if pv[0].any() or (pv[1] if nchw else pv[3]).any():
                raise GraphImportError(f"{src.name}: padding on batch/channel axes feeding a conv")
            pad = (pad[0] + ph[0], pad[1] + ph[1], pad[2] + pw[0], pad[3] + pw[1])
    out = n.name
    out_pad = 0
    if kind == S.UNIT_TCONV:
        # the output size of the transposed convolution and any crop after it give (pad, out_pad)
        oshape = [int(x) for x in g.const(osz_name)]
        ih, iw = shapes[x_name][2:4] if nchw else shapes[x_name][1:3]
        oh, ow = (oshape[2], oshape[3]) if nchw else (oshape[1], oshape[2])
        kh = w.shape[2]
        # out[y] = full[y + th], full[j] = sum over i*s + k == j; th = the forward conv's leading pad
        # for an output of oshape (0 for VALID)
        th = _same_pad(oh, kh, sh, 1)[0] if padding == "SAME" else 0
        tw = _same_pad(ow, w.shape[3], sw, 1)[0] if padding == "SAME" else 0
        ch, cw = oh, ow
        cons = [c for c in g.consumers[n.name] if c.op not in PASS]
        if len(cons) == 1 and cons[0].op in ("Slice", "StridedSlice"):
            sl = cons[0]
            begin = [int(x) for x in g.const(sl.inputs[1])]
            size = [int(x) for x in g.const(sl.inputs[2])]
            if sl.op == "StridedSlice":
                size = [(e if e > 0 else oshape[i] + e) - b for i, (b, e) in enumerate(zip(begin, size))]
            size = [oshape[i] - begin[i] if sz == -1 else sz for i, sz in enumerate(size)]
            bh, bw = (begin[2], begin[3]) if nchw else (begin[1], begin[2])
            ch, cw = (size[2], size[3]) if nchw else (size[1], size[2])
            th, tw = th + bh, tw + bw
            out = sl.name
        # PyTorch / ONNX ConvTranspose(p, out_pad): out[y] = full[y + p], (ih-1)*s - 2p + k + out_pad rows
        p = th
        op_ = ch - ((ih - 1) * sh - 2 * p + kh)
        op_w = cw - ((iw - 1) * sw - 2 * tw + w.shape[3])
        if th != tw or op_ != op_w or not (0 <= op_ < sh) or p < 0:
            raise GraphImportError(f"{n.name}: transposed-conv output crop ({th},{tw}) -> {ch}x{cw} is not a "
                                   "(pad, out_pad) pair")
        pad = (p, p, p, p)
        out_pad = op_
    if pad[0] != pad[1] and not (kind == S.UNIT_CONV and sh == 2 and pad[0] + 1 == pad[1]) or pad[2] != pad[3] \
            and not (kind == S.UNIT_CONV and sh == 2 and pad[2] + 1 == pad[3]):
        raise GraphImportError(f"{n.name}: asymmetric padding {pad}")
    return ConvInfo(n, kind, np.ascontiguousarray(w, np.float32), sh, dh, pad, nchw, out, out_pad)


def elementwise_closure(g: Graph, root: str, act_ends: bool = False):
    """Nodes reachable from tensor `root` through elementwise ops whose other inputs are constant or
    inside the closure, and its single exit (the node whose value leaves the closure).
    Single-input Concat / identity-like ops are pass-through. act_ends: nothing past an activation
    (Relu / Relu6) joins, and an activation joins only as the sole consumer of its input — a ReLU
    that also has an un-rectified reader beside it belongs to the next layer (pre-activation nets)."""
    inside = {_src(root)[0]}
    members: list = []
    acts = set()
    changed = True
    while changed:
        changed = False
        for name in list(inside):
            for c in g.consumers.get(name, []):
                if c.name in inside:
                    continue
                ok = c.op in ELEMENTWISE or (c.op == "ConcatV2" and len(c.inputs) == 2)
                if not ok:
                    continue
                data_in = c.inputs[:-1] if c.op == "ConcatV2" else c.inputs
                if c.op.startswith("FusedBatchNorm"):
                    data_in = c.inputs[:1]
                    if not all(g.is_const(s) for s in c.inputs[1:5]):
                        continue
                if act_ends:
                    if any(_src(s)[0] in acts for s in data_in):
                        continue
                    if c.op in ("Relu", "Relu6") and len(g.consumers.get(_src(c.inputs[0])[0], [])) != 1:
                        continue
                if all(_src(s)[0] in inside or g.is_const(s) for s in data_in):
                    inside.add(c.name)
                    members.append(c)
                    if c.op in ("Relu", "Relu6"):
                        acts.add(c.name)
                    changed = True
    # exits: members (or the root) consumed outside the closure, or not consumed at all
    exits = []
    for name in [_src(root)[0]] + [m.name for m in members]:
        cons = g.consumers.get(name, [])
        if not cons or any(c.name not in inside for c in cons):
            exits.append(name)
    return members, exits


def _run_closure(g: Graph, root: str, members: list, x: np.ndarray, exit_name: str):
    vals = {_src(root)[0]: x}

    def get(s):
        nm, idx = _src(s)
        if nm in vals:
            return vals[nm]
        return g.const(s)

    for m in sorted(members, key=lambda n: g.order[n.name]):
        args = [get(s) for s in m.inputs]
        vals[m.name] = eval_op(m, args) if m.op != "ConcatV2" else args[0]
    return vals[exit_name]


def probe_affine_act(g: Graph, root: str, shape: tuple, nchw: bool):
    """The closure after tensor `root` (shape `shape`) as act(a*x + b) per channel:
    -> (a, b, s, exit node name). s = negative-side slope (PReLU); checked piecewise linear."""
    members, exits = elementwise_closure(g, root)
    if len(exits) != 1:
        raise GraphImportError(f"the ops after {root} leave through {len(exits)} tensors ({exits})")
    ex = exits[0]
    C = shape[1] if nchw else shape[-1]
    cshape = (1, C, 1, 1) if nchw else (1, 1, 1, C)

    def f(v):
        x = np.broadcast_to(np.asarray(v, np.float64).reshape(cshape), (1,) + tuple(shape[1:])).copy()
        y = _run_closure(g, root, members, x, ex)
        y = np.asarray(y, np.float64)
        return y[0, :, 0, 0] if nchw else y[0, 0, 0, :]

    if not members:
        return np.ones(C), np.zeros(C), np.ones(C), ex
    zero = f(np.zeros(C))
    big = 1e4
    # find the kink: a*x + b = 0. Probe far right / far left to get both slopes.
    fr1, fr2 = f(np.full(C, big)), f(np.full(C, 2 * big))
    fl1, fl2 = f(np.full(C, -big)), f(np.full(C, -2 * big))
    sr, sl = (fr2 - fr1) / big, (fl1 - fl2) / big
    # for a > 0 the right side is the positive branch (slope a); for a < 0 it is the left side
    a = np.where(np.abs(sr) >= np.abs(sl), sr, sl)
    pos_right = np.abs(sr) >= np.abs(sl)
    s = np.where(pos_right, np.divide(sl, sr, out=np.ones(C), where=sr != 0),
                 np.divide(sr, sl, out=np.ones(C), where=sl != 0))
    b = np.where(pos_right, fr1 - sr * big, fl1 + sl * big)
    # check: act(a x + b) reproduces the closure at points around the kink
    for t in (-3.0, -1.0, -0.25, 0.5, 2.0):
        x = np.where(a != 0, (t - b) / np.where(a != 0, a, 1), t)
        want = f(x)
        z = a * x + b
        got = np.where(z >= 0, z, s * z)
        if not np.allclose(want, got, rtol=1e-6, atol=1e-6 * (1 + np.abs(want))):
            raise GraphImportError(f"the ops after {root} are not act(a*x + b) with a PReLU/ReLU activation")
    if not np.allclose(f(np.zeros(C)), zero):
        raise GraphImportError(f"the ops after {root} are not deterministic")
    return a, b, s, ex


# ---------------------------------------------------------------------------------------------
# shapes by propagation (only what the importer needs: conv / pool / pad / concat / reshape)
def infer_shapes(g: Graph, input_name: str, input_shape: tuple) -> dict:
    """Static shapes of every tensor reachable from the input, computed without data."""
    shp = {input_name: tuple(input_shape), _src(input_name)[0]: tuple(input_shape)}

    def get(s):
        nm, idx = _src(s)
        if s in shp:
            return shp[s]
        if idx == 0 and nm in shp:
            return shp[nm]
        if f"{nm}:{idx}" in shp:
            return shp[f"{nm}:{idx}"]
        if g.is_const(s):
            return tuple(np.shape(g.const(s)))
        return None

    for n in g.nodes:
        if n.name in shp:
            continue
        ins = [get(s) for s in n.inputs]
        if n.op == "Const" or any(i is None for i in ins[:1]):
            continue
        x = ins[0]
        op = n.op
        out = None
        if op in ELEMENTWISE or op == "BiasAdd":
            cand = [i for i in ins[:2] if i is not None and len(i) == len(x)]
            out = tuple(max(d) for d in zip(*cand)) if cand else x
        elif op in ("Conv2D", "DepthwiseConv2dNative", "MaxPool", "MaxPoolWithArgmax", "AvgPool"):
            nchw = _s(n.attr.get("data_format", b"NHWC")) == "NCHW"
            sh, _ = _geom_attr(n, "strides", nchw)
            dh, _ = _geom_attr(n, "dilations", nchw) if op != "MaxPool" else (1, 1)
            if op.startswith("MaxPool") or op == "AvgPool":
                k = _geom_attr(n, "ksize", nchw)[0]
                cout = x[1] if nchw else x[3]
            else:
                w = g.const(n.inputs[1])
                k = w.shape[0]
                cout = w.shape[3] if op == "Conv2D" else w.shape[2] * w.shape[3]
            H, W = (x[2], x[3]) if nchw else (x[1], x[2])
            padding = _s(n.attr.get("padding", b"VALID"))
            if padding == "SAME":
                oh, ow = -(-H // sh), -(-W // sh)
            else:
                ph = pw = 0
                if padding == "EXPLICIT":
                    ep = [int(v) for v in n.attr.get("explicit_paddings")]
                    ph, pw = (ep[4] + ep[5], ep[6] + ep[7]) if nchw else (ep[2] + ep[3], ep[4] + ep[5])
                ke = (k - 1) * dh + 1
                oh, ow = (H + ph - ke) // sh + 1, (W + pw - ke) // sh + 1
            out = (x[0], cout, oh, ow) if nchw else (x[0], oh, ow, cout)
            if op == "MaxPoolWithArgmax":
                shp[f"{n.name}:1"] = out
        elif op == "Conv2DBackpropInput":
            out = tuple(int(v) for v in g.const(n.inputs[0]))
        elif op in ("Pad", "PadV2", "MirrorPad"):
            pv = g.const(n.inputs[1]).astype(int)
            out = tuple(d + p[0] + p[1] for d, p in zip(x, pv))
        elif op == "ConcatV2":
            ax = int(g.const(n.inputs[-1]))
            parts = [i for i in ins[:-1]]
            if any(p is None for p in parts):
                continue
            ax = ax % len(parts[0])
            out = tuple(sum(p[ax] for p in parts) if d == ax else parts[0][d] for d in range(len(parts[0])))
        elif op == "Transpose":
            perm = [int(v) for v in g.const(n.inputs[1])]
            out = tuple(x[p] for p in perm)
        elif op == "Reshape":
            tgt = [int(v) for v in g.const(n.inputs[1])]
            if -1 in tgt:
                k = int(np.prod([t for t in tgt if t != -1]))
                tgt[tgt.index(-1)] = int(np.prod(x)) // max(k, 1)
            out = tuple(tgt)
        elif op in ("Slice",):
            size = [int(v) for v in g.const(n.inputs[2])]
            begin = [int(v) for v in g.const(n.inputs[1])]
            out = tuple(d - b if s == -1 else s for d, b, s in zip(x, begin, size))
        elif op == "StridedSlice":
            b = [int(v) for v in g.const(n.inputs[1])]
            e = [int(v) for v in g.const(n.inputs[2])]
            out = tuple((ei if ei > 0 else d + ei) - bi for d, bi, ei in zip(x, b, e))
        elif op == "ScatterNd":
            out = tuple(int(v) for v in g.const(n.inputs[2]))
        elif op in ("Identity", "StopGradient", "Snapshot"):
            out = x
        if out is not None:
            shp[n.name] = out
            shp[f"{n.name}:0"] = out
    return shp


# ---------------------------------------------------------------------------------------------
# the ENet import
def _find_input(g: Graph, name: str | None):
    if name:
        return g.node(name).name
    ph = [n for n in g.nodes if n.op == "Placeholder"]
    if len(ph) != 1:
        raise GraphImportError(f"expected one Placeholder input, found {[n.name for n in ph]}")
    return ph[0].name


def import_enet(data: bytes, input_name: str | None = None, input_shape: tuple | None = None,
                num_classes: int | None = None) -> list:
    """Frozen ENet GraphDef -> enet_spec block list (weights only; topology checked against the
    canonical layout). input_shape: the feed's NCHW shape (models.py:94: (1, 3, 256, 512))."""
    g = Graph(parse_graphdef(data))
    inp = _find_input(g, input_name)
    in_node = g.node(inp)
    shape = input_shape
    if shape is None:
        s = in_node.attr.get("shape")
        shape = tuple(d if d and d > 0 else 1 for d in s) if s else (1, 3, 256, 512)
        if not s or any(d is None or d <= 0 for d in s[1:]):
            shape = (1, 3, 256, 512)
    shapes = infer_shapes(g, inp, tuple(shape))
    convs = [n for n in g.nodes if n.op in CONV_OPS and n.name in shapes]
    if any(n.op == "DepthwiseConv2dNative" for n in convs):
        raise GraphImportError("depthwise convolutions are not part of ENet")
    infos = [_conv_info(g, n, shapes) for n in convs]

    def unit_from(ci: ConvInfo, affine=None):
        """Unit with the conv's closure probed (or the given affine/act for the initial block)."""
        w = ci.w
        if ci.kind == S.UNIT_CONV:
            cout, cin, kh, kw = w.shape
        else:
            cin, cout, kh, kw = w.shape
        if affine is None:
            oshape = shapes.get(ci.out) or shapes.get(ci.node.name)
            a, b, s, ex = probe_affine_act(g, ci.out, oshape, ci.nchw)
        else:
            a, b, s, ex = affine
        u = S.Unit(ci.kind, cout, cin, kh, kw, ci.stride, ci.pad[0], ci.pad[2], ci.dil, ci.dil, ci.out_pad, 0.0,
                   w, np.zeros(cout, np.float32), a.astype(np.float32), b.astype(np.float32),
                   np.zeros(cout, np.float32), np.ones(cout, np.float32), s.astype(np.float32))
        return u, ex

    blocks: list = []
    k = 0
    layout = S.canonical_enet_layout(num_classes or S.NUM_CLASSES)

    def need(n):
        if k + n > len(infos):
            raise GraphImportError(f"graph has {len(infos)} convolutions, the canonical ENet needs more")

    def check(u, cout, cin, kh, kw, what):
        if (u.cout, u.cin, u.kh, u.kw) != (cout, cin, kh, kw):
            raise GraphImportError(f"{what}: expected conv {cout}x{cin}x{kh}x{kw}, graph has "
                                   f"{u.cout}x{u.cin}x{u.kh}x{u.kw} ({infos[k].node.name})")

    def block_out(ex: str):
        """The residual merge after a branch exit and the activation after it -> out slope."""
        cons = [c for c in g.consumers[ex] if c.op in ("Add", "AddV2")]
        if len(cons) != 1:
            raise GraphImportError(f"no residual add after {ex}")
        add = cons[0]
        a, b, s, ex2 = probe_affine_act(g, add.name, shapes[add.name], infos[k - 1].nchw)
        if not (np.allclose(a, 1) and np.allclose(b, 0)):
            raise GraphImportError(f"{add.name}: the block output has an affine, not just an activation")
        return s.astype(np.float32)

    for typ, name, at in layout:
        if typ == "initial":
            need(1)
            ci = infos[k]
            # conv (+bias) -> concat with the pooled input -> BN -> act over the concatenation
            members, exits = elementwise_closure(g, ci.out)
            cat = [c for c in g.consumers[exits[0]] if c.op == "ConcatV2"]
            if len(exits) != 1 or len(cat) != 1:
                raise GraphImportError(f"{name}: expected the conv output to be concatenated with a max-pool")
            cat = cat[0]
            cb_a, cb_b, cb_s, _ = probe_affine_act(g, ci.out, shapes[ci.out], ci.nchw)
            if not np.allclose(cb_a, 1) or not np.allclose(cb_s, 1):
                raise GraphImportError(f"{name}: unexpected ops between the conv and the concat")
            a, b, s, _ = probe_affine_act(g, cat.name, shapes[cat.name], ci.nchw)
            cc = ci.w.shape[0]
            pool = [g.producer_chain(x, PASS) for x in cat.inputs[:-1]]
            pool = [p for p in pool if p.op.startswith("MaxPool")]
            if len(pool) != 1:
                raise GraphImportError(f"{name}: no max-pool branch")
            pk = _geom_attr(pool[0], "ksize", _s(pool[0].attr.get("data_format", b"NHWC")) == "NCHW")[0]
            # fold the conv bias into beta: a*(conv + cb) + b
            u, _ = unit_from(ci, (a[:cc], b[:cc] + a[:cc] * cb_b, s[:cc], None))
            check(u, at["cconv"], at["cin"], 3, 3, name)
            cin = at["cin"]
            ex_ = dict(pool_gamma=a[cc:cc + cin].astype(np.float32), pool_beta=b[cc:cc + cin].astype(np.float32),
                       pool_mean=np.zeros(cin, np.float32), pool_var=np.ones(cin, np.float32),
                       pool_eps=np.array([0.0], np.float32), pool_slope=s[cc:cc + cin].astype(np.float32))
            blocks.append(S.Block("initial", name, dict(cin=cin, cconv=at["cconv"], pool_k=pk), [u], ex_))
            k += 1
        elif typ == "down":
            need(3)
            cin, cout = at["cin"], at["cout"]
            us = []
            for j, (co, ci_, kk) in enumerate(((cin // 4, cin, 2), (cin // 4, cin // 4, 3), (cout, cin // 4, 1))):
                u, ex = unit_from(infos[k])
                check(u, co, ci_, kk, kk, f"{name} unit {j}")
                us.append(u)
                k += 1
            blocks.append(S.Block("down", name, dict(cin=cin, cout=cout), us, dict(out_slope=block_out(ex))))
        elif typ == "regular":
            ch, it = at["ch"], at["ch"] // 4
            asym = at["conv"] == "asymmetric"
            need(4 if asym else 3)
            specs = [(it, ch, 1, 1)] + ([(it, it, at["k"], 1), (it, it, 1, at["k"])] if asym else
                                        [(it, it, 3, 3)]) + [(ch, it, 1, 1)]
            us = []
            for j, (co, ci_, kh, kw) in enumerate(specs):
                u, ex = unit_from(infos[k])
                check(u, co, ci_, kh, kw, f"{name} unit {j}")
                if j == 1 and not asym and u.dil_h != at["dil"]:
                    raise GraphImportError(f"{name}: expected dilation {at['dil']}, graph has {u.dil_h}")
                us.append(u)
                k += 1
            blocks.append(S.Block("regular", name, dict(ch=ch), us, dict(out_slope=block_out(ex))))
        elif typ == "up":
            need(4)
            cin, cout, it = at["cin"], at["cout"], at["cin"] // 4
            group = infos[k:k + 4]
            # the main-branch 1x1 (cin -> cout, feeding the unpool) may come first or last
            mains = [i for i, ci in enumerate(group) if ci.kind == S.UNIT_CONV and ci.w.shape[:2] == (cout, cin)]
            if not mains:
                raise GraphImportError(f"{name}: no main-branch 1x1 conv {cout}x{cin}")
            mi = mains[0]
            order = [group[mi]] + [ci for i, ci in enumerate(group) if i != mi]
            us = []
            for j, (ci, (co, c_in, kk)) in enumerate(zip(order, ((cout, cin, 1), (it, cin, 1), (it, it, 2), (cout, it, 1)))):
                u, ex = unit_from(ci)
                if (u.cout, u.cin, u.kh) != (co, c_in, kk):
                    raise GraphImportError(f"{name} unit {j}: expected {co}x{c_in}x{kk}x{kk}, graph has "
                                           f"{u.cout}x{u.cin}x{u.kh}x{u.kw} ({ci.node.name})")
                us.append(u)
            k += 4
            ref = next(i for i, b in enumerate(blocks) if b.name == at["pool_ref"])
            blocks.append(S.Block("up", name, dict(cin=cin, cout=cout, pool_ref=ref), us,
                                  dict(out_slope=block_out(ex))))
        elif typ == "fullconv":
            need(1)
            u, _ = unit_from(infos[k])
            if u.kind != S.UNIT_TCONV or u.cin != at["cin"]:
                raise GraphImportError(f"{name}: expected a transposed conv from {at['cin']} channels")
            if not np.allclose(u.slope, 1):
                raise GraphImportError(f"{name}: activation after the classifier")
            ncls = u.cout
            blocks.append(S.Block("fullconv", name, dict(cin=at["cin"], classes=ncls), [u], {}))
            k += 1
    if k != len(infos):
        raise GraphImportError(f"graph has {len(infos) - k} convolutions beyond the canonical ENet")
    return blocks


def graphdef_to_blob(data: bytes, **kw) -> bytes:
    blocks = import_enet(data, **kw)
    ncls = blocks[-1].attrs["classes"]
    return S.serialize(blocks, ncls)


if __name__ == "__main__":
    import sys
    if len(sys.argv) != 3:
        print("usage: python -m bugcar_image_segmentation_amd.graphdef enet.pb enet.bsg1", file=sys.stderr)
        sys.exit(2)
    with open(sys.argv[1], "rb") as f:
        blob = graphdef_to_blob(f.read(), input_name="input0")
    with open(sys.argv[2], "wb") as f:
        f.write(blob)
    print(f"{sys.argv[2]}: {len(blob)} bytes")
