"""Test helper: write an enet_spec block list as a frozen TensorFlow GraphDef (protobuf wire format),
in two encodings an ENet export can take, to exercise the GraphDef importer
(bugcar_image_segmentation_amd/graphdef.py) without TensorFlow:

* style "nhwc": a Keras-like graph — input transposed to NHWC, explicit Pad + VALID Conv2D,
  BiasAdd, FusedBatchNormV3, PReLU as relu(x) - alpha * relu(-x), MaxPoolWithArgmax + ScatterNd
  max-unpooling, Conv2DBackpropInput + Slice for the transposed convolutions;
* style "nchw": an ONNX-to-TF-like graph — NCHW Conv2D with EXPLICIT padding, filters stored OIHW
  behind a Transpose node, batch norm as Sub / Mul / Add with Rsqrt(var + eps) * gamma folded from
  reshaped 1-D constants, PReLU as max(x, 0) + slope * min(x, 0), pooling through NHWC transposes.

Both end in the reference's output node name (``CATkrIDy/concat``, models.py:16) fed from the
placeholder ``input0`` (models.py:15), NCHW (B, 3, H, W). The semantics are those of the engine /
oracle/enet_oracle.py (PyTorch conventions), written with TF ops.
"""
from __future__ import annotations

import struct

import numpy as np

from bugcar_image_segmentation_amd import enet_spec as S


# ---- protobuf encoding
def _vi(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(f, wt):
    return _vi((f << 3) | wt)


def _ld(f, payload: bytes) -> bytes:
    return _key(f, 2) + _vi(len(payload)) + payload


def _int(f, v) -> bytes:
    return _key(f, 0) + _vi(int(v))


DT = {np.dtype(np.float32): 1, np.dtype(np.float64): 2, np.dtype(np.int32): 3, np.dtype(np.int64): 9}


def _shape(dims) -> bytes:
    return b"".join(_ld(2, _int(1, d)) for d in dims)


def _tensor(a: np.ndarray) -> bytes:
    a = np.array(a, order="C")          # (ascontiguousarray would turn a 0-d scalar into shape (1,))
    return _int(1, DT[a.dtype]) + _ld(2, _shape(a.shape)) + _ld(4, a.tobytes())


def _attr(v) -> bytes:
    if isinstance(v, tuple) and v and v[0] == "type":
        return _int(6, v[1])
    if isinstance(v, tuple) and v and v[0] == "shape":
        return _ld(7, _shape(v[1]))
    if isinstance(v, np.ndarray):
        return _ld(8, _tensor(v))
    if isinstance(v, bool):
        return _int(5, v)
    if isinstance(v, str):
        return _ld(2, v.encode())
    if isinstance(v, float):
        return _key(4, 5) + struct.pack("<f", v)
    if isinstance(v, int):
        return _int(3, v)
    if isinstance(v, list):
        return _ld(1, _ld(3, b"".join(_vi(int(x)) for x in v)))
    raise TypeError(v)


class GraphBuilder:
    def __init__(self):
        self.nodes: list = []
        self.n = 0

    def node(self, op, inputs=(), name=None, **attr) -> str:
        self.n += 1
        name = name or f"n{self.n}_{op}"
        body = _ld(1, name.encode()) + _ld(2, op.encode()) + b"".join(_ld(3, i.encode()) for i in inputs)
        for k, v in attr.items():
            body += _ld(5, _ld(1, k.encode()) + _ld(2, _attr(v)))
        self.nodes.append(_ld(1, body))
        return name

    def const(self, a, dtype=np.float32) -> str:
        a = np.asarray(a, dtype)
        return self.node("Const", dtype=("type", DT[a.dtype]), value=a)

    def bytes(self) -> bytes:
        return b"".join(self.nodes)


F32 = ("type", 1)


# ---- the two encodings
class _Writer:
    def __init__(self, style: str, H: int, W: int, B: int = 1):
        self.g = GraphBuilder()
        self.style = style
        self.nchw = style == "nchw"
        self.B = B
        self.argmax: dict = {}

    # layout helpers
    def fmt(self):
        return "NCHW" if self.nchw else "NHWC"

    def hw4(self, a, b):
        return [1, 1, a, b] if self.nchw else [1, a, b, 1]

    def cdim(self):
        return 1 if self.nchw else 3

    def chshape(self, c):
        return (1, c, 1, 1) if self.nchw else (c,)

    def cvec(self, v):
        """Per-channel constant broadcast against the activation layout."""
        v = np.asarray(v, np.float32)
        if self.nchw:
            return self.g.node("Reshape", [self.g.const(v), self.g.const(np.array([1, -1, 1, 1], np.int32), np.int32)],
                               T=F32, Tshape=("type", 3))
        return self.g.const(v)

    def conv(self, x, u, shape):
        g = self.g
        w = u.w.astype(np.float32)                                     # OIHW
        if self.nchw:
            filt = g.node("Transpose", [g.const(w), g.const(np.array([2, 3, 1, 0], np.int32), np.int32)], T=F32,
                          Tperm=("type", 3))
            y = g.node("Conv2D", [x, filt], T=F32, strides=self.hw4(u.stride, u.stride), padding="EXPLICIT",
                       explicit_paddings=[0, 0, 0, 0, u.pad_h, u.pad_h, u.pad_w, u.pad_w], data_format="NCHW",
                       dilations=self.hw4(u.dil_h, u.dil_w))
        else:
            if u.pad_h or u.pad_w:
                x = g.node("Pad", [x, g.const(np.array([[0, 0], [u.pad_h, u.pad_h], [u.pad_w, u.pad_w], [0, 0]], np.int32),
                                              np.int32)], T=F32, Tpaddings=("type", 3))
            y = g.node("Conv2D", [x, g.const(np.transpose(w, (2, 3, 1, 0)))], T=F32, strides=self.hw4(u.stride, u.stride),
                       padding="VALID", data_format="NHWC", dilations=self.hw4(u.dil_h, u.dil_w))
        B, C, Hh, Ww = shape
        oh = (Hh + 2 * u.pad_h - u.dil_h * (u.kh - 1) - 1) // u.stride + 1
        ow = (Ww + 2 * u.pad_w - u.dil_w * (u.kw - 1) - 1) // u.stride + 1
        return self.bias(y, u), (B, u.cout, oh, ow)

    def tconv(self, x, u, shape):
        g = self.g
        B, C, Hh, Ww = shape
        fh, fw = (Hh - 1) * u.stride + u.kh, (Ww - 1) * u.stride + u.kw
        sizes = [B, u.cout, fh, fw] if self.nchw else [B, fh, fw, u.cout]
        filt = np.transpose(u.w.astype(np.float32), (2, 3, 1, 0))      # IOHW -> [kh, kw, out, in]
        y = g.node("Conv2DBackpropInput", [g.const(np.array(sizes, np.int32), np.int32), g.const(filt), x], T=F32,
                   strides=self.hw4(u.stride, u.stride), padding="VALID", data_format=self.fmt())
        oh = (Hh - 1) * u.stride - 2 * u.pad_h + u.kh + u.out_pad
        ow = (Ww - 1) * u.stride - 2 * u.pad_w + u.kw + u.out_pad
        if (oh, ow) != (fh, fw) or u.pad_h:
            begin = [0, 0, u.pad_h, u.pad_w] if self.nchw else [0, u.pad_h, u.pad_w, 0]
            size = [B, u.cout, oh, ow] if self.nchw else [B, oh, ow, u.cout]
            y = g.node("Slice", [y, g.const(np.array(begin, np.int32), np.int32), g.const(np.array(size, np.int32), np.int32)],
                       T=F32, Index=("type", 3))
        return self.bias(y, u), (B, u.cout, oh, ow)

    def bias(self, y, u):
        if u.b is None or not np.any(u.b):
            return y
        return self.g.node("BiasAdd", [y, self.g.const(u.b.astype(np.float32))], T=F32, data_format=self.fmt())

    def bn(self, x, gamma, beta, mean, var, eps):
        g = self.g
        gamma, beta, mean, var = (np.asarray(t, np.float32) for t in (gamma, beta, mean, var))
        if np.all(gamma == 1) and not beta.any() and not mean.any() and np.all(var == 1):
            return x
        if not self.nchw:
            return g.node("FusedBatchNormV3", [x, g.const(gamma), g.const(beta), g.const(mean), g.const(var)],
                          T=F32, U=F32, epsilon=float(eps), data_format="NHWC", is_training=False)
        # (x - mean) * (gamma * rsqrt(var + eps)) + beta, the factor a constant sub-graph
        inv = g.node("Rsqrt", [g.node("AddV2", [self.cvec(var), g.const(np.float32(eps))], T=F32)], T=F32)
        sc = g.node("Mul", [inv, self.cvec(gamma)], T=F32)
        y = g.node("Sub", [x, self.cvec(mean)], T=F32)
        y = g.node("Mul", [y, sc], T=F32)
        return g.node("AddV2", [y, self.cvec(beta)], T=F32)

    def act(self, x, slope):
        g = self.g
        slope = np.asarray(slope, np.float32)
        if np.all(slope == 1):
            return x
        if np.all(slope == 0):
            return g.node("Relu", [x], T=F32)
        if not self.nchw:
            pos = g.node("Relu", [x], T=F32)
            neg = g.node("Relu", [g.node("Neg", [x], T=F32)], T=F32)
            neg = g.node("Mul", [g.const(-slope), neg], T=F32)
            return g.node("AddV2", [pos, neg], T=F32)
        pos = g.node("Maximum", [x, g.const(np.float32(0))], T=F32)
        neg = g.node("Minimum", [x, g.const(np.float32(0))], T=F32)
        return g.node("AddV2", [pos, g.node("Mul", [self.cvec(slope), neg], T=F32)], T=F32)

    def unit(self, x, u, shape):
        y, shp = (self.tconv if u.kind == S.UNIT_TCONV else self.conv)(x, u, shape)
        return self.act(self.bn(y, u.gamma, u.beta, u.mean, u.var, u.eps), u.slope), shp

    def to_nhwc(self, x):
        if not self.nchw:
            return x
        return self.g.node("Transpose", [x, self.g.const(np.array([0, 2, 3, 1], np.int32), np.int32)], T=F32,
                           Tperm=("type", 3))

    def from_nhwc(self, x):
        if not self.nchw:
            return x
        return self.g.node("Transpose", [x, self.g.const(np.array([0, 3, 1, 2], np.int32), np.int32)], T=F32,
                           Tperm=("type", 3))

    def pad_channels(self, x, extra):
        p = np.zeros((4, 2), np.int32)
        p[self.cdim(), 1] = extra
        return self.g.node("Pad", [x, self.g.const(p, np.int32)], T=F32, Tpaddings=("type", 3))

    def write(self, blocks, H, W) -> bytes:
        g = self.g
        B = self.B
        x = g.node("Placeholder", [], name="input0", dtype=F32, shape=("shape", [B, 3, H, W]))
        if not self.nchw:
            x = g.node("Transpose", [x, g.const(np.array([0, 2, 3, 1], np.int32), np.int32)], T=F32, Tperm=("type", 3))
        shape = (B, 3, H, W)
        for bi, b in enumerate(blocks):
            if b.type == "initial":
                u, e = b.units[0], b.extra
                conv, cs = self.conv(x, u, shape)
                k = b.attrs["pool_k"]
                px = x
                if k == 3:
                    p = np.zeros((4, 2), np.int32)
                    p[(2, 3) if self.nchw else (1, 2), :] = 1
                    px = g.node("PadV2", [x, g.const(p, np.int32), g.const(np.float32(-np.inf))], T=F32,
                                Tpaddings=("type", 3))
                pool = g.node("MaxPool", [px], T=F32, ksize=self.hw4(k, k), strides=self.hw4(2, 2), padding="VALID",
                              data_format=self.fmt())
                cat = g.node("ConcatV2", [conv, pool, g.const(np.int32(self.cdim()), np.int32)], T=F32, N=2,
                             Tidx=("type", 3))
                if self.nchw or float(u.eps) != float(e["pool_eps"][0]):
                    y = self.bn(cat, np.concatenate([u.gamma, e["pool_gamma"]]), np.concatenate([u.beta, e["pool_beta"]]),
                                np.concatenate([u.mean, e["pool_mean"]]), np.concatenate([u.var, e["pool_var"]]), u.eps)
                else:
                    y = self.bn(cat, np.concatenate([u.gamma, e["pool_gamma"]]), np.concatenate([u.beta, e["pool_beta"]]),
                                np.concatenate([u.mean, e["pool_mean"]]), np.concatenate([u.var, e["pool_var"]]), u.eps)
                x = self.act(y, np.concatenate([u.slope, e["pool_slope"]]))
                shape = (B, cs[1] + b.attrs["cin"], cs[2], cs[3])
            elif b.type == "down":
                ext, es = x, shape
                for u in b.units:
                    ext, es = self.unit(ext, u, es)
                pm = g.node("MaxPoolWithArgmax", [self.to_nhwc(x)], T=F32, Targmax=("type", 9), ksize=[1, 2, 2, 1],
                            strides=[1, 2, 2, 1], padding="VALID", include_batch_in_index=False)
                self.argmax[bi] = (pm + ":1", shape)
                main = self.pad_channels(self.from_nhwc(pm), b.attrs["cout"] - b.attrs["cin"])
                x = self.act(g.node("AddV2", [main, ext], T=F32), b.extra["out_slope"])
                shape = es
            elif b.type == "regular":
                ext, es = x, shape
                for u in b.units:
                    ext, es = self.unit(ext, u, es)
                x = self.act(g.node("AddV2", [x, ext], T=F32), b.extra["out_slope"])
            elif b.type == "up":
                um = b.units[0]
                main, ms = self.unit(x, um, shape)
                am, (Bp, Cp, Hp, Wp) = self.argmax[b.attrs["pool_ref"]]
                idx = g.node("Reshape", [am, g.const(np.array([-1, 1], np.int32), np.int32)], T=("type", 9),
                             Tshape=("type", 3))
                upd = g.node("Reshape", [self.to_nhwc(main), g.const(np.array([-1], np.int32), np.int32)], T=F32,
                             Tshape=("type", 3))
                sc = g.node("ScatterNd", [idx, upd, g.const(np.array([Hp * Wp * Cp], np.int64), np.int64)], T=F32,
                            Tindices=("type", 9))
                unpooled = self.from_nhwc(g.node("Reshape", [sc, g.const(np.array([1, Hp, Wp, Cp], np.int32), np.int32)],
                                                 T=F32, Tshape=("type", 3)))
                ext, es = x, shape
                for u in b.units[1:]:
                    ext, es = self.unit(ext, u, es)
                x = self.act(g.node("AddV2", [unpooled, ext], T=F32), b.extra["out_slope"])
                shape = es
            elif b.type == "fullconv":
                u = b.units[0]
                y, shape = self.unit(x, u, shape)
                if not self.nchw:
                    y = g.node("Transpose", [y, g.const(np.array([0, 3, 1, 2], np.int32), np.int32)], T=F32,
                               Tperm=("type", 3))
                g.node("ConcatV2", [y, g.const(np.int32(1), np.int32)], name="CATkrIDy/concat", T=F32, N=1,
                       Tidx=("type", 3))
        return g.bytes()


def write_enet_graphdef(blocks, H: int, W: int, style: str = "nhwc") -> bytes:
    """enet_spec block list -> frozen GraphDef bytes (batch 1, input0 NCHW (1, 3, H, W))."""
    if style not in ("nhwc", "nchw"):
        raise ValueError(style)
    return _Writer(style, H, W).write(blocks, H, W)


def with_biases(blocks, seed: int = 7):
    """A copy of `blocks` whose convolutions carry non-zero biases (exercises bias import)."""
    import copy
    out = copy.deepcopy(blocks)
    rng = np.random.default_rng(seed)
    for b in out:
        for u in b.units:
            u.b = rng.normal(0, 0.05, u.cout).astype(np.float32)
    return out
