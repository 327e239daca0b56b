"""Frozen TF DeepLab GraphDef (``deeplab.pb``) -> deeplab_spec.DeepLab weights. SURVEY.md §8(f) rows 1 + 3.

The reference loads ``pretrained_models/deeplab.pb`` into a TF session (models.py:104-110) and feeds
``import/ImageTensor:0`` (models.py:115-125). That file is absent here (.MISSING_LARGE_BLOBS:1); this
importer reads the frozen graph of the standard TF DeepLab export over MobileNetV2
(deeplab/export_model.py; topology in deeplab_spec.py) with the wire-format reader and constant
folding of graphdef.py, and returns the network the engine runs:

* convolutions are taken in graph order: ``Conv2D`` and ``DepthwiseConv2dNative`` (filters behind
  ``Identity`` read nodes are folded); dilation comes from the op's ``dilations`` attribute or, in
  the ``tf.nn.atrous_conv2d`` / ``with_space_to_batch`` encoding TF1 uses for slim's atrous layers,
  from the ``SpaceToBatchND`` block shape around a VALID convolution (``BatchToSpaceND`` after it);
* each convolution's elementwise closure (``FusedBatchNorm*`` with constant statistics, ``BiasAdd``,
  Sub / Mul / Add encodings of a folded batch norm) is probed per channel as ``a x + b`` followed by
  an activation read from the closure's exit op (``Relu6``, ``Relu`` or none); a lone
  ``FusedBatchNorm`` keeps its own (gamma, beta, mean, var, eps) so the oracle evaluates it unfolded
  exactly as TF does;
* roles follow the graph's data flow, not node names: the stem (3 input channels), then inverted
  residual blocks (optional 1x1 expansion -> depthwise -> linear 1x1 projection, residual when the
  projection's output is added to the block input), then the ASPP convolutions classified by what
  feeds them (a spatial ``Mean`` / ``AvgPool`` of the backbone output: image pooling; the backbone
  output itself: the 1x1 branch or a 3x3 atrous branch; the ``ConcatV2`` of the branches: the
  projection), and the final 1x1 with bias as the logits;
* the projection's input channels are permuted from the graph's concat order to the engine's
  [image pooling, 1x1, atrous...] order.

The other two backbone families are told apart by the root: a second full 3x3 convolution is the
Xception-65 root (``_import_xception``: modules of separable convs, separable ASPP, decoder), a third one
the ResNet-v1-beta root (``_import_resnet``: a 3x3 s2 ``MaxPool``, then bottleneck units found by data
flow — 1x1 + ReLU, 3x3 + ReLU, linear 1x1 meeting the shortcut at an ``Add`` + ``Relu`` — and the dense
ASPP head shared with MobileNetV2, ``_dense_aspp``).

The crop size IS read from the graph: deeplab/input_preprocess.py pads every image to
``image_size + max(crop - image_size, 0)`` per axis, which a frozen export holds as
``Maximum(Sub(Const crop, StridedSlice(Shape(image), [axis])), 0)`` — the two ``Const`` operands give
(crop height, crop width), the lower axis being the height (read_crop). Not read from the graph: the
pad value 127.5, ``(2/255) x - 1`` and the final bilinear resize + argmax, the export's fixed
semantics and the engine's own (deeplab_spec.py).

Parity: pinned against graphs written by tests/deeplab_graph_writer.py (run by the NumPy GraphDef
interpreter oracle/tf_graph.py as the sess.run stand-in); UNPINNED against TF on the real deeplab.pb.
"""
from __future__ import annotations

import numpy as np

from . import deeplab_spec as D
from .graphdef import (PASS, Graph, GraphImportError, _run_closure, _s, _src, elementwise_closure,
                       parse_graphdef)

CONV_OPS = ("Conv2D", "DepthwiseConv2dNative")
_ACT = {"Relu6": D.ACT_RELU6, "Relu": D.ACT_RELU}
_ACT_NAME = {D.ACT_NONE: "none", D.ACT_RELU: "ReLU", D.ACT_RELU6: "ReLU6"}
# ops that carry a branch output to the ASPP concat unchanged in value per channel (the image-pooling
# branch is broadcast back to the feature size)
_BROADCAST = PASS | {"ResizeBilinear", "ResizeNearestNeighbor", "Tile", "BroadcastTo", "ResizeBilinearV2"}


class _Conv:
    """One convolution node of the graph, its geometry and its output closure."""

    def __init__(self, g: Graph, n):
        self.node = n
        self.depthwise = n.op == "DepthwiseConv2dNative"
        if _s(n.attr.get("data_format", b"NHWC")) != "NHWC":
            raise GraphImportError(f"{n.name}: only NHWC DeepLab graphs are supported")
        st = [int(v) for v in (n.attr.get("strides") or [1, 1, 1, 1])]
        dl = [int(v) for v in (n.attr.get("dilations") or [1, 1, 1, 1])]
        if st[1] != st[2] or dl[1] != dl[2]:
            raise GraphImportError(f"{n.name}: anisotropic stride / dilation")
        self.stride, self.dil = st[1], dl[1]
        w = g.const(n.inputs[1])                                         # HWIO / HW C mult
        if self.depthwise:
            if w.shape[3] != 1:
                raise GraphImportError(f"{n.name}: depthwise channel multiplier {w.shape[3]} (MobileNetV2 uses 1)")
            self.w = np.ascontiguousarray(np.transpose(w, (2, 3, 0, 1)), np.float32)   # (C, 1, kh, kw)
        else:
            self.w = np.ascontiguousarray(np.transpose(w, (3, 2, 0, 1)), np.float32)   # OIHW
        if self.w.shape[2] != self.w.shape[3]:
            raise GraphImportError(f"{n.name}: non-square kernel {self.w.shape[2:]}")
        self.input = n.inputs[0]
        self.out = n.name
        self.explicit = None     # (pad before, pad after) of an explicit Pad + VALID convolution
        padding = _s(n.attr.get("padding", b"SAME"))
        # the space-to-batch encoding of an atrous convolution
        src = g.producer_chain(self.input, PASS)
        if padding == "VALID" and src.op in ("Pad", "PadV2"):
            # resnet_utils / xception fixed_padding ahead of a strided convolution
            p = np.asarray(g.const(src.inputs[1]), np.int64).reshape(-1, 2)
            if len(src.inputs) > 2 and float(np.asarray(g.const(src.inputs[2]))) != 0.0:
                raise GraphImportError(f"{src.name}: non-zero pad value ahead of {n.name}")
            if p.shape != (4, 2) or p[0].any() or p[3].any() or not (p[1] == p[2]).all():
                raise GraphImportError(f"{src.name}: paddings {p.tolist()} ahead of {n.name}")
            self.explicit = (int(p[1][0]), int(p[1][1]))
            self.input = src.inputs[0]
        elif padding == "VALID" and src.op != "SpaceToBatchND":
            kh = int(g.const(n.inputs[1]).shape[0])
            if kh != 1:
                raise GraphImportError(f"{n.name}: VALID {kh}x{kh} convolution without an explicit pad")
        if src.op == "SpaceToBatchND":
            bs = [int(v) for v in g.const(src.inputs[1])]
            if len(bs) != 2 or bs[0] != bs[1]:
                raise GraphImportError(f"{src.name}: block shape {bs}")
            if self.stride != 1 or self.dil != 1:
                raise GraphImportError(f"{n.name}: strided / dilated convolution inside SpaceToBatchND")
            self.dil = bs[0]
            self.input = src.inputs[0]
            cons = [c for c in g.consumers[n.name] if c.op not in PASS]
            if len(cons) != 1 or cons[0].op != "BatchToSpaceND":
                raise GraphImportError(f"{n.name}: SpaceToBatchND without a BatchToSpaceND after the convolution")
            self.out = cons[0].name
        self.cin = self.w.shape[0] if self.depthwise else self.w.shape[1]
        self.cout = self.w.shape[0]
        self.k = self.w.shape[2]

    def src(self, g: Graph):
        """Name of the node producing this convolution's input (through identity-like ops)."""
        return g.producer_chain(self.input, PASS).name


def _affine_act(g: Graph, c: _Conv, act_ends: bool = False):
    """The closure after the convolution as act(a x + b) per channel -> (fields for D.Conv, exit)."""
    members, exits = elementwise_closure(g, c.out, act_ends)
    if len(exits) != 1:
        raise GraphImportError(f"the ops after {c.node.name} leave through {len(exits)} tensors ({exits})")
    ex = exits[0]
    act = D.ACT_NONE
    lin_members, lin_exit = members, ex
    exn = g.node(ex)
    if ex != _src(c.out)[0] and exn.op in _ACT:
        act = _ACT[exn.op]
        lin_members = [m for m in members if m.name != ex]
        lin_exit = _src(exn.inputs[0])[0]
    if any(m.op in _ACT or m.op in ("Maximum", "Minimum", "LeakyRelu", "Select", "SelectV2") for m in lin_members):
        raise GraphImportError(f"the ops after {c.node.name} are not batch norm / bias followed by one activation")
    C = c.cout
    fields: dict = {}
    if len(lin_members) == 1 and lin_members[0].op.startswith("FusedBatchNorm"):
        bn = lin_members[0]
        sc, of, mu, var = (np.asarray(g.const(s), np.float32) for s in bn.inputs[1:5])
        fields = dict(gamma=sc, beta=of, mean=mu, var=var, eps=float(bn.attr.get("epsilon", 1e-4)))
    elif lin_members:
        def f(v):
            x = np.asarray(v, np.float64).reshape(1, 1, 1, C)
            return np.asarray(_run_closure(g, c.out, lin_members, x, lin_exit), np.float64).reshape(-1)
        b = f(np.zeros(C))
        a = f(np.ones(C)) - b
        for t in (-3.0, 0.5, 7.0):
            if not np.allclose(f(np.full(C, t)), a * t + b, rtol=1e-6, atol=1e-6 * (1 + np.abs(b))):
                raise GraphImportError(f"the ops after {c.node.name} are not per-channel affine before the activation")
        if np.allclose(a, 1.0, rtol=0, atol=1e-7):
            fields = dict(b=b.astype(np.float32))
        else:
            fields = dict(gamma=a.astype(np.float32), beta=b.astype(np.float32), mean=np.zeros(C, np.float32),
                          var=np.ones(C, np.float32), eps=0.0)
    return fields, act, ex


def _make(c: _Conv, fields: dict, act: int) -> D.Conv:
    return D.Conv(w=c.w, act=act, stride=c.stride, dil=c.dil, depthwise=c.depthwise, **fields)


def _expect(cond, msg):
    if not cond:
        raise GraphImportError(msg)


def read_crop(g: Graph):
    """(crop height, crop width) from the export's pad-to-crop arithmetic, or None when the graph has
    none (see the module docstring)."""
    found = {}
    for n in g.nodes:
        if n.op != "Sub" or len(n.inputs) != 2 or not g.is_const(n.inputs[0]) or g.is_const(n.inputs[1]):
            continue
        v = np.asarray(g.const(n.inputs[0]))
        if v.size != 1 or v.dtype.kind not in "iu" or not any(c.op == "Maximum" for c in g.consumers[n.name]):
            continue
        ss = g.producer_chain(n.inputs[1], PASS)
        if ss.op != "StridedSlice" or len(ss.inputs) < 2 or g.producer_chain(ss.inputs[0], PASS).op != "Shape" \
                or not g.is_const(ss.inputs[1]):
            continue
        found[int(np.atleast_1d(g.const(ss.inputs[1]))[0])] = int(v.reshape(()))
    if len(found) != 2:
        return None
    (_, h), (_, w) = sorted(found.items())
    _expect(h >= 2 and w >= 2, f"graph pads to a {h}x{w} crop")
    return h, w


def _aspp_concat_perm(g: Graph, concat, by_exit: dict, pool_k, aspp0_k, widths: dict, proj_cin: int):
    """The ASPP concat's branch order -> (permutation of the projection's input channels into the
    engine's [pool, 1x1, atrous...] order, the atrous branch keys in concat order). by_exit: branch
    output tensor -> key; widths: key -> channels."""
    parts = []
    for s in concat.inputs[:-1]:
        n = g.node(s)
        while n.op in _BROADCAST and n.name not in by_exit:
            n = g.node(n.inputs[0])
        _expect(n.name in by_exit, f"{concat.name}: input {s} is not an ASPP branch output")
        parts.append(by_exit[n.name])
    _expect(int(g.const(concat.inputs[-1])) % 4 == 3, f"{concat.name}: not a channel concat")
    _expect(sorted(parts) == sorted(by_exit.values()), f"{concat.name}: branches {parts}")
    atr_sorted = [a for a in parts if a not in (pool_k, aspp0_k)]
    order = [pool_k, aspp0_k] + atr_sorted
    off, start = 0, {}
    for j in parts:
        start[j] = off
        off += widths[j]
    _expect(off == proj_cin, f"projection takes {proj_cin} channels, concat has {off}")
    return np.concatenate([np.arange(start[j], start[j] + widths[j]) for j in order]), atr_sorted


def _fixed(c: _Conv) -> bool:
    """A strided convolution padded the xception / resnet_utils way (fixed_padding + VALID)."""
    ke = c.k + (c.k - 1) * (c.dil - 1)
    return c.explicit == ((ke - 1) // 2, ke - 1 - (ke - 1) // 2)


def _import_xception(g: Graph, convs: list, closures: list, crop_h: int, crop_w: int):
    """The DeepLabV3+ Xception-65 export (deeplab_xception.py documents the topology) by data flow:
    root convs, xception modules (three depthwise + pointwise pairs; a ``Relu`` ahead of each pair in
    the pre-activation modules; an ``Add`` with the module input or with a 1x1 shortcut conv of it),
    then the ASPP (image pooling, 1x1, separable atrous branches, projection) and the decoder
    (``ResizeBilinear`` of the projection, concat with a 1x1 over a low-level pointwise output, two
    separable convs) feeding the logits."""
    from . import deeplab_xception as X
    exit_of = {id(c): ex for c, (_, _, ex) in zip(convs, closures)}
    ex = lambda i: exit_of[id(convs[i])]  # noqa: E731
    act = lambda i: closures[i][1]  # noqa: E731

    def conv_at(i):
        f, a, _ = closures[i]
        return _make(convs[i], f, a)

    def need_act(i, want, role):
        _expect(act(i) == want, f"{role} ({convs[i].node.name}): expected {_ACT_NAME[want]} after it, "
                                f"graph has {_ACT_NAME[act(i)]}")

    def strided_ok(i):
        c = convs[i]
        if c.stride > 1 and c.k > 1:
            _expect(_fixed(c), f"{c.node.name}: strided convolution without fixed_padding")
        else:
            _expect(c.explicit is None, f"{c.node.name}: explicit padding on a stride-1 convolution")

    n = len(convs)
    # shortcut convs: 1x1 convs whose output meets a pointwise output at an Add
    consumers_add = {}
    for i in range(n):
        for a in g.consumers[ex(i)]:
            if a.op in ("Add", "AddV2"):
                consumers_add.setdefault(a.name, []).append(i)
    shortcut_of = {}          # add name -> shortcut conv index
    for add, idx in consumers_add.items():
        if len(idx) == 2:
            sc = [i for i in idx if not convs[i].depthwise and convs[i].k == 1 and
                  not (i > 0 and convs[i - 1].depthwise and convs[i].src(g) == ex(i - 1))]
            _expect(len(sc) == 1, f"{add}: cannot tell the shortcut from the residual branch")
            shortcut_of[add] = sc[0]
    shortcuts = set(shortcut_of.values())
    seq = [i for i in range(n) if i not in shortcuts]

    r0, r1 = seq[0], seq[1]
    strided_ok(r0)
    strided_ok(r1)
    need_act(r0, D.ACT_RELU, "root conv")
    need_act(r1, D.ACT_RELU, "root conv")
    _expect(convs[r1].src(g) == ex(r0) and convs[r1].cin == convs[r0].cout, f"{convs[r1].node.name}: root chain")
    cur, cur_c = ex(r1), convs[r1].cout
    modules, pw_pos = [], {}
    k = 2
    def starts_module(k):
        if k + 1 >= len(seq) or not convs[seq[k]].depthwise:
            return False
        inp = convs[seq[k]].input
        return g.producer_chain(inp, PASS).name == cur or _relu_of(g, inp) == cur

    while starts_module(k):
        mod_in, mod_c = cur, cur_c
        seps = []
        src_t = cur
        for j in range(3):
            _expect(k + 1 < len(seq), "graph ends inside an xception module")
            di, pi = seq[k], seq[k + 1]
            dw, pw = convs[di], convs[pi]
            _expect(dw.depthwise and dw.k == 3, f"{dw.node.name}: expected a 3x3 depthwise convolution")
            _expect(not pw.depthwise and pw.k == 1 and pw.src(g) == ex(di),
                    f"{pw.node.name}: expected the 1x1 pointwise convolution of {dw.node.name}")
            if g.producer_chain(dw.input, PASS).name == src_t:
                pre = False
            else:
                _expect(_relu_of(g, dw.input) == src_t, f"{dw.node.name}: input is neither {src_t} nor its ReLU")
                pre = True
            strided_ok(di)
            _expect(act(di) in (D.ACT_NONE, D.ACT_RELU) and act(pi) in (D.ACT_NONE, D.ACT_RELU),
                    f"{dw.node.name}: activation other than ReLU in a separable conv")
            _expect(dw.cin == cur_c, f"{dw.node.name}: channel count")
            dwc, pwc = conv_at(di), conv_at(pi)
            if act(di) == D.ACT_NONE:
                # pre-activation form: a ReLU between two separable convs that is the pointwise's only
                # reader joined its closure; it is this conv's input ReLU (same values either way)
                if j and seps[-1].pw.act == D.ACT_RELU:
                    seps[-1].pw.act = D.ACT_NONE
                    pre = True
                _expect(pre, f"{dw.node.name}: depthwise without ReLU before or after it")
            else:
                _expect(not pre and act(pi) == D.ACT_RELU, f"{dw.node.name}: a separable conv is either "
                                                           "pre-activated or activated inside")
            seps.append(X.SepConv(dwc, pwc, pre))
            pw_pos[ex(pi)] = (len(modules), j)
            src_t, cur_c = ex(pi), pw.cout
            k += 2
        _expect(len({sp.pre_relu for sp in seps}) == 1, "module mixes pre-activated and activated separable convs")
        if seps[0].pre_relu:
            _expect(seps[2].pw.act == D.ACT_NONE, f"{convs[seq[k - 1]].node.name}: activation before the module sum")
        adds = [a for a in g.consumers[src_t] if a.op in ("Add", "AddV2")]
        skip, sc = "none", None
        if adds:
            add = adds[0]
            others = [g.producer_chain(t, PASS).name for t in add.inputs]
            others.remove(src_t)
            if add.name in shortcut_of:
                si = shortcut_of[add.name]
                _expect(convs[si].src(g) == mod_in and ex(si) == others[0] and convs[si].cin == mod_c,
                        f"{convs[si].node.name}: shortcut not over the module input")
                need_act(si, D.ACT_NONE, "shortcut")
                skip, sc = "conv", conv_at(si)
            else:
                _expect(others == [mod_in] and mod_c == cur_c, f"{add.name}: residual over a shape change")
                skip = "sum"
            cur = add.name
        else:
            cur = src_t
        modules.append(X.XModule(seps, skip, sc))
    _expect(len(modules) >= 2, "fewer than two xception modules after the root")
    backbone, feat_c = cur, cur_c
    # ASPP + decoder + logits
    pool = aspp0 = project = logits = low_proj = None
    pool_k = aspp0_k = proj_i = low_i = None
    atrous = {}               # pointwise exit -> SepConv
    dec = []
    concat = None
    rest = seq[k:]
    used = set()
    for q, j in enumerate(rest):
        if j in used:
            continue
        c = convs[j]
        src = g.node(c.src(g))
        if c.depthwise:
            _expect(q + 1 < len(rest), f"{c.node.name}: depthwise convolution at the end of the graph")
            pi = rest[q + 1]
            pw = convs[pi]
            _expect(not pw.depthwise and pw.k == 1 and pw.src(g) == ex(j), f"{c.node.name}: no pointwise after it")
            _expect(act(j) == D.ACT_RELU and act(pi) == D.ACT_RELU, f"{c.node.name}: separable conv without ReLUs")
            used.add(pi)
            sepc = X.SepConv(conv_at(j), conv_at(pi))
            if src.name == backbone:
                atrous[ex(pi)] = sepc
            else:
                dec.append((j, pi, sepc))
        elif src.op in ("Mean", "AvgPool") and g.producer_chain(src.inputs[0], PASS).name == backbone:
            if src.op == "Mean":
                ax = sorted(int(v) % 4 for v in np.atleast_1d(g.const(src.inputs[1])))
                _expect(ax == [1, 2], f"{src.name}: mean over axes {ax}, expected the spatial axes")
            _expect(pool is None and c.k == 1, f"{c.node.name}: second / non-1x1 image-pooling convolution")
            need_act(j, D.ACT_RELU, "image pooling")
            pool, pool_k = conv_at(j), ex(j)
        elif src.name == backbone:
            _expect(aspp0 is None and c.k == 1, f"{c.node.name}: second / non-1x1 dense ASPP branch (the Xception "
                                                "ASPP's atrous branches are separable)")
            need_act(j, D.ACT_RELU, "ASPP branch")
            aspp0, aspp0_k = conv_at(j), ex(j)
        elif src.op == "ConcatV2" and project is None:
            _expect(c.k == 1, f"{c.node.name}: non-1x1 concat projection")
            need_act(j, D.ACT_RELU, "concat projection")
            project, proj_i, concat = conv_at(j), j, src
        elif src.name in pw_pos and low_proj is None:
            _expect(c.k == 1, f"{c.node.name}: non-1x1 low-level projection")
            need_act(j, D.ACT_RELU, "low-level projection")
            low_proj, low_i, low_at = conv_at(j), j, pw_pos[src.name]
        elif c.k == 1 and logits is None and act(j) == D.ACT_NONE:
            logits, logits_src = conv_at(j), src.name
        else:
            raise GraphImportError(f"{c.node.name}: convolution fed by {src.name} ({src.op}) has no DeepLab role")
    _expect(pool is not None and aspp0 is not None and project is not None and logits is not None,
            "missing ASPP parts: " + ", ".join(nm for nm, v in (("image pooling", pool), ("1x1 branch", aspp0),
                                                                ("projection", project), ("logits", logits))
                                                if v is None))
    by_exit = {pool_k: "pool", aspp0_k: "aspp0", **{e: e for e in atrous}}
    widths = {"pool": pool.cout, "aspp0": aspp0.cout, **{e: a.pw.cout for e, a in atrous.items()}}
    perm, atr_sorted = _aspp_concat_perm(g, concat, by_exit, "pool", "aspp0", widths, project.w.shape[1])
    project.w = np.ascontiguousarray(project.w[:, perm])
    atrous_seps = [atrous[e] for e in atr_sorted]
    Dd = aspp0.cout
    _expect(pool.cout == Dd and all(a.pw.cout == Dd for a in atrous_seps) and project.cout == Dd,
            "ASPP branches and projection differ in depth")
    decoder = []
    if low_proj is not None:
        _expect(len(dec) == 2, f"decoder has {len(dec)} separable convs, expected 2")
        d0 = convs[dec[0][0]]
        cat2 = g.node(d0.src(g))
        _expect(cat2.op == "ConcatV2" and len(cat2.inputs) == 3, f"{d0.node.name}: decoder input is not a 2-way concat")
        first = g.node(cat2.inputs[0])
        while first.op in PASS:
            first = g.node(first.inputs[0])
        _expect(first.op in ("ResizeBilinear", "ResizeBilinearV2") and
                g.producer_chain(first.inputs[0], PASS).name == ex(proj_i) and
                g.producer_chain(cat2.inputs[1], PASS).name == ex(low_i),
                f"{cat2.name}: expected [resized ASPP output, low-level projection]")
        _expect(bool(first.attr.get("align_corners", False)), f"{first.name}: decoder resize without align_corners")
        _expect(convs[dec[1][0]].src(g) == ex(dec[0][1]), f"{convs[dec[1][0]].node.name}: decoder chain")
        decoder = [dec[0][2], dec[1][2]]
        _expect(logits_src == ex(dec[1][1]), "logits not over the decoder output")
    else:
        _expect(not dec and logits_src == ex(proj_i), "logits not over the ASPP projection")
    os_ = convs[r0].stride
    for m in modules:
        os_ *= m.seps[2].dw.stride
    return X.DeepLabXception([conv_at(r0), conv_at(r1)], modules, low_at if low_proj is not None else (1, 1), pool,
                             aspp0, atrous_seps, project, low_proj, decoder, logits, logits.cout, os_, crop_h,
                             meta=dict(source="graphdef", backbone="xception_65",
                                       atrous_rates=tuple(a.dw.dil for a in atrous_seps)),
                             crop_w=crop_w if crop_w != crop_h else 0)


def _dense_aspp(g: Graph, convs: list, rest: list, backbone: str, exit_of: dict, conv_at, need_act):
    """The DeepLabV3 head over `backbone` with dense ASPP branches (MobileNetV2, ResNet): convolutions
    `rest` classified by what feeds them — a spatial Mean / AvgPool of the backbone: image pooling; the
    backbone itself: the 1x1 branch or a 3x3 atrous branch; the branches' ConcatV2: the projection; the
    projection's output: the logits — and the projection's input channels permuted from the graph's
    concat order to the engine's [pool, 1x1, atrous...] -> (pool, aspp0, atrous convs, project, logits)."""
    pool = aspp0 = project = logits = None
    pool_i = aspp0_i = proj_i = None
    atrous = []            # (index, conv)
    concat = None
    for j in rest:
        c = convs[j]
        _expect(not c.depthwise, f"{c.node.name}: depthwise convolution in the ASPP head (separable ASPP is "
                                 "the Xception variant; not supported)")
        src = g.node(c.src(g))
        if src.op in ("Mean", "AvgPool") and g.producer_chain(src.inputs[0], PASS).name == backbone:
            if src.op == "Mean":
                ax = sorted(int(v) % 4 for v in np.atleast_1d(g.const(src.inputs[1])))
                _expect(ax == [1, 2], f"{src.name}: mean over axes {ax}, expected the spatial axes")
            _expect(pool is None and c.k == 1, f"{c.node.name}: second / non-1x1 image-pooling convolution")
            need_act(j, D.ACT_RELU, "image pooling")
            pool, pool_i = conv_at(j), j
        elif src.name == backbone:
            need_act(j, D.ACT_RELU, "ASPP branch")
            if c.k == 1:
                _expect(aspp0 is None, f"{c.node.name}: second 1x1 ASPP branch")
                aspp0, aspp0_i = conv_at(j), j
            else:
                _expect(c.k == 3, f"{c.node.name}: ASPP branch kernel {c.k}")
                atrous.append((j, conv_at(j)))
        elif src.op == "ConcatV2":
            _expect(project is None and c.k == 1, f"{c.node.name}: second / non-1x1 concat projection")
            need_act(j, D.ACT_RELU, "concat projection")
            project, proj_i = conv_at(j), j
            concat = src
        elif proj_i is not None and c.src(g) == exit_of[id(convs[proj_i])]:
            _expect(logits is None and c.k == 1, f"{c.node.name}: second / non-1x1 logits convolution")
            need_act(j, D.ACT_NONE, "logits")
            logits = conv_at(j)
        else:
            raise GraphImportError(f"{c.node.name}: convolution fed by {src.name} ({src.op}) has no DeepLab role")
    _expect(pool is not None and aspp0 is not None and project is not None and logits is not None,
            "missing ASPP parts: " + ", ".join(n for n, v in (("image pooling", pool), ("1x1 branch", aspp0),
                                                               ("projection", project), ("logits", logits)) if v is None))
    # concat order -> engine order [pool, aspp0, atrous...]
    by_exit = {exit_of[id(convs[j])]: j for j in [pool_i, aspp0_i] + [a for a, _ in atrous]}
    perm, atr_sorted = _aspp_concat_perm(g, concat, by_exit, pool_i, aspp0_i,
                                         {j: convs[j].cout for j in by_exit.values()}, project.w.shape[1])
    project.w = np.ascontiguousarray(project.w[:, perm])
    atrous_convs = [dict(atrous)[j] for j in atr_sorted]
    Dd = aspp0.cout
    _expect(pool.cout == Dd and all(a.cout == Dd for a in atrous_convs) and project.cout == Dd,
            "ASPP branches and projection differ in depth")
    return pool, aspp0, atrous_convs, project, logits


def _import_resnet(g: Graph, convs: list, closures: list, crop_h: int, crop_w: int):
    """The DeepLabV3 ResNet-v1-beta export (deeplab_resnet.py documents the topology) by data flow:
    three root convs (the first strided with fixed_padding), a 3x3 s2 ``MaxPool``, then bottleneck units
    — a 1x1 + ReLU reading the unit input, a 3x3 + ReLU after it, a linear 1x1 whose output meets the
    shortcut (the unit input, its 1x1 ``MaxPool`` subsample, or a linear 1x1 conv of it) at an ``Add``
    followed by ``Relu`` — until no unit starts at the current tensor; then the dense ASPP head."""
    from . import deeplab_resnet as R
    exit_of = {id(c): ex for c, (_, _, ex) in zip(convs, closures)}
    ex = lambda i: exit_of[id(convs[i])]  # noqa: E731
    act = lambda i: closures[i][1]  # noqa: E731

    def conv_at(i):
        f, a, _ = closures[i]
        return _make(convs[i], f, a)

    def need_act(i, want, role):
        _expect(act(i) == want, f"{role} ({convs[i].node.name}): expected {_ACT_NAME[want]} after it, "
                                f"graph has {_ACT_NAME[act(i)]}")

    def strided_ok(i):
        c = convs[i]
        if c.stride > 1 and c.k > 1:
            _expect(_fixed(c), f"{c.node.name}: strided convolution without fixed_padding")
        else:
            _expect(c.explicit is None, f"{c.node.name}: explicit padding on a stride-1 convolution")

    n = len(convs)
    for i in range(3):
        strided_ok(i)
        need_act(i, D.ACT_RELU, "root conv")
        _expect(not convs[i].depthwise and convs[i].k == 3, f"{convs[i].node.name}: root conv")
        if i:
            _expect(convs[i].src(g) == ex(i - 1) and convs[i].cin == convs[i - 1].cout, f"{convs[i].node.name}: root chain")
    pools = [m for m in g.consumers[ex(2)] if m.op == "MaxPool"]
    _expect(len(pools) == 1, f"{convs[2].node.name}: no max pool after the root")
    mp = pools[0]
    _expect([int(v) for v in mp.attr.get("ksize")] == [1, 3, 3, 1] and [int(v) for v in mp.attr.get("strides")] == [1, 2, 2, 1]
            and _s(mp.attr.get("padding", b"")) == "SAME", f"{mp.name}: expected a 3x3 stride-2 SAME max pool")
    by_src: dict = {}
    for j in range(3, n):
        by_src.setdefault(convs[j].src(g), []).append(j)
    cur, cur_c = mp.name, convs[2].cout
    units, used = [], set(range(3))
    os_ = convs[0].stride * 2
    while True:
        found = None
        for j1 in by_src.get(cur, []):
            c1 = convs[j1]
            if c1.depthwise or c1.k != 1 or act(j1) != D.ACT_RELU:
                continue
            n2 = by_src.get(ex(j1), [])
            if len(n2) != 1 or convs[n2[0]].depthwise or convs[n2[0]].k != 3 or act(n2[0]) != D.ACT_RELU:
                continue
            n3 = by_src.get(ex(n2[0]), [])
            if len(n3) != 1 or convs[n3[0]].depthwise or convs[n3[0]].k != 1 or act(n3[0]) != D.ACT_NONE:
                continue
            adds = [a for a in g.consumers[ex(n3[0])] if a.op in ("Add", "AddV2")]
            if len(adds) == 1:
                found = (j1, n2[0], n3[0], adds[0])
                break
        if found is None:
            break
        j1, j2, j3, add = found
        others = [g.producer_chain(t, PASS) for t in add.inputs if g.producer_chain(t, PASS).name != ex(j3)]
        _expect(len(others) == 1, f"{add.name}: not a two-way residual add")
        o, stride = others[0], convs[j2].stride
        strided_ok(j2)
        _expect(convs[j1].cin == cur_c and convs[j2].cin == convs[j1].cout and convs[j3].cin == convs[j2].cout,
                f"{convs[j1].node.name}: bottleneck channel counts")
        sc = None
        if o.name == cur:
            _expect(stride == 1 and convs[j3].cout == cur_c, f"{add.name}: identity shortcut over a shape change")
        elif o.op == "MaxPool" and g.producer_chain(o.inputs[0], PASS).name == cur:
            _expect([int(v) for v in o.attr.get("ksize")] == [1, 1, 1, 1] and
                    [int(v) for v in o.attr.get("strides")] == [1, stride, stride, 1] and convs[j3].cout == cur_c,
                    f"{o.name}: shortcut subsample does not match the unit stride")
        else:
            js = [j for j in by_src.get(cur, []) if ex(j) == o.name]
            _expect(len(js) == 1 and convs[js[0]].k == 1 and not convs[js[0]].depthwise and convs[js[0]].stride == stride
                    and convs[js[0]].cout == convs[j3].cout, f"{add.name}: shortcut is not a 1x1 conv of the unit input")
            need_act(js[0], D.ACT_NONE, "shortcut")
            sc = conv_at(js[0])
            used.add(js[0])
        relus = [r for r in g.consumers[add.name] if r.op == "Relu"]
        _expect(len(relus) == 1, f"{add.name}: no ReLU after the residual add")
        units.append(R.Unit(conv_at(j1), conv_at(j2), conv_at(j3), sc, stride))
        used.update((j1, j2, j3))
        cur, cur_c = relus[0].name, convs[j3].cout
        os_ *= stride
    _expect(units, "no bottleneck units after the root")
    rest = [j for j in range(n) if j not in used]
    pool, aspp0, atrous_convs, project, logits = _dense_aspp(g, convs, rest, cur, exit_of, conv_at, need_act)
    return R.DeepLabResNet([conv_at(0), conv_at(1), conv_at(2)], units, pool, aspp0, atrous_convs, project, logits,
                           logits.cout, os_, crop_h,
                           meta=dict(source="graphdef", backbone="resnet_v1_beta", atrous_rates=tuple(a.dil for a in atrous_convs)),
                           crop_w=crop_w if crop_w != crop_h else 0)


def _relu_of(g: Graph, name: str):
    """If `name` is (through identity-like ops) a Relu, the tensor it rectifies; else None."""
    n = g.producer_chain(name, PASS)
    return g.producer_chain(n.inputs[0], PASS).name if n.op == "Relu" else None


def import_deeplab(data: bytes, crop=None, default_crop: int = D.CROP) -> D.DeepLab:
    """Frozen DeepLab GraphDef bytes -> the engine's network (weights + topology): deeplab_spec.DeepLab
    (MobileNetV2), deeplab_xception.DeepLabXception or deeplab_resnet.DeepLabResNet, told apart by the
    root's convolutions.
    crop: None reads the export's crop from the graph (read_crop; ``default_crop`` when the graph
    holds none), an int or (height, width) overrides it."""
    g = Graph(parse_graphdef(data))
    if crop is None:
        crop = read_crop(g) or default_crop
    crop_h, crop_w = (int(crop), int(crop)) if np.ndim(crop) == 0 else (int(crop[0]), int(crop[1]))
    convs = [_Conv(g, n) for n in g.nodes if n.op in CONV_OPS]
    _expect(len(convs) >= 6, f"graph has {len(convs)} convolutions; not a DeepLab export")
    st = convs[0]
    _expect(not st.depthwise and st.cin == 3 and st.k == 3, f"{st.node.name}: the first convolution is not a "
                                                            "3x3 stem over the RGB input")
    if not convs[1].depthwise and convs[1].k == 3:
        # a second full 3x3 convolution: the Xception root (MobileNetV2 goes on with a depthwise one); a third
        # one: the ResNet-v1-beta root (Xception goes on with a depthwise one)
        closures = [_affine_act(g, c, act_ends=True) for c in convs]
        if len(convs) > 2 and not convs[2].depthwise and convs[2].k == 3:
            return _import_resnet(g, convs, closures, crop_h, crop_w)
        return _import_xception(g, convs, closures, crop_h, crop_w)
    closures = [_affine_act(g, c) for c in convs]
    exit_of = {id(c): ex for c, (_, _, ex) in zip(convs, closures)}

    def conv_at(i):
        f, act, _ = closures[i]
        return _make(convs[i], f, act)

    def need_act(i, want, role):
        _expect(closures[i][1] == want, f"{role} ({convs[i].node.name}): expected {_ACT_NAME[want]} after it, "
                                        f"graph has {_ACT_NAME[closures[i][1]]}")

    # stem
    for c in convs:
        _expect(c.explicit is None, f"{c.node.name}: explicit padding in a MobileNetV2 graph")
    need_act(0, D.ACT_RELU6, "stem")
    stem = conv_at(0)
    cur = exit_of[id(st)]
    cur_c = st.cout
    # inverted residual blocks
    blocks = []
    i = 1
    while i + 1 < len(convs):
        c0 = convs[i]
        if c0.depthwise:
            ex_i, dw_i = None, i
        elif c0.k == 1 and convs[i + 1].depthwise and convs[i + 1].src(g) == exit_of[id(c0)]:
            ex_i, dw_i = i, i + 1
        else:
            break
        pj_i = dw_i + 1
        _expect(pj_i < len(convs), "graph ends inside an inverted residual block")
        first = convs[ex_i if ex_i is not None else dw_i]
        _expect(first.src(g) == cur, f"{first.node.name}: block input is {first.src(g)}, expected {cur}")
        dw, pj = convs[dw_i], convs[pj_i]
        _expect(dw.k == 3, f"{dw.node.name}: depthwise kernel {dw.k}x{dw.k}")
        _expect(not pj.depthwise and pj.k == 1 and pj.src(g) == exit_of[id(dw)],
                f"{pj.node.name}: expected the 1x1 projection of {dw.node.name}")
        if ex_i is not None:
            _expect(c0.cin == cur_c, f"{c0.node.name}: {c0.cin} input channels, block input has {cur_c}")
            need_act(ex_i, D.ACT_RELU6, "expansion")
        _expect(dw.cin == (convs[ex_i].cout if ex_i is not None else cur_c), f"{dw.node.name}: channel count")
        need_act(dw_i, D.ACT_RELU6, "depthwise")
        need_act(pj_i, D.ACT_NONE, "projection")
        pex = exit_of[id(pj)]
        adds = [a for a in g.consumers[pex] if a.op in ("Add", "AddV2")
                and cur in [g.producer_chain(s, PASS).name for s in a.inputs]]
        residual = bool(adds)
        if residual:
            _expect(pj.cout == cur_c and dw.stride == 1, f"{adds[0].name}: residual over a shape change")
            cur = adds[0].name
        else:
            cur = pex
        blocks.append(D.Block(conv_at(ex_i) if ex_i is not None else None, conv_at(dw_i), conv_at(pj_i), residual))
        cur_c = pj.cout
        i = pj_i + 1
    _expect(blocks, "no inverted residual blocks after the stem")
    backbone = cur
    pool, aspp0, atrous_convs, project, logits = _dense_aspp(g, convs, list(range(i, len(convs))), backbone, exit_of,
                                                             conv_at, need_act)
    # output stride: product of the strides on the way to the backbone output
    os_ = stem.stride
    for b in blocks:
        os_ *= b.dw.stride
    net = D.DeepLab(stem, blocks, pool, aspp0, atrous_convs, project, logits, logits.cout, os_, crop_h,
                    meta=dict(source="graphdef", atrous_rates=tuple(a.dil for a in atrous_convs)),
                    crop_w=crop_w if crop_w != crop_h else 0)
    return net


def graphdef_to_npz(data: bytes, path, crop=None) -> D.DeepLab:
    net = import_deeplab(data, crop=crop)
    D.save(net, path)
    return net


if __name__ == "__main__":
    import sys
    if len(sys.argv) != 3:
        print("usage: python -m bugcar_image_segmentation_amd.deeplab_graphdef deeplab.pb deeplab.npz", file=sys.stderr)
        sys.exit(2)
    with open(sys.argv[1], "rb") as f:
        net = graphdef_to_npz(f.read(), sys.argv[2])
    body = net.blocks if hasattr(net, "blocks") else net.modules if hasattr(net, "modules") else net.units
    print(f"{sys.argv[2]}: {type(net).__name__}, {len(body)} blocks, {net.num_classes} classes, output stride "
          f"{net.output_stride}, crop {D.crop_hw(net)}")
