"""DeepLabV3+ over the aligned Xception-65 backbone: topology, synthetic weights and lowering to the
executor's op list. SURVEY.md §8(f) row 3 / config 4 — the other backbone a frozen ``deeplab.pb``
of the TF DeepLab model zoo can hold (``xception65_coco_voc_trainaug``: output stride 16, atrous
rates 6/12/18, decoder output stride 4, crop 513). The reference (models.py:98-136) feeds the export
u8 RGB and reads int64 class ids; which backbone its absent ``deeplab.pb`` carries is unknown
(SURVEY.md §2 #7), so both zoo forms run on the same op kinds.

Topology (deeplab/core/xception.py ``xception_65``, deeplab/model.py):

* root: ``conv2d_same`` 3x3 s2 32 + BN + ReLU (stride 2: explicit ``fixed_padding``, then VALID),
  3x3 s1 64 + BN + ReLU;
* xception modules of three separable convs (3x3 depthwise + BN, 1x1 pointwise + BN), the third one
  carrying the module stride (explicit fixed padding when strided):
    entry  [128]x3 s2, [256]x3 s2, [728]x3 s2      skip: 1x1 conv (stride) + BN, added
    middle 16 x [728]x3 s1                          skip: identity sum
    exit   [728, 1024, 1024] s2                     skip: 1x1 conv + BN
           [1536, 1536, 2048] s1                    no skip; ReLU inside the separable convs
  every other module applies ReLU to its input ahead of each separable conv
  (``activation_fn_in_separable_conv=False``); the skip takes the un-rectified input;
* output stride: once reached, strides turn into atrous rates (``stack_blocks_dense``: stride 1,
  rate = running rate, rate *= stride), the exit flow's last module at rate x ``multi_grid``;
* ASPP: image pooling (global mean at the crop, 1x1 256 + BN + ReLU, broadcast), 1x1 256 + BN +
  ReLU, one *separable* atrous branch per rate (3x3 depthwise at the rate + BN + ReLU, 1x1 256 +
  BN + ReLU), concat [pool, 1x1, atrous...], 1x1 projection 256 + BN + ReLU;
* decoder (``refine_by_decoder``, decoder output stride 4): the ASPP output resized (bilinear,
  align_corners) to the size of the low-level features — entry block 2's second pointwise output
  (``entry_flow/block2/unit_1/xception_module/separable_conv2_pointwise``, BN, before any ReLU) —
  concat with their 1x1 48 + BN + ReLU projection, two separable 3x3 convs 256 (ReLU after the
  depthwise and after the pointwise);
* logits 1x1 with bias at the decoder resolution; bilinear resize to the crop; argmax.

The oracle is ``oracle/deeplab_oracle.py`` (its Xception forward) on the same synthetic weights;
parity is UNPINNED against TF on the real file (absent).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import deeplab_spec as D
from .deeplab_spec import ACT_NONE, ACT_RELU, Conv, _Init, _r, _r8, same_pad

LOW_LEVEL_DEPTH = 48
DECODER_DEPTH = 256
# (depths, skip, stride, number of units) per xception_65 block; the exit flow's last block has the
# activation inside its separable convs
X65_BLOCKS = [((128, 128, 128), "conv", 2, 1), ((256, 256, 256), "conv", 2, 1), ((728, 728, 728), "conv", 2, 1),
              ((728, 728, 728), "sum", 1, 16),
              ((728, 1024, 1024), "conv", 2, 1), ((1536, 1536, 2048), "none", 1, 1)]


@dataclass
class SepConv:
    """split_separable_conv2d / separable_conv2d_same: 3x3 depthwise + BN (+ act), 1x1 + BN (+ act)."""
    dw: Conv
    pw: Conv
    pre_relu: bool = False       # ReLU on the input first (activation_fn_in_separable_conv=False)


@dataclass
class XModule:
    seps: list                   # three SepConv; the third carries the stride
    skip: str                    # "conv" | "sum" | "none"
    shortcut: Conv | None = None


@dataclass
class DeepLabXception:
    root: list                   # [3x3 s2 32, 3x3 64]
    modules: list
    low_level: tuple             # (module index, separable conv index): its pointwise output feeds the decoder
    pool: Conv
    aspp0: Conv
    atrous: list                 # SepConv per atrous rate
    project: Conv
    low_proj: Conv | None        # decoder: 1x1 48 over the low-level features (None: no decoder)
    decoder: list                # decoder: two SepConv
    logits: Conv
    num_classes: int = D.NUM_CLASSES
    output_stride: int = 16
    crop: int = D.CROP
    meta: dict = field(default_factory=dict)
    crop_w: int = 0


def scale_dimension(dim: int, scale: float) -> int:
    """deeplab/core/utils.py scale_dimension: int((dim - 1) * scale + 1)."""
    return int((float(dim) - 1.0) * scale + 1.0)


def xgeom(n: int, k: int, s: int, d: int):
    """Output size and pad-before of a resnet_utils conv2d_same / separable_conv2d_same: stride 1 is
    SAME; a strided one pads the input explicitly by fixed_padding ((k_eff - 1) // 2 before) and runs
    VALID."""
    if s == 1:
        return same_pad(n, k, s, d)
    ke = k + (k - 1) * (d - 1)
    return (n + ke - 1 - ke) // s + 1, (ke - 1) // 2


def _sep(ini: _Init, cin, cout, act, *, stride=1, dil=1, pre_relu=False, pw_gamma=(0.5, 1.5)) -> SepConv:
    dw = ini.conv(cin, cin, 3, act, stride=stride, dil=dil, depthwise=True)
    pw = ini.conv(cout, cin, 1, act, gamma=pw_gamma)
    if act == ACT_NONE:          # its input is not rectified: unit gain instead of He's sqrt(2)
        pw.w = (pw.w / np.sqrt(2.0)).astype(np.float32)
    return SepConv(dw, pw, pre_relu)


def build_deeplab_xception(seed: int = 6543, num_classes: int = D.NUM_CLASSES, output_stride: int = 16,
                           atrous_rates=(6, 12, 18), crop=D.CROP, width: float = 1.0, middle: int = 16,
                           decoder: bool = True, multi_grid=(1, 1, 1)) -> DeepLabXception:
    """Synthetic-weight DeepLabV3+ Xception-65 (He-normal convs, BN as in deeplab_spec.build_deeplab;
    the last pointwise BN of every residual module draws gamma from U(0.05, 0.15) and the linear
    1x1s take unit gain, so the 21-module residual stream stays O(1) without trained statistics). `width` scales channel counts and
    `middle` the middle-flow repeats (tests use small ones); `crop` an int or (height, width)."""
    crop_h, crop_w = (int(crop), 0) if np.ndim(crop) == 0 else (int(crop[0]), int(crop[1]))
    ini = _Init(seed)
    ch = lambda c: max(8, int(round(c * width / 8)) * 8)  # noqa: E731
    root = [ini.conv(ch(32), 3, 3, ACT_RELU, stride=2), ini.conv(ch(64), ch(32), 3, ACT_RELU)]
    modules = []
    cin = ch(64)
    cur_stride, rate = 2, 1
    blocks = [(d, sk, s, middle if sk == "sum" else n) for d, sk, s, n in X65_BLOCKS]
    for bi, (depths, skip, stride, units) in enumerate(blocks):
        last_block = bi == len(blocks) - 1
        for _ in range(units):
            if output_stride is not None and cur_stride == output_stride:
                ustride, urate = 1, rate
                rate *= stride
            else:
                ustride, urate = stride, 1
                cur_stride *= stride
            seps = []
            c = cin
            for i, dep in enumerate(depths):
                r = urate * (multi_grid[i] if last_block else 1)
                last = i == 2
                small = last and skip != "none"
                seps.append(_sep(ini, c, ch(dep), ACT_RELU if last_block else ACT_NONE,
                                 stride=ustride if last else 1, dil=r, pre_relu=not last_block,
                                 pw_gamma=(0.05, 0.15) if small else (0.5, 1.5)))
                c = ch(dep)
            sc = ini.conv(c, cin, 1, ACT_NONE, stride=ustride) if skip == "conv" else None
            if sc is not None:
                sc.w = (sc.w / np.sqrt(2.0)).astype(np.float32)
            modules.append(XModule(seps, skip, sc))
            cin = c
    Dd = D.ASPP_DEPTH if width >= 1.0 else ch(D.ASPP_DEPTH)
    pool = ini.conv(Dd, cin, 1, ACT_RELU)
    aspp0 = ini.conv(Dd, cin, 1, ACT_RELU)
    atrous = [_sep(ini, cin, Dd, ACT_RELU, dil=int(r)) for r in atrous_rates]
    project = ini.conv(Dd, Dd * (2 + len(atrous)), 1, ACT_RELU)
    low_proj, dec = None, []
    if decoder:
        low_c = modules[1].seps[1].pw.cout
        low_proj = ini.conv(ch(LOW_LEVEL_DEPTH), low_c, 1, ACT_RELU)
        dd = DECODER_DEPTH if width >= 1.0 else ch(DECODER_DEPTH)
        dec = [_sep(ini, Dd + low_proj.cout, dd, ACT_RELU), _sep(ini, dd, dd, ACT_RELU)]
        head_c = dd
    else:
        head_c = Dd
    logits = ini.conv(num_classes, head_c, 1, ACT_NONE, bn=False, bias=True)
    logits.w = (ini.r.standard_normal(logits.w.shape) * np.sqrt(1.0 / head_c)).astype(np.float32)
    return DeepLabXception(root, modules, (1, 1), pool, aspp0, atrous, project, low_proj, dec, logits, num_classes,
                           output_stride, crop_h, meta=dict(seed=seed, atrous_rates=tuple(int(r) for r in atrous_rates),
                                                             width=width, middle=middle, backbone="xception_65"),
                           crop_w=crop_w if crop_w != crop_h else 0)


def feature_sizes(net: DeepLabXception, H: int, W: int):
    """-> ((h, w) of the backbone output, (h, w) of the low-level features) for an H x W crop."""
    sizes = []
    for n in (H, W):
        n, _ = xgeom(n, 3, 2, 1)
        n, _ = xgeom(n, 3, 1, 1)
        low = None
        for mi, m in enumerate(net.modules):
            for si, sp in enumerate(m.seps):
                n, _ = xgeom(n, 3, sp.dw.stride, sp.dw.dil)
                if (mi, si) == tuple(net.low_level):
                    low = n
        sizes.append((n, low))
    return (sizes[0][0], sizes[1][0]), (sizes[0][1], sizes[1][1])


def lower_xception(net: DeepLabXception, B: int, bf16: bool, nb=None, fuse_prep: bool = True):
    """-> (weight blob, ops, buffer bytes, info) as deeplab_spec.lower. Buffers: 0 input, 1/2 module
    ping-pong, 3 depthwise out, 4 pointwise out inside a module, 5 module shortcut, 6 low-level
    features, 7 logits (f32), 8/9/10 image pooling (partials, per-image projection bias, branch
    output; f32), 11 ASPP concat, 12 ASPP projection / decoder output, 13 decoder concat, 14 ASPP /
    decoder depthwise out, 15 decoder pointwise out."""
    L = D.Lowering(B, bf16, 16, nb)
    es = L.es
    Hc, Wc = D.crop_hw(net)
    L.use(0, B * Hc * Wc * 8 * es)
    if not fuse_prep:
        L.op([D.OP_PREP, 0], "prep", 0, B * Hc * Wc * (3 + 8 * es))

    def geom(c: Conv, H, W):
        Ho, pt = xgeom(H, c.k, c.stride, c.dil)
        Wo, pl = xgeom(W, c.k, c.stride, c.dil)
        return Ho, pt, Wo, pl

    r0, r1 = net.root
    H, W = L.conv(r0, 0, Hc, Wc, 8, 2, _r8(r0.cout), tag="conv stem", rgb=fuse_prep, geom=geom(r0, Hc, Wc))
    if fuse_prep and int(L.ops[-1][31]) != 2:
        raise ValueError("fuse_prep needs the tap-packed stem (3x3 over the 8-channel input)")
    H, W = L.conv(r1, 2, H, W, r0.cout, 1, r1.cout, tag="conv root", geom=geom(r1, H, W))
    cur, C = 1, r1.cout
    low = None
    for mi, m in enumerate(net.modules):
        nxt = 2 if cur == 1 else 1
        X, Cx, Hx, Wx = cur, C, H, W
        src = X
        for si, sp in enumerate(m.seps):
            Ho, Wo = L.dw(sp.dw, src, 3, H, W, C, in_relu=sp.pre_relu, geom=geom(sp.dw, H, W),
                          tag="dw" if sp.dw.stride == 1 else "dw s2")
            res = -1
            if si == 2:
                dst = nxt
                if m.skip == "conv":
                    L.conv(m.shortcut, X, Hx, Wx, Cx, 5, m.shortcut.cout, tag="conv shortcut",
                           geom=geom(m.shortcut, Hx, Wx))
                    res = 5
                elif m.skip == "sum":
                    res = X
            else:
                dst = 6 if (mi, si) == tuple(net.low_level) else 4
            L.conv(sp.pw, 3, Ho, Wo, C, dst, sp.pw.cout, res=res, tag="conv pointwise")
            if dst == 6:
                low = (Ho, Wo, sp.pw.cout)
            src, C, H, W = dst, sp.pw.cout, Ho, Wo
        cur = nxt

    # ASPP (image pooling as the projection's per-image bias, as in the MobileNetV2 plan)
    Dd = net.aspp0.cout
    cat_cs = Dd * (1 + len(net.atrous))
    h, w = H, W
    zs = L.aspp_pool(net, cur, h, w, C)
    L.conv(net.aspp0, cur, h, w, C, 11, cat_cs, out_off=0, tag="conv aspp")
    for i, a in enumerate(net.atrous):
        L.dw(a.dw, cur, 14, h, w, C, tag="dw atrous")
        L.conv(a.pw, 14, h, w, C, 11, cat_cs, out_off=Dd * (i + 1), tag="conv atrous pointwise")
    L.conv(L.projection_conv(net), 11, h, w, cat_cs, 12, Dd, bias_img=9, bias_img_stride=zs, zero_bias=True,
           tag="conv project")
    head, hh, hw_, hc = 12, h, w, Dd
    if net.low_proj is not None:
        if low is None:
            raise ValueError("low-level feature point not found")
        lh, lw, lc = low
        dcs = Dd + net.low_proj.cout
        L.resize(12, 13, h, w, Dd, Dd, lh, lw, dcs, 0)
        L.conv(net.low_proj, 6, lh, lw, lc, 13, dcs, out_off=Dd, tag="conv low-level")
        s0, s1 = net.decoder
        L.dw(s0.dw, 13, 14, lh, lw, dcs, tag="dw decoder")
        L.conv(s0.pw, 14, lh, lw, dcs, 15, s0.pw.cout, tag="conv decoder")
        L.dw(s1.dw, 15, 14, lh, lw, s0.pw.cout, tag="dw decoder")
        L.conv(s1.pw, 14, lh, lw, s0.pw.cout, 12, s1.pw.cout, tag="conv decoder")
        head, hh, hw_, hc = 12, lh, lw, s1.pw.cout
    LCS = _r(net.num_classes, 8)
    L.conv(net.logits, head, hh, hw_, hc, 7, LCS, out_f32=True, cout=LCS, tag="conv logits")
    L.argmax(7, hh, hw_, LCS, net.num_classes, Hc, Wc)
    L.info.update(feature=(hh, hw_), lcs=LCS, backbone=(h, w))
    return L.result()


# ---------------------------------------------------------------- weight file (.npz, no pickle)
_SKIP = {"none": 0, "sum": 1, "conv": 2}


def _named_convs(net: DeepLabXception):
    yield "root0", net.root[0]
    yield "root1", net.root[1]
    for i, m in enumerate(net.modules):
        for j, sp in enumerate(m.seps):
            yield f"m{i}.s{j}.dw", sp.dw
            yield f"m{i}.s{j}.pw", sp.pw
        if m.shortcut is not None:
            yield f"m{i}.shortcut", m.shortcut
    yield "pool", net.pool
    yield "aspp0", net.aspp0
    for i, a in enumerate(net.atrous):
        yield f"atrous{i}.dw", a.dw
        yield f"atrous{i}.pw", a.pw
    yield "project", net.project
    if net.low_proj is not None:
        yield "low_proj", net.low_proj
        for i, sp in enumerate(net.decoder):
            yield f"dec{i}.dw", sp.dw
            yield f"dec{i}.pw", sp.pw
    yield "logits", net.logits


def save_xception(net: DeepLabXception, path) -> None:
    arrs = {}
    D.conv_arrays(arrs, _named_convs(net))
    arrs["net.xattrs"] = np.array([net.num_classes, net.output_stride or 0, net.crop, net.crop_w or 0,
                                   len(net.modules), len(net.atrous), int(net.low_proj is not None),
                                   net.low_level[0], net.low_level[1]], np.int32)
    arrs["net.xmodules"] = np.array([[_SKIP[m.skip]] + [int(sp.pre_relu) for sp in m.seps] for m in net.modules],
                                    np.int32)
    np.savez(path, **arrs)


def load_xception(z, path="") -> DeepLabXception:
    conv = lambda name: D.conv_from(z, name, path)  # noqa: E731
    ncls, os_, crop, crop_w, nmod, natr, dec, lm, ls = (int(v) for v in z["net.xattrs"])
    inv = {v: k for k, v in _SKIP.items()}
    modules = []
    for i, row in enumerate(z["net.xmodules"]):
        seps = [SepConv(conv(f"m{i}.s{j}.dw"), conv(f"m{i}.s{j}.pw"), bool(row[1 + j])) for j in range(3)]
        skip = inv[int(row[0])]
        modules.append(XModule(seps, skip, conv(f"m{i}.shortcut") if skip == "conv" else None))
    if len(modules) != nmod:
        raise ValueError(f"{path}: {len(modules)} modules, attributes say {nmod}")
    atrous = [SepConv(conv(f"atrous{i}.dw"), conv(f"atrous{i}.pw")) for i in range(natr)]
    low_proj = conv("low_proj") if dec else None
    decoder = [SepConv(conv(f"dec{i}.dw"), conv(f"dec{i}.pw")) for i in range(2)] if dec else []
    return DeepLabXception([conv("root0"), conv("root1")], modules, (lm, ls), conv("pool"), conv("aspp0"), atrous,
                           conv("project"), low_proj, decoder, conv("logits"), ncls, os_ or None, crop,
                           meta=dict(source=str(path), backbone="xception_65"), crop_w=crop_w)
