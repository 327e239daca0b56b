"""DeepLabV3 over a ResNet-v1 "beta" backbone: topology, synthetic weights and lowering to the
executor's op list. SURVEY.md §8(f) row 3 / config 4 — the third backbone family a frozen
``deeplab.pb`` of the TF DeepLab code base can hold (deeplab/core/feature_extractor.py
``resnet_v1_50_beta`` / ``resnet_v1_101_beta``; which backbone the reference's absent file carries is
unknown). The reference feeds the export u8 RGB and reads int64 class ids
(models.py:98-136); every op here is one the MobileNetV2 / Xception plans already run, plus max
pooling and a residual epilogue with the ReLU after the add.

Topology (deeplab/core/resnet_v1_beta.py, slim resnet_utils, deeplab/model.py):

* preprocessing: ``_preprocess_zero_mean_unit_range`` (the beta variants), pad to the crop with 127.5,
  ``(2/255) x - 1`` — the same fused stem input as the other backbones;
* root block: ``conv2d_same`` 3x3 s2 64 (explicit fixed padding, then VALID), 3x3 64, 3x3 128, each
  + BN + ReLU, then ``max_pool2d`` 3x3 s2 SAME;
* four blocks of v1 bottleneck units (base depth d, output 4d): block1 (64, units 3, stride 2), block2
  (128, 4, 2), block3 (256, 6 | 23, 2), block4 (512, 3, 1) with ``multi_grid`` unit rates; the block
  stride sits on its LAST unit. A unit: shortcut = ``subsample`` (1x1 max pool, the stride) when the
  depth is unchanged, else 1x1 conv (stride) + BN; residual = 1x1 d + BN + ReLU, ``conv2d_same`` 3x3 d
  (stride, rate) + BN + ReLU, 1x1 4d + BN; out = ReLU(shortcut + residual);
* output stride (``stack_blocks_dense``): once reached, unit strides become atrous rates (stride 1,
  rate = running rate, rate *= stride), block4's units at rate x multi_grid;
* ASPP (deeplab/model.py, ``aspp_with_separable_conv`` off): image pooling, 1x1 256 + BN + ReLU, one
  dense atrous 3x3 256 + BN + ReLU per rate, concat [pool, 1x1, atrous...], 1x1 projection 256 + BN +
  ReLU; logits 1x1 with bias; bilinear resize (align_corners) to the crop; argmax.

The oracle is ``oracle/deeplab_oracle.py`` (``forward_resnet``) on the same synthetic weights;
parity is UNPINNED against TF on a real file (absent).
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field

import numpy as np

from . import deeplab_spec as D
from .deeplab_spec import ACT_NONE, ACT_RELU, Conv, _Init, _r, _r8, same_pad
from .deeplab_xception import xgeom

ACT_RELU_POST = 3          # executor CONV act code: ReLU after the residual add (deeplab_internal.h)
# (base depth, units, stride) per block of resnet_v1_{50,101}_beta
RESNET_BLOCKS = {50: [(64, 3, 2), (128, 4, 2), (256, 6, 2), (512, 3, 1)],
                 101: [(64, 3, 2), (128, 4, 2), (256, 23, 2), (512, 3, 1)]}


@dataclass
class Unit:
    """slim resnet_v1 bottleneck: conv1 1x1 + ReLU, conv2 3x3 (stride, rate) + ReLU, conv3 1x1 (linear),
    shortcut (1x1 conv + BN, or None: identity / subsample by the stride); out = ReLU(shortcut + conv3)."""
    conv1: Conv
    conv2: Conv
    conv3: Conv
    shortcut: Conv | None
    stride: int


@dataclass
class DeepLabResNet:
    root: list                   # [3x3 s2 64, 3x3 64, 3x3 128], then the 3x3 s2 max pool
    units: list
    pool: Conv                   # image pooling 1x1
    aspp0: Conv
    atrous: list                 # dense 3x3 atrous branches
    project: Conv
    logits: Conv
    num_classes: int = D.NUM_CLASSES
    output_stride: int = 16
    crop: int = D.CROP
    meta: dict = field(default_factory=dict)
    crop_w: int = 0


def build_deeplab_resnet(depth: int = 101, seed: int = 7654, num_classes: int = D.NUM_CLASSES, output_stride: int = 16,
                         atrous_rates=(6, 12, 18), multi_grid=(1, 2, 4), crop=D.CROP, width: float = 1.0,
                         units=None) -> DeepLabResNet:
    """Synthetic-weight DeepLabV3 ResNet-v1-{50,101}-beta (He-normal convs, BN as in
    deeplab_spec.build_deeplab; every unit's last BN draws gamma from U(0.05, 0.15) and the projection
    shortcuts take unit gain, so the 16- / 33-unit residual stream stays O(1) without trained
    statistics). `width` scales channel counts, `units` overrides the units per block (tests use small
    ones); `crop` an int or (height, width)."""
    crop_h, crop_w = (int(crop), 0) if np.ndim(crop) == 0 else (int(crop[0]), int(crop[1]))
    ini = _Init(seed)
    ch = lambda c: max(8, int(round(c * width / 8)) * 8)  # noqa: E731
    root = [ini.conv(ch(64), 3, 3, ACT_RELU, stride=2), ini.conv(ch(64), ch(64), 3, ACT_RELU),
            ini.conv(ch(128), ch(64), 3, ACT_RELU)]
    blocks = RESNET_BLOCKS[depth]
    if units is not None:
        blocks = [(d, int(n), s) for (d, _n, s), n in zip(blocks, units)]
    cin = ch(128)
    cur_stride, rate = 4, 1
    out_units = []
    for bi, (base, n, stride) in enumerate(blocks):
        last_block = bi == len(blocks) - 1
        for i in range(n):
            s = stride if i == n - 1 else 1
            if output_stride is not None and cur_stride == output_stride:
                ustride, urate = 1, rate
                rate *= s
            else:
                ustride, urate = s, 1
                cur_stride *= s
            r = urate * (multi_grid[i % len(multi_grid)] if last_block else 1)
            dep, bott = ch(4 * base), ch(base)
            c1 = ini.conv(bott, cin, 1, ACT_RELU)
            c2 = ini.conv(bott, bott, 3, ACT_RELU, stride=ustride, dil=r)
            c3 = ini.conv(dep, bott, 1, ACT_NONE, gamma=(0.05, 0.15))
            sc = None
            if dep != cin:
                sc = ini.conv(dep, cin, 1, ACT_NONE, stride=ustride)
                sc.w = (sc.w / np.sqrt(2.0)).astype(np.float32)
            out_units.append(Unit(c1, c2, c3, sc, ustride))
            cin = dep
    Dd = D.ASPP_DEPTH if width >= 1.0 else ch(D.ASPP_DEPTH)
    pool = ini.conv(Dd, cin, 1, ACT_RELU)
    aspp0 = ini.conv(Dd, cin, 1, ACT_RELU)
    atrous = [ini.conv(Dd, cin, 3, ACT_RELU, dil=int(r)) for r in atrous_rates]
    project = ini.conv(Dd, Dd * (2 + len(atrous)), 1, ACT_RELU)
    logits = ini.conv(num_classes, Dd, 1, ACT_NONE, bn=False, bias=True)
    logits.w = (ini.r.standard_normal(logits.w.shape) * np.sqrt(1.0 / Dd)).astype(np.float32)
    return DeepLabResNet(root, out_units, pool, aspp0, atrous, project, logits, num_classes, output_stride, crop_h,
                         meta=dict(seed=seed, depth=depth, atrous_rates=tuple(int(r) for r in atrous_rates),
                                   multi_grid=tuple(multi_grid), width=width, backbone=f"resnet_v1_{depth}_beta"),
                         crop_w=crop_w if crop_w != crop_h else 0)


def _geom(c: Conv, H, W):
    """(Hout, pad_t, Wout, pad_l) of a conv2d_same (fixed padding when strided, SAME otherwise)."""
    Ho, pt = xgeom(H, c.k, c.stride, c.dil)
    Wo, pl = xgeom(W, c.k, c.stride, c.dil)
    return Ho, pt, Wo, pl


def feature_size(net: DeepLabResNet, n: int) -> int:
    """Spatial size of the backbone output for an n-pixel crop side."""
    for c in net.root:
        n, _ = xgeom(n, 3, c.stride, c.dil)
    n, _ = same_pad(n, 3, 2, 1)                     # the root's max pool
    for u in net.units:
        n, _ = xgeom(n, 3, u.conv2.stride, u.conv2.dil)
    return n


def lower_resnet(net: DeepLabResNet, B: int, bf16: bool, nb=None, fuse_prep: bool = True):
    """-> (weight blob, ops, buffer bytes, info) as deeplab_spec.lower. Buffers: 0 input, 1/2 unit
    ping-pong, 3 / 4 root and bottleneck intermediates, 5 shortcut, 6 (unused), 7 logits (f32),
    8/9/10 image pooling (partials, per-image projection bias, branch output; f32), 11 ASPP concat,
    12 ASPP projection."""
    L = D.Lowering(B, bf16, 13, nb)
    es = L.es
    Hc, Wc = D.crop_hw(net)
    L.use(0, B * Hc * Wc * 8 * es)
    if not fuse_prep:
        L.op([D.OP_PREP, 0], "prep", 0, B * Hc * Wc * (3 + 8 * es))
    r0, r1, r2 = net.root
    H, W = L.conv(r0, 0, Hc, Wc, 8, 3, _r8(r0.cout), tag="conv stem", rgb=fuse_prep, geom=_geom(r0, Hc, Wc))
    if fuse_prep and int(L.ops[-1][31]) != 2:
        raise ValueError("fuse_prep needs the tap-packed stem (3x3 over the 8-channel input)")
    H, W = L.conv(r1, 3, H, W, r0.cout, 4, r1.cout, tag="conv root", geom=_geom(r1, H, W))
    H, W = L.conv(r2, 4, H, W, r1.cout, 3, r2.cout, tag="conv root", geom=_geom(r2, H, W))
    C = r2.cout
    H, W = L.maxpool(3, 1, H, W, C, 3, 2, tag="maxpool root")
    cur = 1
    for u in net.units:
        nxt = 2 if cur == 1 else 1
        if u.shortcut is not None:
            L.conv(u.shortcut, cur, H, W, C, 5, u.shortcut.cout, tag="conv shortcut", geom=_geom(u.shortcut, H, W))
            res = 5
        elif u.stride > 1:
            L.maxpool(cur, 5, H, W, C, 1, u.stride, tag="subsample")
            res = 5
        else:
            res = cur
        L.conv(u.conv1, cur, H, W, C, 3, u.conv1.cout, tag="conv reduce")
        Ho, Wo = L.conv(u.conv2, 3, H, W, u.conv1.cout, 4, u.conv2.cout, tag="conv 3x3" if u.stride == 1 else "conv 3x3 s2",
                        geom=_geom(u.conv2, H, W))
        L.conv(dataclasses.replace(u.conv3, act=ACT_RELU_POST), 4, Ho, Wo, u.conv2.cout, nxt, u.conv3.cout, res=res,
               tag="conv expand")
        H, W, C, cur = Ho, Wo, u.conv3.cout, nxt

    # ASPP (image pooling as the projection's per-image bias, as in the MobileNetV2 plan)
    Dd = net.aspp0.cout
    cat_cs = Dd * (1 + len(net.atrous))
    h, w = H, W
    zs = L.aspp_pool(net, cur, h, w, C)
    L.conv(net.aspp0, cur, h, w, C, 11, cat_cs, out_off=0, tag="conv aspp")
    for i, a in enumerate(net.atrous):
        L.conv(a, cur, h, w, C, 11, cat_cs, out_off=Dd * (i + 1), tag="conv atrous")
    L.conv(L.projection_conv(net), 11, h, w, cat_cs, 12, Dd, bias_img=9, bias_img_stride=zs, zero_bias=True,
           tag="conv project")
    LCS = _r(net.num_classes, 8)
    L.conv(net.logits, 12, h, w, Dd, 7, LCS, out_f32=True, cout=LCS, tag="conv logits")
    L.argmax(7, h, w, LCS, net.num_classes, Hc, Wc)
    L.info.update(feature=(h, w), lcs=LCS, backbone=(h, w))
    return L.result()


# ---------------------------------------------------------------- weight file (.npz, no pickle)
def _named_convs(net: DeepLabResNet):
    for i, c in enumerate(net.root):
        yield f"root{i}", c
    for i, u in enumerate(net.units):
        yield f"u{i}.conv1", u.conv1
        yield f"u{i}.conv2", u.conv2
        yield f"u{i}.conv3", u.conv3
        if u.shortcut is not None:
            yield f"u{i}.shortcut", u.shortcut
    yield "pool", net.pool
    yield "aspp0", net.aspp0
    for i, a in enumerate(net.atrous):
        yield f"atrous{i}", a
    yield "project", net.project
    yield "logits", net.logits


def save_resnet(net: DeepLabResNet, path) -> None:
    arrs = {}
    D.conv_arrays(arrs, _named_convs(net))
    arrs["net.rattrs"] = np.array([net.num_classes, net.output_stride or 0, net.crop, net.crop_w or 0,
                                   len(net.units), len(net.atrous), int(net.meta.get("depth", 0))], np.int32)
    arrs["net.runits"] = np.array([[u.stride, int(u.shortcut is not None)] for u in net.units], np.int32)
    np.savez(path, **arrs)


def load_resnet(z, path="") -> DeepLabResNet:
    conv = lambda name: D.conv_from(z, name, path)  # noqa: E731
    ncls, os_, crop, crop_w, nunits, natr, depth = (int(v) for v in z["net.rattrs"])
    units = []
    for i, (stride, has_sc) in enumerate(z["net.runits"]):
        units.append(Unit(conv(f"u{i}.conv1"), conv(f"u{i}.conv2"), conv(f"u{i}.conv3"),
                          conv(f"u{i}.shortcut") if has_sc else None, int(stride)))
    if len(units) != nunits:
        raise ValueError(f"{path}: {len(units)} units, attributes say {nunits}")
    return DeepLabResNet([conv(f"root{i}") for i in range(3)], units, conv("pool"), conv("aspp0"),
                         [conv(f"atrous{i}") for i in range(natr)], conv("project"), conv("logits"), ncls, os_ or None,
                         crop, meta=dict(source=str(path), depth=depth, backbone=f"resnet_v1_{depth}_beta"),
                         crop_w=crop_w)
