"""DeepLabV3 graph builder: topology, synthetic weights, batch-norm folding, weight packing and
lowering to the executor's op list (libbugseg.so, bugseg_dl_*). SURVEY.md §8(f) row 3 / config 4.

What the reference runs (models.py:98-136) is a frozen TF DeepLab export fed through
``import/ImageTensor:0`` (u8 RGB, batch of images) and read from ``import/SemanticPredictions:0``
(int64 class ids). ``deeplab.pb`` is absent (.MISSING_LARGE_BLOBS:1), so the network here is the
standard export that name denotes — deeplab/export_model.py over the MobileNetV2 feature extractor
of the TF DeepLab model zoo (``mobilenet_v2``, depth multiplier 1, output stride 8, crop 513):

* preprocessing: pad to the crop with the mean pixel 127.5, then ``(2/255) x - 1``;
* MobileNetV2 ``V2_DEF`` (slim): 3x3 s2 conv 32 + ReLU6, then inverted residuals
  (t, c, n, s) = (1,16,1,1) (6,24,2,2) (6,32,3,2) (6,64,4,2) (6,96,3,1) (6,160,3,2) (6,320,1,1):
  1x1 expand + ReLU6 (absent for t = 1), 3x3 depthwise + ReLU6, linear 1x1 projection, residual when
  stride 1 and channels match; once the output stride is reached, strides become atrous rates the
  way slim's ``mobilenet_base`` does it (layer stride 1, layer rate = running rate, rate *= stride);
  every convolution SAME-padded, batch norm (eps 1e-3) after each;
* ASPP (deeplab/model.py ``extract_features``): image pooling (global mean, 1x1 256 + BN + ReLU,
  broadcast back), 1x1 256 + BN + ReLU, optional atrous 3x3 branches (``atrous_rates``: none for the
  MobileNetV2 zoo models; 6/12/18 at output stride 16 for the ResNet / Xception ones, here dense
  convs), concat [pool, 1x1, atrous...], 1x1 projection 256 + BN + ReLU (dropout: identity);
* logits: 1x1 conv with bias; bilinear resize (align_corners=True) to the crop; argmax.

Parity is UNPINNED against TF on the real deeplab.pb (neither exists here); the oracle is
``oracle/deeplab_oracle.py`` on the same synthetic weights.

Op list (``lower``): int32 records of ``OP_FIELDS`` fields, interpreted by deeplab_runtime.cpp:
  PREP   [1, dst]
  CONV   [2, src, dst, res, Hin, Win, CS, Hout, Wout, kh, kw, stride, dil, pad_t, pad_l, cinP, NP,
          w_off, b_off, act, res_cs, out_cs, out_off, cout, out_f32, bias_img_buf, bias_img_stride]
  DW     [3, src, dst, Hin, Win, C, Hout, Wout, stride, dil, pad_t, pad_l, w_off, b_off, act, in_relu]
  POOL   [4, src, part, z, H, W, C, CS, chunk_px, nchunks, cmid, cout, wp_off, bp_off, wq_off, bq_off, z_stride, y]
  ARGMAX [5, logits, h, w, LCS, ncls]
  RESIZE [6, src, dst, h, w, in_cs, C, Hout, Wout, out_cs, out_off]   (bilinear, align_corners; DeepLabV3+ decoder)
  MAXPOOL [7, src, dst, Hin, Win, C, Hout, Wout, k, stride, pad_t, pad_l]   (ResNet root pool / subsample)
CONV act: 0 none, 1 ReLU, 2 ReLU6 (before the residual add), 3 ReLU after the residual add (ResNet).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np
import torch

OP_FIELDS = 32
OP_PREP, OP_CONV, OP_DW, OP_POOL, OP_ARGMAX, OP_RESIZE, OP_MAXPOOL = 1, 2, 3, 4, 5, 6, 7
ACT_NONE, ACT_RELU, ACT_RELU6 = 0, 1, 2
BN_EPS = 1e-3
CROP = 513
NUM_CLASSES = 21
ASPP_DEPTH = 256
# slim mobilenet_v2 V2_DEF: (expansion t, output channels c, repeats n, first stride s)
MNV2_BLOCKS = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2), (6, 320, 1, 1)]


@dataclass
class Conv:
    """One convolution + (optional) inference batch norm + activation. w: (cout, cin/groups, kh, kw)."""
    w: np.ndarray
    b: np.ndarray | None = None        # conv bias (logits only)
    gamma: np.ndarray | None = None    # batch norm (None: no BN)
    beta: np.ndarray | None = None
    mean: np.ndarray | None = None
    var: np.ndarray | None = None
    eps: float = BN_EPS
    act: int = ACT_NONE
    stride: int = 1
    dil: int = 1
    depthwise: bool = False

    @property
    def cout(self):
        return self.w.shape[0]

    @property
    def k(self):
        return self.w.shape[2]

    def folded(self):
        """(w, b) with the batch norm folded in, float64."""
        w = self.w.astype(np.float64)
        b = np.zeros(self.cout) if self.b is None else self.b.astype(np.float64)
        if self.gamma is not None:
            s = self.gamma.astype(np.float64) / np.sqrt(self.var.astype(np.float64) + self.eps)
            w = w * s.reshape(-1, 1, 1, 1)
            b = (b - self.mean) * s + self.beta
        return w, b


@dataclass
class Block:
    """MobileNetV2 inverted residual (slim expanded_conv)."""
    expand: Conv | None
    dw: Conv
    project: Conv
    residual: bool


@dataclass
class DeepLab:
    stem: Conv
    blocks: list
    pool: Conv                   # image pooling 1x1
    aspp0: Conv
    atrous: list                 # 3x3 dense atrous branches
    project: Conv                # concat projection over [pool, aspp0, atrous...]
    logits: Conv
    num_classes: int = NUM_CLASSES
    output_stride: int = 8
    crop: int = CROP             # crop height (the export's crop_size[0])
    meta: dict = field(default_factory=dict)
    crop_w: int = 0              # crop width when the export's crop is not square (0: = crop)


def crop_hw(net: "DeepLab") -> tuple:
    """(crop height, crop width): the padded size every image runs at (pad_to_bounding_box)."""
    return int(net.crop), int(net.crop_w or net.crop)


def same_pad(n_in: int, k: int, s: int, d: int):
    """TF 'SAME': out = ceil(in / s), pad_total = max((out - 1) s + (k - 1) d + 1 - in, 0),
    pad_before = pad_total // 2."""
    out = -(-n_in // s)
    tot = max((out - 1) * s + (k - 1) * d + 1 - n_in, 0)
    return out, tot // 2


class _Init:
    def __init__(self, seed: int):
        self.r = np.random.default_rng(seed)

    def conv(self, cout, cin, k, act, *, stride=1, dil=1, depthwise=False, bn=True, gamma=(0.5, 1.5), bias=False):
        r = self.r
        fan_in = (1 if depthwise else cin) * k * k
        w = (r.standard_normal((cout, 1 if depthwise else cin, k, k)) * np.sqrt(2.0 / fan_in)).astype(np.float32)
        c = Conv(w=w, act=act, stride=stride, dil=dil, depthwise=depthwise)
        if bn:
            c.gamma = r.uniform(*gamma, cout).astype(np.float32)
            c.beta = (r.standard_normal(cout) * 0.1).astype(np.float32)
            c.mean = (r.standard_normal(cout) * 0.1).astype(np.float32)
            c.var = r.uniform(0.5, 1.5, cout).astype(np.float32)
        if bias:
            c.b = (r.standard_normal(cout) * 0.1).astype(np.float32)
        return c


def build_deeplab(seed: int = 4321, num_classes: int = NUM_CLASSES, output_stride: int = 8,
                  atrous_rates=(), crop=CROP, width: float = 1.0) -> DeepLab:
    """Synthetic-weight DeepLabV3-MobileNetV2 (He-normal convs, BN gamma~U(0.5,1.5), beta~N(0,0.1),
    mean~N(0,0.1), var~U(0.5,1.5); the linear projections of residual blocks draw gamma from
    U(0.1,0.3) so the residual stream stays O(1) without trained statistics). `width` scales the
    channel counts (tests use small widths; multiples of 8 are kept). `crop`: an int or (height,
    width)."""
    crop_h, crop_w = (int(crop), 0) if np.ndim(crop) == 0 else (int(crop[0]), int(crop[1]))
    ini = _Init(seed)
    ch = lambda c: max(8, int(round(c * width / 8)) * 8)  # noqa: E731
    stem = ini.conv(ch(32), 3, 3, ACT_RELU6, stride=2)
    blocks = []
    cin = ch(32)
    cur_stride, rate = 2, 1
    for t, c, n, s in MNV2_BLOCKS:
        cout = ch(c) if c != 16 else ch(16)
        for i in range(n):
            st = s if i == 0 else 1
            if output_stride is not None and cur_stride == output_stride:
                lstride, lrate = 1, rate
                rate *= st
            else:
                lstride, lrate = st, 1
                cur_stride *= st
            inner = cin * t
            expand = ini.conv(inner, cin, 1, ACT_RELU6) if t != 1 else None
            dw = ini.conv(inner, inner, 3, ACT_RELU6, stride=lstride, dil=lrate, depthwise=True)
            res = lstride == 1 and cin == cout
            proj = ini.conv(cout, inner, 1, ACT_NONE, gamma=(0.1, 0.3) if res else (0.5, 1.5))
            blocks.append(Block(expand, dw, proj, res))
            cin = cout
    D = ASPP_DEPTH if width >= 1.0 else ch(ASPP_DEPTH)
    pool = ini.conv(D, cin, 1, ACT_RELU)
    aspp0 = ini.conv(D, cin, 1, ACT_RELU)
    atrous = [ini.conv(D, cin, 3, ACT_RELU, dil=int(r)) for r in atrous_rates]
    project = ini.conv(D, D * (2 + len(atrous)), 1, ACT_RELU)
    logits = ini.conv(num_classes, D, 1, ACT_NONE, bn=False, bias=True)
    logits.w = (ini.r.standard_normal(logits.w.shape) * np.sqrt(1.0 / D)).astype(np.float32)
    return DeepLab(stem, blocks, pool, aspp0, atrous, project, logits, num_classes, output_stride, crop_h,
                   meta=dict(seed=seed, atrous_rates=tuple(int(r) for r in atrous_rates), width=width),
                   crop_w=crop_w if crop_w != crop_h else 0)


def feature_size(net: DeepLab, n: int) -> int:
    """Spatial size of the backbone output for an n-pixel crop side."""
    n, _ = same_pad(n, 3, 2, 1)
    for b in net.blocks:
        n, _ = same_pad(n, 3, b.dw.stride, b.dw.dil)
    return n


def _r8(c):
    return (c + 7) // 8 * 8


def _r(c, m):
    return (c + m - 1) // m * m


def _round(a: np.ndarray, bf16: bool) -> np.ndarray:
    """f64/f32 -> f32 holding values representable in the compute type."""
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))
    if bf16:
        t = t.to(torch.bfloat16).to(torch.float32)
    return t.numpy()


class _Blob:
    def __init__(self, bf16: bool):
        self.bf16 = bf16
        self.parts: list[bytes] = []
        self.size = 0

    def add(self, a: np.ndarray, as_compute_type: bool) -> int:
        off = self.size
        t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))
        if as_compute_type and self.bf16:
            raw = t.to(torch.bfloat16).view(torch.int16).numpy().tobytes()
        else:
            raw = t.numpy().tobytes()
        pad = (-len(raw)) % 256
        self.parts.append(raw + b"\0" * pad)
        self.size += len(raw) + pad
        return off

    def bytes(self) -> bytes:
        return b"".join(self.parts)


def pack_conv(c: Conv, cinS: int, bf16: bool, tap_packed: bool = False):
    """-> (packed [NP][taps][cinP] f32 array (values rounded to the compute type), bias [NP], cinP, NP).
    Input channel c of tap (ky, kx) sits at k = (ky * kw + kx) * cinP + c; tap_packed (inputs of at
    most 8 channels): [NP][ceil(taps / 4) * 32] with k = tap * 8 + c."""
    w, b = c.folded()
    cout, cin, kh, kw = w.shape
    cinP, NP = _r(max(cinS, cin), 32), _r(cout, 64)
    if tap_packed:
        assert cinS == 8 and cin <= 8
        taps = kh * kw
        p = np.zeros((NP, (taps + 3) // 4 * 32), np.float64)
        q = np.zeros((cout, taps, 8))
        q[:, :, :cin] = w.transpose(0, 2, 3, 1).reshape(cout, taps, cin)
        p[:cout, :taps * 8] = q.reshape(cout, taps * 8)
    else:
        p = np.zeros((NP, kh * kw, cinP), np.float64)
        p[:cout, :, :cin] = w.transpose(0, 2, 3, 1).reshape(cout, kh * kw, cin)
    bb = np.zeros(NP, np.float64)
    bb[:cout] = b
    return _round(p, bf16), bb.astype(np.float32), cinP, NP


def _pick_nb(tag: str, hw: int, K: int, cout: int, B: int = 16) -> int:
    """Measured on MI355X (bench_deeplab.py per-op times, 16 frames): 4 pixel fragments per wave pay
    for wide, deep 1x1s (960 -> 320: 219 -> 169 us, 576 -> 160: 87 -> 72 us); 2 win for shallow K
    (expansions, 24 -> 144: 30 -> 34 us with 4). BUGSEG_DL_NB=2|4 forces one for A/B runs."""
    env = os.environ.get("BUGSEG_DL_NB")
    if env:
        return int(env)
    if hw <= 4225 and B * hw >= 131072:
        # the output-stride-8 layers at B >= 32 (per-op sweep at B = 64, all 31 convs at 65x65): 4 fragments
        # win from K = 64 / cout = 64 up (960 -> 160: 434 -> 408 us, 160 -> 960: 367 -> 331 us), 8 only
        # for 960 -> 320 (603 -> 548 us); 2 stays best for the 32-channel blocks
        if K >= 576 and cout >= 320:
            return 8
        return 4 if (K >= 64 and cout >= 64) or K >= 256 else 2
    if K >= 576 and cout >= 160:
        return 8    # bf16 only (the launcher uses 4 in fp32): 960 -> 320 165 -> 149 us, elsewhere slower
    return 4 if K >= 192 and cout >= 64 else 2


class Lowering:
    """Op-list builder shared by the backbones (lower, deeplab_xception.lower_xception): the weight
    blob, the op records, each buffer's size and the per-op (tag, flops, bytes) accounting."""

    def __init__(self, B: int, bf16: bool, nbufs: int, nb=None):
        self.B, self.bf16, self.es, self.nb = B, bf16, (2 if bf16 else 4), nb
        self.blob = _Blob(bf16)
        self.ops = []
        self.need = [256] * nbufs
        self.info = dict(flops=0.0, bytes=0.0, per_op=[])

    def use(self, buf, nbytes):
        self.need[buf] = max(self.need[buf], int(nbytes))

    def op(self, rec, tag, flops, nbytes):
        self.ops.append(list(rec) + [0] * (OP_FIELDS - len(rec)))
        self.info["per_op"].append((tag, float(flops), float(nbytes)))
        self.info["flops"] += flops
        self.info["bytes"] += nbytes

    def conv(self, c: Conv, src, H, W, CS, dst, out_cs, out_off=0, res=-1, out_f32=False, bias_img=-1,
             bias_img_stride=0, zero_bias=False, cout=None, tag="conv", dwf=None, rgb=False, geom=None):
        """-> (Hout, Wout). rgb: the input is the raw u8 RGB frame batch, padded and normalised on load
        (the stem with fuse_prep; tap field 2). geom: (Hout, pad_t, Wout, pad_l) instead of SAME."""
        B, es, blob = self.B, self.es, self.blob
        k = c.k
        if geom is None:
            Ho, pt = same_pad(H, k, c.stride, c.dil)
            Wo, pl = same_pad(W, k, c.stride, c.dil)
        else:
            Ho, pt, Wo, pl = geom
        extra = [-1, -1, 0]
        Hin, Win = H, W
        if dwf is not None:   # (dw conv, its input H, W): this 1x1 runs over the dw output grid
            d, Hin, Win = dwf
            Ho, dpt = same_pad(Hin, 3, d.stride, d.dil)
            Wo, dpl = same_pad(Win, 3, d.stride, d.dil)
            wd, bd = d.folded()
            extra = [blob.add(wd.reshape(CS, 9).T, True), blob.add(bd.astype(np.float32), False),
                     d.stride | d.dil << 8 | dpt << 16 | dpl << 24]
        tp = CS == 8 and dwf is None and k > 1
        wp, bias, cinP, NP = pack_conv(c, CS, self.bf16, tap_packed=tp)
        if zero_bias:
            bias = np.zeros_like(bias)
        w_off = blob.add(wp, True)
        b_off = blob.add(bias, False)
        cw = c.cout if cout is None else cout
        oes = 4 if out_f32 else es
        self.use(dst, B * Ho * Wo * out_cs * oes)
        cin = c.w.shape[1]
        flops = 2.0 * B * Ho * Wo * c.cout * cin * k * k + (2.0 * B * Ho * Wo * CS * 9 if dwf else 0)
        nbytes = (B * Hin * Win * 3 if rgb else B * Hin * Win * CS * es) + B * Ho * Wo * cw * oes + \
            (B * Ho * Wo * cw * es if res >= 0 else 0) + wp.size * es
        t = tag if dwf is None else "conv dw+project"
        nb = self.nb
        f30 = nb(t, Ho * Wo, cinP * k * k, cw) if callable(nb) else (nb or _pick_nb(t, Ho * Wo, cinP * k * k, cw, B))
        self.op([OP_CONV, src, dst, res, Hin, Win, CS, Ho, Wo, k, k, c.stride, c.dil, pt, pl, cinP, NP, w_off, b_off,
                 c.act, out_cs if res >= 0 else 0, out_cs, out_off, cw, int(out_f32), bias_img, bias_img_stride] +
                extra + [f30, 2 if (rgb and tp) else int(tp)], t, flops, nbytes)
        return Ho, Wo

    def dw(self, d: Conv, src, dst, H, W, C, in_relu=False, geom=None, tag="dw"):
        """3x3 depthwise (+ folded BN, activation d.act; in_relu: ReLU on the loaded input) -> (Hout, Wout)."""
        B, es = self.B, self.es
        if geom is None:
            Ho, pt = same_pad(H, 3, d.stride, d.dil)
            Wo, pl = same_pad(W, 3, d.stride, d.dil)
        else:
            Ho, pt, Wo, pl = geom
        wd, bd = d.folded()
        w_off = self.blob.add(wd.reshape(C, 9).T, True)   # [9][C] in the compute type
        b_off = self.blob.add(bd.astype(np.float32), False)
        self.use(dst, B * Ho * Wo * C * es)
        self.op([OP_DW, src, dst, H, W, C, Ho, Wo, d.stride, d.dil, pt, pl, w_off, b_off, d.act, int(in_relu)], tag,
                2.0 * B * Ho * Wo * C * 9, B * (H * W + Ho * Wo) * C * es)
        return Ho, Wo

    def maxpool(self, src, dst, H, W, C, k, s, tag="maxpool"):
        """k x k max pool, stride s: TF SAME for k > 1 (slim max_pool2d in resnet_arg_scope), VALID for the
        1x1 subsample (resnet_utils.subsample) -> (Hout, Wout)."""
        B, es = self.B, self.es
        if k == 1:
            Ho, pt, Wo, pl = (H - 1) // s + 1, 0, (W - 1) // s + 1, 0
        else:
            Ho, pt = same_pad(H, k, s, 1)
            Wo, pl = same_pad(W, k, s, 1)
        self.use(dst, B * Ho * Wo * C * es)
        self.op([OP_MAXPOOL, src, dst, H, W, C, Ho, Wo, k, s, pt, pl], tag, float(B * Ho * Wo * C * k * k),
                B * (H * W + Ho * Wo) * C * es)
        return Ho, Wo

    def aspp_pool(self, net, src, h, w, C, part=8, z=9, y=10):
        """Image pooling folded into the projection as a per-image bias (buffers part, z, y) -> z stride."""
        B, es = self.B, self.es
        D = net.aspp0.cout
        chunk = 64
        nch = -(-(h * w) // chunk)
        self.use(part, B * nch * C * 4)
        zs = _r(D, 64)
        self.use(z, B * zs * 4)
        wpool, bpool = net.pool.folded()
        wproj, bproj = net.project.folded()
        self.use(y, B * D * 4)
        wp_off = self.blob.add(_round(wpool.reshape(D, C), self.bf16), False)             # [D][C]
        bp_off = self.blob.add(bpool.astype(np.float32), False)
        wq_off = self.blob.add(_round(wproj.reshape(D, -1)[:, :D], self.bf16), False)     # [D (out)][D (pooled ch)]
        bq_off = self.blob.add(bproj.astype(np.float32), False)
        self.op([OP_POOL, src, part, z, h, w, C, C, chunk, nch, D, D, wp_off, bp_off, wq_off, bq_off, zs, y], "pool",
                2.0 * B * (D * C + D * D) + B * h * w * C, B * h * w * C * es)
        return zs

    def projection_conv(self, net):
        """The ASPP projection over the concat minus its pooled part (that part arrives as the per-image bias)."""
        D = net.aspp0.cout
        return Conv(w=net.project.w[:, D:], gamma=net.project.gamma, beta=net.project.beta, mean=net.project.mean,
                    var=net.project.var, eps=net.project.eps, act=net.project.act)

    def resize(self, src, dst, h, w, in_cs, C, Ho, Wo, out_cs, out_off):
        es = self.es
        self.use(dst, self.B * Ho * Wo * out_cs * es)
        self.op([OP_RESIZE, src, dst, h, w, in_cs, C, Ho, Wo, out_cs, out_off], "resize", 8.0 * self.B * Ho * Wo * C,
                self.B * (h * w + Ho * Wo) * C * es)

    def argmax(self, logits, h, w, LCS, ncls, Hc, Wc):
        self.op([OP_ARGMAX, logits, h, w, LCS, ncls], "argmax", 0, self.B * (h * w * LCS * 4 + Hc * Wc * 8))

    def result(self):
        self.info["nops"] = len(self.ops)
        return self.blob.bytes(), np.asarray(self.ops, np.int32), np.asarray(self.need, np.uint64), self.info


def lower(net, B: int, bf16: bool, fuse_dw: bool = False, nb=None, fuse_prep: bool = True):
    """-> (weight blob bytes, ops int32 (nops, OP_FIELDS), buffer bytes uint64 (nbufs,), info dict).
    Buffers: 0 input, 1/2 block ping-pong, 3 expanded, 4 depthwise out, 5 ASPP concat, 6 projection,
    7 logits (f32), 8 pooling partials (f32), 9 per-image projection bias (f32), 10 image-pooling
    branch output (f32).
    nb: pixel fragments per wave of the conv kernel (CONV field 30): 2 or 4, a callable
    (tag, Hout * Wout, K, cout) -> 2 | 4, or None for the measured default (_pick_nb).
    fuse_dw: each block's depthwise conv runs inside its projection's operand loads (CONV fields
    27-29: dw weight / bias offsets, stride | dil << 8 | pad_t << 16 | pad_l << 24; field 31: the
    stem's tap packing, 4 taps x 8 channels per k-step); bit-identical to
    the default plan (separate DW ops through buffer 4) but measured 2.4x slower (5.1 vs 2.2 ms per
    16-frame forward for the pair): the 9 tap loads of every operand chunk serialise ahead of the
    MFMAs and are recomputed for every 64-channel output tile.
    An Xception network (deeplab_xception.DeepLabXception) lowers through lower_xception, a ResNet one
    (deeplab_resnet.DeepLabResNet) through lower_resnet."""
    if not isinstance(net, DeepLab):
        from .deeplab_resnet import DeepLabResNet, lower_resnet
        if isinstance(net, DeepLabResNet):
            if fuse_dw:
                raise ValueError("fuse_dw applies to the MobileNetV2 blocks only")
            return lower_resnet(net, B, bf16, nb=nb, fuse_prep=fuse_prep)
        from .deeplab_xception import lower_xception
        if fuse_dw:
            raise ValueError("fuse_dw applies to the MobileNetV2 blocks only")
        return lower_xception(net, B, bf16, nb=nb, fuse_prep=fuse_prep)
    L = Lowering(B, bf16, 11, nb)
    es = L.es
    Hc, Wc = crop_hw(net)
    L.use(0, B * Hc * Wc * 8 * es)
    if not fuse_prep:
        L.op([OP_PREP, 0], "prep", 0, B * Hc * Wc * (3 + 8 * es))
    # stem
    H, W = L.conv(net.stem, 0, Hc, Wc, 8, 1, _r8(net.stem.cout), tag="conv stem", rgb=fuse_prep)
    if fuse_prep and int(L.ops[-1][31]) != 2:
        raise ValueError("fuse_prep needs the tap-packed stem (3x3 over the 8-channel input)")
    C = net.stem.cout
    cur = 1
    for bi, blk in enumerate(net.blocks):
        nxt = 2 if cur == 1 else 1
        x_in, Cin = cur, C
        if blk.expand is not None:
            L.conv(blk.expand, x_in, H, W, Cin, 3, blk.expand.cout, tag="conv expand")
            src, Cm = 3, blk.expand.cout
        else:
            src, Cm = x_in, Cin
        d = blk.dw
        Cout = blk.project.cout
        if fuse_dw:
            Ho, _ = same_pad(H, 3, d.stride, d.dil)
            Wo, _ = same_pad(W, 3, d.stride, d.dil)
            L.conv(blk.project, src, H, W, Cm, nxt, Cout, res=x_in if blk.residual else -1, dwf=(d, H, W))
            H, W = Ho, Wo
            cur, C = nxt, Cout
            continue
        H, W = L.dw(d, src, 4, H, W, Cm)
        L.conv(blk.project, 4, H, W, Cm, nxt, Cout, res=x_in if blk.residual else -1, tag="conv project")
        cur, C = nxt, Cout

    # ASPP
    D = net.aspp0.cout
    cat_cs = D * (1 + len(net.atrous))
    h, w = H, W
    zs = L.aspp_pool(net, cur, h, w, C)
    L.conv(net.aspp0, cur, h, w, C, 5, cat_cs, out_off=0, tag="conv aspp")
    for i, a in enumerate(net.atrous):
        L.conv(a, cur, h, w, C, 5, cat_cs, out_off=D * (i + 1), tag="conv atrous")
    L.conv(L.projection_conv(net), 5, h, w, cat_cs, 6, D, bias_img=9, bias_img_stride=zs, zero_bias=True,
           tag="conv project")
    LCS = _r(net.num_classes, 8)
    L.conv(net.logits, 6, h, w, D, 7, LCS, out_f32=True, cout=LCS, tag="conv logits")
    L.argmax(7, h, w, LCS, net.num_classes, Hc, Wc)
    L.info.update(feature=(h, w), lcs=LCS)
    return L.result()


# ---------------------------------------------------------------- weight file (.npz, no pickle)
_CONV_FIELDS = ("w", "b", "gamma", "beta", "mean", "var")


def _convs(net: DeepLab):
    yield "stem", net.stem
    for i, b in enumerate(net.blocks):
        if b.expand is not None:
            yield f"b{i}.expand", b.expand
        yield f"b{i}.dw", b.dw
        yield f"b{i}.project", b.project
    yield "pool", net.pool
    yield "aspp0", net.aspp0
    for i, a in enumerate(net.atrous):
        yield f"atrous{i}", a
    yield "project", net.project
    yield "logits", net.logits


def conv_arrays(arrs: dict, named_convs) -> None:
    """Each (name, Conv) as plain arrays: name.{w,b,gamma,beta,mean,var}, name.attrs, name.eps."""
    for name, c in named_convs:
        for f in _CONV_FIELDS:
            v = getattr(c, f)
            if v is not None:
                arrs[f"{name}.{f}"] = np.asarray(v, np.float32)
        arrs[f"{name}.attrs"] = np.array([c.act, c.stride, c.dil, int(c.depthwise)], np.int32)
        arrs[f"{name}.eps"] = np.array([c.eps], np.float64)


def conv_from(z, name, path="") -> Conv:
    if f"{name}.w" not in z:
        raise KeyError(f"{path}: missing {name}.w")
    act, stride, dil, dw = (int(v) for v in z[f"{name}.attrs"])
    c = Conv(w=z[f"{name}.w"], act=act, stride=stride, dil=dil, depthwise=bool(dw), eps=float(z[f"{name}.eps"][0]))
    for f in _CONV_FIELDS[1:]:
        if f"{name}.{f}" in z:
            setattr(c, f, z[f"{name}.{f}"])
    return c


def save(net, path) -> None:
    """Weights + topology attributes as a plain .npz (loadable with allow_pickle=False); either
    backbone (an Xception network is written by deeplab_xception.save_xception)."""
    if not isinstance(net, DeepLab):
        from .deeplab_resnet import DeepLabResNet, save_resnet
        if isinstance(net, DeepLabResNet):
            return save_resnet(net, path)
        from .deeplab_xception import save_xception
        return save_xception(net, path)
    arrs = {}
    conv_arrays(arrs, _convs(net))
    arrs["net.residual"] = np.array([int(b.residual) for b in net.blocks], np.int32)
    arrs["net.expand"] = np.array([int(b.expand is not None) for b in net.blocks], np.int32)
    arrs["net.attrs"] = np.array([net.num_classes, net.output_stride or 0, net.crop, len(net.atrous)], np.int32)
    arrs["net.crop_w"] = np.array([net.crop_w or 0], np.int32)
    np.savez(path, **arrs)


def load(path):
    z = np.load(path, allow_pickle=False)
    if "net.xattrs" in z:
        from .deeplab_xception import load_xception
        return load_xception(z, path)
    if "net.rattrs" in z:
        from .deeplab_resnet import load_resnet
        return load_resnet(z, path)

    def conv(name):
        return conv_from(z, name, path)

    ncls, os_, crop, natr = (int(v) for v in z["net.attrs"])
    blocks = []
    for i, (res, ex) in enumerate(zip(z["net.residual"], z["net.expand"])):
        blocks.append(Block(conv(f"b{i}.expand") if ex else None, conv(f"b{i}.dw"), conv(f"b{i}.project"), bool(res)))
    return DeepLab(conv("stem"), blocks, conv("pool"), conv("aspp0"), [conv(f"atrous{i}") for i in range(natr)],
                   conv("project"), conv("logits"), ncls, os_ or None, crop,
                   crop_w=int(z["net.crop_w"][0]) if "net.crop_w" in z else 0)
