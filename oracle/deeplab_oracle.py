"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by the product package).

CPU restatement of the DeepLab inference the reference runs through TF ``sess.run``
(models.py:115-125: ``ImageTensor`` u8 -> ``SemanticPredictions`` int64) for the standard TF
DeepLab export over MobileNetV2 (deeplab_spec.py documents the topology), on PyTorch-CPU ops with
TF's semantics written out:

* ``preprocess``  deeplab input_preprocess + mobilenet ``_preprocess_zero_mean_unit_range``: pad to
                  the crop with 127.5 (pad_to_bounding_box), ``f32(2/255) * x - 1`` in f32;
* ``forward``     SAME padding (pad_before = total // 2), conv / depthwise conv, inference batch
                  norm NOT folded, ReLU6 / ReLU, residual adds, image pooling (spatial mean, 1x1,
                  broadcast), ASPP concat in TF's order [pool, 1x1, atrous...], projection, logits;
* ``resize_bilinear_tf``  TF1 ResizeBilinear, align_corners=True, legacy scaler, lerp order
                  ``top + (bottom - top) * y_lerp`` (resize_bilinear_op.cc) in f32;
* ``predict``     argmax over classes (first maximum) -> int64, sliced to the un-padded image.

``bf16_storage=True`` emulates the engine's bf16 mode: batch norm folded (independently of the
engine's packer), weights and every stored activation rounded to bf16, arithmetic in f32.

Parity status: UNPINNED against TensorFlow on deeplab.pb — neither TF nor the weights exist in this
image (.MISSING_LARGE_BLOBS:1).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def crop_hw(net):
    """(crop height, crop width) of the export (a square crop stores only ``crop``)."""
    return int(net.crop), int(getattr(net, "crop_w", 0) or net.crop)


def preprocess(rgb: np.ndarray, crop) -> np.ndarray:
    """(B, H, W, 3) u8 -> (B, crop_h, crop_w, 3) f32; ``crop`` an int or (height, width)."""
    ch, cw = (crop, crop) if np.ndim(crop) == 0 else crop
    B, H, W, _ = rgb.shape
    assert H <= ch and W <= cw
    x = np.full((B, ch, cw, 3), 127.5, np.float32)
    x[:, :H, :W] = rgb.astype(np.float32)
    return (np.float32(2.0 / 255.0) * x - np.float32(1.0)).astype(np.float32)


def _same(x, k, s, d):
    H, W = x.shape[2], x.shape[3]
    pads = []
    for n in (W, H):
        out = -(-n // s)
        tot = max((out - 1) * s + (k - 1) * d + 1 - n, 0)
        pads += [tot // 2, tot - tot // 2]
    return F.pad(x, pads)


class _Num:
    def __init__(self, dtype, bf16):
        self.dtype, self.bf16 = dtype, bf16

    def t(self, a):
        return torch.as_tensor(np.asarray(a), dtype=self.dtype)

    def store(self, y):
        return y.to(torch.bfloat16).to(self.dtype) if self.bf16 else y

    def wb(self, c):
        """Weights / bias as used: raw (+ separate BN) in exact mode, folded and rounded in bf16 mode."""
        if not self.bf16:
            return self.t(c.w), (None if c.b is None else self.t(c.b))
        w = np.asarray(c.w, np.float64)
        b = np.zeros(c.w.shape[0]) if c.b is None else np.asarray(c.b, np.float64)
        if c.gamma is not None:
            s = np.asarray(c.gamma, np.float64) / np.sqrt(np.asarray(c.var, np.float64) + c.eps)
            w = w * s[:, None, None, None]
            b = (b - np.asarray(c.mean, np.float64)) * s + np.asarray(c.beta, np.float64)
        wt = torch.as_tensor(w, dtype=torch.float32).to(torch.bfloat16).to(self.dtype)
        return wt, torch.as_tensor(b, dtype=torch.float32).to(self.dtype)

    def bn_act(self, y, c, act=True):
        if not self.bf16 and c.gamma is not None:
            y = F.batch_norm(y, self.t(c.mean), self.t(c.var), self.t(c.gamma), self.t(c.beta), training=False,
                             eps=float(c.eps))
        if act and c.act == 1:
            y = F.relu(y)
        elif act and c.act == 2:
            y = torch.clamp(y, 0.0, 6.0)
        return y


def _conv(n: _Num, x, c, groups=1):
    w, b = n.wb(c)
    y = F.conv2d(_same(x, c.w.shape[2], c.stride, c.dil), w, b, stride=c.stride, dilation=c.dil, groups=groups)
    return n.bn_act(y, c)


def forward(net, rgb: np.ndarray, dtype=torch.float64, bf16_storage: bool = False) -> torch.Tensor:
    """(B, H, W, 3) u8 RGB -> logits (B, classes, h, w) at the backbone resolution, f32."""
    n = _Num(torch.float32 if bf16_storage else dtype, bf16_storage)
    x = torch.from_numpy(preprocess(rgb, crop_hw(net))).permute(0, 3, 1, 2).to(n.dtype)
    x = n.store(x)
    x = n.store(_conv(n, x, net.stem))
    for blk in net.blocks:
        inp = x
        if blk.expand is not None:
            x = n.store(_conv(n, x, blk.expand))
        x = n.store(_conv(n, x, blk.dw, groups=x.shape[1]))
        y = _conv(n, x, blk.project)
        if blk.residual:
            y = y + inp
        x = n.store(y)
    h, w = x.shape[2], x.shape[3]
    pooled = n.store(x.mean(dim=(2, 3), keepdim=True))
    img = n.store(_conv(n, pooled, net.pool)).expand(-1, -1, h, w)
    branches = [img, n.store(_conv(n, x, net.aspp0))] + [n.store(_conv(n, x, a)) for a in net.atrous]
    cat = torch.cat(branches, dim=1)
    p = n.store(_conv(n, cat, net.project))
    logits = _conv(n, p, net.logits)
    return logits.to(torch.float32)


def resize_bilinear_tf(logits: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """(B, C, h, w) f32 -> (B, C, out_h, out_w) f32, TF1 ResizeBilinear align_corners=True."""
    B, C, h, w = logits.shape
    f = np.float32
    sy = f(h - 1) / f(out_h - 1) if out_h > 1 else f(0)
    sx = f(w - 1) / f(out_w - 1) if out_w > 1 else f(0)
    iy = np.arange(out_h, dtype=np.float32) * f(sy)
    ix = np.arange(out_w, dtype=np.float32) * f(sx)
    y0 = np.floor(iy).astype(np.int64)
    x0 = np.floor(ix).astype(np.int64)
    y1 = np.minimum(y0 + 1, h - 1)
    x1 = np.minimum(x0 + 1, w - 1)
    ly = (iy - y0.astype(np.float32)).astype(np.float32)[:, None]
    lx = (ix - x0.astype(np.float32)).astype(np.float32)[None, :]
    L = logits.astype(np.float32)
    tl = L[:, :, y0][:, :, :, x0]
    tr = L[:, :, y0][:, :, :, x1]
    bl = L[:, :, y1][:, :, :, x0]
    br = L[:, :, y1][:, :, :, x1]
    top = tl + (tr - tl) * lx
    bot = bl + (br - bl) * lx
    return (top + (bot - top) * ly).astype(np.float32)


def predict(net, rgb: np.ndarray, logits: torch.Tensor | np.ndarray | None = None, **kw) -> np.ndarray:
    """-> (B, H, W) int64 = SemanticPredictions for the un-padded image."""
    B, H, W, _ = rgb.shape
    if logits is None:
        logits = forward(net, rgb, **kw)
    L = np.asarray(logits.numpy() if isinstance(logits, torch.Tensor) else logits, np.float32)
    up = resize_bilinear_tf(L, *crop_hw(net))
    return np.argmax(up, axis=1)[:, :H, :W].astype(np.int64)
