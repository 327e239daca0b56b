"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by the product package).

CPU restatement of the reference's ENet inference path on PyTorch-CPU ops (the plain fp32/fp64
reference the HIP kernels are checked against):

* ``forward``      : the ENet forward the reference runs inside TF ``sess.run``
                     (models.py:43-44), layer by layer as the block list describes it —
                     conv, batch-norm (inference), PReLU, maxpool-with-indices, max-unpool,
                     transposed conv — with BN NOT folded (folding is the engine's business).
* ``predict``      : argmax over classes + 3-class remap, models.py:55-58,67-69.
* ``predict_binary``: argmax + (c==0)|(c==1), models.py:78-82.
* ``preprocess``   : models.py:84-95 (resize via ocv restatement, BGR->RGB, /256, mean/std).

Parity status: UNPINNED against TensorFlow on enet.pb — neither TF nor the weights exist in this
image (.MISSING_LARGE_BLOBS:2). The topology is the canonical ENet of SURVEY.md
Appendix A with the synthetic weights of ``enet_spec.build_enet``.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

# models.py:17-18
IMAGE_MEAN = np.array([0.485, 0.456, 0.406])
IMAGE_STD = np.array([0.229, 0.224, 0.225])
# models.py:56-58: {2,9} -> 0, {0,1} -> 1, others -> 2
LUT3 = np.array([1, 1, 0, 2, 2, 2, 2, 2, 2, 0, 2, 2, 2, 2, 2], dtype=np.uint8)
# models.py:79-80
LUT_BINARY = np.array([1, 1] + [0] * 13, dtype=np.uint8)


def _t(a, dtype):
    return torch.as_tensor(np.asarray(a), dtype=dtype)


def _bn(y, mean, var, gamma, beta, eps, dtype):
    """Inference batch norm; eps == 0 (units imported with BN already reduced to an affine, or
    without BN) is evaluated directly (F.batch_norm requires eps > 0)."""
    if float(eps) > 0:
        return F.batch_norm(y, _t(mean, dtype), _t(var, dtype), _t(gamma, dtype), _t(beta, dtype),
                            training=False, eps=float(eps))
    v = lambda a: _t(a, dtype).view(1, -1, 1, 1)  # noqa: E731
    return (y - v(mean)) / torch.sqrt(v(var)) * v(gamma) + v(beta)


def _identity_bn(u) -> bool:
    return (np.all(np.asarray(u.gamma) == 1) and not np.any(u.beta) and not np.any(u.mean)
            and np.all(np.asarray(u.var) == 1))


def _unit(x, u, dtype, act=True):
    w = _t(u.w, dtype)
    if u.kind == 0:
        y = F.conv2d(x, w, _t(u.b, dtype), stride=u.stride, padding=(u.pad_h, u.pad_w),
                     dilation=(u.dil_h, u.dil_w))
    else:
        y = F.conv_transpose2d(x, w, _t(u.b, dtype), stride=u.stride, padding=(u.pad_h, u.pad_w),
                               output_padding=u.out_pad)
    y = _bn(y, u.mean, u.var, u.gamma, u.beta, u.eps, dtype)
    if act:
        y = _prelu(y, u.slope, dtype)
    return y


def _prelu(x, slope, dtype):
    s = _t(slope, dtype).view(1, -1, 1, 1)
    return torch.where(x > 0, x, x * s)


def forward(blocks, x: np.ndarray, dtype=torch.float32) -> np.ndarray:
    """x: (B,3,H,W) NCHW float -> logits (B,classes,H,W) as numpy."""
    with torch.no_grad():
        h = _t(x, dtype)
        pools = {}
        for i, b in enumerate(blocks):
            if b.type == "initial":
                u = b.units[0]
                main = F.conv2d(h, _t(u.w, dtype), _t(u.b, dtype), stride=2, padding=1)
                k = b.attrs["pool_k"]
                ext = F.max_pool2d(h, k, stride=2, padding=(k - 1) // 2)
                y = torch.cat([main, ext], 1)
                e = b.extra
                if float(u.eps) == float(e["pool_eps"][0]):
                    y = _bn(y, np.concatenate([u.mean, e["pool_mean"]]), np.concatenate([u.var, e["pool_var"]]),
                            np.concatenate([u.gamma, e["pool_gamma"]]), np.concatenate([u.beta, e["pool_beta"]]),
                            u.eps, dtype)
                else:
                    c = u.cout
                    y = torch.cat([_bn(y[:, :c], u.mean, u.var, u.gamma, u.beta, u.eps, dtype),
                                   _bn(y[:, c:], e["pool_mean"], e["pool_var"], e["pool_gamma"], e["pool_beta"],
                                       e["pool_eps"][0], dtype)], 1)
                h = _prelu(y, np.concatenate([u.slope, e["pool_slope"]]), dtype)
            elif b.type == "down":
                main, idx = F.max_pool2d(h, 2, stride=2, return_indices=True)
                pools[i] = (idx, h.shape[2:])
                ext = h
                for u in b.units:
                    ext = _unit(ext, u, dtype)
                pad = ext.shape[1] - main.shape[1]
                main = torch.cat([main, main.new_zeros((main.shape[0], pad) + main.shape[2:])], 1)
                h = _prelu(main + ext, b.extra["out_slope"], dtype)
            elif b.type == "regular":
                ext = h
                for u in b.units:
                    ext = _unit(ext, u, dtype)
                h = _prelu(h + ext, b.extra["out_slope"], dtype)
            elif b.type == "up":
                idx, size = pools[b.attrs["pool_ref"]]
                main = _unit(h, b.units[0], dtype, act=False)
                main = F.max_unpool2d(main, idx, 2, stride=2, output_size=size)
                ext = h
                for u in b.units[1:]:
                    ext = _unit(ext, u, dtype)
                h = _prelu(main + ext, b.extra["out_slope"], dtype)
            elif b.type == "fullconv":
                u = b.units[0]
                h = F.conv_transpose2d(h, _t(u.w, dtype), _t(u.b, dtype), stride=2,
                                       padding=(u.pad_h, u.pad_w), output_padding=u.out_pad)
                if not _identity_bn(u):       # the engine folds a classifier BN like any other
                    h = _bn(h, u.mean, u.var, u.gamma, u.beta, u.eps, dtype)
        return h.numpy()


def argmax_classes(logits: np.ndarray) -> np.ndarray:
    """tf.math.argmax(segmap, axis=1): first maximal index on ties (models.py:55)."""
    return np.argmax(logits, axis=1)


def predict(blocks, x, dtype=torch.float32) -> np.ndarray:
    """ENET.predict: models.py:43-69 -> uint8 (B,H,W) in {0,1,2}."""
    return LUT3[argmax_classes(forward(blocks, x, dtype))]


def predict_binary(blocks, x, dtype=torch.float32) -> np.ndarray:
    """ENET.predict_binary: models.py:71-82 -> uint8 (B,H,W) in {0,1}."""
    return LUT_BINARY[argmax_classes(forward(blocks, x, dtype))]


def normalize_lut() -> np.ndarray:
    """(v/256.0 - mean)/std for every u8 value v, per RGB channel, in float64 (models.py:91)."""
    v = np.arange(256, dtype=np.float64)[:, None]
    return (v / 256.0 - IMAGE_MEAN[None, :]) / IMAGE_STD[None, :]     # (256, 3)


def preprocess(bgr: np.ndarray, width: int = 512, height: int = 256) -> np.ndarray:
    """ENET.preprocess: models.py:84-95 -> (1,3,height,width) float64 NCHW RGB."""
    from . import ocv_np
    resized = ocv_np.resize_linear(bgr, (width, height))                    # models.py:87
    rgb = resized[..., ::-1]                                                # models.py:89
    normalized = (rgb / 256.0 - IMAGE_MEAN) / IMAGE_STD                     # models.py:91
    return np.expand_dims(np.moveaxis(normalized, -1, 0), 0)               # models.py:92-94


# ---------------------------------------------------------------- bf16-storage emulation
_STORE = torch.bfloat16      # the storage type forward_bf16_storage rounds to (forward_storage sets it)


def _bf16(t):
    """Round to the emulated storage type (bf16 unless forward_storage selected f16) and back."""
    return t.to(_STORE).to(torch.float32)


def _fold(u):
    """BN folded into the conv in float64 (what the engine does), as float32 tensors (w, bias)."""
    s = np.asarray(u.gamma, np.float64) / np.sqrt(np.asarray(u.var, np.float64) + float(u.eps))
    shift = (np.asarray(u.b, np.float64) - np.asarray(u.mean, np.float64)) * s + np.asarray(u.beta, np.float64)
    w = np.asarray(u.w, np.float64)
    w = w * (s[:, None, None, None] if u.kind == 0 else s[None, :, None, None])
    return torch.as_tensor(w.astype(np.float32)), torch.as_tensor(shift.astype(np.float32))


def _unit_bf16(x, u, act=True):
    w, b = _fold(u)
    w = _bf16(w)
    if u.kind == 0:
        y = F.conv2d(x, w, b, stride=u.stride, padding=(u.pad_h, u.pad_w), dilation=(u.dil_h, u.dil_w))
    else:
        y = F.conv_transpose2d(x, w, b, stride=u.stride, padding=(u.pad_h, u.pad_w), output_padding=u.out_pad)
    return _prelu(y, u.slope, torch.float32) if act else y


def forward_bf16_storage(blocks, x: np.ndarray) -> np.ndarray:
    """The engine's bf16 mode numerics: BN-folded weights and every stored activation rounded to
    bf16, products/accumulation/epilogue in fp32 (residual added in fp32 before the output is
    rounded). Checks the bf16 kernels against matching numerics, not against fp32."""
    f32 = torch.float32
    with torch.no_grad():
        h = _bf16(torch.as_tensor(np.asarray(x, np.float32)))
        pools = {}
        for i, b in enumerate(blocks):
            if b.type == "initial":
                u = b.units[0]
                w, bias = _fold(u)
                main = F.conv2d(h, _bf16(w), bias, stride=2, padding=1)
                k = b.attrs["pool_k"]
                e = b.extra
                ps = np.asarray(e["pool_gamma"], np.float64) / np.sqrt(np.asarray(e["pool_var"], np.float64) + float(e["pool_eps"][0]))
                pb = np.asarray(e["pool_beta"], np.float64) - np.asarray(e["pool_mean"], np.float64) * ps
                pool = F.max_pool2d(h, k, stride=2, padding=(k - 1) // 2)
                pool = pool * torch.as_tensor(ps.astype(np.float32)).view(1, -1, 1, 1) + \
                    torch.as_tensor(pb.astype(np.float32)).view(1, -1, 1, 1)
                y = torch.cat([main, pool], 1)
                h = _bf16(_prelu(y, np.concatenate([u.slope, e["pool_slope"]]), f32))
            elif b.type == "down":
                main, idx = F.max_pool2d(h, 2, stride=2, return_indices=True)
                pools[i] = (idx, h.shape[2:])
                ext = h
                for j, u in enumerate(b.units):
                    ext = _unit_bf16(ext, u)
                    if j + 1 < len(b.units):
                        ext = _bf16(ext)
                pad = ext.shape[1] - main.shape[1]
                main = torch.cat([main, main.new_zeros((main.shape[0], pad) + main.shape[2:])], 1)
                h = _bf16(_prelu(main + ext, b.extra["out_slope"], f32))
            elif b.type == "regular":
                ext = h
                for j, u in enumerate(b.units):
                    ext = _unit_bf16(ext, u)
                    if j + 1 < len(b.units):
                        ext = _bf16(ext)
                h = _bf16(_prelu(h + ext, b.extra["out_slope"], f32))
            elif b.type == "up":
                idx, size = pools[b.attrs["pool_ref"]]
                main = _bf16(_unit_bf16(h, b.units[0], act=False))
                main = F.max_unpool2d(main, idx, 2, stride=2, output_size=size)
                ext = h
                for u in b.units[1:]:
                    ext = _unit_bf16(ext, u)
                    if u is not b.units[-1]:
                        ext = _bf16(ext)
                h = _bf16(_prelu(main + ext, b.extra["out_slope"], f32))
            elif b.type == "fullconv":
                h = _unit_bf16(h, b.units[0], act=False)
        return h.numpy()


def forward_storage(blocks, x: np.ndarray, dtype=torch.bfloat16) -> np.ndarray:
    """forward_bf16_storage with the stored activations and folded weights rounded to `dtype`
    (torch.bfloat16: the bf16 mode; torch.float16: the fp16 mode), f32 products and accumulation."""
    global _STORE
    prev, _STORE = _STORE, dtype
    try:
        return forward_bf16_storage(blocks, x)
    finally:
        _STORE = prev
