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


def forward(blocks, x: np.ndarray, dtype=torch.float32, ties: "PoolTies | None" = None) -> np.ndarray:
    """x: (B,3,H,W) NCHW float -> logits (B,classes,H,W) as numpy. ties: a ``PoolTies`` that records
    every max-pool of the run (windows, argmax positions, top-2 gaps) and the block sequence, so the
    footprint of a set of windows can be propagated to the logits afterwards."""
    return _forward(blocks, x, dtype, ties)


class PoolTies:
    """Max-pool near-ties and where they can move a value, propagated to the logits.

    MaxPoolWithArgmax (the down blocks) is continuous in its pooled VALUE but not in
    its argmax INDEX: when a 2x2 window's top two inputs differ by less than the rounding error of an
    f32 evaluation, another evaluation order can pick the other one, and the paired upsampling block's
    max-unpool (a2.4) then writes the main branch's value to another pixel of the window. Logits that
    depend on that window's unpooled 2x2 block may then differ from the fp64 result by O(the values
    themselves) — a discontinuity of the network, not an arithmetic fault.

    Recorded per down block i (the pool input h of a frame, window w = (n, c, y, x)):
    * ``pos[i]``: the first-maximum window position 2*dy + dx (the engine's index byte);
    * ``gap[i]``: (top1 - top2) / max|h| of the frame.
    ``near_ties(kappa)``: windows with 0 < gap <= kappa. Exact ties (gap 0) are not near-ties: an exact
    fp64 tie between two different computations does not happen in practice, and between identical
    computations (the initial block's pool channels, where overlapping 3x3 windows share a maximum)
    every evaluation ties exactly and takes the first index — one that did not would be a real fault.
    ``footprint(windows)``: the logits pixels those windows can reach — at an up block, the unpool's
    2x2 block of every listed window of its paired pool (any channel), OR the up-sampled footprint so
    far; through every later block grown by its receptive field (per unit (k-1)/2 * dilation, rows and
    columns separately; a transposed conv: x2 and (k-1)/2). A superset of the pixels a flip reaches."""

    def __init__(self):
        self.pos, self.gap, self.events = {}, {}, []

    # -- recording (called by _forward)
    def pool(self, i, h):
        B, C, H, W = h.shape
        win = h[:, :, :H // 2 * 2, :W // 2 * 2].reshape(B, C, H // 2, 2, W // 2, 2)
        win = win.permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
        top = win.topk(2, dim=-1).values
        scale = h.abs().amax(dim=(1, 2, 3)).view(B, 1, 1, 1)
        self.gap[i] = ((top[..., 0] - top[..., 1]) / scale).float()
        self.pos[i] = win.argmax(-1).to(torch.uint8)      # torch: the first maximum, as the engine

    def event(self, *e):
        self.events.append(e)

    # -- queries
    def near_ties(self, kappa: float) -> dict:
        return {i: ((g > 0) & (g <= kappa)) for i, g in self.gap.items()}

    def flips(self, engine_pos: dict) -> dict:
        """(B,C,h,w) bool per down block: windows whose engine index (NHWC (B,h,w,CS) u8) differs from
        the fp64 argmax position."""
        out = {}
        for i, p in self.pos.items():
            e = torch.as_tensor(np.asarray(engine_pos[i]))[..., :p.shape[1]].permute(0, 3, 1, 2)
            out[i] = e != p
        return out

    def footprint(self, windows: dict) -> np.ndarray:
        """windows: down block -> (B,C,h,w) or (B,h,w) bool -> (B,H,W) bool at the logits."""
        win = {i: (w.any(1) if w.dim() == 4 else w) for i, w in windows.items()}
        m = None
        for e in self.events:
            if e[0] == "down" and m is not None:
                units, size = e[1], e[2]
                m = F.max_pool2d(m[:, None].float(), 2, stride=2, ceil_mode=True)[:, 0, :size[0], :size[1]] > 0
                m = self._grow(m, *self._radius(units[1:]))
            elif e[0] == "regular" and m is not None:
                m = self._grow(m, *self._radius(e[1]))
            elif e[0] == "up":
                ref, units, size = e[1], e[2], e[3]
                t = self._up2(win[ref], size)
                m = t if m is None else (t | self._grow(self._up2(m, size), *self._radius(units[1:])))
            elif e[0] == "fullconv":
                size, k = e[1], e[3]
                B = next(iter(self.pos.values())).shape[0] if self.pos else e[2]
                m = (torch.zeros((B,) + tuple(size), dtype=torch.bool) if m is None
                     else self._grow(self._up2(m, size), (k - 1) // 2, (k - 1) // 2))
        return m.numpy()

    @staticmethod
    def _up2(m, size):
        m = m.repeat_interleave(2, 1).repeat_interleave(2, 2)
        out = m.new_zeros((m.shape[0],) + tuple(size))
        hh, ww = min(size[0], m.shape[1]), min(size[1], m.shape[2])
        out[:, :hh, :ww] = m[:, :hh, :ww]
        return out

    @staticmethod
    def _grow(m, rh, rw):
        if rh == 0 and rw == 0:
            return m
        f = F.max_pool2d(m[:, None].float(), (2 * rh + 1, 2 * rw + 1), stride=1, padding=(rh, rw))
        return f[:, 0] > 0

    @staticmethod
    def _radius(units):
        rh = rw = 0
        for u in units:
            kh, kw = np.asarray(u.w).shape[2:4]
            rh += (kh - 1) // 2 * max(1, int(u.dil_h))
            rw += (kw - 1) // 2 * max(1, int(u.dil_w))
        return rh, rw


def _forward(blocks, x, dtype, fp):
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
                if fp is not None:
                    fp.pool(i, h)
                main, idx = F.max_pool2d(h, 2, stride=2, return_indices=True)
                pools[i] = (idx, h.shape[2:])
                ext = h
                for u in b.units:
                    ext = _unit(ext, u, dtype)
                pad = ext.shape[1] - main.shape[1]
                main = torch.cat([main, main.new_zeros((main.shape[0], pad) + main.shape[2:])], 1)
                h = _prelu(main + ext, b.extra["out_slope"], dtype)
                if fp is not None:
                    fp.event("down", b.units, tuple(h.shape[2:]))
            elif b.type == "regular":
                ext = h
                for u in b.units:
                    ext = _unit(ext, u, dtype)
                h = _prelu(h + ext, b.extra["out_slope"], dtype)
                if fp is not None:
                    fp.event("regular", b.units)
            elif b.type == "up":
                idx, size = pools[b.attrs["pool_ref"]]
                main = _unit(h, b.units[0], dtype, act=False)
                main = F.max_unpool2d(main, idx, 2, stride=2, output_size=size)
                ext = h
                for u in b.units[1:]:
                    ext = _unit(ext, u, dtype)
                h = _prelu(main + ext, b.extra["out_slope"], dtype)
                if fp is not None:
                    fp.event("up", b.attrs["pool_ref"], b.units, tuple(h.shape[2:]))
            elif b.type == "fullconv":
                u = b.units[0]
                h = F.conv_transpose2d(h, _t(u.w, dtype), _t(u.b, dtype), stride=2,
                                       padding=(u.pad_h, u.pad_w), output_padding=u.out_pad)
                if not _identity_bn(u):       # the engine folds a classifier BN like any other
                    h = _bn(h, u.mean, u.var, u.gamma, u.beta, u.eps, dtype)
                if fp is not None:
                    fp.event("fullconv", tuple(h.shape[2:]), h.shape[0], int(np.asarray(u.w).shape[2]))
        return h.numpy()


def down_blocks(blocks) -> list:
    """Indices of the downsampling blocks (the max-pools whose indices an up block unpools)."""
    return [i for i, b in enumerate(blocks) if b.type == "down"]


# the fp32 range bar (tests/test_gpu_range.py, smoke): per pixel e = max over classes |dlogit| / max|logit|
RANGE_REL, RANGE_REL99, RANGE_MAX_OFF, RANGE_KAPPA = 5e-6, 2e-6, 5e-3, 1e-5


def range_verdict(got, ref, ties: PoolTies, engine_idx: dict, what: str):
    """The fp32 mode against the fp64 oracle over the f32 range, with every excused pixel ATTRIBUTED
    (errors relative to each frame's own max |logit|).

    got: the engine's logits (B,C,H,W); ref: ``forward(..., torch.float64, ties=ties)``; engine_idx:
    down block -> the engine's pooling indices of the same run (NHWC u8, bugseg_debug_pool_indices).
    Criterion (-> (ok, message, stats)):
    * every logit finite; 99% of the pixels within RANGE_REL99 of the max;
    * every window whose engine index differs from the fp64 first-maximum position is a near-tie of
      the fp64 pool input (0 < top-2 gap <= RANGE_KAPPA of the frame's max|pool input|: ~16x the
      fp32 oracle's own max deviation there) — an index flipped anywhere else is a fault;
    * every pixel beyond RANGE_REL lies inside the footprint of the flipped windows
      (``PoolTies.footprint``), and at most RANGE_MAX_OFF of a frame (>= 2 x 32 x 32 pixels) is beyond;
    * classes exact on every pixel outside that footprint whose fp64 top-2 margin exceeds 2.5x its error."""
    if not np.isfinite(got).all():
        return False, f"{what}: {int((~np.isfinite(got)).sum())} non-finite logits", {}
    amax = np.abs(ref).reshape(ref.shape[0], -1).max(1)          # per frame: a batch may mix scales
    err_px = np.abs(got - ref).max(1)
    e = err_px / amax[:, None, None]
    off = e > RANGE_REL
    p99 = float(np.percentile(e, 99))
    flips = ties.flips(engine_idx)
    bad_flip, n_flip, max_gap = 0, 0, 0.0
    for i, f in flips.items():
        g = ties.gap[i]
        n_flip += int(f.sum())
        if f.any():
            max_gap = max(max_gap, float(g[f].max()))
        bad_flip += int((f & ~((g > 0) & (g <= RANGE_KAPPA))).sum())
    fp = ties.footprint(flips)
    outside = off & ~fp
    s = np.sort(ref, axis=1)
    dec = ((s[:, -1] - s[:, -2]) > 2.5 * err_px) & ~fp
    cls_ok = bool((got.argmax(1)[dec] == ref.argmax(1)[dec]).all())
    n_off = off.reshape(off.shape[0], -1).sum(1)
    allowed = max(RANGE_MAX_OFF * off[0].size, 2 * 32 * 32)
    e_out = e[~fp]
    stats = {"p99": p99, "max": float(e.max()), "beyond": int(off.sum()), "flipped_windows": n_flip,
             "p99_outside_footprint": float(np.percentile(e_out, 99)) if e_out.size else 0.0,
             "flips_not_near_tie": bad_flip, "max_flip_gap": max_gap, "footprint": int(fp.sum()),
             "beyond_outside_footprint": int(outside.sum()),
             "max_outside_footprint": float(np.where(fp, 0.0, e).max())}
    msg = (f"{what}: max|logit| {amax.min():.3e}..{amax.max():.3e}; error / max: p50 {np.percentile(e, 50):.1e} p99 {p99:.1e} max "
           f"{e.max():.1e} ({stats['max_outside_footprint']:.1e} outside the footprint); {n_flip} pool indices "
           f"differ from fp64 ({bad_flip} not near-ties, largest gap {max_gap:.1e}), footprint {int(fp.sum())} px; "
           f"{int(off.sum())} of {off.size} pixels beyond {RANGE_REL:g}, {int(outside.sum())} of them outside it; "
           f"classes {'exact' if cls_ok else 'DIFFER'} on {int(dec.sum())} decided pixels")
    ok = (p99 <= RANGE_REL99 and bad_flip == 0 and int(outside.sum()) == 0 and bool((n_off <= allowed).all())
          and cls_ok)
    return ok, msg, stats


def engine_pool_indices(ctx, blocks, ties: PoolTies, B: int, H: int, W: int) -> dict:
    """The engine's pooling indices of its last forward at (B, H, W) for every down block, as numpy
    (B, h, w, channel stride) — shapes from the oracle's recorded pools."""
    out = {}
    for i in down_blocks(blocks):
        _b, c, h, w = ties.pos[i].shape
        out[i] = ctx.pool_indices(B, H, W, i, (h, w, (c + 7) // 8 * 8)).cpu().numpy()
    return out


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
