"""Model plugins with the reference's API (models.py), running on the native MI355X engine.

Drop-in for `models.py` of the reference: same class names, class constants, method names,
argument meaning and return dtypes/shapes. Underneath, `sess.run` on a frozen TF graph
(models.py:43-44) and the TF-eager argmax/remap (models.py:55-58, 78-80) are replaced by one
launch plan of hand-written gfx950 kernels (libbugseg.so) with the argmax + class remap fused into
the final transposed-convolution epilogue. There is no CPU fallback: without the library or a GPU
every call raises.

Additions beyond the reference API (device fast paths for batching): `predict_device`,
`logits`, `preprocess_device`.
"""
from __future__ import annotations

import os
from abc import ABC

import numpy as np
import torch

from . import _native as N
from . import enet_spec


class InferenceModel(ABC):
    """models.py:8-13. (The reference declares `preprocess(rgb_image)` under @classmethod, which
    binds the image to `cls`; subclasses here take `(cls, bgr_frame)` as ENET does.)"""

    def predict(self, preprocessed_image):
        pass

    @classmethod
    def preprocess(cls, bgr_frame):
        pass


def _as_device_tensor(x, dtype=None, device: int | None = None) -> torch.Tensor:
    """Host array / tensor -> contiguous tensor on HIP device `device` (default: the current one).
    A tensor already on another device is refused rather than silently used with this context's
    stream (the kernels would run on the context's device with a foreign pointer)."""
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    if isinstance(x, torch.Tensor):
        t = x
    else:
        t = torch.from_numpy(np.ascontiguousarray(x))
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    if not t.is_cuda:
        t = t.to(dev, non_blocking=False)
    elif t.device != dev:
        raise ValueError(f"input is on {t.device}, but the model runs on {dev}")
    return t.contiguous()


def _load_blob(path: str) -> bytes:
    """Weight file -> BSG1 blob: a BSG1 file as is, or a frozen TF GraphDef (the reference's enet.pb,
    models.py:25-30) through the importer (graphdef.py), which checks it is the canonical ENet."""
    if not os.path.exists(path):
        # TF's GFile raises NotFoundError here (models.py:25); FileNotFoundError is its Python twin
        raise FileNotFoundError(f"{path}: no such file")
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] == b"BSG1":
        return data
    from . import graphdef
    return graphdef.graphdef_to_blob(data, input_name=ENET.INPUT_TENSOR_NAME.split(":")[0])


class ENET(InferenceModel):
    """models.py:14-95 on the MI355X engine."""
    INPUT_TENSOR_NAME = "input0:0"
    OUTPUT_TENSOR_NAME = "CATkrIDy/concat:0"
    IMAGE_MEAN = np.array([0.485, 0.456, 0.406])
    IMAGE_STD = np.array([0.229, 0.224, 0.225])
    INPUT_WIDTH, INPUT_HEIGHT = (512, 256)

    def __init__(self, GRAPH_PB_PATH=None, *, weights=None, precision: str = "fp32", device: int | None = None):
        """GRAPH_PB_PATH: weight file (default "./pretrained_models/enet.pb", models.py:23-24).
        weights: a BSG1 blob (bytes) or an enet_spec block list, instead of a file.
        precision: "fp32" (parity mode: f32 storage and accumulation; each f32 product is computed as
        three f16 MFMA products of split operands, hi = f16(v), lo = f16(v - hi), ~2^-21 relative per
        product; every operand is first brought into the f16 window by an exact power of two —
        measured per tensor, bounded for a fused block's internals, static for the weights — clamped
        to 2^+-40, so tensors whose max |v| lies in [2^-26, 2^54] split exactly and beyond that the
        split loses precision gracefully. Tested: logits within 1e-3 absolute of the fp32 oracle on
        the default weights; over the f32 range a relative bar against fp64 (p99 of the per-pixel error
        <= 2e-6 of the max |logit|, pixels beyond 5e-6 only at max-pool near-ties,
        tests/test_gpu_range.py), "bf16" or "fp16" (throughput modes: 2-byte activations and weights,
        f32 accumulation; fp16 keeps 3 more mantissa bits than bf16, so its class maps agree more
        closely with fp32, but values beyond fp16's +-65504 become inf — a graph whose activations
        leave that range needs fp32 or bf16)."""
        if precision not in ("fp32", "bf16", "fp16"):
            raise ValueError("precision must be 'fp32', 'bf16' or 'fp16'")
        if weights is None:
            if GRAPH_PB_PATH is None:
                GRAPH_PB_PATH = "./pretrained_models/enet.pb"
            blob = _load_blob(GRAPH_PB_PATH)
        elif isinstance(weights, (bytes, bytearray)):
            blob = bytes(weights)
        else:
            blob = enet_spec.serialize(weights)
        self.precision = precision
        self.ctx = N.Context(device, {"fp32": N.FP32, "bf16": N.BF16, "fp16": N.F16}[precision])
        self.ctx.load_weights(blob)
        self.blob = blob
        self.num_classes = self.ctx.num_classes
        self._bufs: dict = {}
        self.test = None

    # -- device fast paths --------------------------------------------------------------------
    def _buf(self, key, shape, dtype):
        t = self._bufs.get(key)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype or t.device.index != self.ctx.device:
            t = torch.empty(shape, dtype=dtype, device=torch.device("cuda", self.ctx.device))
            self._bufs[key] = t
        return t

    def engine_input(self, preprocessed) -> torch.Tensor:
        """NCHW (B,3,H,W) float (numpy or torch) -> engine input tensor (B,H,W,8) on the device."""
        x = _as_device_tensor(preprocessed, device=self.ctx.device)
        if x.dtype not in (torch.float32, torch.float64):
            x = x.to(torch.float32)
        if x.dim() != 4 or x.shape[1] != 3:
            raise ValueError(f"expected (B, 3, H, W) input, got {tuple(x.shape)}")
        B, _, H, W = x.shape
        es = 4 if self.precision == "fp32" else 2
        out = self._buf("in", (B, H, W, 8 * es), torch.uint8)
        self.ctx.nchw_to_input(x, B, H, W, out, self._stream())
        return out

    def _stream(self):
        return torch.cuda.current_stream(torch.device("cuda", self.ctx.device))

    def predict_device(self, engine_in: torch.Tensor, out_kind: int = N.OUT_CLASS3_U8, out: torch.Tensor | None = None):
        """Forward on an engine-input tensor (B,H,W,8*elem bytes u8 view) -> device tensor."""
        B, H, W = engine_in.shape[:3]
        dev = torch.device("cuda", self.ctx.device)
        if engine_in.device != dev:
            raise ValueError(f"input is on {engine_in.device}, but the model runs on {dev}")
        if out is None:
            if out_kind == N.OUT_LOGITS_F32:
                out = torch.empty((B, self.num_classes, H, W), dtype=torch.float32, device=dev)
            else:
                out = torch.empty((B, H, W), dtype=torch.uint8, device=dev)
        self.ctx.forward(engine_in, B, H, W, out_kind, out, self._stream())
        return out

    def logits(self, preprocessed_imgs) -> np.ndarray:
        """The TF output tensor OUTPUT_TENSOR_NAME: (B, classes, H, W) float32 NCHW (models.py:43-44,52)."""
        return self.predict_device(self.engine_input(preprocessed_imgs), N.OUT_LOGITS_F32).cpu().numpy()

    # -- reference API ------------------------------------------------------------------------
    def predict(self, preprocessed_imgs) -> np.ndarray:
        """models.py:42-69: uint8 (B,H,W); 1 road(+lane marking), 0 flat non-road (pavement,
        vegetation), 2 everything else. Argmax ties go to the lowest class (tf.math.argmax)."""
        return self.predict_device(self.engine_input(preprocessed_imgs), N.OUT_CLASS3_U8).cpu().numpy()

    def predict_binary(self, preprocessed_imgs) -> np.ndarray:
        """models.py:70-82: uint8 (B,H,W), 1 where the class is road or lane marking."""
        return self.predict_device(self.engine_input(preprocessed_imgs), N.OUT_BINARY_U8).cpu().numpy()

    @classmethod
    def preprocess_device(cls, bgr, layout: int = N.PRE_NCHW_F64, ctx: "N.Context | None" = None,
                          width: int | None = None, height: int | None = None) -> torch.Tensor:
        """Batched models.py:84-95 on the device: bgr (B,H0,W0,3) or (H0,W0,3) uint8."""
        x = _as_device_tensor(bgr, torch.uint8, None if ctx is None else ctx.device)
        if x.dim() == 3:
            x = x.unsqueeze(0)
        if x.dim() != 4 or x.shape[3] != 3:
            raise ValueError(f"expected a BGR uint8 frame (H, W, 3), got {tuple(x.shape)}")
        W = cls.INPUT_WIDTH if width is None else width
        H = cls.INPUT_HEIGHT if height is None else height
        B, H0, W0 = x.shape[:3]
        c = ctx if ctx is not None else N.shared_context(x.device.index)
        dev = x.device
        if layout == N.PRE_NCHW_F64:
            out = torch.empty((B, 3, H, W), dtype=torch.float64, device=dev)
        elif layout == N.PRE_NCHW_F32:
            out = torch.empty((B, 3, H, W), dtype=torch.float32, device=dev)
        else:
            out = torch.empty((B, H, W, 8 * (4 if c.precision == N.FP32 else 2)), dtype=torch.uint8, device=dev)
        c.preprocess(x, B, H0, W0, H, W, layout, out, torch.cuda.current_stream(dev))
        return out

    @classmethod
    def preprocess(cls, bgr_frame) -> np.ndarray:
        """models.py:84-95: BGR uint8 frame -> (1, 3, INPUT_HEIGHT, INPUT_WIDTH) float64 RGB,
        (x/256 - mean)/std. Bit-identical to the reference's NumPy float64 arithmetic given the
        same resized image (cv2.resize INTER_LINEAR restated in fixed point on the device)."""
        return cls.preprocess_device(bgr_frame, N.PRE_NCHW_F64).cpu().numpy()


class DeepLabV3(InferenceModel):
    """models.py:98-136 on the MI355X engine (BASELINE config 4).

    The reference feeds ``[img]`` to ``import/ImageTensor:0`` and returns
    ``import/SemanticPredictions:0`` (models.py:115-125): u8 RGB images in, int64 class ids out,
    with padding to the export's crop (513 in the model zoo), normalisation, MobileNetV2 + ASPP, logits, bilinear resize and
    argmax all inside the frozen graph. Here the same graph (deeplab_spec.py) runs as one op list of
    gfx950 kernels (libbugseg.so, bugseg_dl_*).

    Deviations, because the reference wrapper is broken as written:
    ``predict`` takes the ImageTensor layout itself — (H, W, 3) or (B, H, W, 3) u8 RGB, H, W at most
    the crop — instead of unpacking a 4-D NCHW shape and wrapping it in a list (models.py:116,124);
    ``preprocess`` (whose reference body uses undefined ``cls.input_size`` / ``IMAGE_MEAN``,
    models.py:129,132) returns the RGB u8 frame resized so the longer side is at most the crop — the
    resize the DeepLab demo applies before feeding the graph. The node-name printing
    (models.py:112-113, 116, 121) is dropped.

    The crop (height, width) is the export's own: read from the graph's pad-to-crop arithmetic by
    deeplab_graphdef.import_deeplab (``CROP_SIZE`` only when a graph does not hold it). Images larger
    than the crop are refused: the export sizes its image-pooling window and resize from the crop
    (deeplab/model.py, ``crop_size`` given at export), so the graph itself cannot run them.

    Backbones: MobileNetV2 (DeepLabV3, dense or no atrous branches) and Xception-65 (DeepLabV3+:
    separable ASPP, decoder at output stride 4), the two model-zoo forms (deeplab_xception.py), and
    ResNet-v1-50 / 101 "beta" (DeepLabV3, dense atrous ASPP; deeplab_resnet.py).

    Weights: GRAPH_PB_PATH may be a frozen TF DeepLab-MobileNetV2 GraphDef (``deeplab.pb``, read by
    deeplab_graphdef.import_deeplab; the file itself is absent, .MISSING_LARGE_BLOBS:1), a
    ``deeplab_spec.save`` .npz, or None for the seeded synthetic network (``deeplab_spec.build_deeplab``)."""
    INPUT_TENSOR_NAME = "import/ImageTensor:0"
    OUTPUT_TENSOR_NAME = "import/SemanticPredictions:0"
    INPUT_SIZE = 1024
    FROZEN_GRAPH_NAME = "deeplab.pb"
    CROP_SIZE = 513

    def __init__(self, GRAPH_PB_PATH=None, *, net=None, precision: str = "fp32", device: int | None = None,
                 fuse_dw: bool | None = None, fuse_prep: bool = True, backbone: str = "mobilenet_v2"):
        """precision: "fp32" (default: the parity mode, logits within 1e-3 of the fp32 graph, as a
        drop-in for the reference's TF fp32 sess.run) or "bf16" (the throughput mode the bench uses;
        class ids can differ from fp32 where two logits are close).
        fuse_dw=True computes each depthwise conv inside its projection's operand loads
        (bit-identical, measured slower; deeplab_spec.lower). fuse_prep=False runs the padding +
        normalisation as its own launch instead of inside the stem's operand loads (bit-identical).
        backbone: the seeded synthetic network when neither a file nor ``net`` is given —
        "mobilenet_v2" (deeplab_spec), "xception_65" (DeepLabV3+, deeplab_xception) or
        "resnet_v1_50_beta" / "resnet_v1_101_beta" (DeepLabV3, deeplab_resnet)."""
        from . import deeplab_spec
        if precision not in ("fp32", "bf16"):
            raise ValueError("precision must be 'fp32' or 'bf16'")
        if net is None:
            if GRAPH_PB_PATH is None:
                if backbone == "xception_65":
                    from .deeplab_xception import build_deeplab_xception
                    net = build_deeplab_xception()
                elif backbone == "mobilenet_v2":
                    net = deeplab_spec.build_deeplab()
                elif backbone in ("resnet_v1_50_beta", "resnet_v1_101_beta"):
                    from .deeplab_resnet import build_deeplab_resnet
                    net = build_deeplab_resnet(depth=50 if "50" in backbone else 101)
                else:
                    raise ValueError("backbone must be 'mobilenet_v2', 'xception_65', 'resnet_v1_50_beta' or "
                                     "'resnet_v1_101_beta'")
            else:
                if not os.path.exists(GRAPH_PB_PATH):
                    raise FileNotFoundError(f"{GRAPH_PB_PATH}: no such file")
                with open(GRAPH_PB_PATH, "rb") as f:
                    magic = f.read(4)
                if magic[:2] == b"PK":
                    net = deeplab_spec.load(GRAPH_PB_PATH)
                else:
                    # a frozen TF DeepLab export (models.py:104-110 reads it as a GraphDef)
                    from .deeplab_graphdef import import_deeplab
                    with open(GRAPH_PB_PATH, "rb") as f:
                        net = import_deeplab(f.read(), crop=None, default_crop=self.CROP_SIZE)
        self.net = net
        self.precision = precision
        self.ctx = N.DeepLabContext(device, N.BF16 if precision == "bf16" else N.FP32)
        self._spec = deeplab_spec
        self._blob = None
        self._plan_B = None
        self.plan_info = None
        self.fuse_dw = bool(int(os.environ.get("BUGSEG_DL_FUSE_DW", "0"))) if fuse_dw is None else fuse_dw
        self.fuse_prep = fuse_prep

    def _ensure_plan(self, B: int) -> None:
        if self._plan_B == B:
            return
        blob, ops, bufs, info = self._spec.lower(self.net, B, self.precision == "bf16", fuse_dw=self.fuse_dw,
                                                 fuse_prep=self.fuse_prep)
        if self._blob is None:
            self.ctx.load_weights(blob)
            self._blob = blob
        self.ctx.set_plan(ops, bufs, B, *self._spec.crop_hw(self.net))
        self._plan_B = B
        self.plan_info = info

    def predict_device(self, rgb, out: torch.Tensor | None = None) -> torch.Tensor:
        """(B, H, W, 3) u8 RGB (device or host) -> (B, H, W) int64 device tensor."""
        x = _as_device_tensor(rgb, torch.uint8, self.ctx.device)
        if x.dim() == 3:
            x = x.unsqueeze(0)
        if x.dim() != 4 or x.shape[3] != 3:
            raise ValueError(f"expected u8 RGB images (B, H, W, 3), got {tuple(x.shape)}")
        B, H, W = x.shape[:3]
        Hc, Wc = self._spec.crop_hw(self.net)
        if H > Hc or W > Wc:
            raise ValueError(f"image {H}x{W} exceeds the export's {Hc}x{Wc} crop: resize it first "
                             "(DeepLabV3.preprocess)")
        self._ensure_plan(B)
        if out is None:
            out = torch.empty((B, H, W), dtype=torch.int64, device=x.device)
        self.ctx.forward(x, B, H, W, out, torch.cuda.current_stream(x.device))
        return out

    def logits_device(self) -> torch.Tensor:
        """The last forward's logits (B, h, w, classes padded to 4) f32 at the backbone resolution."""
        h, w = self.plan_info["feature"]
        t = torch.empty((self._plan_B, h, w, self.plan_info["lcs"]), dtype=torch.float32,
                        device=torch.device("cuda", self.ctx.device))
        self.ctx.read_buffer(7, t, torch.cuda.current_stream(t.device))
        return t

    def predict(self, img) -> np.ndarray:
        """models.py:115-125: SemanticPredictions, (B, H, W) int64."""
        return self.predict_device(img).cpu().numpy()

    @classmethod
    def preprocess(cls, bgr_frame) -> np.ndarray:
        """BGR u8 frame -> RGB u8 frame whose longer side is at most CROP_SIZE (nearest-pixel
        downscale when larger; the reference body is broken, see the class docstring). For an export
        with another crop, set CROP_SIZE on the class (or resize to the model's net.crop)."""
        f = np.asarray(bgr_frame)
        if f.ndim != 3 or f.shape[2] != 3 or f.dtype != np.uint8:
            raise ValueError("expected a BGR uint8 frame (H, W, 3)")
        rgb = f[:, :, ::-1]
        H, W = rgb.shape[:2]
        r = cls.CROP_SIZE / max(H, W)
        if r < 1.0:
            h, w = max(1, int(r * H)), max(1, int(r * W))
            ys = np.minimum((np.arange(h) * (H / h)).astype(np.int64), H - 1)
            xs = np.minimum((np.arange(w) * (W / w)).astype(np.int64), W - 1)
            rgb = rgb[ys][:, xs]
        return np.ascontiguousarray(rgb)
