"""ctypes binding of libbugseg.so (include/bugseg.h).

There is no fallback: if the library is missing or no HIP device is visible, every product call
raises. torch is imported first so that the library binds to torch's already-loaded HIP runtime
(same soname libamdhip64.so.7) and torch device pointers / streams are valid for it.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

import torch  # noqa: F401  (must precede loading the library: shared HIP runtime)

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("BUGSEG_LIB", _PKG / "libbugseg.so"))

OK, EINVAL, ENOMEM, EHIP, EFORMAT, ESTATE = 0, -1, -2, -3, -4, -5
FP32, BF16, F16 = 0, 1, 2
OUT_LOGITS_F32, OUT_CLASS15_U8, OUT_CLASS3_U8, OUT_BINARY_U8 = 0, 1, 2, 3
PRE_ENGINE, PRE_NCHW_F64, PRE_NCHW_F32, PRE_BGR_U8 = 0, 1, 2, 3

EXPORTED = ("bugseg_version", "bugseg_create", "bugseg_destroy", "bugseg_load_weights", "bugseg_num_classes",
            "bugseg_input_bytes", "bugseg_preprocess", "bugseg_nchw_to_input", "bugseg_enet_forward",
            "bugseg_enet_forward_bgr", "bugseg_enet_forward_bgr_ops",
            "bugseg_bev_occgrid", "bugseg_bev_workspace_bytes", "bugseg_bev_occgrid_ws", "bugseg_plan_info", "bugseg_plan_op", "bugseg_plan_launch_op",
            "bugseg_last_error",
            "bugseg_dl_create", "bugseg_dl_destroy", "bugseg_dl_load_weights", "bugseg_dl_set_plan",
            "bugseg_dl_forward", "bugseg_dl_launch_op", "bugseg_dl_read_buffer", "bugseg_dl_last_error",
            "bugseg_debug_parse_pack", "bugseg_debug_polar_tables", "bugseg_debug_ctx_info", "bugseg_debug_set_spans", "bugseg_debug_pool_indices",
            "bugseg_dl_debug_check_plan")
DL_OP_FIELDS = 32


class BevParams(ctypes.Structure):
    _fields_ = [("M", ctypes.c_double * 9), ("in_rows", ctypes.c_int), ("in_cols", ctypes.c_int),
                ("warp_w", ctypes.c_int), ("warp_h", ctypes.c_int), ("occ_w_px", ctypes.c_int),
                ("occ_h_px", ctypes.c_int), ("occ_w", ctypes.c_int), ("occ_h", ctypes.c_int),
                ("left_x", ctypes.c_int), ("top_y", ctypes.c_int), ("ros_layout", ctypes.c_int),
                ("variant", ctypes.c_int), ("laserscan", ctypes.c_int)]


class BugsegError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"bugseg error {code}: {msg}")
        self.code = code


_lib = None
_lock = threading.Lock()


def load_library(path: Path | str | None = None) -> ctypes.CDLL:
    """Load (once) and prototype libbugseg.so. Raises if it is missing."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = Path(path) if path else LIB_PATH
        if not p.exists():
            raise FileNotFoundError(f"{p} not found: build it with `python -m bugcar_image_segmentation_amd.build` "
                                    "(or __graft_entry__.build())")
        lib = ctypes.CDLL(str(p))
        vp, i, sz, cp = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_char_p
        proto = {
            "bugseg_version": (i, []),
            "bugseg_create": (i, [i, i, ctypes.POINTER(vp)]),
            "bugseg_destroy": (i, [vp]),
            "bugseg_load_weights": (i, [vp, vp, sz]),
            "bugseg_num_classes": (i, [vp]),
            "bugseg_input_bytes": (sz, [vp, i, i, i]),
            "bugseg_preprocess": (i, [vp, vp, i, i, i, i, i, i, vp, vp]),
            "bugseg_nchw_to_input": (i, [vp, vp, i, i, i, i, vp, vp]),
            "bugseg_enet_forward": (i, [vp, vp, i, i, i, i, vp, vp]),
            "bugseg_enet_forward_bgr": (i, [vp, vp, i, i, i, i, vp, vp]),
            "bugseg_enet_forward_bgr_ops": (i, [vp, vp, i, i, i, i, vp, i, i, vp]),
            "bugseg_bev_occgrid": (i, [vp, vp, i, ctypes.POINTER(BevParams), vp, vp]),
            "bugseg_bev_workspace_bytes": (sz, [ctypes.POINTER(BevParams), i]),
            "bugseg_bev_occgrid_ws": (i, [vp, vp, i, ctypes.POINTER(BevParams), vp, vp, sz, vp]),
            "bugseg_plan_info": (i, [vp, i, i, i, i, i, ctypes.POINTER(i), ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
            "bugseg_plan_op": (i, [vp, i, i, i, i, cp, i, ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
            "bugseg_plan_launch_op": (i, [vp, i, i, i, i, vp]),
            "bugseg_last_error": (cp, [vp]),
            "bugseg_dl_create": (i, [i, i, ctypes.POINTER(vp)]),
            "bugseg_dl_destroy": (i, [vp]),
            "bugseg_dl_load_weights": (i, [vp, vp, sz]),
            "bugseg_dl_set_plan": (i, [vp, vp, i, vp, i, i, i, i]),
            "bugseg_dl_forward": (i, [vp, vp, i, i, i, vp, vp]),
            "bugseg_dl_launch_op": (i, [vp, i, vp]),
            "bugseg_dl_read_buffer": (i, [vp, i, vp, sz, vp]),
            "bugseg_dl_last_error": (cp, [vp]),
            "bugseg_debug_parse_pack": (i, [vp, sz, i, ctypes.POINTER(i)]),
            "bugseg_debug_polar_tables": (i, [i, i, i, vp, sz, vp, sz, ctypes.POINTER(i), ctypes.POINTER(i)]),
            "bugseg_debug_ctx_info": (i, [vp, i, i]),
            "bugseg_debug_set_spans": (i, [vp, vp, i]),
            "bugseg_debug_pool_indices": (i, [vp, i, i, i, i, vp, sz, ctypes.POINTER(ctypes.c_int), vp]),
            "bugseg_dl_debug_check_plan": (i, [vp, i, vp, i, i, i, i, i, sz]),
        }
        for name, (res, args) in proto.items():
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        _lib = lib
        return lib


def check(code: int, ctx=None) -> None:
    if code != OK:
        lib = load_library()
        msg = lib.bugseg_last_error(ctx).decode(errors="replace")
        if code == EINVAL:
            raise ValueError(msg)
        raise BugsegError(code, msg)


def require_gpu() -> None:
    if not torch.cuda.is_available():
        raise RuntimeError("bugseg needs a HIP GPU (MI355X / gfx950); none is visible — there is no CPU fallback")


def stream_handle(stream: torch.cuda.Stream | None = None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


class Context:
    """Owns one bugseg_ctx (device + precision + weights + activation arena)."""

    def __init__(self, device: int | None = None, precision: int = FP32):
        require_gpu()
        self.lib = load_library()
        self.device = torch.cuda.current_device() if device is None else int(device)
        self.precision = precision
        h = ctypes.c_void_p()
        check(self.lib.bugseg_create(self.device, precision, ctypes.byref(h)))
        self.h = h

    def close(self) -> None:
        if getattr(self, "h", None) and self.h.value:
            self.lib.bugseg_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_weights(self, blob: bytes) -> None:
        buf = ctypes.create_string_buffer(blob, len(blob))
        check(self.lib.bugseg_load_weights(self.h, buf, len(blob)), self.h)

    @property
    def num_classes(self) -> int:
        return int(self.lib.bugseg_num_classes(self.h))

    def input_bytes(self, B: int, H: int, W: int) -> int:
        return int(self.lib.bugseg_input_bytes(self.h, B, H, W))

    def preprocess(self, bgr, B, H0, W0, H, W, layout, out, stream=None):
        check(self.lib.bugseg_preprocess(self.h, bgr.data_ptr(), B, H0, W0, H, W, layout, out.data_ptr(),
                                         stream_handle(stream)), self.h)

    def nchw_to_input(self, x, B, H, W, out, stream=None):
        check(self.lib.bugseg_nchw_to_input(self.h, x.data_ptr(), int(x.dtype == torch.float64), B, H, W,
                                            out.data_ptr(), stream_handle(stream)), self.h)

    def forward(self, x, B, H, W, out_kind, out, stream=None):
        check(self.lib.bugseg_enet_forward(self.h, x.data_ptr(), B, H, W, out_kind, out.data_ptr(),
                                           stream_handle(stream)), self.h)

    def forward_bgr(self, bgr, B, H, W, out_kind, out, stream=None):
        check(self.lib.bugseg_enet_forward_bgr(self.h, bgr.data_ptr(), B, H, W, out_kind, out.data_ptr(),
                                               stream_handle(stream)), self.h)

    def forward_bgr_ops(self, bgr, B, H, W, out_kind, out, first_op, last_op, stream=None):
        """Launches [first_op, last_op) of forward_bgr's plan only (last_op = -1: to the end)."""
        check(self.lib.bugseg_enet_forward_bgr_ops(self.h, bgr.data_ptr(), B, H, W, out_kind, out.data_ptr(),
                                                   first_op, last_op, stream_handle(stream)), self.h)

    def bev(self, seg, B, params: BevParams, out, stream=None):
        """bugseg_bev_occgrid_ws: the laserscan scratch comes from torch's caching allocator on the
        stream the work runs on (reuse is stream-ordered; under graph capture it is the graph's pool),
        so the library never allocates or synchronises for it."""
        st = stream if stream is not None else torch.cuda.current_stream(seg.device)
        nws = int(self.lib.bugseg_bev_workspace_bytes(ctypes.byref(params), B))
        ws = None
        if nws:
            with torch.cuda.stream(st):
                ws = torch.empty(nws, dtype=torch.uint8, device=seg.device)
        check(self.lib.bugseg_bev_occgrid_ws(self.h, seg.data_ptr(), B, ctypes.byref(params), out.data_ptr(),
                                             0 if ws is None else ws.data_ptr(), nws, stream_handle(st)), self.h)

    def plan_info(self, B, H, W, out_kind, bgr_input=False):
        """-> (launches, per-layer algorithmic bytes, plan compulsory bytes, flops) of one forward."""
        n = ctypes.c_int()
        lb = ctypes.c_double()
        pb = ctypes.c_double()
        fl = ctypes.c_double()
        check(self.lib.bugseg_plan_info(self.h, B, H, W, out_kind, int(bool(bgr_input)), ctypes.byref(n),
                                        ctypes.byref(lb), ctypes.byref(pb), ctypes.byref(fl)), self.h)
        return n.value, lb.value, pb.value, fl.value

    def plan_op(self, B, H, W, op):
        """Profiling hook: -> (kernel tag, per-layer algorithmic bytes, bytes the launch moves, flops)
        of launch `op` of the plan the last forward at (B, H, W) ran."""
        buf = ctypes.create_string_buffer(64)
        lb, pb, fl = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        check(self.lib.bugseg_plan_op(self.h, B, H, W, op, buf, 64, ctypes.byref(lb), ctypes.byref(pb),
                                      ctypes.byref(fl)), self.h)
        return buf.value.decode(), lb.value, pb.value, fl.value

    def launch_op(self, B, H, W, op, stream=None):
        """Profiling hook: enqueue launch `op` of that plan alone (its buffers must still be alive)."""
        check(self.lib.bugseg_plan_launch_op(self.h, B, H, W, op, ctypes.c_void_p(stream_handle(stream))), self.h)

    def debug_info(self, what: int, arg: int = 0) -> int:
        """Test hook (bugseg_debug_ctx_info): 0 = exact affine byte normalisation in use, 1 = fp32 range
        scaling off, 2 = weight exponent of packed convolution `arg`."""
        return int(self.lib.bugseg_debug_ctx_info(self.h, what, arg))

    def set_spans(self, spans=None):
        """Measurement hook (bugseg_debug_set_spans): a CUDA int64 tensor of 512 words per plan op (64
        [entry, exit] slots, 64 B apart) that later launches fold their clock into (None disarms); ops
        beyond the tensor's size are never armed."""
        if spans is None:
            check(self.lib.bugseg_debug_set_spans(self.h, ctypes.c_void_p(0), 0), self.h)
            return
        if not spans.is_cuda or spans.dtype != torch.int64 or not spans.is_contiguous() or spans.numel() % 512:
            raise ValueError("spans must be a contiguous CUDA int64 tensor of 512 words per op")
        check(self.lib.bugseg_debug_set_spans(self.h, ctypes.c_void_p(spans.data_ptr()), spans.numel() // 512), self.h)

    def pool_indices(self, B: int, H: int, W: int, block: int, shape: tuple, stream=None) -> torch.Tensor:
        """Test hook (bugseg_debug_pool_indices): the pooling indices the last forward at (B, H, W) wrote
        for downsampling block `block`, as a uint8 (B, h, w, idx_cs) device tensor; shape = (h, w, idx_cs)."""
        out = torch.empty((B,) + tuple(shape), dtype=torch.uint8, device=torch.device("cuda", self.device))
        cs = ctypes.c_int(0)
        check(self.lib.bugseg_debug_pool_indices(self.h, B, H, W, block, ctypes.c_void_p(out.data_ptr()), out.numel(),
                                                 ctypes.byref(cs), ctypes.c_void_p(stream_handle(stream))), self.h)
        if cs.value != shape[-1]:
            raise ValueError(f"index tensor has channel stride {cs.value}, not {shape[-1]}")
        return out


_shared: dict[int, Context] = {}


def shared_context(device: int | None = None) -> Context:
    """Per-device context for the weight-free ops (preprocess classmethod, BEV rasteriser)."""
    require_gpu()
    d = torch.cuda.current_device() if device is None else int(device)
    with _lock:
        c = _shared.get(d)
    if c is None:
        c = Context(d, FP32)
        with _lock:
            _shared.setdefault(d, c)
            c = _shared[d]
    return c


class DeepLabContext:
    """Owns one bugseg_dl (DeepLabV3 executor: weights + op list + activation arena), include/bugseg.h."""

    def __init__(self, device: int | None = None, precision: int = BF16):
        require_gpu()
        self.lib = load_library()
        self.device = torch.cuda.current_device() if device is None else int(device)
        self.precision = precision
        h = ctypes.c_void_p()
        self._check(self.lib.bugseg_dl_create(self.device, precision, ctypes.byref(h)), None)
        self.h = h

    def _check(self, code, h):
        if code != OK:
            msg = self.lib.bugseg_dl_last_error(h).decode(errors="replace")
            if code == EINVAL:
                raise ValueError(msg)
            raise BugsegError(code, msg)

    def close(self) -> None:
        if getattr(self, "h", None) and self.h.value:
            self.lib.bugseg_dl_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_weights(self, blob: bytes) -> None:
        buf = ctypes.create_string_buffer(blob, len(blob))
        self._check(self.lib.bugseg_dl_load_weights(self.h, buf, len(blob)), self.h)

    def set_plan(self, ops, buf_bytes, B: int, Hc: int, Wc: int) -> None:
        import numpy as np
        o = np.ascontiguousarray(ops, dtype=np.int32)
        assert o.ndim == 2 and o.shape[1] == DL_OP_FIELDS
        b = np.ascontiguousarray(buf_bytes, dtype=np.uint64)
        self._check(self.lib.bugseg_dl_set_plan(self.h, o.ctypes.data, o.shape[0], b.ctypes.data, b.shape[0], B, Hc, Wc),
                    self.h)

    def forward(self, rgb, B, H, W, out, stream=None):
        self._check(self.lib.bugseg_dl_forward(self.h, rgb.data_ptr(), B, H, W, out.data_ptr(), stream_handle(stream)),
                    self.h)

    def launch_op(self, op, stream=None):
        self._check(self.lib.bugseg_dl_launch_op(self.h, op, ctypes.c_void_p(stream_handle(stream))), self.h)

    def read_buffer(self, buf, out, stream=None):
        self._check(self.lib.bugseg_dl_read_buffer(self.h, buf, out.data_ptr(), out.numel() * out.element_size(),
                                                   ctypes.c_void_p(stream_handle(stream))), self.h)
