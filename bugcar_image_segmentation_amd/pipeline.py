"""Batched, device-resident frame -> occupancy-grid path (BASELINE config 3):

    BGR u8 frames (B,H0,W0,3)  --[resize kernel, only if H0xW0 != HxW]-->  BGR u8 (B,H,W,3)
      --29 launches, one per ENet block (the initial block normalises the raw bytes as it loads
        them, argmax + 3-class remap in the class layer's epilogue)-->  u8 (B,H,W)
      --BEV rasteriser kernel-->  int8 grids (B,h,w)   [or ROS data order]

Everything stays in HBM; there is no host round trip between stages. With streams > 1 every frame
shard runs all three stages on its own context and stream. This is the
loop the reference's (absent) ROS node runs per frame (README.md:19), batched.
"""
from __future__ import annotations

import torch

from . import _native as N
from .bev import bev_transform_tools
from .models import ENET


class OccupancyPipeline:
    """streams > 1 splits the batch into that many frame shards, each run by its own engine context
    (own activation arena) on its own HIP stream, so the launches of different shards overlap on the
    device (one shard's compute phases beside another's memory phases). Results are identical."""

    def __init__(self, model: ENET, bev: bev_transform_tools, grid_w_m: float, grid_h_m: float, cell_m: float,
                 model_hw: tuple[int, int] | None = None, ros_layout: bool = False, streams: int = 1,
                 binary: bool = False, stream_priority: int = 0, chain_forwards: bool = False, shard_offset: int = 0):
        """binary=True is the predict_binary + create_occupancy_grid_binary pairing (models.py:70-82,
        bev.py:97-165): class maps through the binary LUT, the binary rasteriser; in the laserscan-like
        mode its output is the reference's pair, (2, B, ...) (bev.py:164). stream_priority is the HIP
        priority of the side shards' streams (shard 0 runs on the caller's stream; lower = higher).
        chain_forwards=True starts shard i's forward when shard i-1's forward has finished, so each
        shard's BEV rasteriser runs beside the next shard's forward (only the last one is exposed)
        instead of all shards' forwards running together and their BEVs together at the end.
        shard_offset=k > 0 starts shard i+1 when shard i has reached its k-th launch (an
        event between launches k-1 and k of its forward), so the shards run different layers side by
        side instead of the same layer at the same time."""
        self.model = model
        self.binary = binary
        self.bev = bev
        self.grid = (grid_w_m, grid_h_m, cell_m)
        self.H, self.W = model_hw if model_hw is not None else (ENET.INPUT_HEIGHT, ENET.INPUT_WIDTH)
        self.ros_layout = ros_layout
        if (self.H, self.W) != (bev.input_width, bev.input_height):
            raise ValueError(f"model output {self.H}x{self.W} must equal the calibration's input image size "
                             f"{bev.input_width}x{bev.input_height} (bev.py:169)")
        if streams < 1:
            raise ValueError("streams must be >= 1")
        self.streams = streams
        self.stream_priority = stream_priority
        self.chain_forwards = chain_forwards
        self.shard_offset = int(shard_offset)
        self._ctxs = [model.ctx]
        self._streams = []
        self._x = None
        self._seg = None
        self._grid = None

    def _shard_ctxs(self, dev: torch.device):
        while len(self._ctxs) < self.streams:
            c = N.Context(dev.index, self.model.ctx.precision)
            c.load_weights(self.model.blob)
            self._ctxs.append(c)
            self._streams.append(torch.cuda.Stream(device=dev, priority=self.stream_priority))
        return self._ctxs, self._streams

    def _bufs(self, B: int, dev: torch.device):
        if self._x is None or self._x.shape[0] != B or self._x.device != dev:
            self._x = torch.empty((B, self.H, self.W, 3), dtype=torch.uint8, device=dev)   # resized BGR
            self._seg = torch.empty((B, self.H, self.W), dtype=torch.uint8, device=dev)
            self._grid = torch.empty(self._grid_shape(B), dtype=torch.int8, device=dev)
        return self._x, self._seg, self._grid

    def _params(self):
        return self.bev.occupancy_params(*self.grid, ros_layout=self.ros_layout, binary=self.binary)

    def _grid_shape(self, B):
        p = self._params()
        shape = (B, p.occ_w, p.occ_h) if self.ros_layout else (B, p.occ_h, p.occ_w)
        return ((2,) + shape) if self.binary and p.laserscan else shape

    def run(self, frames_bgr: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        if frames_bgr.dim() != 4 or frames_bgr.shape[3] != 3 or frames_bgr.dtype != torch.uint8 or not frames_bgr.is_cuda:
            raise ValueError("frames must be a (B, H0, W0, 3) uint8 device tensor")
        B, H0, W0 = frames_bgr.shape[:3]
        x, seg, grid = self._bufs(B, frames_bgr.device)
        if grid.shape != self._grid_shape(B):       # the calibration's laserscan flag changed
            self._grid = grid = torch.empty(self._grid_shape(B), dtype=torch.int8, device=frames_bgr.device)
        frames = frames_bgr.contiguous()
        out = grid if out is None else out
        if tuple(out.shape) != tuple(grid.shape) or out.dtype != torch.int8 or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous int8 tensor of shape {tuple(grid.shape)}")
        p = self._params()
        if self.streams == 1 or B < self.streams:
            self._run_shard(self.model.ctx, frames, x, seg, out, p, None)
            return out
        pair = self.binary and bool(p.laserscan)
        ctxs, streams = self._shard_ctxs(frames.device)
        main = torch.cuda.current_stream(frames.device)
        ready = main.record_event()
        bounds = [B * i // self.streams for i in range(self.streams + 1)]
        for i in range(self.streams):
            s, e = bounds[i], bounds[i + 1]
            st = main if i == 0 else streams[i - 1]
            if i:
                st.wait_event(ready)
            split_done = self.chain_forwards or (self.shard_offset > 0 and i + 1 < self.streams)
            with torch.cuda.stream(st):
                if self.shard_offset > 0 and i + 1 < self.streams:
                    self._run_forward(ctxs[i], frames[s:e], x[s:e], seg[s:e], st, split=self.shard_offset)
                    ready = self._split_event
                elif self.chain_forwards:
                    self._run_forward(ctxs[i], frames[s:e], x[s:e], seg[s:e], st)
                    ready = torch.cuda.Event()
                    ready.record(st)                  # the next shard's forward starts here
                if pair:
                    # the kernel writes a shard's pair as one contiguous (2, e - s, ...) block; the
                    # batch's pair (2, B, ...) holds it as two slabs, so stage it and copy
                    tmp = self._pair_buf(i, (2, e - s) + tuple(out.shape[2:]), out.device)
                    self._run_shard(ctxs[i], frames[s:e], x[s:e], seg[s:e], tmp, p, st, forward=not split_done)
                    out[:, s:e].copy_(tmp)
                else:
                    self._run_shard(ctxs[i], frames[s:e], x[s:e], seg[s:e], out[s:e], p, st, forward=not split_done)
        for st in streams[: self.streams - 1]:
            main.wait_stream(st)
        return out

    def _pair_buf(self, i, shape, dev):
        if not hasattr(self, "_pairs"):
            self._pairs = {}
        t = self._pairs.get(i)
        if t is None or tuple(t.shape) != shape or t.device != dev:
            t = self._pairs[i] = torch.empty(shape, dtype=torch.int8, device=dev)
        return t

    def capture(self, frames_bgr: torch.Tensor, out: torch.Tensor | None = None, warm: bool = True):
        """Record one ``run`` over these frame / output buffers as a HIP graph (every shard's launches
        and the stream fork / join between them) and return (replay, out): ``replay()`` re-launches the
        whole step with one call, reading whatever the frame buffer holds at that time. The buffers
        must stay alive and keep their addresses. warm=True runs the step once eagerly first;
        warm=False captures the very first call at this shape and geometry (the library allocates
        arenas and builds its tables on its own stream during the capture; only the shard contexts
        and streams are created beforehand)."""
        dev = frames_bgr.device
        if warm:
            self.run(frames_bgr, out)
        elif self.streams > 1 and frames_bgr.shape[0] >= self.streams:
            self._shard_ctxs(dev)
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            res = self.run(frames_bgr, out)
        return graph.replay, res

    def _run_forward(self, ctx, frames, x, seg, stream, split=0):
        B, H0, W0 = frames.shape[:3]
        if (H0, W0) != (self.H, self.W):
            # resize only (models.py:87); colour swap + normalisation are fused into the initial block
            ctx.preprocess(frames, B, H0, W0, self.H, self.W, N.PRE_BGR_U8, x, stream)
            frames = x
        kind = N.OUT_BINARY_U8 if self.binary else N.OUT_CLASS3_U8
        if split <= 0:
            ctx.forward_bgr(frames, B, self.H, self.W, kind, seg, stream)
            return
        # launches [0, split), an event (the next shard starts there), then the rest
        ctx.forward_bgr_ops(frames, B, self.H, self.W, kind, seg, 0, split, stream)
        self._split_event = torch.cuda.Event()
        self._split_event.record(stream)
        ctx.forward_bgr_ops(frames, B, self.H, self.W, kind, seg, split, -1, stream)

    def _run_shard(self, ctx, frames, x, seg, out, p, stream, forward=True):
        if forward:
            self._run_forward(ctx, frames, x, seg, stream)
        # the shard's own context: its laserscan scratch is never shared with another shard's stream
        ctx.bev(seg, frames.shape[0], p, out, stream)
