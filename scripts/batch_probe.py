"""Debug: per-kernel-tag launch durations (HIP events around every launch, single stream) of the
bf16 forward at several batch sizes, to separate per-tile cost from launch quantisation / tail.

usage: python scripts/batch_probe.py [B ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import kernel_table  # noqa: E402
from bugcar_image_segmentation_amd import _native as N  # noqa: E402
from bugcar_image_segmentation_amd import enet_spec, synthetic  # noqa: E402
from bugcar_image_segmentation_amd.models import ENET  # noqa: E402

H, W = 480, 640
blocks = enet_spec.build_enet()
m = ENET(weights=blocks, precision=os.environ.get("PREC", "bf16"))
stream = torch.cuda.current_stream()
for B in [int(v) for v in (sys.argv[1:] or ["8", "16", "32", "64", "128"])]:
    frames = torch.from_numpy(synthetic.uniform_frames(B, H, W)).cuda()
    seg = torch.empty((B, H, W), dtype=torch.uint8, device="cuda")
    for _ in range(3):
        m.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS3_U8, seg)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(stream)
    for _ in range(10):
        m.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS3_U8, seg)
    ev[1].record(stream)
    ev[1].synchronize()
    fwd = ev[0].elapsed_time(ev[1]) / 10
    k = kernel_table(m.ctx, B, H, W, 5, stream)
    print(f"B={B}: forward {fwd:.3f} ms = {fwd * 1e3 / B:.2f} us/frame ({B / fwd * 1e3:.0f} frames/s)", flush=True)
    for tag, v in sorted(k.items(), key=lambda kv: -kv[1]["total_us"]):
        print(f"   {tag:18s} n={v['launches']:2d} {v['us_per_launch']:8.2f} us/launch {v['us_per_launch'] / B:6.3f} us/frame/launch "
              f"{v['bytes_per_launch'] / v['us_per_launch'] / 1e3:7.0f} GB/s", flush=True)
    del frames, seg
