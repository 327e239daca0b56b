"""Debug: in-kernel phase clocks of the fused bottleneck (libbugseg_stamps.so, -DBUGSEG_STAMPS).

Runs one forward (bf16 unless given) at batch B, then launches each fused-bottleneck op of the plan alone with the
stamp buffer armed and prints, per op, the mean shader-clock cycles of each tile phase:
  wait0  top-of-tile barrier (previous tile's phase 3 of the slowest wave)
  ph1    projection over tile + halo (global loads -> MFMA -> t0 in LDS)
  bar1   barrier after phase 1
  ph2    middle conv MFMA loop (t0 from LDS)
  mid    barrier + t1 to LDS + barrier + t1 fragments to registers + barrier
  ph3    expansion + residual + stores issued
and the span of the launch in clocks next to its HIP-event duration (-> effective clock).

usage: python scripts/stamp_probe.py [B] [precision: bf16 | fp16 | fp32]   (build: python -m bugcar_image_segmentation_amd.build --stamps)"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["BUGSEG_LIB"] = os.path.join(ROOT, "bugcar_image_segmentation_amd", "libbugseg_stamps.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bugcar_image_segmentation_amd import _native as N  # noqa: E402
from bugcar_image_segmentation_amd import enet_spec, synthetic  # noqa: E402
from bugcar_image_segmentation_amd.models import ENET  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
H, W = 480, 640
lib = N.load_library()
lib.bugseg_debug_set_stamps.argtypes = [ctypes.c_void_p]
m = ENET(weights=enet_spec.build_enet(), precision=sys.argv[2] if len(sys.argv) > 2 else "bf16")
frames = torch.from_numpy(synthetic.uniform_frames(B, H, W)).cuda()
seg = torch.empty((B, H, W), dtype=torch.uint8, device="cuda")
for _ in range(3):
    m.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS3_U8, seg)
torch.cuda.synchronize()
n = m.ctx.plan_info(B, H, W, 2)[0]
stamps = torch.zeros(1 << 20, dtype=torch.int64, device="cuda")
stream = torch.cuda.current_stream()
seen = set()
for i in range(n):
    tag = m.ctx.plan_op(B, H, W, i)[0]
    if not (tag.startswith("bneck") or tag.startswith("down")) or tag in seen:
        continue
    seen.add(tag)
    for _ in range(3):
        m.ctx.launch_op(B, H, W, i, stream)
    stamps.zero_()
    torch.cuda.synchronize()
    assert lib.bugseg_debug_set_stamps(ctypes.c_void_p(stamps.data_ptr())) == 0
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(stream)
    m.ctx.launch_op(B, H, W, i, stream)
    ev[1].record(stream)
    torch.cuda.synchronize()
    assert lib.bugseg_debug_set_stamps(ctypes.c_void_p(0)) == 0
    us = ev[0].elapsed_time(ev[1]) * 1e3
    allst = stamps.cpu().numpy()
    ent = allst[1 << 19:].reshape(-1, 2)
    nwg = int((ent[:, 0] != 0).sum())
    ent = ent[:nwg]
    s = allst[:1 << 19].reshape(-1, 8)
    s = s[s[:, 0] != 0]
    d = np.diff(s[:, :7], axis=1).astype(np.float64)
    names = ["wait0", "ph1", "bar1", "ph2", "mid", "ph3"]
    wg = s[:, 7]
    per_wg = np.bincount(wg.astype(np.int64))
    per_wg = per_wg[per_wg > 0]
    # span per XCD (clocks of different XCDs need not agree): blockIdx & 7 is the XCD in round-robin dispatch
    spans = []
    for x in range(8):
        sx = s[(wg & 7) == x]
        if len(sx):
            spans.append(sx[:, 6].max() - sx[:, 0].min())
    tile_cyc = (s[:, 6] - s[:, 0]).mean()
    # entry / exit of every workgroup on the 100 MHz real-time clock, from the first entry (us)
    e = (ent[:, 0] - ent[:, 0].min()) / 100.0
    x = (ent[:, 1] - ent[:, 0].min()) / 100.0
    life = x - e
    print(f"     realtime: entry p50/p90/max {np.percentile(e, 50):.1f}/{np.percentile(e, 90):.1f}/{e.max():.1f} us  "
          f"WG life p10/p50/p90 {np.percentile(life, 10):.1f}/{np.percentile(life, 50):.1f}/{np.percentile(life, 90):.1f}  "
          f"exit p10/p50/p90/max {np.percentile(x, 10):.1f}/{np.percentile(x, 50):.1f}/{np.percentile(x, 90):.1f}/{x.max():.1f} us", flush=True)
    h, _ = np.histogram(e, bins=10, range=(0, x.max()))
    hx, _ = np.histogram(x, bins=10, range=(0, x.max()))
    print(f"     entries per tenth of the span: {h.tolist()}  exits: {hx.tolist()}", flush=True)
    print(f"op {i:2d} {tag:16s} B={B}: {len(s)} tiles on {len(per_wg)} WGs ({per_wg.min()}-{per_wg.max()} tiles/WG); "
          f"{us:.1f} us; span {np.mean(spans):.0f} cyc -> {np.mean(spans) / us / 1e3:.2f} GHz; tile {tile_cyc:.0f} cyc", flush=True)
    print("     " + "  ".join(f"{nm}={d[:, k].mean():7.0f} (p90 {np.percentile(d[:, k], 90):7.0f})" for k, nm in enumerate(names)), flush=True)
    # tiles 1.. of each WG (steady state, weights already staged)
    first = np.zeros(len(s), bool)
    order = np.lexsort((s[:, 0], wg))
    first[order[np.r_[True, wg[order][1:] != wg[order][:-1]]]] = True
    if (~first).any():
        print("     later tiles: " + "  ".join(f"{nm}={d[~first, k].mean():7.0f}" for k, nm in enumerate(names)), flush=True)
        print("     first tiles: " + "  ".join(f"{nm}={d[first, k].mean():7.0f}" for k, nm in enumerate(names)), flush=True)
