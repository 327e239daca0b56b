"""Debug: the BEV rasteriser right after a forward (cold caches, as bench.py's stage timing runs it) vs
back to back (warm), per repetition, at the bench shard (32 frames of 480x640, fp16).

usage: python scripts/bev_cold_probe.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bugcar_image_segmentation_amd import _native as N  # noqa: E402
from bugcar_image_segmentation_amd import enet_spec, synthetic  # noqa: E402
from bugcar_image_segmentation_amd.models import ENET  # noqa: E402

B, H, W = 32, 480, 640
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
model = ENET(weights=enet_spec.build_enet(), precision="fp16")
bev = synthetic.synthetic_bev(H, W)
grid = (synthetic.GRID_W_M, synthetic.GRID_H_M, synthetic.CELL_M)
frames = torch.from_numpy(synthetic.uniform_frames(B, H, W)).cuda()
seg = torch.empty((B, H, W), dtype=torch.uint8, device="cuda")
stream = torch.cuda.current_stream()
model.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS3_U8, seg)
g = bev.create_occupancy_grid_device(seg, *grid)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
cold, warm = [], []
for _ in range(reps):
    ev[0].record(stream)
    model.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS3_U8, seg)
    ev[1].record(stream)
    bev.create_occupancy_grid_device(seg, *grid, out=g)
    ev[2].record(stream)
    ev[2].synchronize()
    cold.append(ev[1].elapsed_time(ev[2]) * 1e3)
for _ in range(reps):
    ev[1].record(stream)
    bev.create_occupancy_grid_device(seg, *grid, out=g)
    ev[2].record(stream)
    ev[2].synchronize()
    warm.append(ev[1].elapsed_time(ev[2]) * 1e3)
print("after a forward (us):", " ".join(f"{v:.1f}" for v in cold))
print("back to back    (us):", " ".join(f"{v:.1f}" for v in warm))
