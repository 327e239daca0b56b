"""Debug: BEV rasteriser time per 32-frame batch on the bench's class maps (the kernel variant is
chosen by BUGSEG_BEV_F, read once per process), for rocprofv3 counter passes (scripts/gpu_bevpmc.sh).

usage: python scripts/bev_probe.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bugcar_image_segmentation_amd import _native as N  # noqa: E402
from bugcar_image_segmentation_amd import enet_spec, synthetic  # noqa: E402
from bugcar_image_segmentation_amd.models import ENET  # noqa: E402

B, H, W = 32, 480, 640
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
model = ENET(weights=enet_spec.build_enet(), precision="bf16")
bev = synthetic.synthetic_bev(H, W)
grid = (synthetic.GRID_W_M, synthetic.GRID_H_M, synthetic.CELL_M)
frames = torch.from_numpy(synthetic.uniform_frames(B, H, W)).cuda()
seg = torch.empty((B, H, W), dtype=torch.uint8, device="cuda")
model.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS3_U8, seg)
print("class histogram", torch.bincount(seg.flatten().long(), minlength=3).tolist())
g = bev.create_occupancy_grid_device(seg, *grid)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
for _ in range(reps):
    bev.create_occupancy_grid_device(seg, *grid, out=g)
ev[1].record()
ev[1].synchronize()
print(f"BEV_F={os.environ.get('BUGSEG_BEV_F', 'default')}: {ev[0].elapsed_time(ev[1]) / reps * 1000:8.1f} us per {B} frames",
      flush=True)
