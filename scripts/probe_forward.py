"""Profiling workload: `reps` forwards (+ BEV) of one B-frame 480x640 shard in one precision on one
stream — what rocprofv3 --pmc passes attach to (scripts/gpu_r4_sq.sh). Kernel launches of the
warm-up are in the trace too; the summaries average every dispatch of a kernel.

usage: python scripts/probe_forward.py [prec=fp16] [B=32] [reps=5]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bugcar_image_segmentation_amd import _native as N  # noqa: E402
from bugcar_image_segmentation_amd import enet_spec, synthetic  # noqa: E402
from bugcar_image_segmentation_amd.models import ENET  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp16"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
H, W = 480, 640
m = ENET(weights=enet_spec.build_enet(), precision=prec)
bev = synthetic.synthetic_bev(H, W)
grid = (synthetic.GRID_W_M, synthetic.GRID_H_M, synthetic.CELL_M)
frames = torch.from_numpy(synthetic.uniform_frames(B, H, W)).cuda()
seg = torch.empty((B, H, W), dtype=torch.uint8, device="cuda")
for _ in range(reps):
    m.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS3_U8, seg)
    bev.create_occupancy_grid_device(seg, *grid)
torch.cuda.synchronize()
print("probe done", prec, B, reps)
