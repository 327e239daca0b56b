"""Debug (ablation A/B): HIP-event time of the default BEV rasteriser (32 frames of 480x640, the bench
class maps) and of every forward kernel tag at the bench shard (fp16, B = 32), for whichever library
BUGSEG_LIB names (scripts/build_variants.sh builds the ablation variants: wrong results, timing only).

usage: BUGSEG_LIB=... python scripts/abl_probe.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import kernel_table  # noqa: E402
from bugcar_image_segmentation_amd import _native as N  # noqa: E402
from bugcar_image_segmentation_amd import enet_spec, synthetic  # noqa: E402
from bugcar_image_segmentation_amd.models import ENET  # noqa: E402

B, H, W = 32, 480, 640
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
model = ENET(weights=enet_spec.build_enet(), precision=os.environ.get("PREC", "fp16"))
bev = synthetic.synthetic_bev(H, W)
grid = (synthetic.GRID_W_M, synthetic.GRID_H_M, synthetic.CELL_M)
frames = torch.from_numpy(synthetic.uniform_frames(B, H, W)).cuda()
seg = torch.empty((B, H, W), dtype=torch.uint8, device="cuda")
stream = torch.cuda.current_stream()
model.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS3_U8, seg)
torch.cuda.synchronize()
g = bev.create_occupancy_grid_device(seg, *grid)
torch.cuda.synchronize()
graph = torch.cuda.CUDAGraph()          # replayed: eager back-to-back calls are host-bound
with torch.cuda.graph(graph):
    for _ in range(reps):
        bev.create_occupancy_grid_device(seg, *grid, out=g)
graph.replay()
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
graph.replay()
ev[1].record()
ev[1].synchronize()
print(f"{os.path.basename(os.environ.get('BUGSEG_LIB', 'default'))}: bev {ev[0].elapsed_time(ev[1]) / reps * 1000:.1f} us / 32 frames", flush=True)
k = kernel_table(model.ctx, B, H, W, 5, stream)
print("   " + "  ".join(f"{t}: {v['us_per_launch']:.1f}" for t, v in sorted(k.items(), key=lambda kv: -kv[1]["total_us"])), flush=True)
