"""Debug: every form of the BEV rasteriser (bev_kernels.hip; BUGSEG_BEV_F = frames per thread of the
gather kernel, BUGSEG_BEV_FG = frames per workgroup of the LDS-staged kernel; both read per call) at
the bench shard (32 frames of 480x640, the bench's class maps), HIP-event time per launch (a graph of
`reps` launches replayed: eager back-to-back calls are host-bound), and a
check that every form gives the same grids.

usage: python scripts/bev_sweep.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bugcar_image_segmentation_amd import _native as N  # noqa: E402
from bugcar_image_segmentation_amd import enet_spec, synthetic  # noqa: E402
from bugcar_image_segmentation_amd.models import ENET  # noqa: E402

B, H, W = 32, 480, 640
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
model = ENET(weights=enet_spec.build_enet(), precision="fp16")
bev = synthetic.synthetic_bev(H, W)
grid = (synthetic.GRID_W_M, synthetic.GRID_H_M, synthetic.CELL_M)
frames = torch.from_numpy(synthetic.uniform_frames(B, H, W)).cuda()
seg = torch.empty((B, H, W), dtype=torch.uint8, device="cuda")
model.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS3_U8, seg)
print("class histogram", torch.bincount(seg.flatten().long(), minlength=3).tolist())
ref = None
for f, fg in [(None, None), ("FB2", None), ("1", None), ("2", None), ("1", "4"), (None, None), ("FB2", None), ("1", None)]:
    os.environ.pop("BUGSEG_BEV_FB", None)
    if f == "FB2":
        os.environ["BUGSEG_BEV_FB"] = "2"
        f = None
    if f is None:
        os.environ.pop("BUGSEG_BEV_F", None)      # the default: the band-staged kernel
    else:
        os.environ["BUGSEG_BEV_F"] = f
    if fg is None:
        os.environ.pop("BUGSEG_BEV_FG", None)
    else:
        os.environ["BUGSEG_BEV_FG"] = fg
    for ls in (False, True):
        bev.laserscan_like_occupancy_grid = ls
        g = bev.create_occupancy_grid_device(seg, *grid)
        torch.cuda.synchronize()
        # timed as a replayed graph of `reps` calls: back-to-back eager calls are bound by the host's
        # per-call work (~20 us), not by the kernel
        graph = torch.cuda.CUDAGraph()
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
        if not ls:
            if ref is None:
                ref = g.clone()
            same = bool(torch.equal(ref, g))
        print(f"F={f} FG={fg} FB={os.environ.get('BUGSEG_BEV_FB', 'default')} laserscan={ls}: {ev[0].elapsed_time(ev[1]) / reps * 1000:8.1f} us per {B} frames"
              + ("" if ls else f"  same grids: {same}"), flush=True)
bev.laserscan_like_occupancy_grid = False
