"""Debug: in-kernel phase clocks of the BEV band kernel (libbugseg_stamps.so, -DBUGSEG_STAMPS).

One 32-frame call on the bench class maps with the stamp buffer armed; per workgroup (one work item of
one frame) the constant 100 MHz clock at: entry, box staged (barrier), pass 1 done (barrier), pass 2
done, grid stores issued. Prints the launch span, the spread of entry / exit times (dispatch ramp,
tail) and per-phase percentiles, near vs far bands.

usage: python scripts/bev_stamp_probe.py   (build: python -m bugcar_image_segmentation_amd.build --stamps)"""
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

B, H, W = 32, 480, 640
lib = N.load_library()
lib.bugseg_debug_set_bev_stamps.argtypes = [ctypes.c_void_p]
model = ENET(weights=enet_spec.build_enet(), precision="fp16")
bev = synthetic.synthetic_bev(H, W)
grid = (synthetic.GRID_W_M, synthetic.GRID_H_M, synthetic.CELL_M)
frames = torch.from_numpy(synthetic.uniform_frames(B, H, W)).cuda()
seg = torch.empty((B, H, W), dtype=torch.uint8, device="cuda")
model.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS3_U8, seg)
g = bev.create_occupancy_grid_device(seg, *grid)
torch.cuda.synchronize()
st = torch.zeros(1 << 16, dtype=torch.int64, device="cuda")
for rep in range(3):
    st.zero_()
    assert lib.bugseg_debug_set_bev_stamps(ctypes.c_void_p(st.data_ptr())) == 0
    bev.create_occupancy_grid_device(seg, *grid, out=g)
    torch.cuda.synchronize()
    assert lib.bugseg_debug_set_bev_stamps(ctypes.c_void_p(0)) == 0
    s = st.cpu().numpy().reshape(-1, 8)
    s = s[s[:, 0] > 0]
    t = s[:, :5].astype(np.float64)
    t0 = t[:, 0].min()
    us = (t - t0) / 100.0                        # 100 MHz -> us
    info = s[:, 6]
    nw, band, n = info & 0xffff, (info >> 16) & 0xffff, info >> 32
    span = us[:, 4].max()
    print(f"rep {rep}: {len(s)} workgroups, span {span:.1f} us (entry .. last stores issued)")
    pct = lambda x: " ".join(f"{np.percentile(x, q):6.2f}" for q in (5, 50, 95, 100))  # noqa: E731
    print("  entry time         p5/p50/p95/max:", pct(us[:, 0]))
    print("  exit time          p5/p50/p95/max:", pct(us[:, 4]))
    for name, a_, b_ in (("staging", 0, 1), ("pass 1", 1, 2), ("pass 2", 2, 3), ("stores", 3, 4), ("whole", 0, 4)):
        d = us[:, b_] - us[:, a_]
        print(f"  {name:8s} duration  p5/p50/p95/max:", pct(d))
    nb = band.max() + 1
    for lo, hi, name in ((0, nb // 2, "far half"), (nb // 2, nb - 4, "near"), (nb - 4, nb, "nearest 4")):
        m = (band >= lo) & (band < hi)
        if m.any():
            print(f"  {name:10s} bands: {m.sum():4d} wgs, whole p50 {np.median(us[m, 4] - us[m, 0]):.2f} us, "
                  f"work list p50 {np.median(nw[m]):.0f} of cells p50 {np.median(n[m]):.0f}, exit p95 {np.percentile(us[m, 4], 95):.2f}")
