"""Debug: a few single-stream bench-workload forwards (B = 32) to run under rocprofv3 (--kernel-trace
or --pmc; scripts/gpu_sqpmc.sh, scripts/gpu_layers.sh). The argument list is kept for the earlier
in-kernel ablation runs (round-1 record in DESIGN.md); the ablation hooks are gone from the kernel,
so every argument now runs the same baseline."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bugcar_image_segmentation_amd import _native as N  # noqa: E402
from bugcar_image_segmentation_amd import enet_spec, synthetic  # noqa: E402
from bugcar_image_segmentation_amd.models import ENET  # noqa: E402

B, H, W = int(os.environ.get("BUGSEG_B", "32")), 480, 640
blocks = enet_spec.build_enet()
frames = torch.from_numpy(synthetic.uniform_frames(B, H, W)).cuda()
seg = torch.empty((B, H, W), dtype=torch.uint8, device="cuda")
for flags in [int(v) for v in (sys.argv[1:] or ["0", "1", "2", "4", "7"])]:
    os.environ["BUGSEG_BNECK_ABLATE"] = str(flags)
    m = ENET(weights=blocks, precision=os.environ.get("BUGSEG_PREC", "fp16"))
    for _ in range(4):
        m.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS3_U8, seg)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(5):
        m.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS3_U8, seg)
    ev[1].record()
    ev[1].synchronize()
    print(f"ablate={flags}: forward {ev[0].elapsed_time(ev[1]) / 5:.3f} ms", flush=True)
    del m
