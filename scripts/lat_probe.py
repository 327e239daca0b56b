import sys, torch, json
sys.path.insert(0, '.')
from bugcar_image_segmentation_amd import _native as N, enet_spec, synthetic
from bugcar_image_segmentation_amd.models import ENET
m = ENET(weights=enet_spec.build_enet(), precision="fp16")
for B in (1, 2, 4, 32):
    fr = torch.from_numpy(synthetic.uniform_frames(B, 480, 640)).cuda()
    seg = torch.empty((B, 480, 640), dtype=torch.uint8, device="cuda")
    tags = [m.ctx.plan_op(B, 480, 640, i)[0] for i in range(m.ctx.plan_info(B, 480, 640, 2)[0])]
    for _ in range(5): m.ctx.forward_bgr(fr, B, 480, 640, N.OUT_CLASS3_U8, seg)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(50): m.ctx.forward_bgr(fr, B, 480, 640, N.OUT_CLASS3_U8, seg)
    e[1].record(); e[1].synchronize()
    print(B, f"{e[0].elapsed_time(e[1]) / 50:.4f} ms/forward", sorted(set(t for t in tags if 'bneck' in t)), flush=True)
