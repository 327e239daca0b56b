"""Parity at the configuration bench.py times: 64 frames of 480x640 per GPU,
split by OccupancyPipeline into 2 shards of 32 frames on 2 streams (each shard its own context), in
the 2-byte storage modes. At B = 32 the runtime picks its large-batch bottleneck tiles and the
multi-tile workgroup walks, so this is what these checks exercise.

For frames taken from BOTH shards, the logits come from the same shard context at B = 32 and are
compared with the oracle's storage emulation (oracle/enet_oracle.py forward_storage: BN-folded
weights and every stored activation rounded to the mode's type, f32 products). Bounds: fp16 — mean
|dlogit| < 5e-3, class agreement >= 0.995 (as tests/test_gpu_parity.py); bf16 — mean < 6e-2, agreement
>= 0.97. Two emulations that differ ONLY in accumulation order (f32 vs f64 sums, same storage
rounding) already differ by mean 1.3e-2 / agree 0.9936 (bf16) and 3.9e-3 / 0.9981 (fp16) on frame 0
(scripts/storage_spread.py): bf16's 8-bit mantissa turns last-bit differences of a sum into
rounding flips that the 29 layers amplify. The pipeline's own class maps must be the LUT of those logits' argmax (exact),
and its grids the C restatement's rasteriser on those class maps (bit-exact). Reference:
models.py:43-58 (sess.run + argmax + remap), bev.py:166-246.
"""
import numpy as np
import pytest
import torch

from bugcar_image_segmentation_amd import _native as N
from bugcar_image_segmentation_amd import synthetic
from bugcar_image_segmentation_amd.models import ENET
from bugcar_image_segmentation_amd.pipeline import OccupancyPipeline
from oracle import enet_oracle as eo
from oracle import ocv_c

pytestmark = pytest.mark.gpu

BOUNDS = {"fp16": (torch.float16, 5e-3, 0.995), "bf16": (torch.bfloat16, 6e-2, 0.97)}


@pytest.mark.parametrize("prec", ["fp16", "bf16"])
def test_timed_configuration_vs_storage_oracle(gpu, blocks, prec):
    dtype, mean_tol, agree_tol = BOUNDS[prec]
    H, W, B, S = 480, 640, 64, 2
    model = ENET(weights=blocks, precision=prec)
    bev = synthetic.synthetic_bev(H, W)
    grid = (synthetic.GRID_W_M, synthetic.GRID_H_M, synthetic.CELL_M)
    pipe = OccupancyPipeline(model, bev, *grid, model_hw=(H, W), streams=S)
    frames = torch.from_numpy(synthetic.uniform_frames(B, H, W, seed=0)).to(gpu)   # bench.py's rank-0 frames
    grids = pipe.run(frames).clone()
    torch.cuda.synchronize()
    seg = pipe._seg.clone()
    assert len(pipe._ctxs) == S
    Bs = B // S
    picks = {0: (0, 17, 31), 1: (32, 45, 63)}            # frames of both shards, first / middle / last
    lut3 = torch.tensor(eo.LUT3, device=gpu)
    worst = []
    for shard, ctx in enumerate(pipe._ctxs):
        s = shard * Bs
        logits = torch.empty((Bs, model.num_classes, H, W), dtype=torch.float32, device=gpu)
        ctx.forward_bgr(frames[s:s + Bs], Bs, H, W, N.OUT_LOGITS_F32, logits)   # same context, B = 32
        torch.cuda.synchronize()
        # the timed step's class maps are exactly the remap of these logits' argmax (models.py:55-58)
        assert torch.equal(seg[s:s + Bs], lut3[logits.argmax(1)].to(torch.uint8))
        for i in picks[shard]:
            x = ENET.preprocess_device(frames[i].cpu().numpy(), width=W, height=H).cpu().numpy().astype(np.float32)
            emu = eo.forward_storage(blocks, x, dtype)[0]
            got = logits[i - s].cpu().numpy()
            d = np.abs(got - emu)
            agree = float((got.argmax(0) == emu.argmax(0)).mean())
            print(f"{prec} frame {i} (shard {shard}): mean|d| {d.mean():.2e} max|d| {d.max():.3f} "
                  f"class agreement with the {prec}-storage oracle {agree:.5f}")
            assert np.isfinite(got).all()
            assert d.mean() < mean_tol
            assert agree >= agree_tol
            worst.append(agree)
    # the grids of the timed step: the oracle's rasteriser on the step's own class maps, bit-exact
    seg_np = seg.cpu().numpy()
    g_np = grids.cpu().numpy()
    for i in (0, 31, 32, 63):
        want = ocv_c.create_occupancy_grid(seg_np[i], bev._bev_matrix, bev.after_warp_width, bev.after_warp_height,
                                           bev.cm_per_px, *grid)
        assert np.array_equal(g_np[i], want), i
    print(f"{prec}: worst per-frame agreement {min(worst):.5f}")
