"""GPU parity: every kernel through the C ABI against the CPU oracle (oracle/), same seeded inputs.

Tolerances (written here, as north_star states them): fp32 mode — logits within 1e-3 absolute of
the fp32 oracle, class maps exact on every pixel whose oracle top-2 logit margin exceeds 2.5x this
run's measured max |logit error| (floor 1e-5; with every logit within e of the oracle, a margin
above 2e is provably decided identically — 2.5e leaves room for the margin's own f32 rounding — so
only true near-ties are excused; their count is printed and bounded); bf16 / fp16 modes — against the oracle with the same storage numerics, agreement rate
reported and bounded. Integer / byte paths (preprocess, BEV rasteriser) bit-exact.
"""
import os
from pathlib import Path

import numpy as np
import pytest
import torch

from bugcar_image_segmentation_amd import _native as N
from bugcar_image_segmentation_amd import enet_spec, synthetic
from bugcar_image_segmentation_amd.bev import bev_transform_tools
from bugcar_image_segmentation_amd.models import ENET
from bugcar_image_segmentation_amd.pipeline import OccupancyPipeline
from oracle import enet_oracle as eo
from oracle import ocv_c, ocv_np

pytestmark = pytest.mark.gpu

LOGIT_TOL = 1e-3


def _margin(logits):
    s = np.sort(logits, axis=1)
    return s[:, -1] - s[:, -2]


def _decided(ref, got, max_excused=1e-3, what=""):
    """Mask of the pixels whose oracle top-2 margin exceeds 2.5 x max|got - ref| (floor 1e-5): the
    pixels on which class equality is asserted. Prints and bounds the excused (near-tie) share."""
    err = float(np.abs(got - ref).max())
    thr = max(2.5 * err, 1e-5)
    dec = _margin(ref) > thr
    n_exc = int(dec.size - dec.sum())
    print(f"{what} max|dlogit| {err:.2e}; margin threshold {thr:.2e}; excused {n_exc} of {dec.size} pixels "
          f"({n_exc / dec.size:.2e})")
    assert n_exc / dec.size <= max_excused
    return dec


@pytest.fixture(scope="module")
def fp32_model(gpu, blocks):
    return ENET(weights=blocks, precision="fp32")


@pytest.fixture(scope="module")
def bf16_model(gpu, blocks):
    return ENET(weights=blocks, precision="bf16")


@pytest.mark.parametrize("B,H,W", [(1, 32, 48), (2, 64, 96), (1, 120, 160)])
def test_enet_fp32_logits_and_classes(fp32_model, blocks, B, H, W):
    x = np.random.default_rng(B * 1000 + H).normal(size=(B, 3, H, W)).astype(np.float32)
    ref = eo.forward(blocks, x)
    got = fp32_model.logits(x)
    assert got.shape == ref.shape and got.dtype == np.float32
    assert np.abs(got - ref).max() < LOGIT_TOL
    decided = _decided(ref, got, what=f"fp32 {B}x{H}x{W}")
    cls_ref = eo.argmax_classes(ref)
    raw = fp32_model.predict_device(fp32_model.engine_input(x), N.OUT_CLASS15_U8).cpu().numpy()
    assert (raw[decided] == cls_ref[decided]).all()
    p3 = fp32_model.predict(x)
    assert p3.dtype == np.uint8 and p3.shape == (B, H, W)
    assert (p3[decided] == eo.LUT3[cls_ref][decided]).all()
    pb = fp32_model.predict_binary(x)
    assert (pb[decided] == eo.LUT_BINARY[cls_ref][decided]).all()


def test_enet_fp32_model_resolution(fp32_model, blocks):
    """configs[1] shape (480x640) through the fp32 parity mode, one frame."""
    x = np.random.default_rng(7).normal(size=(1, 3, 480, 640)).astype(np.float32)
    ref = eo.forward(blocks, x)
    got = fp32_model.logits(x)
    assert np.abs(got - ref).max() < LOGIT_TOL
    decided = _decided(ref, got, max_excused=1e-4, what="fp32 480x640")
    assert (got.argmax(1)[decided] == eo.argmax_classes(ref)[decided]).all()
    assert (fp32_model.predict(x)[decided] == eo.LUT3[eo.argmax_classes(ref)][decided]).all()


def test_enet_bf16_vs_bf16_storage_oracle(bf16_model, blocks):
    """bf16 mode against the oracle with the SAME storage numerics (BN-folded bf16 weights, bf16
    activations, fp32 accumulate/epilogue): only accumulation order differs. Agreement with the
    fp32 oracle is inherent to bf16 storage (the CPU emulation alone agrees ~95% on this untrained
    network) and is reported, not asserted tight."""
    x = np.random.default_rng(11).normal(size=(2, 3, 96, 128)).astype(np.float32)
    emu = eo.forward_bf16_storage(blocks, x)
    ref = eo.forward(blocks, x)
    got = bf16_model.logits(x)
    d = np.abs(got - emu)
    agree_emu = (np.argmax(got, 1) == np.argmax(emu, 1)).mean()
    agree_f32 = (np.argmax(got, 1) == eo.argmax_classes(ref)).mean()
    print(f"bf16 vs bf16-storage oracle: mean|d| {d.mean():.2e} max|d| {d.max():.3f} class agree {agree_emu:.5f}; "
          f"vs fp32 oracle class agree {agree_f32:.5f}")
    assert d.mean() < 2e-2
    assert agree_emu > 0.99


def test_enet_fp16_vs_fp16_storage_oracle(gpu, blocks):
    """fp16 mode against the oracle with the same storage numerics (forward_storage, float16): only
    accumulation order differs, so it tracks its emulation as bf16 does; and its class agreement
    with the fp32 oracle is far closer than bf16's (3 more mantissa bits), which is the point of the
    mode: asserted > 97% here on these untrained weights (bf16's is ~91%)."""
    import torch as _t
    m = ENET(weights=blocks, precision="fp16")
    x = np.random.default_rng(11).normal(size=(2, 3, 96, 128)).astype(np.float32)
    emu = eo.forward_storage(blocks, x, _t.float16)
    ref = eo.forward(blocks, x)
    got = m.logits(x)
    assert np.isfinite(got).all()
    d = np.abs(got - emu)
    agree_emu = (np.argmax(got, 1) == np.argmax(emu, 1)).mean()
    agree_f32 = (np.argmax(got, 1) == eo.argmax_classes(ref)).mean()
    print(f"fp16 vs fp16-storage oracle: mean|d| {d.mean():.2e} max|d| {d.max():.3f} class agree {agree_emu:.5f}; "
          f"vs fp32 oracle class agree {agree_f32:.5f}")
    assert d.mean() < 5e-3
    assert agree_emu > 0.995
    assert agree_f32 > 0.97


def test_fullconv_k2_and_pool2_variants(gpu):
    """Topology is data: the 2x2 final deconv / 2x2 initial pool variants of ENet."""
    bl = enet_spec.build_enet(seed=5, fullconv_k=2, initial_pool_k=2)
    m = ENET(weights=bl, precision="fp32")
    x = np.random.default_rng(3).normal(size=(1, 3, 64, 64)).astype(np.float32)
    ref = eo.forward(bl, x)
    assert np.abs(m.logits(x) - ref).max() < LOGIT_TOL


@pytest.mark.parametrize("ncls", [3, 16])
def test_class_counts(gpu, ncls):
    """The class layer at other class counts (the kernel masks padding classes): 3 (the reference's
    road / obstacle / background head) and 16 (no padding), fp32 against the oracle."""
    bl = enet_spec.build_enet(seed=20 + ncls, num_classes=ncls)
    m = ENET(weights=bl, precision="fp32")
    assert m.num_classes == ncls
    x = np.random.default_rng(ncls).normal(size=(1, 3, 64, 96)).astype(np.float32)
    ref = eo.forward(bl, x)
    got = m.logits(x)
    assert got.shape == ref.shape == (1, ncls, 64, 96)
    assert np.abs(got - ref).max() < LOGIT_TOL
    decided = _decided(ref, got, what=f"fp32 {ncls} classes")
    raw = m.predict_device(m.engine_input(x), N.OUT_CLASS15_U8).cpu().numpy()
    assert (raw[decided] == eo.argmax_classes(ref)[decided]).all()


@pytest.mark.parametrize("shape,dsize", [((512, 512), (512, 256)), ((480, 640), (512, 256)),
                                         ((256, 512), (512, 256)), ((100, 130), (64, 48)),
                                         ((512, 1024), (512, 256)), ((37, 41), (96, 80))])
def test_preprocess_bit_exact(gpu, shape, dsize):
    bgr = np.random.default_rng(shape[0]).integers(0, 256, size=shape + (3,), dtype=np.uint8)
    ref = eo.preprocess(bgr, *dsize)
    got = ENET.preprocess_device(bgr, width=dsize[0], height=dsize[1]).cpu().numpy()
    assert got.dtype == np.float64 and got.shape == ref.shape == (1, 3, dsize[1], dsize[0])
    assert np.array_equal(got, ref)
    f32 = ENET.preprocess_device(bgr, N.PRE_NCHW_F32, width=dsize[0], height=dsize[1]).cpu().numpy()
    assert np.array_equal(f32, ref.astype(np.float32))


def test_preprocess_classmethod_reference_api(gpu):
    bgr = np.random.default_rng(2).integers(0, 256, size=(512, 512, 3), dtype=np.uint8)
    out = ENET.preprocess(bgr)
    assert out.shape == (1, 3, 256, 512) and out.dtype == np.float64
    assert np.array_equal(out, eo.preprocess(bgr))


def _bev_case(rows, cols, ww, wh, seed):
    rng = np.random.default_rng(seed)
    bev = synthetic.synthetic_bev(rows, cols, ww, wh)
    M = bev._bev_matrix @ np.array([[1 + 0.05 * rng.normal(), 0.02 * rng.normal(), rng.normal() * 5],
                                    [0.02 * rng.normal(), 1 + 0.05 * rng.normal(), rng.normal() * 5],
                                    [1e-5 * rng.normal(), 1e-5 * rng.normal(), 1.0]])
    bev._bev_matrix = M
    return bev


@pytest.mark.parametrize("form", [None, "NEAR", "FB2", "G", "FG4", "F2"])
@pytest.mark.parametrize("rows,cols,ww,wh,grid,seed", [
    (480, 640, 1000, 1000, (10.0, 10.0, 0.05), 0),
    (120, 160, 300, 260, (3.0, 2.0, 0.05), 1),
    (96, 128, 250, 180, (3.1, 2.7, 0.07), 2),     # template wider than the warp (negative left_x/top_y)
    (64, 80, 200, 150, (1.0, 1.0, 0.1), 3),
])
def test_bev_occgrid_bit_exact(gpu, rows, cols, ww, wh, grid, seed, form, monkeypatch):
    """Every form of the rasteriser (bev_kernels.hip: the default band-staged kernel, 2 frames per
    band workgroup, the gather kernel, the block-staged one, 2 frames per thread; NEAR: the band
    kernel's work items nearest band first, the earlier order, if this context builds the table) is bit-exact against
    the C restatement; class maps with labels past the 3-class range (up to 255: segmap + 1 wraps in
    uint8 as np.add does, bev.py:177) included."""
    if form == "G":
        monkeypatch.setenv("BUGSEG_BEV_BAND", "0")
    elif form == "FB2":
        monkeypatch.setenv("BUGSEG_BEV_FB", "2")
    elif form == "FG4":
        monkeypatch.setenv("BUGSEG_BEV_FG", "4")
    elif form == "F2":
        monkeypatch.setenv("BUGSEG_BEV_F", "2")
    elif form == "NEAR":
        monkeypatch.setenv("BUGSEG_BEV_NEAR_FIRST", "1")
    bev = _bev_case(rows, cols, ww, wh, seed)
    rng = np.random.default_rng(seed)
    # blocky class maps (realistic regions + speckles) and pure noise
    blocky = np.kron(rng.integers(0, 3, size=(rows // 8, cols // 8)), np.ones((8, 8), np.int64)).astype(np.uint8)
    noise = rng.integers(0, 3, size=(rows, cols)).astype(np.uint8)
    wide = rng.integers(0, 256, size=(rows, cols)).astype(np.uint8)
    # 3-class noise with sparse outliers (7, 255): some band boxes take the 2-bit quad form, some not
    sparse = noise.copy()
    pick = rng.random((rows, cols))
    sparse[pick < 0.002] = 7
    sparse[(pick >= 0.002) & (pick < 0.004)] = 255
    segs = np.stack([blocky, noise, wide, sparse])
    ref = np.stack([ocv_c.create_occupancy_grid(s, bev._bev_matrix, ww, wh, 1.0, *grid) for s in segs])
    got = bev.create_occupancy_grid_device(torch.from_numpy(segs).cuda(), *grid).cpu().numpy()
    assert got.dtype == np.int8 and got.shape == ref.shape
    assert np.array_equal(got, ref)
    ros = bev.create_occupancy_grid_device(torch.from_numpy(segs).cuda(), *grid, ros_layout=True).cpu().numpy()
    assert np.array_equal(ros, np.stack([ocv_np.ros_layout(r) for r in ref]))
    # reference API, one frame, numpy in/out
    one = bev.create_occupancy_grid(blocky, *grid)
    assert one.dtype == np.int8 and np.array_equal(one, ref[0])


@pytest.mark.parametrize("rows,cols,ww,wh,grid,seed", [
    (480, 640, 1000, 1000, (10.0, 10.0, 0.05), 4),
    (96, 128, 250, 180, (3.1, 2.7, 0.07), 5),
])
def test_bev_occgrid_binary_bit_exact(gpu, rows, cols, ww, wh, grid, seed):
    """create_occupancy_grid_binary (bev.py:97-165) vs its C restatement: predict_binary maps ({0,1})
    and 3-class maps (the reference's uint8 encoding turns class 2 into -100)."""
    bev = _bev_case(rows, cols, ww, wh, seed)
    rng = np.random.default_rng(seed)
    segs = np.stack([np.kron(rng.integers(0, k, size=(rows // 8, cols // 8)), np.ones((8, 8), np.int64)).astype(np.uint8)
                     for k in (2, 3)] + [rng.integers(0, 2, size=(rows, cols)).astype(np.uint8)])
    ref = np.stack([ocv_c.create_occupancy_grid_binary(s, bev._bev_matrix, ww, wh, 1.0, *grid) for s in segs])
    got = bev.create_occupancy_grid_device(torch.from_numpy(segs).cuda(), *grid, binary=True).cpu().numpy()
    assert np.array_equal(got, ref)
    one = bev.create_occupancy_grid_binary(segs[0], *grid)
    assert one.dtype == np.int8 and np.array_equal(one, ref[0])


@pytest.mark.parametrize("rows,cols,ww,wh,grid,seed", [
    (480, 640, 1000, 1000, (10.0, 10.0, 0.05), 6),
    (120, 160, 300, 260, (3.0, 2.0, 0.05), 7),       # wide grid: the polar radius follows the width
    (96, 128, 250, 180, (3.1, 2.7, 0.07), 8),        # odd grid width: half-pixel polar centre
    (64, 80, 200, 150, (1.0, 1.6, 0.1), 9),          # tall grid
])
def test_bev_laserscan_bit_exact(gpu, rows, cols, ww, wh, grid, seed):
    """Laserscan-like mode (bev.py:216-240; binary variant bev.py:143-164) vs the C restatement: the
    per-ray nearest obstacle, the stamped pluses and the re-projection, batched, in both layouts."""
    bev = _bev_case(rows, cols, ww, wh, seed)
    bev.laserscan_like_occupancy_grid = True
    rng = np.random.default_rng(seed)
    blocky = np.kron(rng.integers(0, 3, size=(rows // 8, cols // 8)), np.ones((8, 8), np.int64)).astype(np.uint8)
    sparse = np.ones((rows, cols), np.uint8)
    sparse[rng.random((rows, cols)) < 0.05] = 2
    none = np.ones((rows, cols), np.uint8)           # no obstacle on any ray
    segs = np.stack([blocky, sparse, none, rng.integers(0, 3, size=(rows, cols)).astype(np.uint8)])
    M = bev._bev_matrix
    ref = np.stack([ocv_c.create_occupancy_grid_laserscan(s, M, ww, wh, 1.0, *grid) for s in segs])
    dev = torch.from_numpy(segs).cuda()
    got = bev.create_occupancy_grid_device(dev, *grid).cpu().numpy()
    assert np.array_equal(got, ref)
    ros = bev.create_occupancy_grid_device(dev, *grid, ros_layout=True).cpu().numpy()
    assert np.array_equal(ros, np.stack([ocv_np.ros_layout(r) for r in ref]))
    assert np.array_equal(bev.create_occupancy_grid(blocky, *grid), ref[0])
    # binary variant: the reference's returned pair
    bref = [ocv_c.create_occupancy_grid_binary_laserscan(s, M, ww, wh, 1.0, *grid) for s in segs]
    bgot = bev.create_occupancy_grid_device(dev, *grid, binary=True).cpu().numpy()
    assert bgot.shape[0] == 2
    assert np.array_equal(bgot[0], np.stack([r[0] for r in bref]))
    assert np.array_equal(bgot[1], np.stack([r[1] for r in bref]))
    g, n = bev.create_occupancy_grid_binary(segs[1], *grid)
    assert np.array_equal(g, bref[1][0]) and np.array_equal(n, bref[1][1])
    # a non-laserscan call on the same context after the laserscan ones is unaffected
    bev.laserscan_like_occupancy_grid = False
    assert np.array_equal(bev.create_occupancy_grid(blocky, *grid),
                          ocv_c.create_occupancy_grid(blocky, M, ww, wh, 1.0, *grid))


@pytest.mark.parametrize("prec", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("pool_k", [3, 2])
def test_forward_bgr_equals_preprocess_then_forward(gpu, prec, pool_k):
    """The fused-preprocess entry (raw BGR into the initial block) is bit-identical to
    preprocess(ENGINE) + forward, including the maxpool channels (pool over raw bytes)."""
    bl = enet_spec.build_enet(seed=17, initial_pool_k=pool_k)
    m = ENET(weights=bl, precision=prec)
    B, H, W = 2, 64, 96
    bgr = torch.from_numpy(synthetic.road_frames(B, H, W, seed=4)).cuda()
    x = ENET.preprocess_device(bgr, N.PRE_ENGINE, ctx=m.ctx, width=W, height=H)
    a = m.predict_device(x, N.OUT_LOGITS_F32)
    b = torch.empty_like(a)
    m.ctx.forward_bgr(bgr, B, H, W, N.OUT_LOGITS_F32, b)
    assert torch.equal(a, b)
    # resize-only preprocess + fused forward == full preprocess + forward
    big = torch.from_numpy(synthetic.road_frames(B, 100, 150, seed=5)).cuda()
    x2 = ENET.preprocess_device(big, N.PRE_ENGINE, ctx=m.ctx, width=W, height=H)
    r = torch.empty((B, H, W, 3), dtype=torch.uint8, device=gpu)
    m.ctx.preprocess(big, B, 100, 150, H, W, N.PRE_BGR_U8, r)
    c = torch.empty_like(a)
    m.ctx.forward_bgr(r, B, H, W, N.OUT_LOGITS_F32, c)
    assert torch.equal(m.predict_device(x2, N.OUT_LOGITS_F32), c)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_init_affine_normalisation_equals_table(gpu, blocks, prec, monkeypatch):
    """bf16 / fp16: the fused initial block normalises each byte as one fmaf with per-channel constants
    the context found exact on the device (bugseg_runtime.cpp, init_kernels.hip naff_search_kernel);
    the table form (BUGSEG_INIT_TABLE=1) gives the same logits bit for bit, at the bench shape."""
    B, H, W = 2, 480, 640
    bgr = torch.from_numpy(synthetic.uniform_frames(B, H, W)).cuda()
    m = ENET(weights=blocks, precision=prec)
    # the device search found exact constants for every channel, so the fmaf form really runs (ADVICE r4:
    # otherwise both runs would use the table and this test would compare the table with itself)
    assert m.ctx.debug_info(0) == 1
    a = torch.empty((B, 15, H, W), dtype=torch.float32, device=gpu)
    m.ctx.forward_bgr(bgr, B, H, W, N.OUT_LOGITS_F32, a)
    monkeypatch.setenv("BUGSEG_INIT_TABLE", "1")
    b = torch.empty_like(a)
    m.ctx.forward_bgr(bgr, B, H, W, N.OUT_LOGITS_F32, b)
    assert torch.equal(a, b)


@pytest.mark.parametrize("pool_k", [3, 2])
def test_init_packed_pool_equals_scan(gpu, pool_k, monkeypatch):
    """fp16: the initial block's pool maxima as packed f16 pairs from 5-dword window rows
    (init_kernels.hip) equal the per-tap scan (BUGSEG_INIT_POOL_SCAN=1) bit for bit — frame edges (the
    excluded -inf taps) and pool_k 2's window included, raw-BGR and engine-input entries alike."""
    bl = enet_spec.build_enet(seed=19, initial_pool_k=pool_k)
    m = ENET(weights=bl, precision="fp16")
    B, H, W = 2, 72, 104
    bgr = torch.from_numpy(synthetic.road_frames(B, H, W, seed=9)).cuda()
    x = ENET.preprocess_device(bgr, N.PRE_ENGINE, ctx=m.ctx, width=W, height=H)
    outs = []
    for scan in (False, True):
        if scan:
            monkeypatch.setenv("BUGSEG_INIT_POOL_SCAN", "1")
        a = torch.empty((B, 15, H, W), dtype=torch.float32, device=gpu)
        m.ctx.forward_bgr(bgr, B, H, W, N.OUT_LOGITS_F32, a)
        outs.append((a, m.predict_device(x, N.OUT_LOGITS_F32)))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("variant", [None, "0", "1", "2", "3", "4"])
@pytest.mark.parametrize("prec", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("H,W", [(64, 96), (72, 104), (120, 160), (480, 640)])
def test_fused_bottlenecks_equal_unfused(gpu, blocks, prec, H, W, variant, monkeypatch):
    """The fused bottleneck kernel (projection + middle conv + expansion + residual, internals in
    LDS) rounds the internal tensors exactly as the unfused conv chain stores them: bit-identical.
    `variant` forces one tile shape for every fused layer (bypassing the efficiency rule, so the
    d = 8 / 16 blocks run fused through the dilated tiling too); None = the runtime's choice."""
    B = 2 if H < 480 else 1
    bgr = torch.from_numpy(synthetic.road_frames(B, H, W, seed=H)).cuda()
    if variant is not None:
        monkeypatch.setenv("BUGSEG_BNECK_VARIANT", variant)
    fused = ENET(weights=blocks, precision=prec)
    a = torch.empty((B, 15, H, W), dtype=torch.float32, device=gpu)
    fused.ctx.forward_bgr(bgr, B, H, W, N.OUT_LOGITS_F32, a)
    monkeypatch.delenv("BUGSEG_BNECK_VARIANT", raising=False)
    monkeypatch.setenv("BUGSEG_NO_FUSE", "1")
    plain = ENET(weights=blocks, precision=prec)
    b = torch.empty_like(a)
    plain.ctx.forward_bgr(bgr, B, H, W, N.OUT_LOGITS_F32, b)
    n_fused = fused.ctx.plan_info(B, H, W, N.OUT_LOGITS_F32)[0]
    n_plain = plain.ctx.plan_info(B, H, W, N.OUT_LOGITS_F32)[0]
    assert n_plain == 88 and n_fused < n_plain      # 89 convolutions; the up5 main + extension 1x1 pair is one launch
    # (BUGSEG_NO_FUSE also turns off the fused upsampling blocks: this compares them too)
    assert torch.equal(a, b)


@pytest.mark.parametrize("H,W", [(72, 104), (120, 160), (480, 640)])
def test_bneck2_two_tile_form_equals_unfused(gpu, blocks, H, W, monkeypatch):
    """The fp32 C128 two-phase-shifted-tiles kernel (bneck2_kernels.hip, BUGSEG_BNECK2=1; measured slower
    and off by default) is bit-identical to the unfused chain: same products, same order."""
    B = 2
    bgr = torch.from_numpy(synthetic.road_frames(B, H, W, seed=H + 1)).cuda()
    monkeypatch.setenv("BUGSEG_BNECK2", "1")
    monkeypatch.setenv("BUGSEG_BNECK_VARIANT_C128", "5")     # every symmetric C128 layer, any efficiency
    fused = ENET(weights=blocks, precision="fp32")
    a = torch.empty((B, 15, H, W), dtype=torch.float32, device=gpu)
    fused.ctx.forward_bgr(bgr, B, H, W, N.OUT_LOGITS_F32, a)
    n = fused.ctx.plan_info(B, H, W, N.OUT_LOGITS_F32)[0]
    tags = [fused.ctx.plan_op(B, H, W, i)[0] for i in range(n)]
    assert any(t.startswith("bneck2") for t in tags), tags
    monkeypatch.delenv("BUGSEG_BNECK2")
    monkeypatch.delenv("BUGSEG_BNECK_VARIANT_C128")
    monkeypatch.setenv("BUGSEG_NO_FUSE", "1")
    plain = ENET(weights=blocks, precision="fp32")
    b = torch.empty_like(a)
    plain.ctx.forward_bgr(bgr, B, H, W, N.OUT_LOGITS_F32, b)
    assert torch.equal(a, b)


@pytest.mark.parametrize("grid", ["8", "-2"])
@pytest.mark.parametrize("variant", [None, "0", "2", "4"])
@pytest.mark.parametrize("prec", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("H,W", [(72, 104), (480, 640)])
def test_fused_bottlenecks_multi_tile_walks(gpu, blocks, prec, H, W, variant, grid, monkeypatch):
    """Every fused bottleneck launch on a small grid (BUGSEG_BNECK_GRID: 8 workgroups, or half the
    resident slots), so each workgroup walks several tiles: bit-identical to the unfused chain."""
    B = 2
    bgr = torch.from_numpy(synthetic.road_frames(B, H, W, seed=H + 1)).cuda()
    if variant is not None:
        monkeypatch.setenv("BUGSEG_BNECK_VARIANT", variant)
    monkeypatch.setenv("BUGSEG_BNECK_GRID", grid)
    fused = ENET(weights=blocks, precision=prec)
    a = torch.empty((B, 15, H, W), dtype=torch.float32, device=gpu)
    fused.ctx.forward_bgr(bgr, B, H, W, N.OUT_LOGITS_F32, a)
    torch.cuda.synchronize()
    monkeypatch.delenv("BUGSEG_BNECK_VARIANT", raising=False)
    monkeypatch.delenv("BUGSEG_BNECK_GRID", raising=False)
    monkeypatch.setenv("BUGSEG_NO_FUSE", "1")
    plain = ENET(weights=blocks, precision=prec)
    b = torch.empty_like(a)
    plain.ctx.forward_bgr(bgr, B, H, W, N.OUT_LOGITS_F32, b)
    assert torch.equal(a, b)


_CLASS_KINDS = (N.OUT_CLASS15_U8, N.OUT_CLASS3_U8, N.OUT_BINARY_U8)


@pytest.mark.parametrize("grid", [None, "8"])
@pytest.mark.parametrize("prec", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("B,H,W", [(3, 72, 104), (2, 64, 96), (2, 120, 160), (1, 480, 640)])
def test_class_fusion_equals_separate_launches(gpu, blocks, prec, B, H, W, grid, monkeypatch):
    """ENet's last bottleneck and the class layer as ONE launch (class fusion, bneck_kernels.hip FC:
    tiles 15 apart, the block output in LDS) against the two launches (BUGSEG_CLS_FUSE=0): every class
    map (raw ids, the 3-class and the binary map) equal byte for byte — edge tiles included (the C16
    maps 36 x 52 / 32 x 48 are not multiples of 15), and with grid "8" every workgroup walks many tiles.
    The fused form (opt-in: BUGSEG_CLS_FUSE=1, measured slower) runs for class maps only."""
    bgr = torch.from_numpy(synthetic.road_frames(B, H, W, seed=H + 3)).cuda()
    monkeypatch.setenv("BUGSEG_CLS_FUSE", "1")
    if grid is not None:
        monkeypatch.setenv("BUGSEG_BNECK_GRID", grid)
    fused = ENET(weights=blocks, precision=prec)
    got = {}
    for kind in _CLASS_KINDS:
        seg = torch.empty((B, H, W), dtype=torch.uint8, device=gpu)
        fused.ctx.forward_bgr(bgr, B, H, W, kind, seg)
        got[kind] = seg
    n = fused.ctx.plan_info(B, H, W, N.OUT_CLASS3_U8, bgr_input=True)[0]
    tags = [fused.ctx.plan_op(B, H, W, i)[0] for i in range(n)]
    assert tags[-2] == "bneck C16+classes 16x16" and tags[-1] == "fused", tags[-3:]
    torch.cuda.synchronize()
    monkeypatch.delenv("BUGSEG_BNECK_GRID", raising=False)
    monkeypatch.setenv("BUGSEG_CLS_FUSE", "0")
    plain = ENET(weights=blocks, precision=prec)
    for kind in _CLASS_KINDS:
        ref = torch.empty((B, H, W), dtype=torch.uint8, device=gpu)
        plain.ctx.forward_bgr(bgr, B, H, W, kind, ref)
        assert plain.ctx.plan_op(B, H, W, n - 1)[0] == "classes"
        diff = int((got[kind] != ref).sum())
        assert diff == 0, f"kind {kind}: {diff} of {ref.numel()} pixels differ"


def test_class_fusion_under_range_scaling(gpu):
    """fp32 with the survey's undamped weights (activations past f16's range): the fused class phase
    scales its input by the TILE's measured max (the class kernel: the batch's), so its logits differ
    from the separate launches' in the last bits where either exponent is non-zero — the class maps
    then agree wherever the top-2 logit margin exceeds 1e-5 of the frame's max |logit|, and the fused
    map equals LUT[first argmax] of the separate launch's logits there."""
    bl = enet_spec.build_enet(res_gamma=(0.5, 1.5))
    B, H, W = 2, 240, 320
    os.environ["BUGSEG_CLS_FUSE"] = "1"
    bgr = torch.from_numpy(synthetic.road_frames(B, H, W, seed=12)).cuda()
    try:
        m = ENET(weights=bl, precision="fp32")
        lg = torch.empty((B, m.num_classes, H, W), dtype=torch.float32, device=gpu)
        m.ctx.forward_bgr(bgr, B, H, W, N.OUT_LOGITS_F32, lg)       # (the plan, and its fusion choice, is built here)
    finally:
        del os.environ["BUGSEG_CLS_FUSE"]
    seg = torch.empty((B, H, W), dtype=torch.uint8, device=gpu)
    m.ctx.forward_bgr(bgr, B, H, W, N.OUT_CLASS15_U8, seg)
    assert m.ctx.plan_op(B, H, W, m.ctx.plan_info(B, H, W, N.OUT_CLASS15_U8)[0] - 1)[0] == "fused"
    la = lg.cpu().numpy()
    assert np.abs(la).max() > 1e4          # the case really scales
    mx = np.abs(la).reshape(B, -1).max(1)[:, None, None]
    dec = _margin(la) > 1e-5 * mx
    s = seg.cpu().numpy()
    print(f"undamped fp32 class fusion: {int((~dec).sum())} near-tie pixels of {dec.size}; "
          f"{int(((s != la.argmax(1)) & dec).sum())} decided pixels differ")
    assert (~dec).mean() < 1e-3
    assert np.array_equal(s[dec], la.argmax(1)[dec])


@pytest.mark.parametrize("prec", ["fp32", "bf16", "fp16"])
def test_up_block_pair_equals_separate(gpu, blocks, prec, monkeypatch):
    """The upsampling blocks' main and extension 1x1 convolutions merged into one launch (one read
    of the block input, the tconv reading the extension half) are bit-identical to the separate
    launches (BUGSEG_NO_PAIR=1)."""
    H, W = 120, 160
    bgr = torch.from_numpy(synthetic.road_frames(2, H, W, seed=4)).cuda()
    monkeypatch.setenv("BUGSEG_NO_FUSE", "1")
    paired = ENET(weights=blocks, precision=prec)
    a = torch.empty((2, 15, H, W), dtype=torch.float32, device=gpu)
    paired.ctx.forward_bgr(bgr, 2, H, W, N.OUT_LOGITS_F32, a)
    monkeypatch.setenv("BUGSEG_NO_PAIR", "1")
    monkeypatch.setenv("BUGSEG_NO_FUSE", "1")        # (the fused upsampling kernel would take both)
    sep = ENET(weights=blocks, precision=prec)
    b = torch.empty_like(a)
    sep.ctx.forward_bgr(bgr, 2, H, W, N.OUT_LOGITS_F32, b)
    assert paired.ctx.plan_info(2, H, W, N.OUT_LOGITS_F32)[0] < sep.ctx.plan_info(2, H, W, N.OUT_LOGITS_F32)[0]
    assert torch.equal(a, b)


@pytest.mark.parametrize("prec", ["fp32", "bf16", "fp16"])
def test_class_layer_kernel_matches_conv_path(gpu, blocks, prec, monkeypatch):
    """The class-layer kernel (cls_kernels.hip: 32x32 MFMA, all 16 logits of an output pixel in one
    lane, in-register argmax) against the generic implicit-GEMM path (BUGSEG_CLS_CONV=1) on the same
    network: the two sum the 64 products in different orders, so logits agree to rounding and class
    maps wherever the top-2 margin is not a near-tie; the argmax itself is checked exactly against the
    kernel's own logits."""
    H, W = 120, 160
    bgr = torch.from_numpy(synthetic.road_frames(2, H, W, seed=6)).cuda()
    model = ENET(weights=blocks, precision=prec)
    a = torch.empty((2, 15, H, W), dtype=torch.float32, device=gpu)
    model.ctx.forward_bgr(bgr, 2, H, W, N.OUT_LOGITS_F32, a)
    raw = torch.empty((2, H, W), dtype=torch.uint8, device=gpu)
    model.ctx.forward_bgr(bgr, 2, H, W, N.OUT_CLASS15_U8, raw)
    tags = [model.ctx.plan_op(2, H, W, i)[0] for i in range(model.ctx.plan_info(2, H, W, N.OUT_CLASS15_U8)[0])]
    assert tags[-1] == "classes"
    monkeypatch.setenv("BUGSEG_CLS_CONV", "1")
    ref = ENET(weights=blocks, precision=prec)
    b = torch.empty_like(a)
    ref.ctx.forward_bgr(bgr, 2, H, W, N.OUT_LOGITS_F32, b)
    la, lb = a.cpu().numpy(), b.cpu().numpy()
    tol = 1e-4 if prec == "fp32" else 2e-2
    np.testing.assert_allclose(la, lb, rtol=0, atol=tol * max(1.0, float(np.abs(lb).max())))
    # the kernel's class map is exactly tf.math.argmax of its own logits (lowest index on ties)
    assert np.array_equal(raw.cpu().numpy(), la.argmax(axis=1))
    decided = _decided(lb, la, what=f"class kernel vs conv path ({prec})") if prec == "fp32" else _margin(lb) > 0.1
    assert (la.argmax(axis=1)[decided] == lb.argmax(axis=1)[decided]).all()


@pytest.mark.parametrize("prec", ["fp32", "fp16"])
@pytest.mark.parametrize("tied", [False, True])
def test_class_layer_group_argmax_is_lut_of_first_maximum(gpu, blocks, prec, tied):
    """The remapped maps (CLASS3, BINARY) take the class kernel's group-maxima argmax (LK = 1 / 2 in
    cls_kernels.hip); it must equal LUT[first-index argmax] of the same kernel's logits exactly. With
    ``tied`` class 3 is given class 0's weights and bias, so every pixel whose maximum is class 0 ties
    across groups ({0, 1} vs the rest) and takes the full-scan fallback: the first maximum, class 0."""
    import copy
    bl = blocks
    if tied:
        bl = copy.deepcopy(blocks)
        u = bl[-1].units[0]
        ax = [i for i, s in enumerate(u.w.shape) if s == 15][0]
        w = np.moveaxis(u.w, ax, 0)
        w[3] = w[0]
        u.b[0] += 3.0                            # make class 0 win often enough
        u.b[3] = u.b[0]
    H, W = 120, 160
    bgr = torch.from_numpy(synthetic.road_frames(2, H, W, seed=7)).cuda()
    model = ENET(weights=bl, precision=prec)
    lg = torch.empty((2, 15, H, W), dtype=torch.float32, device=gpu)
    model.ctx.forward_bgr(bgr, 2, H, W, N.OUT_LOGITS_F32, lg)
    first = lg.cpu().numpy().argmax(axis=1)
    if tied:
        assert (first == 0).mean() > 0.01        # the tie path is taken on a fair share of pixels
    for kind, lut in ((N.OUT_CLASS3_U8, eo.LUT3), (N.OUT_BINARY_U8, eo.LUT_BINARY)):
        seg = torch.empty((2, H, W), dtype=torch.uint8, device=gpu)
        model.ctx.forward_bgr(bgr, 2, H, W, kind, seg)
        assert np.array_equal(seg.cpu().numpy(), lut[first]), kind


def test_canonical_plan_is_one_launch_per_block(gpu, blocks, monkeypatch):
    """At the bench shape every ENet block of the canonical graph runs as ONE fused launch: initial
    block, 2 downsampling, 23 regular / dilated / asymmetric bottlenecks, 2 upsampling blocks and
    the class layer (29 launches); the unfused reference plan has one launch per convolution."""
    B, H, W = 2, 480, 640
    m = ENET(weights=blocks, precision="bf16")
    bgr = torch.from_numpy(synthetic.uniform_frames(B, H, W)).cuda()
    seg = torch.empty((B, H, W), dtype=torch.uint8, device=gpu)
    m.ctx.forward_bgr(bgr, B, H, W, N.OUT_CLASS3_U8, seg)
    n = m.ctx.plan_info(B, H, W, N.OUT_CLASS3_U8, bgr_input=True)[0]
    tags = [m.ctx.plan_op(B, H, W, i)[0] for i in range(n)]
    assert n == 29
    assert tags[0] == "init" and tags[-1] == "classes"
    assert [t.split(" ")[0] + " " + t.split(" ")[1] for t in tags if t.startswith(("down", "up"))] == \
        ["down C64", "down C128", "up C64", "up C16"]
    assert sum(t.startswith("bneck") for t in tags) == 23
    x = ENET.preprocess_device(bgr, N.PRE_ENGINE, ctx=m.ctx, width=W, height=H)
    m.predict_device(x, N.OUT_CLASS3_U8)
    tags = [m.ctx.plan_op(B, H, W, i)[0] for i in range(n)]
    assert tags[0] == "init" and tags[1].startswith("down C64")


def test_bev_shape_assert(gpu):
    bev = synthetic.synthetic_bev(120, 160, 300, 300)
    with pytest.raises(AssertionError):
        bev.create_occupancy_grid(np.zeros((160, 120), np.uint8), 3.0, 3.0, 0.05)


def test_pipeline_end_to_end_fp32(fp32_model, blocks):
    H, W = 480, 640
    frames = synthetic.road_frames(2, H, W, seed=9)
    bev = synthetic.synthetic_bev(H, W)
    grid = (synthetic.GRID_W_M, synthetic.GRID_H_M, synthetic.CELL_M)
    pipe = OccupancyPipeline(fp32_model, bev, *grid, model_hw=(H, W))
    out = pipe.run(torch.from_numpy(frames).cuda()).cpu().numpy()
    cls_ref, grids_ref, logits_ref = ocv_c.pipeline(frames, blocks, bev._bev_matrix, 1000, 1000, 1.0, grid, (H, W))
    # the grid is recomputed from the GPU's own class map by the oracle: exact
    x = np.concatenate([ENET.preprocess_device(f, width=W, height=H).cpu().numpy() for f in frames])
    cls = fp32_model.predict(x)
    own = np.stack([ocv_c.create_occupancy_grid(c, bev._bev_matrix, 1000, 1000, 1.0, *grid) for c in cls])
    assert np.array_equal(out, own)
    decided = _decided(logits_ref, fp32_model.logits(x), max_excused=1e-4, what="pipeline fp32 480x640")
    assert (cls[decided] == cls_ref[decided]).all()
    seg = pipe._seg.cpu().numpy()              # the fused-preprocess class maps of the pipeline itself
    assert (seg[decided] == cls_ref[decided]).all()
    print(f"end-to-end grid agreement vs oracle {(out == grids_ref).mean():.6f}")


def test_multistream_pipeline_identical(bf16_model):
    H, W, B = 96, 128, 10
    frames = torch.from_numpy(synthetic.road_frames(B, H, W, seed=8)).cuda()
    bev = synthetic.synthetic_bev(H, W, 300, 300)
    one = OccupancyPipeline(bf16_model, bev, 3.0, 3.0, 0.05, model_hw=(H, W)).run(frames).clone()
    for s in (2, 3):
        for chain, off in ((False, 0), (True, 0), (False, 7)):   # chain: shard i's forward after shard
            # i-1's (BEV beside it); off: shard i+1 starts at shard i's 7th launch
            many = OccupancyPipeline(bf16_model, bev, 3.0, 3.0, 0.05, model_hw=(H, W), streams=s,
                                     chain_forwards=chain, shard_offset=off)
            for _ in range(2):
                got = many.run(frames)
            torch.cuda.synchronize()
            assert torch.equal(one, got)


@pytest.mark.parametrize("binary", [False, True])
def test_multistream_pipeline_laserscan(bf16_model, binary):
    """Laserscan-like mode through OccupancyPipeline with 2 and 3 frame shards on their own streams
    (B = 10: the uneven 3/3/4 split included), several steps back to back so the shards' kernels
    overlap each other and the previous step: identical to streams = 1, which is itself equal to the
    C restatement recomputed from the GPU's own class maps (bev.py:216-240; the binary pairing
    predict_binary + create_occupancy_grid_binary returns the reference's pair, bev.py:143-164)."""
    H, W, B = 240, 320, 10
    ww = wh = 600
    grid = (6.0, 6.0, 0.05)
    frames = torch.from_numpy(synthetic.road_frames(B, H, W, seed=12)).cuda()
    bev = synthetic.synthetic_bev(H, W, ww, wh)
    bev.laserscan_like_occupancy_grid = True
    one_pipe = OccupancyPipeline(bf16_model, bev, *grid, model_hw=(H, W), binary=binary)
    one = one_pipe.run(frames).clone()
    seg = one_pipe._seg.cpu().numpy()
    M = bev._bev_matrix
    if binary:
        assert set(np.unique(seg).tolist()) <= {0, 1}
        ref = [ocv_c.create_occupancy_grid_binary_laserscan(c, M, ww, wh, 1.0, *grid) for c in seg]
        want = np.stack([np.stack([r[0] for r in ref]), np.stack([r[1] for r in ref])])
    else:
        want = np.stack([ocv_c.create_occupancy_grid_laserscan(c, M, ww, wh, 1.0, *grid) for c in seg])
    assert one.shape == want.shape
    assert np.array_equal(one.cpu().numpy(), want)
    for s in (2, 3):
        many = OccupancyPipeline(bf16_model, bev, *grid, model_hw=(H, W), streams=s, binary=binary)
        outs = [many.run(frames).clone() for _ in range(3)]
        torch.cuda.synchronize()
        for o in outs:
            assert torch.equal(one, o)


def test_shared_context_bev_on_two_streams(gpu):
    """bugseg_bev_occgrid keeps its laserscan scratch per (context, stream): the per-device shared
    context, driven from two streams at once with batches of different sizes (a larger batch grows
    its stream's scratch while the other stream's kernels are in flight), gives the single-stream
    results."""
    rows, cols, ww, wh, grid = 240, 320, 600, 600, (6.0, 6.0, 0.05)
    bev = _bev_case(rows, cols, ww, wh, 13)
    bev.laserscan_like_occupancy_grid = True
    rng = np.random.default_rng(13)
    segs = [torch.from_numpy(np.kron(rng.integers(0, 3, size=(b, rows // 4, cols // 4)),
                                     np.ones((1, 4, 4), np.int64)).astype(np.uint8)).cuda() for b in (6, 16, 4, 24)]
    want = [bev.create_occupancy_grid_device(s, *grid).clone() for s in segs]
    torch.cuda.synchronize()
    sts = [torch.cuda.Stream(), torch.cuda.Stream()]
    got = []
    for rep in range(2):
        for i, s in enumerate(segs):
            st = sts[i % 2]
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                got.append((i, bev.create_occupancy_grid_device(s, *grid)))
    torch.cuda.synchronize()
    for i, g in got:
        assert torch.equal(g, want[i])


def test_config1_reference_resolution_fp32(fp32_model, blocks):
    """BASELINE config 1: a 512x512 BGR frame -> ENET.preprocess (cv2.resize INTER_LINEAR to
    512x256, BGR->RGB, (x/256 - mean)/std; models.py:84-95) -> the fp32 forward at the reference's
    native 256x512 (models.py:19, 42-44) -> logits within 1e-3 of the oracle, class maps (predict and
    predict_binary, models.py:55-58, 78-80) equal on every pixel whose top-2 margin exceeds 2.5x the measured max logit error."""
    frame = synthetic.road_frames(1, 512, 512, seed=21)[0]
    x = ENET.preprocess(frame)
    assert x.shape == (1, 3, 256, 512) and x.dtype == np.float64
    assert np.array_equal(x, eo.preprocess(frame))
    ref = eo.forward(blocks, x.astype(np.float32))
    got = fp32_model.logits(x)
    assert got.shape == ref.shape == (1, 15, 256, 512)
    assert np.abs(got - ref).max() < LOGIT_TOL
    decided = _decided(ref, got, max_excused=1e-4, what="config 1 fp32 256x512")
    cls = eo.argmax_classes(ref)
    p3 = fp32_model.predict(x)
    assert p3.shape == (1, 256, 512) and p3.dtype == np.uint8
    assert (p3[decided] == eo.LUT3[cls][decided]).all()
    assert (fp32_model.predict_binary(x)[decided] == eo.LUT_BINARY[cls][decided]).all()


@pytest.mark.parametrize("streams", [1, 2])
def test_captured_pipeline_identical(bf16_model, streams):
    """OccupancyPipeline.capture: the HIP-graph replay of a step equals the eager step, and re-reads
    the frame buffer at every replay."""
    H, W, B = 96, 128, 8
    bev = synthetic.synthetic_bev(H, W, 300, 300)
    a = torch.from_numpy(synthetic.road_frames(B, H, W, seed=8)).cuda()
    b = torch.from_numpy(synthetic.road_frames(B, H, W, seed=9)).cuda()
    eager = OccupancyPipeline(bf16_model, bev, 3.0, 3.0, 0.05, model_hw=(H, W))
    ref_a, ref_b = eager.run(a).clone(), eager.run(b).clone()
    pipe = OccupancyPipeline(bf16_model, bev, 3.0, 3.0, 0.05, model_hw=(H, W), streams=streams)
    buf = a.clone()
    replay, grids = pipe.capture(buf)
    buf.copy_(b)
    replay()
    torch.cuda.synchronize()
    assert torch.equal(grids, ref_b)
    buf.copy_(a)
    replay()
    torch.cuda.synchronize()
    assert torch.equal(grids, ref_a)


def test_full_size_batch_properties(bf16_model):
    """Full configs[2] shape (B=32, 480x640): value sets, determinism, batch independence."""
    H, W, B = 480, 640, 32
    frames = torch.from_numpy(synthetic.uniform_frames(B, H, W, seed=1)).cuda()
    bev = synthetic.synthetic_bev(H, W)
    pipe = OccupancyPipeline(bf16_model, bev, synthetic.GRID_W_M, synthetic.GRID_H_M, synthetic.CELL_M, model_hw=(H, W))
    a = pipe.run(frames).clone()
    b = pipe.run(frames).clone()
    assert torch.equal(a, b)
    assert set(torch.unique(a).tolist()) <= {-1, 0, 100}
    pipe1 = OccupancyPipeline(bf16_model, bev, synthetic.GRID_W_M, synthetic.GRID_H_M, synthetic.CELL_M, model_hw=(H, W))
    for i in (0, 17, 31):
        single = pipe1.run(frames[i:i + 1].contiguous())
        assert torch.equal(single[0], a[i])


@pytest.mark.parametrize("prec", ["fp16", "bf16"])
def test_multi_tile_workgroups_batch_independent(gpu, blocks, prec):
    """B = 48 at 480x640: more bottleneck tiles than resident workgroup slots (C128: 720 tiles on
    512 slots, C64: 3,840 on 1,280), so workgroups walk several tiles — the later tiles of a walk skip
    the weight-staging wait and the kept-residual forms issue their loads ahead of the ts barrier.
    Every frame's logits equal its single-frame forward bit for bit."""
    H, W, B = 480, 640, 48
    m = ENET(weights=blocks, precision=prec)
    frames = torch.from_numpy(synthetic.road_frames(B, H, W, seed=11)).cuda()
    out = torch.empty((B, 15, H, W), dtype=torch.float32, device=gpu)
    m.ctx.forward_bgr(frames, B, H, W, N.OUT_LOGITS_F32, out)
    one = torch.empty((1, 15, H, W), dtype=torch.float32, device=gpu)
    for i in (0, 23, 47):
        m.ctx.forward_bgr(frames[i:i + 1].contiguous(), 1, H, W, N.OUT_LOGITS_F32, one)
        torch.cuda.synchronize()
        assert torch.equal(one[0], out[i]), i


def test_errors_are_loud(gpu, blocks):
    m = ENET(weights=blocks, precision="fp32")
    with pytest.raises(ValueError):
        m.predict(np.zeros((1, 3, 30, 44), np.float32))      # not a multiple of 8
    with pytest.raises(N.BugsegError):
        ENET(weights=b"BSG1" + b"\0" * 12)


@pytest.mark.parametrize("style", ["nhwc", "nchw"])
def test_enet_from_graphdef_matches_graph_interpreter(gpu, tmp_path, style):
    """The north star's TF-parity check, on a frozen GraphDef written from the synthetic weights
    (tests/graph_writer.py; the real enet.pb is absent): ENET("x.pb") — the reference's constructor
    (models.py:21-31) through the GraphDef importer — against the NumPy interpreter of the same
    graph (oracle/tf_graph.py, the sess.run stand-in): logits within 1e-3 (fp32), classes equal
    wherever the interpreter's top-2 margin exceeds 2.5x the measured max logit error."""
    import sys
    sys.path.insert(0, str(Path(__file__).parent))
    from graph_writer import with_biases, write_enet_graphdef
    from oracle import tf_graph
    H, W = 120, 160
    blocks = with_biases(enet_spec.build_enet(), seed=3)
    pb = write_enet_graphdef(blocks, H, W, style)
    path = tmp_path / "enet.pb"
    path.write_bytes(pb)
    x = np.concatenate([ENET.preprocess_device(f, width=W, height=H).cpu().numpy()
                        for f in synthetic.road_frames(1, H, W, seed=11)]).astype(np.float32)
    want = tf_graph.run(pb, {"input0": x}, ENET.OUTPUT_TENSOR_NAME)
    model = ENET(str(path), precision="fp32")
    got = model.logits(x)
    assert got.shape == want.shape
    err = float(np.abs(got - want).max())
    assert err < 1e-3, err
    decided = _decided(want, got, what=f"graphdef {style}")
    cls = np.argmax(want, axis=1)
    assert (model.predict(x)[decided] == eo.LUT3[cls][decided]).all()


@pytest.mark.skipif(not os.environ.get("BUGSEG_ENET_PB"), reason="set BUGSEG_ENET_PB=path/to/enet.pb (absent here)")
def test_real_enet_pb_tf_parity(gpu):
    """The one-command TF-parity check for when the reference's pretrained_models/enet.pb is
    supplied: BUGSEG_ENET_PB=.../enet.pb pytest tests/test_gpu_parity.py -m gpu -k real_enet_pb.
    Same bar as the synthetic-graph test: logits within 1e-3 of the graph (interpreted), classes
    equal wherever the top-2 margin exceeds 2.5x the measured max logit error, at the reference's 256 x 512 input."""
    from oracle import tf_graph
    path = os.environ["BUGSEG_ENET_PB"]
    pb = Path(path).read_bytes()
    H, W = ENET.INPUT_HEIGHT, ENET.INPUT_WIDTH
    x = np.concatenate([ENET.preprocess_device(f, width=W, height=H).cpu().numpy()
                        for f in synthetic.road_frames(1, 512, 512, seed=5)]).astype(np.float32)
    want = tf_graph.run(pb, {ENET.INPUT_TENSOR_NAME.split(":")[0]: x}, ENET.OUTPUT_TENSOR_NAME)
    model = ENET(path, precision="fp32")
    got = model.logits(x)
    assert np.abs(got - want).max() < 1e-3
    decided = _decided(want, got, max_excused=1e-4, what="enet.pb")
    assert (model.predict(x)[decided] == eo.LUT3[np.argmax(want, axis=1)][decided]).all()
