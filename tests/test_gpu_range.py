"""GPU: the fp32 parity mode over the whole f32 range.

The fp32 mode's products take split-f16 operands (hi = f16(v), lo = f16(v - hi)), exact only for |v| in
the f16 window. bugseg brings every operand into it by exact powers of two (bugseg_internal.h
RangeArgs): stored tensors measured by the launch that writes them, the fused kernels' internal
tensors bounded from those measurements, weights by a static exponent. These tests put activations
and weights far outside the f16 range and compare the logits with the fp64 oracle
(`oracle/enet_oracle.forward`, the restatement of the reference's TF fp32 `sess.run`, models.py:43-44).

The criterion (oracle/enet_oracle.py range_verdict), per pixel e = max over classes |dlogit| / max |logit|:

* every logit finite; 99% of the pixels within 2e-6 of the max (f32 itself: the fp32 oracle is 2.0e-6
  of the max away from fp64 on the undamped 480x640 case, its p99 6e-7);
* every pixel beyond 5e-6 is ATTRIBUTED: the engine's own pooling indices of the same run
  (bugseg_debug_pool_indices) are compared with the fp64 first-maximum positions; every window whose
  index differs must be an fp64 near-tie (0 < top-2 gap <= 1e-5 of the frame's max |pool input|), and
  every pixel beyond the bar must lie inside the footprint of those flipped windows (their unpooled
  2x2 blocks grown through every later block's receptive field, oracle PoolTies.footprint). Where a
  max-pool window's top two inputs lie within rounding of each other, another index moves a value to
  another position through max-unpool — a discontinuity every f32 evaluation order can hit (the fp32
  oracle itself does on some frames). A flip at a window that is not a near-tie, or an error outside
  the flips' footprint, is a fault and fails the test; so do more than 0.5% of a frame's pixels
  (at least 2 x 32 x 32 allowed) beyond the bar. An f16 range failure shows as inf / NaN or as errors
  on most pixels (the negative control below);
* classes exact on every pixel outside the footprint whose fp64 top-2 margin exceeds 2.5x its error.

Cases: SURVEY.md §8(d)'s undamped draw (residual-branch BN gamma ~ U(0.5, 1.5): activations grow ~2.5x
per block, logits ~1e6, past f16's 65504 from the 16th block on), fused and unfused plans, two frames
each, and through the raw-BGR entry; single layers of 1e-6-scale weights (f16 subnormals: ~3% relative
error per weight unscaled) and of 1e5-1e6-scale weights (f16 overflow), the classifier included
(logits ~1e-5: the criterion is relative); and the negative control: with the scaling switched off
(BUGSEG_F32_RANGE=0, the round-4 arithmetic) the undamped case fails this criterion.
"""
import numpy as np
import pytest
import torch

from bugcar_image_segmentation_amd import _native as N
from bugcar_image_segmentation_amd import enet_spec, synthetic
from bugcar_image_segmentation_amd.models import ENET
from oracle import enet_oracle as eo

pytestmark = pytest.mark.gpu

REL = eo.RANGE_REL


def _frames(n, H, W, seed):
    """Normalised road-scene frames (B, 3, H, W): the reference's preprocess output range."""
    bgr = synthetic.road_frames(n, H, W, seed=seed)
    x = (bgr[..., ::-1] / 256.0 - eo.IMAGE_MEAN) / eo.IMAGE_STD
    return np.ascontiguousarray(np.moveaxis(x, -1, 1)).astype(np.float32)


def _reference(blocks, x):
    """fp64 logits and the pool record of the same forward."""
    ties = eo.PoolTies()
    return eo.forward(blocks, x.astype(np.float64), torch.float64, ties=ties), ties


def _verdict(m, blocks, got, ref, ties, what):
    """-> (ok, message) under the criterion of the module docstring; the engine's pooling indices are
    those of m's last forward at got's shape."""
    B, _c, H, W = got.shape
    idx = eo.engine_pool_indices(m.ctx, blocks, ties, B, H, W)
    ok, msg, _stats = eo.range_verdict(got, ref, ties, idx, what)
    return ok, msg


def _check(blocks, x, what):
    m = ENET(weights=blocks, precision="fp32")
    got = m.logits(x)
    ref, ties = _reference(blocks, x)
    ok, msg = _verdict(m, blocks, got, ref, ties, what)
    print(msg)
    assert ok, msg
    return m, ref


def _scaled(blocks, name, unit, factor):
    for b in blocks:
        if b.name == name:
            u = b.units[unit]
            u.w = (u.w.astype(np.float64) * factor).astype(np.float32)
            return blocks
    raise KeyError(name)


@pytest.mark.parametrize("fuse", [True, False])
@pytest.mark.parametrize("seed", [5, 6])
def test_undamped_survey_draw_480x640(gpu, fuse, seed, monkeypatch):
    """§8(d)'s draw as written: logits ~1e6, activations past f16's range in the late blocks."""
    if not fuse:
        monkeypatch.setenv("BUGSEG_NO_FUSE", "1")
    bl = enet_spec.build_enet(res_gamma=(0.5, 1.5))
    _m, ref = _check(bl, _frames(1, 480, 640, seed=seed),
                     f"undamped 480x640 seed {seed} {'fused' if fuse else 'unfused'}")
    assert np.abs(ref).max() > 1e5        # the case really leaves the f16 range


def test_undamped_through_bgr_pipeline(gpu):
    """The product entry (raw BGR frames, preprocess fused into the initial block), 2 frames of
    480x640, undamped weights; the 3-class maps against the fp64 argmax + LUT."""
    bl = enet_spec.build_enet(res_gamma=(0.5, 1.5))
    m = ENET(weights=bl, precision="fp32")
    bgr = synthetic.road_frames(2, 480, 640, seed=9)
    dev = torch.device("cuda", 0)
    frames = torch.from_numpy(bgr).to(dev)
    lg = torch.empty((2, m.num_classes, 480, 640), dtype=torch.float32, device=dev)
    m.ctx.forward_bgr(frames, 2, 480, 640, N.OUT_LOGITS_F32, lg)
    cls3 = torch.empty((2, 480, 640), dtype=torch.uint8, device=dev)
    m.ctx.forward_bgr(frames, 2, 480, 640, N.OUT_CLASS3_U8, cls3)
    torch.cuda.synchronize()
    # the engine's table rounds (v/256 - mean)/std to f32, as the engine-input path stores it
    x = np.ascontiguousarray(np.moveaxis(((bgr[..., ::-1] / 256.0 - eo.IMAGE_MEAN) / eo.IMAGE_STD), -1, 1)).astype(np.float32)
    ref, ties = _reference(bl, x)
    got = lg.cpu().numpy()
    ok, msg = _verdict(m, bl, got, ref, ties, "undamped BGR entry B=2")
    print(msg)
    assert ok, msg
    err = np.abs(got - ref).max(1)
    s = np.sort(ref, axis=1)
    dec = ((s[:, -1] - s[:, -2]) > 2.5 * err) & (err / np.abs(ref).max() <= REL)
    assert (cls3.cpu().numpy()[dec] == eo.LUT3[ref.argmax(1)][dec]).all()


@pytest.mark.parametrize("name,unit,factor", [("regular2_1", 0, 1e-6), ("regular1_2", 1, 1e-6),
                                              ("upsample4_0", 1, 1e-6), ("downsample2_0", 1, 1e6),
                                              ("regular3_4", 2, 1e5), ("asymmetric2_3", 2, 1e6),
                                              ("transposed_conv", 0, 1e-6), ("initial_block", 0, 1e5)])
def test_extreme_weight_scales(gpu, name, unit, factor):
    """One layer's weights far outside the f16 window (subnormal at 1e-6, past 65504 at 1e5-1e6): the
    packer's static weight exponent and the activations' measured / bounded exponents keep the
    products exact."""
    bl = _scaled(enet_spec.build_enet(), name, unit, factor)
    m, _ref = _check(bl, _frames(1, 120, 160, seed=2), f"{name}.units[{unit}] x {factor:g} 120x160")
    sws = [m.ctx.debug_info(2, i) for i in range(256)]
    assert any(abs(v) >= 10 and v != -1000 for v in sws)      # the scaled layer got its exponent


def test_without_scaling_the_undamped_case_fails(gpu, monkeypatch):
    """Negative control: BUGSEG_F32_RANGE=0 (read at load_weights) packs the weights unscaled and runs
    every kernel at exponent 0; the undamped case then fails the criterion (its activations overflow
    the f16 parts) — the tests above measure the scaling, not a criterion any f32 run would pass."""
    monkeypatch.setenv("BUGSEG_F32_RANGE", "0")
    bl = enet_spec.build_enet(res_gamma=(0.5, 1.5))
    m = ENET(weights=bl, precision="fp32")
    assert m.ctx.debug_info(1) == 1
    x = _frames(1, 480, 640, seed=5)
    got = m.logits(x)
    ref, ties = _reference(bl, x)
    ok, msg = _verdict(m, bl, got, ref, ties, "undamped, scaling OFF")
    print(msg)
    assert not ok


def test_damped_fast_path_unchanged(gpu, blocks):
    """The default (damped) network: its activations sit inside the window, so the measured exponents
    stay 0 — the logits equal the fp32 oracle within the round-4 bar."""
    x = _frames(1, 120, 160, seed=1)
    m = ENET(weights=blocks, precision="fp32")
    assert m.ctx.debug_info(1) == 0
    got = m.logits(x)
    ref = eo.forward(blocks, x)
    assert np.abs(got - ref).max() < 1e-3
