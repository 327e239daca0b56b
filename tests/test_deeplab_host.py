"""Host-side DeepLabV3 checks (no GPU): the graph builder's lowering, TF-semantics known answers of
the oracle, the weight-file round trip and the plugin's preprocess (models.py:98-136)."""
import numpy as np
import pytest
import torch

from bugcar_image_segmentation_amd import deeplab_spec as S
from oracle import deeplab_oracle as O


def test_same_padding_known_answers():
    # TF SAME: out = ceil(in/s); pad_before = total // 2 (the extra pixel goes after)
    assert S.same_pad(513, 3, 2, 1) == (257, 1)
    assert S.same_pad(512, 3, 2, 1) == (256, 0)
    assert S.same_pad(65, 3, 1, 4) == (65, 4)
    assert S.same_pad(65, 1, 1, 1) == (65, 0)
    assert S.same_pad(7, 2, 2, 1) == (4, 0)


def test_mobilenet_v2_output_stride_schedule():
    """slim mobilenet_base: strides past the output stride turn into atrous rates."""
    net = S.build_deeplab(output_stride=8)
    sd = [(b.dw.stride, b.dw.dil) for b in net.blocks]
    assert sd == [(1, 1), (2, 1), (1, 1), (2, 1), (1, 1), (1, 1), (1, 1), (1, 2), (1, 2), (1, 2),
                  (1, 2), (1, 2), (1, 2), (1, 2), (1, 4), (1, 4), (1, 4)]
    assert S.feature_size(net, 513) == 65
    net16 = S.build_deeplab(output_stride=16)
    assert S.feature_size(net16, 513) == 33
    assert [b.residual for b in net.blocks].count(True) == 10
    assert net.blocks[0].expand is None and all(b.expand is not None for b in net.blocks[1:])


def test_lowering_is_consistent():
    net = S.build_deeplab(atrous_rates=(12, 24, 36))
    blob, ops, bufs, info = S.lower(net, 2, bf16=True)
    assert ops.shape == (info["nops"], S.OP_FIELDS) and ops.dtype == np.int32
    kinds = list(ops[:, 0])
    assert kinds[0] == S.OP_CONV and kinds[-1] == S.OP_ARGMAX and kinds.count(S.OP_POOL) == 1
    assert ops[0, 31] == 2 and S.OP_PREP not in kinds          # preprocessing fused into the stem's loads
    _, ops_p, _, info_p = S.lower(net, 2, bf16=True, fuse_prep=False)
    assert ops_p[0, 0] == S.OP_PREP and ops_p[1, 31] == 1 and info_p["nops"] == info["nops"] + 1
    assert kinds.count(S.OP_DW) == 17
    _, ops_f, _, info_f = S.lower(net, 2, bf16=True, fuse_dw=True)
    assert list(ops_f[:, 0]).count(S.OP_DW) == 0 and info["nops"] == info_f["nops"] + 17
    assert [t for t, _, _ in info_f["per_op"]].count("conv dw+project") == 17
    assert info["bytes"] > info_f["bytes"] and info["flops"] == info["flops"]
    conv = ops[ops[:, 0] == S.OP_CONV]
    assert np.all(conv[:, 17] % 256 == 0) and np.all(conv[:, 17] < len(blob))   # weight offsets aligned, inside
    assert np.all(conv[:, 15] % 32 == 0) and np.all(conv[:, 16] % 64 == 0)
    # the ASPP branches write disjoint channel ranges of the concat buffer
    cat = conv[conv[:, 2] == 5]
    assert sorted(cat[:, 22]) == [0, 256, 512, 768] and np.all(cat[:, 21] == 1024)
    assert info["feature"] == (65, 65) and info["lcs"] == 24
    assert len(bufs) == 11 and bufs.min() > 0
    # MACs: ~8.5 GMAC/frame at 513 with the zoo head, plus the three dense atrous branches
    assert 2 * 8.0e9 < info["flops"] / 2 < 2 * 20e9


def test_weight_file_round_trip(tmp_path):
    net = S.build_deeplab(width=0.25, crop=65, atrous_rates=(2, 4))
    p = tmp_path / "dl.npz"
    S.save(net, p)
    net2 = S.load(p)
    b1, o1, _, _ = S.lower(net, 1, bf16=False)
    b2, o2, _, _ = S.lower(net2, 1, bf16=False)
    assert b1 == b2 and np.array_equal(o1, o2)


def test_preprocess_pad_and_normalise():
    x = np.array([[[[0, 255, 128]]]], np.uint8)
    y = O.preprocess(x, 3)
    f = np.float32
    assert y[0, 0, 0, 0] == f(-1.0) and y[0, 0, 0, 1] == f(2.0 / 255.0) * f(255) - f(1)
    pad = f(2.0 / 255.0) * f(127.5) - f(1)
    assert np.all(y[0, 1:, :, :] == pad) and np.all(y[0, :, 1:, :] == pad)


def test_resize_bilinear_tf_known_answers():
    L = np.arange(2 * 3 * 3, dtype=np.float32).reshape(1, 2, 3, 3)
    up = O.resize_bilinear_tf(L, 5, 5)
    # align_corners: the corners are the input corners, the midpoints the input pixels
    assert np.array_equal(up[:, :, ::2, ::2], L)
    assert up[0, 0, 1, 1] == np.float32(2.0)   # mean of 0, 1, 3, 4
    # 65 -> 513 uses scale 64/512 = 0.125 exactly
    L = np.random.default_rng(0).normal(size=(1, 1, 65, 65)).astype(np.float32)
    up = O.resize_bilinear_tf(L, 513, 513)
    assert np.array_equal(up[:, :, ::8, ::8], L)


def test_argmax_ties_take_lowest_class():
    net = S.build_deeplab(width=0.25, crop=9)
    L = np.zeros((1, net.num_classes, 2, 2), np.float32)
    L[:, 3] = 1.0
    L[:, 5] = 1.0
    cls = O.predict(net, np.zeros((1, 9, 9, 3), np.uint8), logits=L)
    assert cls.dtype == np.int64 and np.all(cls == 3)


def test_oracle_bf16_emulation_tracks_fp64():
    net = S.build_deeplab(width=0.25, crop=65)
    x = np.random.default_rng(1).integers(0, 256, (1, 65, 60, 3), dtype=np.uint8)
    a = O.forward(net, x, dtype=torch.float64)
    b = O.forward(net, x, bf16_storage=True)
    assert float((a - b).abs().mean()) < 0.1
    assert (O.predict(net, x, logits=a) == O.predict(net, x, logits=b)).mean() > 0.95


def test_plugin_preprocess_rgb_and_resize():
    from bugcar_image_segmentation_amd.models import DeepLabV3
    f = np.random.default_rng(2).integers(0, 256, (600, 1026, 3), dtype=np.uint8)
    r = DeepLabV3.preprocess(f)
    assert r.dtype == np.uint8 and max(r.shape[:2]) <= 513 and r.shape[2] == 3
    small = f[:100, :200]
    assert np.array_equal(DeepLabV3.preprocess(small), small[:, :, ::-1])
    with pytest.raises(ValueError):
        DeepLabV3.preprocess(f[:, :, :2])


def test_non_square_crop_lowering_and_weight_file(tmp_path):
    """An export with crop_size (h, w), h != w: the plan pads to h x w (stem input and the final
    resize), feature size per axis; the .npz keeps the width; the oracle pads and resizes to it."""
    net = S.build_deeplab(width=0.25, crop=(65, 97))
    assert S.crop_hw(net) == (65, 97)
    _, ops, bufs, info = S.lower(net, 2, bf16=False)
    assert tuple(ops[0, 4:6]) == (65, 97)                  # stem input H, W = the crop
    assert info["feature"] == (S.feature_size(net, 65), S.feature_size(net, 97))
    p = tmp_path / "dl.npz"
    S.save(net, p)
    assert S.crop_hw(S.load(p)) == (65, 97)
    sq = S.build_deeplab(width=0.25, crop=65)
    S.save(sq, p)
    assert S.crop_hw(S.load(p)) == (65, 65) and S.load(p).crop_w == 0
    x = np.random.default_rng(4).integers(0, 256, (1, 50, 90, 3), dtype=np.uint8)
    pre = O.preprocess(x, S.crop_hw(net))
    assert pre.shape == (1, 65, 97, 3) and np.all(pre[:, 50:] == np.float32(2 / 255) * np.float32(127.5) - 1)
    lg = O.forward(net, x)
    assert tuple(lg.shape[2:]) == info["feature"]
    assert O.predict(net, x, logits=lg).shape == (1, 50, 90)


def test_resnet_structure_and_lowering():
    """ResNet-v1-beta DeepLabV3 (deeplab_resnet.py): resnet_v1_101_beta's 3 / 4 / 23 / 3 units with the
    block stride on each block's last unit, output stride 16 turning block 3's last stride into rate 2
    and block 4 into rates 2 x multi-grid (1, 2, 4); projection shortcuts exactly where the depth
    changes; the op list's root pool, subsample ops and post-add-ReLU convs, buffer 7 the logits."""
    from bugcar_image_segmentation_amd import deeplab_resnet as R
    net = R.build_deeplab_resnet(depth=101, width=0.25)
    assert len(net.units) == 33
    strides = [u.stride for u in net.units]
    assert strides[2] == 2 and strides[6] == 2 and strides.count(2) == 2      # block 3's stride became a rate
    assert [u.conv2.dil for u in net.units[-3:]] == [2, 4, 8]
    assert [u.conv2.dil for u in net.units[7:29]] == [1] * 22 and net.units[29].conv2.dil == 1
    assert sum(u.shortcut is not None for u in net.units) == 4                 # first unit of every block
    assert R.feature_size(net, 513) == 33
    blob, ops, bufs, info = S.lower(net, 2, True)
    kinds = [int(o[0]) for o in ops]
    assert kinds.count(S.OP_MAXPOOL) == 1 + 2                                  # root pool + 2 subsamples
    post = [o for o in ops if int(o[0]) == S.OP_CONV and int(o[19]) == 3]
    assert len(post) == 33 and all(int(o[3]) >= 0 for o in post)             # every unit: residual, ReLU after
    assert info["feature"] == (33, 33) and int(bufs[7]) >= 2 * 33 * 33 * info["lcs"] * 4


def test_resnet_oracle_maxpool_same_and_subsample():
    """The oracle's TF max-pool restatement: SAME pads with -inf (pad_before = total // 2), so an
    all-negative input keeps its own values at the border; 1x1 VALID subsample = every s-th pixel."""
    x = -torch.arange(1.0, 1.0 + 2 * 3 * 7 * 6, dtype=torch.float64).reshape(2, 3, 7, 6)
    y = O._maxpool_same(x, 3, 2)
    assert y.shape == (2, 3, 4, 3)
    # output (0, 0) covers input rows -1..1 / cols -1..1 (pad 1 before for 7 -> 4): the max is x[0:2, 0:2]'s
    assert float(y[0, 0, 0, 0]) == float(x[0, 0, :2, :2].max())
    assert torch.equal(O._maxpool_same(x, 1, 2), x[:, :, ::2, ::2])


def test_resnet_bf16_emulation_tracks_fp64():
    from bugcar_image_segmentation_amd import deeplab_resnet as R
    net = R.build_deeplab_resnet(depth=50, width=0.25, units=(1, 1, 2, 1), crop=65)
    x = np.random.default_rng(3).integers(0, 256, (1, 65, 60, 3), dtype=np.uint8)
    a = O.forward(net, x).numpy()
    b = O.forward(net, x, bf16_storage=True).numpy()
    assert np.abs(a).max() > 0.1 and np.abs(a - b).mean() < 0.05 * np.abs(a).mean() + 1e-2
