"""Stream order and graphs: the BEV entry points build their tables on
the context's private stream and take their laserscan scratch from the caller (torch's allocator),
so the FIRST call at a new geometry and batch can be captured into a HIP graph — for the rasteriser
alone and for a whole OccupancyPipeline step, laserscan mode included, on 1 and 2 shard streams.

The N > 1 product path on one GPU: two ranks of a gloo
process group, both on cuda:0, each runs OccupancyPipeline over its shard_bounds shard and the
grids go through distributed.gather_grids; and bench.py's distributed branch end to end under
torch.distributed.run with --backend gloo (a functional run, not a timing).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from bugcar_image_segmentation_amd import _native as N
from bugcar_image_segmentation_amd import enet_spec, synthetic
from bugcar_image_segmentation_amd.models import ENET
from bugcar_image_segmentation_amd.pipeline import OccupancyPipeline
from oracle import ocv_c

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fresh_bev(rows, cols, ww, wh, seed):
    """A calibration no earlier call has used (perturbed matrix): its tables do not exist yet."""
    rng = np.random.default_rng(1000 + seed)
    bev = synthetic.synthetic_bev(rows, cols, ww, wh)
    bev._bev_matrix = bev._bev_matrix @ np.array([[1 + 0.03 * rng.normal(), 0.01 * rng.normal(), 3 * rng.normal()],
                                                  [0.01 * rng.normal(), 1 + 0.03 * rng.normal(), 3 * rng.normal()],
                                                  [1e-5 * rng.normal(), 1e-5 * rng.normal(), 1.0]])
    return bev


def _oracle(bev, segs, grid, binary, laserscan):
    M, ww, wh = bev._bev_matrix, bev.after_warp_width, bev.after_warp_height
    if binary and laserscan:
        pairs = [ocv_c.create_occupancy_grid_binary_laserscan(s, M, ww, wh, 1.0, *grid) for s in segs]
        return np.stack([np.stack([p[0] for p in pairs]), np.stack([p[1] for p in pairs])])
    f = {(0, 0): ocv_c.create_occupancy_grid, (0, 1): ocv_c.create_occupancy_grid_laserscan,
         (1, 0): ocv_c.create_occupancy_grid_binary}[(int(binary), int(laserscan))]
    return np.stack([f(s, M, ww, wh, 1.0, *grid) for s in segs])


@pytest.mark.parametrize("binary", [False, True])
@pytest.mark.parametrize("laserscan", [False, True])
def test_capture_first_bev_call_at_new_geometry(gpu, laserscan, binary):
    rows, cols, ww, wh, grid = 120, 160, 300, 260, (3.0, 2.0, 0.05)
    bev = _fresh_bev(rows, cols, ww, wh, 2 * int(laserscan) + int(binary))
    bev.laserscan_like_occupancy_grid = laserscan
    rng = np.random.default_rng(5)
    a = np.kron(rng.integers(0, 3, size=(5, rows // 8, cols // 8)), np.ones((1, 8, 8), np.int64)).astype(np.uint8)
    b = rng.integers(0, 3, size=(5, rows, cols)).astype(np.uint8)
    seg = torch.from_numpy(a).to(gpu)
    p = bev.occupancy_params(*grid, binary=binary)
    shape = (5, p.occ_h, p.occ_w)
    out = torch.empty(((2,) + shape) if binary and laserscan else shape, dtype=torch.int8, device=gpu)
    if laserscan and binary:
        N.shared_context(gpu.index)     # a context created inside the capture is covered by the other cases
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):                         # the first call at this geometry and batch
        bev.create_occupancy_grid_device(seg, *grid, out=out, binary=binary)
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), _oracle(bev, a, grid, binary, laserscan))
    seg.copy_(torch.from_numpy(b))                    # the replay re-reads the class maps
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), _oracle(bev, b, grid, binary, laserscan))
    # eager calls on the same context after the capture: same tables, same results
    assert np.array_equal(bev.create_occupancy_grid_device(seg, *grid, binary=binary).cpu().numpy(),
                          _oracle(bev, b, grid, binary, laserscan))


@pytest.mark.parametrize("warm", [False, True])
@pytest.mark.parametrize("laserscan", [False, True])
@pytest.mark.parametrize("streams", [1, 2])
def test_captured_pipeline_laserscan_and_first_call(gpu, blocks, streams, laserscan, warm):
    """OccupancyPipeline.capture with the laserscan-like mode on and off, on 1 and 2 shard streams;
    warm=False captures the very first step (arenas, tables and scratch come into being during the
    capture). The replay equals an eager pipeline on other contexts."""
    H, W, B = 96, 128, 6
    bev = _fresh_bev(H, W, 300, 300, 10 + 4 * streams + 2 * int(laserscan) + int(warm))
    bev.laserscan_like_occupancy_grid = laserscan
    grid = (3.0, 3.0, 0.05)
    fa = torch.from_numpy(synthetic.road_frames(B, H, W, seed=31)).to(gpu)
    fb = torch.from_numpy(synthetic.road_frames(B, H, W, seed=32)).to(gpu)
    ref_model = ENET(weights=blocks, precision="bf16")
    eager = OccupancyPipeline(ref_model, bev, *grid, model_hw=(H, W))
    ref_a, ref_b = eager.run(fa).clone(), eager.run(fb).clone()
    model = ENET(weights=blocks, precision="bf16")
    pipe = OccupancyPipeline(model, bev, *grid, model_hw=(H, W), streams=streams)
    buf = fa.clone()
    replay, grids = pipe.capture(buf, warm=warm)
    replay()
    torch.cuda.synchronize()
    assert torch.equal(grids, ref_a)
    buf.copy_(fb)
    replay()
    torch.cuda.synchronize()
    assert torch.equal(grids, ref_b)


@pytest.mark.parametrize("warm", [False, True])
def test_captured_pipeline_with_resize_then_other_geometry(gpu, blocks, warm):
    """frames NOT at the model resolution (the resize table of bugseg_preprocess mode 2).
    The capture (warm or the very first call) builds that table on the private stream; an eager
    step at a third source resolution afterwards builds another one and must not free the table
    the graph reads: the replay still equals an eager pipeline."""
    H, W, B = 96, 128, 4
    H0, W0 = 131, 170                                   # not 2x: the fixed-point linear resize
    bev = _fresh_bev(H, W, 300, 300, 40 + int(warm))
    grid = (3.0, 3.0, 0.05)
    fa = torch.from_numpy(synthetic.road_frames(B, H0, W0, seed=51)).to(gpu)
    fb = torch.from_numpy(synthetic.road_frames(B, H0, W0, seed=52)).to(gpu)
    fc = torch.from_numpy(synthetic.road_frames(B, 110, 150, seed=53)).to(gpu)
    eager = OccupancyPipeline(ENET(weights=blocks, precision="fp16"), bev, *grid, model_hw=(H, W))
    ref_a, ref_b, ref_c = eager.run(fa).clone(), eager.run(fb).clone(), eager.run(fc).clone()
    pipe = OccupancyPipeline(ENET(weights=blocks, precision="fp16"), bev, *grid, model_hw=(H, W))
    buf = fa.clone()
    replay, grids = pipe.capture(buf, warm=warm)
    replay()
    torch.cuda.synchronize()
    assert torch.equal(grids, ref_a)
    # an eager step at a third source resolution (another resize table) on the same context
    out_c = torch.empty_like(grids)
    pipe.run(fc, out=out_c)
    torch.cuda.synchronize()
    assert torch.equal(out_c, ref_c)
    buf.copy_(fb)
    replay()
    torch.cuda.synchronize()
    assert torch.equal(grids, ref_b)


def test_weight_reload_keeps_captured_graph_memory(gpu, blocks):
    """load_weights after a capture keeps the old weights (and arena) the graph's kernels
    point at until the context is destroyed, so replaying the old graph still computes with the old
    weights, and eager forwards use the new ones."""
    H, W, B = 64, 96, 2
    frames = torch.from_numpy(synthetic.road_frames(B, H, W, seed=61)).to(gpu)
    other = enet_spec.build_enet(seed=77)
    m = ENET(weights=blocks, precision="fp16")
    seg = torch.empty((B, H, W), dtype=torch.uint8, device=gpu)
    m.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS15_U8, seg)
    want_old = seg.clone()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        m.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS15_U8, seg)
    ref_new = ENET(weights=other, precision="fp16")
    want_new = torch.empty_like(seg)
    ref_new.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS15_U8, want_new)
    m.ctx.load_weights(ref_new.blob)                    # the old weights go to the graveyard
    seg.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(seg, want_old)
    fresh = torch.empty_like(seg)
    m.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS15_U8, fresh)
    torch.cuda.synchronize()
    assert torch.equal(fresh, want_new)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gloo_gpu_worker(rank, world, port, total, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from bugcar_image_segmentation_amd.distributed import gather_grids, shard_bounds
        H, W = 96, 128
        model = ENET(weights=enet_spec.build_enet(), precision="fp16")
        bev = synthetic.synthetic_bev(H, W, 300, 300)
        pipe = OccupancyPipeline(model, bev, 3.0, 3.0, 0.05, model_hw=(H, W), streams=2)
        frames = synthetic.road_frames(total, H, W, seed=40)     # every rank holds the same batch
        s, e = shard_bounds(total, world, rank)
        local = pipe.run(torch.from_numpy(frames[s:e]).cuda())
        full = gather_grids(local, total)
        assert full.is_cuda and full.shape[0] == total
        q.put((rank, full.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_sharded_pipeline_two_ranks_one_gpu(gpu, blocks):
    world, total = 2, 7                              # uneven shards: 4 + 3 frames
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_gpu_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=200) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    H, W = 96, 128
    model = ENET(weights=blocks, precision="fp16")
    bev = synthetic.synthetic_bev(H, W, 300, 300)
    one = OccupancyPipeline(model, bev, 3.0, 3.0, 0.05, model_hw=(H, W)).run(
        torch.from_numpy(synthetic.road_frames(total, H, W, seed=40)).to(gpu)).cpu().numpy()
    for r in range(world):
        assert np.array_equal(got[r], one), r


@pytest.mark.timeout(240)
@pytest.mark.parametrize("overlap", [0, 2])
def test_bench_distributed_branch_gloo_one_gpu(gpu, overlap):
    """bench.py's N > 1 branch (process group, in-step gather_grids, max-over-ranks timing, the
    gathered-grid check) run end to end as `python bench.py --gpus 2 --backend gloo` with NO launcher:
    bench.py starts the 2 ranks itself (a torch.distributed.run child, started before it touches the
    GPU); both ranks share this one GPU. --overlap-gather 2 forces the RCCL run's overlapped form (two
    captured steps, the gather on a communication stream) onto the gloo group, the only multi-rank
    group one GPU can host."""
    cmd = [sys.executable, "bench.py", "--gpus", "2",
           "--backend", "gloo", "--steps", "5", "--warmup", "3", "--batch", "4", "--height", "96", "--width", "128",
           "--extras", "0", "--no-cpu-baseline", "--overlap-gather", str(overlap)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=220, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    print(json.dumps({k: line[k] for k in ("value", "n_gpus", "ms_per_step", "config")}))
    assert line["config"]["global_batch"] == 8 and line["config"]["gather_check"] is True
    assert line["n_gpus"] == 2 and line["config"]["ranks"] == 2 and line["config"]["devices"] == 1
    assert line["config"]["backend"].startswith("gloo") and line["value"] > 0
    assert ("overlapped" in line["config"]["parallelism"]) == (overlap == 2)


@pytest.mark.timeout(240)
def test_bench_rccl_branch_one_rank(gpu):
    """bench.py's process-group branch on RCCL (backend nccl: init_process_group with the device id,
    the in-step all_gather_into_tensor of the grids, the all-reduced gathered-grid check and the
    MAX all-reduce of the elapsed time, all on GPU tensors) run by torch.distributed.run as a 1-rank
    job on this one GPU. Two ranks cannot share a GPU under RCCL; this is the N = 8 product path's
    code, executed end to end with a world of one."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "1",
           "--backend", "nccl", "--steps", "3", "--warmup", "1", "--batch", "4", "--height", "96", "--width", "128",
           "--extras", "0", "--no-cpu-baseline"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=220, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    print(json.dumps({k: line[k] for k in ("value", "n_gpus", "ms_per_step", "config")}))
    assert line["config"]["backend"] == "rccl" and line["config"]["gather_check"] is True
    assert "RCCL all-gather" in line["config"]["parallelism"] and line["config"]["ranks"] == 1
    assert line["n_gpus"] == 1 and line["value"] > 0


@pytest.mark.parametrize("prec", ["fp32", "fp16"])
def test_launch_spans_inside_a_captured_step(gpu, blocks, prec):
    """bench.py's in-step timing hook (bugseg_debug_set_spans): every launch of a replayed graph folds
    its workgroups' entry / exit clock into its own slots — each launch's span is positive, launches
    of one stream follow each other, and the armed launches' results equal unarmed ones bit for bit."""
    B, H, W = 4, 96, 128
    m = ENET(weights=blocks, precision=prec)
    dev = torch.device("cuda", 0)
    frames = torch.from_numpy(synthetic.uniform_frames(B, H, W, seed=5)).to(dev)
    seg0 = torch.empty((B, H, W), dtype=torch.uint8, device=dev)
    m.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS3_U8, seg0)
    n = m.ctx.plan_info(B, H, W, N.OUT_CLASS3_U8, bgr_input=True)[0]
    spans = torch.zeros((n, 64, 8), dtype=torch.int64, device=dev)
    seg = torch.empty_like(seg0)
    torch.cuda.synchronize()
    m.ctx.set_spans(spans)
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            m.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS3_U8, seg, torch.cuda.current_stream())
    finally:
        m.ctx.set_spans(None)
    spans[:, :, 0].fill_(-1)
    spans[:, :, 1].zero_()
    g.replay()
    torch.cuda.synchronize()
    sp = spans.cpu().numpy().view(np.uint64)
    st, en = sp[:, :, 0].min(1), sp[:, :, 1].max(1)
    # (with class fusion, BUGSEG_CLS_FUSE=1, op "fused" ran within the previous launch)
    launched = np.array([m.ctx.plan_op(B, H, W, i)[0] != "fused" for i in range(n)])
    st, en = st[launched], en[launched]
    assert (st < np.uint64(2 ** 63)).all() and (en > st).all()          # every launch stamped
    assert (st[1:] >= en[:-1]).all()                                      # stream order
    assert torch.equal(seg, seg0)
    # disarmed: a later eager forward leaves the slots alone
    before = spans.clone()
    m.ctx.forward_bgr(frames, B, H, W, N.OUT_CLASS3_U8, seg)
    torch.cuda.synchronize()
    assert torch.equal(spans, before)
