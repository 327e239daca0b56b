"""Benchmark of BASELINE config 4: DeepLabV3 (MobileNetV2, output stride 8, ASPP) at 513x513 on MI355X;
``--backbone xception_65`` measures the other model-zoo export, DeepLabV3+ over Xception-65 (output
stride 16, separable ASPP 6/12/18, decoder at stride 4).

One "step" = the DeepLab plugin's forward (models.DeepLabV3.predict_device: pad + normalise,
backbone, ASPP, logits, bilinear resize to 513x513, argmax -> int64) over one batch of synthetic
513x513 RGB frames already resident in HBM. bench.py stays the headline (ENet -> BEV occupancy
grid); this prints ONE JSON line of the same shape for config 4. With WORLD_SIZE > 1 (torchrun)
frames shard across ranks with no collective (weak scaling).

`roofline` describes the dominant kernel tag (largest total time per forward), timed per launch
with HIP events on the stream the kernels run on (bugseg_dl_launch_op): achieved = the launch's
algorithmic bytes (input read once, output written once, residual read, weights once;
deeplab_spec.lower) / its average duration, against 8 TB/s; `forward` adds whole-forward bytes,
flops and the MFMA fraction; `traffic` is the PMC-measured HBM bytes per launch of that op tag from
the committed profile (profiles/dl_pmc_traffic.json, scripts/dl_pmc_summary.py), when it was taken
at the same batch. The CPU baseline is the oracle (PyTorch-CPU fp32, TF semantics) on a bounded
sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0
MFMA_PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3}


def parse():
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=64, help="frames per GPU (measured: 16 / 32 / 64 -> 6.72k / 6.88k / 7.05k frames/s)")
    p.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--backbone", default="mobilenet_v2", choices=["mobilenet_v2", "xception_65", "resnet_v1_101_beta"])
    return p.parse_args()


def cpu_baseline(net, budget_s):
    """The oracle on a bounded sample, on every CPU the process is granted (bench.cpu_cores)."""
    from bench import cpu_cores
    from oracle import deeplab_oracle as O
    x = np.random.default_rng(7).integers(0, 256, (1, net.crop, net.crop, 3), dtype=np.uint8)
    threads, facts = cpu_cores()
    torch.set_num_threads(threads)
    O.predict(net, x, dtype=torch.float32)   # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        O.predict(net, x, dtype=torch.float32)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s and n >= 2:
            break
    return {"value": round(n / el, 3), "unit": "frames/s", "cores": threads, "kind": "port", **facts,
            "sample": f"{n} frames of the same workload ({net.crop}x{net.crop}, fp32 PyTorch-CPU oracle with TF "
                      f"semantics), {el:.1f} s at {threads} threads, one frame per call"}


def pmc_traffic(tag, batch, backbone="mobilenet_v2"):
    """HBM bytes per launch of op tag `tag` from the committed PMC summary
    (profiles/dl_pmc_traffic.json, written by scripts/dl_pmc_summary.py from rocprofv3 FETCH_SIZE /
    WRITE_SIZE passes of this script at the same batch), or None."""
    if backbone not in ("mobilenet_v2", "xception_65"):
        return None
    p = os.path.join(ROOT, "profiles", "dl_pmc_traffic_xception.json" if backbone == "xception_65" else "dl_pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if int(d.get("batch", -1)) != batch:
        return None
    v = d.get("per_launch_bytes", {}).get(tag)
    return None if v is None else round(float(v))


WORKLOAD = {"mobilenet_v2": "DeepLabV3 MobileNetV2 OS8 + ASPP (image pooling + 1x1)",
            "xception_65": "DeepLabV3+ Xception-65 OS16 + separable ASPP 6/12/18 + decoder OS4",
            "resnet_v1_101_beta": "DeepLabV3 ResNet-v1-101-beta OS16 + dense ASPP 6/12/18"}


def measure(dev, B, steps, warmup, precision, world=1, rank=0, backbone="mobilenet_v2"):
    """Time `steps` DeepLab forwards of B frames (barrier + sync on both sides, max over ranks), then
    every launch of the plan with HIP events (untimed). Returns (el seconds, model, per-tag table,
    per-op list, forward us)."""
    from bugcar_image_segmentation_amd.models import DeepLabV3

    # BUGSEG_DL_FUSE_PREP=0 (A/B knob): the separate padding / normalisation launch instead of the stem's fused loads
    model = DeepLabV3(precision=precision, backbone=backbone, fuse_prep=os.environ.get("BUGSEG_DL_FUSE_PREP", "1") != "0")
    C = model.net.crop
    frames = torch.from_numpy(np.random.default_rng(rank).integers(0, 256, (B, C, C, 3), dtype=np.uint8)).to(dev)
    out = torch.empty((B, C, C), dtype=torch.int64, device=dev)

    for _ in range(warmup):
        model.predict_device(frames, out=out)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        model.predict_device(frames, out=out)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    # per-launch HIP-event timing of the plan the timed region ran (untimed region)
    stream = torch.cuda.current_stream()
    info = model.plan_info
    reps = max(3, min(10, steps))
    per = defaultdict(lambda: {"launches": 0, "us": 0.0, "bytes": 0.0, "flops": 0.0})
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fwd_us = 0.0
    per_op = []
    for i, (tag, flops, nbytes) in enumerate(info["per_op"]):
        model.ctx.launch_op(i, stream)
        evs[0].record(stream)
        for _ in range(reps):
            model.ctx.launch_op(i, stream)
        evs[1].record(stream)
        evs[1].synchronize()
        us = evs[0].elapsed_time(evs[1]) * 1e3 / reps
        fwd_us += us
        per_op.append([tag, round(us, 2), round(nbytes / (us * 1e-6) / 1e9, 1)])
        d = per[tag]
        d["launches"] += 1
        d["us"] += us
        d["bytes"] += nbytes
        d["flops"] += flops
    return el, model, per, per_op, fwd_us


def roofline(model, per, fwd_us, B, precision, backbone="mobilenet_v2"):
    """Dominant op tag's roofline. MobileNetV2 is HBM-bound (its dominant tag moves ~1 B per 2 flops);
    Xception-65's dominant tag is the pointwise 1x1 GEMMs (108 GFLOP per frame), priced against the
    dense MFMA peak of the dtype."""
    info = model.plan_info
    tag, k = max(per.items(), key=lambda kv: kv[1]["us"])
    achieved = k["bytes"] / (k["us"] * 1e-6) / 1e9
    peak_tf = MFMA_PEAK_TFLOPS[precision]
    tflops = k["flops"] / (k["us"] * 1e-6) / 1e12
    mfma = backbone != "mobilenet_v2"
    bound = ({"bound": "mfma", "achieved": round(tflops, 1), "peak": peak_tf, "unit": "TFLOP/s",
              "frac": round(tflops / peak_tf, 4), "hbm_achieved_gbs": round(achieved, 1),
              "hbm_frac": round(achieved / HBM_PEAK_GBS, 4)} if mfma else
             {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
              "frac": round(achieved / HBM_PEAK_GBS, 4)})
    return {
        **bound, "traffic": pmc_traffic(tag, B, backbone),
        "kernel": f"{tag}: dominant kernel tag ({k['launches']} launches, {k['us']:.0f} us of {fwd_us:.0f} us "
                  f"per forward); {k['bytes'] / k['launches'] / 1e6:.1f} MB per launch (input once + output "
                  f"once + residual + weights); {k['flops'] / (k['us'] * 1e-6) / 1e12:.1f} TFLOP/s "
                  f"({k['flops'] / (k['us'] * 1e-6) / 1e12 / peak_tf:.3f} of the dense {precision} MFMA peak)",
        "forward": {"launches": len(info["per_op"]), "us": round(fwd_us, 1), "frames": B,
                    "bytes_per_frame": round(info["bytes"] / B), "flops_per_frame": round(info["flops"] / B),
                    "achieved_gbs": round(info["bytes"] / (fwd_us * 1e-6) / 1e9, 1),
                    "mfma_tflops": round(info["flops"] / (fwd_us * 1e-6) / 1e12, 2),
                    "mfma_frac": round(info["flops"] / (fwd_us * 1e-6) / 1e12 / peak_tf, 4)},
    }


def kernel_summary(per):
    return {t: {"launches": v["launches"], "us": round(v["us"], 1),
                "GBps": round(v["bytes"] / (v["us"] * 1e-6) / 1e9, 1),
                "TFLOPs": round(v["flops"] / (v["us"] * 1e-6) / 1e12, 2)}
            for t, v in sorted(per.items(), key=lambda kv: -kv[1]["us"])}


def record(dev, B, steps, warmup, precision, cpu_seconds=0.0, backbone="mobilenet_v2"):
    """The config-4 sub-record bench.py adds to its line (one GPU, measured after its timed loop)."""
    el, model, per, _per_op, fwd_us = measure(dev, B, steps, warmup, precision, backbone=backbone)
    res = {"value": round(B * steps / el, 2), "unit": "frames/s", "ms_per_step": round(el / steps * 1e3, 4),
           "steps": steps, "dtype": precision, "per_gpu_batch": B, "crop": model.net.crop,
           "workload": f"config4: {WORKLOAD[backbone]}, 513x513 u8 RGB -> SemanticPredictions int64",
           "roofline": roofline(model, per, fwd_us, B, precision, backbone)}
    if cpu_seconds > 0:
        res["cpu_baseline"] = cpu_baseline(model.net, cpu_seconds)
    del model
    return res


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    B = a.batch
    el, model, per, per_op, fwd_us = measure(dev, B, a.steps, a.warmup, a.precision, world, rank, a.backbone)
    C = model.net.crop

    if rank == 0:
        value = B * world * a.steps / el
        res = {
            "metric": f"frames/sec {'DeepLabV3+' if a.backbone == 'xception_65' else 'DeepLabV3'} 513x513 -> "
                      "SemanticPredictions (synthetic), whole job",
            "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(el / a.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": a.precision,
            "data": f"synthetic (uniform u8 RGB frames, seed=rank; random-init {a.backbone} weights, "
                    f"seed {model.net.meta.get('seed')})",
            "config": {"workload": f"config4: {WORKLOAD[a.backbone]}, {C}x{C}, batch {B} per GPU, "
                                   "pad/normalise + forward + bilinear resize + argmax int64",
                       "global_batch": B * world, "per_gpu_batch": B, "crop": C,
                       "parallelism": f"frame-sharded dp{world}"},
            "roofline": roofline(model, per, fwd_us, B, a.precision, a.backbone),
            "kernels": kernel_summary(per),
            "per_op": per_op,
        }
        if not a.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(model.net, a.cpu_baseline_seconds)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
