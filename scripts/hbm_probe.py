"""HBM write / read / copy bandwidth of plain torch ops on one MI355X (what the DeepLab 1x1
expansions' 2 TB/s of writes should be compared with). python scripts/hbm_probe.py"""
import torch

dev = torch.device("cuda:0")
n = 1 << 30   # 1 GiB
x = torch.empty(n // 2, dtype=torch.bfloat16, device=dev)
y = torch.empty_like(x)


def t(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


w = t(lambda: x.fill_(1.0))
r = t(lambda: x.sum())
c = t(lambda: y.copy_(x))
print(f"write {n / w / 1e12:.2f} TB/s  read {n / r / 1e12:.2f} TB/s  copy {2 * n / c / 1e12:.2f} TB/s (read+write)")
