"""Debug: what the vendor GEMM (torch.matmul -> hipBLASLt on ROCm) reaches on Xception-65's middle-flow
pointwise shape (34,848 pixels x 728 -> 728 channels, bf16, B = 32 at the 513 crop, OS 16), against
the 2.5 PF dense bf16 peak — to decide whether the 1x1 convs should call the library GEMM."""
import torch

dev = torch.device("cuda", 0)
for (M, K, N) in [(34848, 736, 728), (34848, 728, 728), (34848, 736, 736), (135200, 256, 256), (34848, 1024, 1536)]:
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(N, device=dev, dtype=torch.bfloat16)
    for name, f in [("mm", lambda: x @ w.t()), ("addmm+relu", lambda: torch.relu(torch.addmm(b, x, w.t())))]:
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            f()
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        tf = 2 * M * N * K / us / 1e6
        print(f"{name:11s} M={M} K={K} N={N}: {us:8.1f} us  {tf:7.1f} TFLOP/s  {tf / 2500:.3f} of peak", flush=True)
