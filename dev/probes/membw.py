"""HBM write/copy bandwidth probe (reference point for store-bound kernels)."""
import torch

x = torch.empty(250 * 2**20, dtype=torch.bfloat16, device="cuda")  # 500 MB
y = torch.empty_like(x)
for name, fn, nbytes in (("fill 500MB", lambda: x.fill_(1.0), x.numel() * 2),
                         ("copy 500MB", lambda: y.copy_(x), 2 * x.numel() * 2)):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        fn()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 100
    print(f"{name}: {us:8.1f} us  {nbytes / us / 1e6:.2f} TB/s")
