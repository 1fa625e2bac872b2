"""Probe: ways to reduce an NHWC bf16 gradient (M x C) to an fp32 bias grad."""
import torch, time

def t(fn, n=50):
    for _ in range(5): fn()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / n * 1e6

for M, C in ((18432, 128), (18432, 256), (589824, 64), (147456, 96)):
    gy = torch.randn(M, C, device="cuda").to(torch.bfloat16)
    ref = gy.float().sum(0)
    ones = torch.ones(1, M, device="cuda", dtype=torch.bfloat16)
    S = 64
    cands = {
        "sum_dtype": lambda: gy.sum(0, dtype=torch.float32),
        "float_sum": lambda: gy.float().sum(0),
        "split_sum": lambda: gy.reshape(S, M // S, C).sum(1, dtype=torch.float32).sum(0),
        "gemv_f32": lambda: torch.mm(ones, gy, out_dtype=torch.float32)[0],
        "split_bmm": lambda: torch.bmm(ones[:, : M // S].expand(S, 1, M // S), gy.reshape(S, M // S, C), out_dtype=torch.float32).sum(0)[0],
    }
    for k, f in cands.items():
        err = ((f() - ref).abs().max() / ref.abs().max()).item()
        print(f"M={M} C={C} {k:10s} {t(f):8.1f} us  relerr={err:.1e}", flush=True)
