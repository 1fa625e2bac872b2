"""GPU time per forward (back-to-back, host ahead) for a sequence of engine
modes built in one process, e.g. `probe_modes.py 4 final all final`."""
import sys

import torch

sys.path.insert(0, ".")
from jax_raft_amd import raft_large  # noqa: E402

m, _ = raft_large(seed=0)
m = m.cuda().eval()
B = int(sys.argv[1])
i1 = torch.rand(B, 440, 1024, 3, device="cuda") * 2 - 1
i2 = torch.rand(B, 440, 1024, 3, device="cuda") * 2 - 1
for mode in sys.argv[2:]:
    if mode == "clear":  # drop the autotune cache and the engines (fresh tuning, fresh plans)
        from jax_raft_amd.runtime import engine as _e
        _e._TUNE_CACHE.clear()
        m._engines = {}
        continue
    if mode == "drop":  # drop the built plans, keep engines + autotune cache (plans rebuilt from the cache)
        for e in m._engines.values():
            e._states.clear()
        continue
    if mode == "dumptune":
        from jax_raft_amd.runtime import engine as _e
        for k, v in sorted(_e._TUNE_CACHE.items(), key=str):
            print("  tune", k[:8], k[8:10], "->", v)
        continue
    kw = dict(return_all_iters=mode.startswith("all"), streams="nostreams" not in mode)
    for _ in range(3):
        m(i1, i2, num_flow_updates=32, **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(100_000_000)
    e0.record()
    for _ in range(10):
        o = m(i1, i2, num_flow_updates=32, **kw)
    e1.record()
    torch.cuda.synchronize()
    print(f"{mode:16s} {e0.elapsed_time(e1) / 10:.2f} ms/forward  |flow| {o[-1].abs().mean().item():.3g}", flush=True)
