"""Host-side enqueue cost of one forward (graph replay vs eager plan, lanes on/off):
the batch-1 forward is host-bound when this exceeds its GPU time."""
import sys
import time

import torch

sys.path.insert(0, ".")
from jax_raft_amd import raft_large  # noqa: E402

m, _ = raft_large(seed=0)
m = m.cuda().eval()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
i1 = torch.rand(B, 440, 1024, 3, device="cuda") * 2 - 1
i2 = torch.rand(B, 440, 1024, 3, device="cuda") * 2 - 1
for kw in (dict(use_graph=True), dict(use_graph=True, streams=False), dict(use_graph=False),
           dict(use_graph=False, streams=False)):
    for _ in range(3):
        m(i1, i2, num_flow_updates=32, **kw)
    torch.cuda.synchronize()
    n = 10
    t0 = time.perf_counter()
    for _ in range(n):
        m(i1, i2, num_flow_updates=32, **kw)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    # GPU-only time: one forward behind a long spin so the host is far ahead
    torch.cuda._sleep(200_000_000)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        m(i1, i2, num_flow_updates=32, **kw)
    e1.record()
    torch.cuda.synchronize()
    eng = m.engine(torch.device("cuda", 0), **{k: v for k, v in kw.items() if k != "use_graph"}) if False else None
    print(kw, f"host {1e3 * (t1 - t0) / n:.2f} ms  wall {1e3 * (t2 - t0) / n:.2f} ms  "
          f"gpu(back-to-back, host ahead) {e0.elapsed_time(e1) / n:.2f} ms", flush=True)
