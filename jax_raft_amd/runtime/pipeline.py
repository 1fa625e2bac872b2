"""Host->device input pipelining for batched inference.

The reference times each pair with its host->device transfer in the loop
(scripts/validate_sintel.py:185-186 of jax-raft): a synchronous copy that the
GPU waits for.  A serving loop on MI355X overlaps that copy with the previous
batch's forward instead: `InputPrefetcher` owns a dedicated copy stream and a
ring of device input buffers; batch i+1's pinned-host -> device copy runs on
the copy engine while batch i's hipGraph runs on the compute stream, and
events order both directions (a buffer is refilled only after the forward that
read it has consumed it, and a forward starts only after its copy landed).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch


class InputPrefetcher:
    """Ring of ``depth`` device buffer sets, filled on a private copy stream.

    Usage::

        pf = InputPrefetcher([(B, H, W, 3), (B, H, W, 3)], device)
        pf.put(0, [img1_pinned, img2_pinned])
        for i in range(n):
            a, b = pf.get(i)                   # compute stream waits for copy i
            out = model(a, b, ...)
            pf.release(i)                      # the forward's reads are ordered before reuse
            if i + 1 < n:
                pf.put(i + 1, next_host_batch)  # overlaps with forward i
    """

    def __init__(self, shapes: Sequence[Tuple[int, ...]], device, dtype=torch.float32, depth: int = 2):
        self.device = torch.device(device)
        self.depth = depth
        self.stream = torch.cuda.Stream(device=self.device)
        self.bufs: List[List[torch.Tensor]] = [[torch.empty(s, dtype=dtype, device=self.device) for s in shapes]
                                               for _ in range(depth)]
        self.ready = [torch.cuda.Event() for _ in range(depth)]
        self.free = [torch.cuda.Event() for _ in range(depth)]
        self._released = [True] * depth

    def put(self, i: int, host: Sequence[torch.Tensor]) -> None:
        """Start copying ``host`` tensors (pinned for true overlap) into slot i % depth."""
        k = i % self.depth
        with torch.cuda.stream(self.stream):
            if not self._released[k]:
                raise RuntimeError(f"prefetch slot {k} refilled before release()")
            self.stream.wait_event(self.free[k])
            for dst, src in zip(self.bufs[k], host):
                dst.copy_(src, non_blocking=True)
            self.ready[k].record(self.stream)
            self._released[k] = False

    def get(self, i: int) -> List[torch.Tensor]:
        """Device tensors of batch i; the current stream waits for their copy."""
        k = i % self.depth
        torch.cuda.current_stream(self.device).wait_event(self.ready[k])
        return self.bufs[k]

    def release(self, i: int) -> None:
        """Mark batch i's buffers reusable once the work queued so far on the current stream is done."""
        k = i % self.depth
        self.free[k].record(torch.cuda.current_stream(self.device))
        self._released[k] = True
