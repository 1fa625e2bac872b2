#!/usr/bin/env python3
"""Phase timing of one training step (BASELINE config 5 shape): encoders
forward, fused loop forward / backward plan / weight gradients, encoder
backward, optimizer.  Each phase is bracketed by device synchronisation, so
the sum is an upper bound of the overlapped step; it shows where a step's
time goes, not the step time itself (tools/train_bench.py)."""
import argparse
import collections
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_raft_amd.train import fused as F  # noqa: E402
from jax_raft_amd.train.trainer import TrainConfig, Trainer  # noqa: E402

T_ = collections.defaultdict(float)


def timed(name, fn):
    def w(*a, **k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn(*a, **k)
        torch.cuda.synchronize()
        T_[name] += time.perf_counter() - t0
        return r
    return w


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=6)
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    cfg = TrainConfig(batch=a.batch, iters=a.iters, steps=a.steps + 2, log_every=10 ** 9)
    tr = Trainer(cfg)
    m = tr.model
    from jax_raft_amd.train import fused_encoder as FE

    m.feature_encoder.forward = timed("fe_fwd (autograd)", m.feature_encoder.forward)
    m.context_encoder.forward = timed("ce_fwd (autograd)", m.context_encoder.forward)
    FE.EncoderTrain.forward = timed("encoders_fwd (plans)", FE.EncoderTrain.forward)
    FE.EncoderTrain.run_backward = timed("encoders_bwd (plan + wgrad)", FE.EncoderTrain.run_backward)
    F.FusedLoop.forward_prepared = timed("loop_fwd", F.FusedLoop.forward_prepared)
    from jax_raft_amd.train import loss as L

    L._SeqLoss.forward = staticmethod(timed("loss_fwd", L._SeqLoss.forward))
    orig_backward = F.FusedLoop.backward

    def bwd(self, gout, gen, fe_dy=None):
        if gen != self.gen or self.done_gen == gen:
            return orig_backward(self, gout, gen, fe_dy)
        self.done_gen = gen
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        self.gout.copy_(gout)
        self._run(self.plan_b)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        r = self._finish(fe_dy)
        torch.cuda.synchronize()
        T_["loop_bwd_plan"] += t1 - t0
        T_["loop_wgrad_finish"] += time.perf_counter() - t1
        return r

    F.FusedLoop.backward = bwd
    tr.opt.step = timed("optimizer", tr.opt.step)
    batch = tr.batch_for(0)
    for _ in range(2):
        tr.train_step(batch)
    T_.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.train_step(batch)
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t0) / a.steps * 1e3
    out = {k: round(v / a.steps * 1e3, 2) for k, v in T_.items()}
    out["other (loss, encoder backward, clip, ...)"] = round(tot - sum(out.values()), 2)
    out["step_ms (serialised phases)"] = round(tot, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
