#!/usr/bin/env python3
"""Probe: cross-batch pipelining with the prologue launched EAGERLY on a second
stream (Plan.run_segment(0)) while the previous batch's loop graph
(Plan.replay_part(1)) replays on the main stream -- vs the one-graph
pipelining of RaftEngine.pipelined (whose prologue branch the executor only
starts near the end of the loop branch, profiles/r3_b1_pipeline_experiments.txt).

  python tools/pipe_streams.py [--arch raft_large] [--batch 1] [--steps 40]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="raft_large")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--iters", type=int, default=32)
    ap.add_argument("--steps", type=int, default=40)
    a = ap.parse_args()
    import jax_raft_amd as J
    from jax_raft_amd.runtime.engine import RaftEngine

    model = getattr(J, a.arch)()[0].eval().cuda()
    dev = torch.device("cuda", 0)
    eng = RaftEngine(model, dev)
    B, H, W, n = a.batch, 440, 1024, a.iters
    g = torch.Generator(device="cuda").manual_seed(0)
    imgs = [(torch.rand(B, H, W, 3, device=dev, generator=g) * 2 - 1,
             torch.rand(B, H, W, 3, device=dev, generator=g) * 2 - 1) for _ in range(2)]

    # reference: the one-graph pipelining
    for _ in range(5):
        eng.pipelined(*imgs[0], n)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        eng.pipelined(*imgs[k & 1], n)
    torch.cuda.synchronize()
    one_graph = (time.perf_counter() - t0) / a.steps * 1e3
    eng.flush()

    key = (B, H, W, n, True)
    sts = [eng._slot_state(key, s) for s in (0, 1)]
    for st in sts:
        if st.plan.captured_part_iters(1) != n:
            st.plan.capture_part(1, n)
    main_s = torch.cuda.current_stream()
    pro_s = torch.cuda.Stream(priority=0)
    ev_pro = [torch.cuda.Event() for _ in range(2)]
    ev_loop = [torch.cuda.Event() for _ in range(2)]
    for e in ev_loop:
        e.record(main_s)

    def step(k, first=False):
        s = k & 1
        st = sts[s]
        with torch.cuda.stream(pro_s):
            pro_s.wait_event(ev_loop[s])          # this slot's previous loop has read its buffers
            st.inp1.copy_(imgs[k & 1][0])
            st.inp2.copy_(imgs[k & 1][1])
            st.plan.run_segment(0, 0)             # eager prologue on the side stream
            ev_pro[s].record(pro_s)
        if not first:
            p = sts[s ^ 1]
            main_s.wait_event(ev_pro[s ^ 1])
            p.plan.replay_part(1)
            ev_loop[s ^ 1].record(main_s)

    step(0, first=True)
    for k in range(1, 6):
        step(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(6, 6 + a.steps):
        step(k)
    torch.cuda.synchronize()
    two_stream = (time.perf_counter() - t0) / a.steps * 1e3
    print(f"{a.arch} batch {B}: one-graph pipelining {one_graph:.3f} ms/step ({B * 1e3 / one_graph:.1f} pairs/s); "
          f"eager prologue on a 2nd stream + loop graph {two_stream:.3f} ms/step ({B * 1e3 / two_stream:.1f} pairs/s)",
          flush=True)


if __name__ == "__main__":
    main()
