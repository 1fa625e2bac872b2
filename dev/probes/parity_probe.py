#!/usr/bin/env python3
"""Engine vs fp32 golden EPE per iteration over tests/test_engine_gpu.py::test_engine_matches_golden's
configurations (the measured basis of that test's bound)."""
import sys, torch
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from test_engine_gpu import _inputs, _epe
from jax_raft_amd import raft_large, raft_small
for factory in (raft_small, raft_large):
    for use_graph in (False, True):
        for B, W in ((2, 160), (2, 256), (4, 256)):
            torch.manual_seed(0)
            model, variables = factory()
            i1, i2 = _inputs(B, 128, W)
            ref = model.apply(variables, i1, i2, train=False, num_flow_updates=4)
            model = model.cuda()
            out = model(i1.cuda(), i2.cuda(), num_flow_updates=4, use_graph=use_graph).cpu()
            mag = ref.norm(dim=-1).mean().item()
            es = [_epe(out[it], ref[it]) for it in range(4)]
            print(factory.__name__, use_graph, B, W, "mag %.3f" % mag, "epe", " ".join("%.4f" % e for e in es),
                  "max rel %.4f" % (max(es) / mag), flush=True)
