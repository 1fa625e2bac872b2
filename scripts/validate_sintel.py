#!/usr/bin/env python3
"""Sintel (train) validation of raft_large / raft_small: EPE, 1/3/5px, FPS.

Equivalent of the reference scripts/validate_sintel.py (its __main__ runs
both models with pretrained weights at 32 iterations).  Usage:

  python scripts/validate_sintel.py /path/to/Sintel [--model raft_large] [--weights w.msgpack]
      [--iters 32] [--max-pairs N]

Multi-GPU (data-parallel, one rank per GPU over RCCL):
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 scripts/validate_sintel.py /path/to/Sintel
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_raft_amd import raft_large, raft_small  # noqa: E402
from jax_raft_amd.eval.sintel import validate_sintel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("data_root")
    ap.add_argument("--model", choices=["raft_large", "raft_small", "both"], default="both")
    ap.add_argument("--weights", default=None, help="Flax msgpack checkpoint (default: pretrained release file)")
    ap.add_argument("--iters", type=int, default=32)
    ap.add_argument("--max-pairs", type=int, default=None)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cpu") if args.cpu or not torch.cuda.is_available() else torch.device("cuda", torch.cuda.current_device())
    names = ["raft_large", "raft_small"] if args.model == "both" else [args.model]
    out = {}
    for name in names:
        factory = raft_large if name == "raft_large" else raft_small
        if args.weights:
            model, _ = factory(weights=args.weights)
        else:
            model, _ = factory(pretrained=True)
        out[name] = validate_sintel(model, args.data_root, iters=args.iters, device=device, max_pairs=args.max_pairs)
    if args.json and (world == 1 or torch.distributed.get_rank() == 0):
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
