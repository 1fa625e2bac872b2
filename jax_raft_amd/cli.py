"""Console entry points (reference CLIs: scripts/convert_checkpoint.py:59-68,
scripts/validate_sintel.py:250-263).  ``scripts/*.py`` are thin wrappers so the
repository works uninstalled; ``pip install .`` exposes the same functions as
``jax-raft-amd-convert`` / ``jax-raft-amd-validate``."""
from __future__ import annotations

import argparse
import json
import os
import sys
from typing import Optional, Sequence


def convert_main(argv: Optional[Sequence[str]] = None) -> int:
    """``convert <input.pth> <output.msgpack>``: torchvision state_dict -> Flax msgpack
    (read with ``torch.load(weights_only=True)``: tensors only, nothing executed)."""
    from .utils.checkpoint import convert_checkpoint

    argv = list(sys.argv[1:] if argv is None else argv)
    if len(argv) != 2:
        print("Usage: python convert_checkpoint.py <input_file> <output_file>")
        return 1
    if not argv[1].endswith(".msgpack"):
        print("output file must end in .msgpack")
        return 1
    convert_checkpoint(argv[0], argv[1])
    return 0


def validate_main(argv: Optional[Sequence[str]] = None) -> int:
    """Sintel (train split) EPE / 1-3-5px / FPS of raft_large and/or raft_small,
    data-parallel over RCCL when launched by torchrun."""
    import torch

    from . import raft_large, raft_small
    from .eval.sintel import validate_sintel

    ap = argparse.ArgumentParser(prog="validate_sintel")
    ap.add_argument("data_root")
    ap.add_argument("--model", choices=["raft_large", "raft_small", "both"], default="both")
    ap.add_argument("--weights", default=None, help="Flax msgpack checkpoint (default: pretrained release file)")
    ap.add_argument("--iters", type=int, default=32)
    ap.add_argument("--max-pairs", type=int, default=None)
    ap.add_argument("--batch-size", type=int, default=1, help="pairs per forward (1 = the reference protocol)")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"],
                    help="native engine precision (fp32 = the reference's own, runtime/engine_f32.py)")
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--json", default=None)
    args = ap.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        from .parallel.dp import init_distributed

        init_distributed("gloo" if args.cpu else None)
    device = (torch.device("cpu") if args.cpu or not torch.cuda.is_available()
              else torch.device("cuda", torch.cuda.current_device()))
    names = ["raft_large", "raft_small"] if args.model == "both" else [args.model]
    out = {}
    for name in names:
        factory = raft_large if name == "raft_large" else raft_small
        model, _ = factory(weights=args.weights) if args.weights else factory(pretrained=True)
        out[name] = validate_sintel(model, args.data_root, iters=args.iters, device=device, max_pairs=args.max_pairs,
                                    batch_size=args.batch_size,
                                    **({} if device.type == "cpu" else dict(precision=args.precision)))
    if args.json and (world == 1 or torch.distributed.get_rank() == 0):
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)
    if world > 1:
        torch.distributed.destroy_process_group()
    return 0
