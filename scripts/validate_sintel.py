#!/usr/bin/env python3
"""Sintel (train) validation of raft_large / raft_small: EPE, 1/3/5px, FPS.

Equivalent of the reference scripts/validate_sintel.py (its __main__ runs
both models with pretrained weights at 32 iterations).  Usage:

  python scripts/validate_sintel.py /path/to/Sintel [--model raft_large] [--weights w.msgpack]
      [--iters 32] [--max-pairs N]

Multi-GPU (data-parallel, one rank per GPU over RCCL):
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 scripts/validate_sintel.py /path/to/Sintel
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from jax_raft_amd.cli import validate_main  # noqa: E402

if __name__ == "__main__":
    sys.exit(validate_main())
