#!/usr/bin/env python3
"""Convert an official torchvision RAFT checkpoint (.pth state_dict) to the
jax-raft Flax msgpack format (reference scripts/convert_checkpoint.py).

  python scripts/convert_checkpoint.py raft_large_C_T_SKHT_V2.pth raft_large.msgpack

The .pth is read with torch.load(weights_only=True): tensors only, nothing executed.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from jax_raft_amd.cli import convert_main  # noqa: E402

if __name__ == "__main__":
    sys.exit(convert_main())
