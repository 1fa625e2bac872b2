#!/usr/bin/env python3
"""Minimal usage example (reference examples/demo.py): estimate the flow
between two frames and save a colour-coded visualisation.

  python examples/demo.py frame1.png frame2.png [--weights raft_small.msgpack] [--out flow.png]

Without frames on the command line a synthetic translated pair is used.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from jax_raft_amd import raft_small  # noqa: E402
from jax_raft_amd.utils.flow_io import InputPadder, flow_to_color, normalize_image, read_image  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("frames", nargs="*")
    ap.add_argument("--weights", default=None)
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--out", default="flow.png")
    args = ap.parse_args()
    if len(args.frames) == 2:
        image1, image2 = normalize_image(read_image(args.frames[0])), normalize_image(read_image(args.frames[1]))
    else:
        rng = np.random.default_rng(0)
        base = rng.integers(0, 255, (260, 340, 3), dtype=np.uint8)
        image1, image2 = normalize_image(base[2:258, 2:338]), normalize_image(base[:256, 4:340])
    padder = InputPadder(image1.shape, channels_last=True)
    image1, image2 = padder.pad(image1, image2)
    raft, variables = raft_small(weights=args.weights) if args.weights else raft_small()
    if torch.cuda.is_available():
        raft = raft.cuda()
        image1, image2 = image1.cuda(), image2.cuda()
    flow_predictions = raft.apply(variables if not torch.cuda.is_available() else raft.variables(), image1, image2,
                                  train=False, num_flow_updates=args.iters)
    flow = padder.unpad(flow_predictions[-1])
    print("Flow shape:", tuple(flow.shape))
    from PIL import Image

    Image.fromarray(flow_to_color(flow[0].detach().float().cpu().numpy())).save(args.out)
    print("saved", args.out)


if __name__ == "__main__":
    main()
