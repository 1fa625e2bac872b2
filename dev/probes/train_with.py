#!/usr/bin/env python3
"""tools/train_bench.py with fused-training class attributes overridden (A/B):
    python dev/probes/train_with.py FusedModel.SIDE_ENCODER=0 -- --steps 20"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from jax_raft_amd.train import fused, fused_encoder  # noqa: E402


def main():
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    for item in argv[:cut]:
        k, v = item.split("=")
        cls, attr = k.split(".")
        obj = getattr(fused, cls, None) or getattr(fused_encoder, cls)
        old = getattr(obj, attr)
        val = (v not in ("0", "false", "False")) if isinstance(old, bool) else type(old)(v)
        setattr(obj, attr, val)
        print(f"{k} = {val!r} (default {old!r})", file=sys.stderr, flush=True)
    sys.argv = [os.path.join(ROOT, "tools", "train_bench.py")] + argv[cut + 1:]
    runpy.run_path(sys.argv[0], run_name="__main__")


if __name__ == "__main__":
    main()
