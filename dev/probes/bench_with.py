#!/usr/bin/env python3
"""Run bench.py with engine class attributes overridden (A/B of the lowering choices that are
class attributes, jax_raft_amd/knobs.py):

    python dev/probes/bench_with.py MASK_PARITY=1 GRU=halo -- --extras off --steps 20
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from jax_raft_amd.runtime.engine import RaftEngine  # noqa: E402


def main():
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    for item in argv[:cut]:
        k, v = item.split("=")
        old = getattr(RaftEngine, k)
        val = (v not in ("0", "false", "False")) if isinstance(old, bool) else type(old)(v)
        setattr(RaftEngine, k, val)
        print(f"RaftEngine.{k} = {val!r} (default {old!r})", file=sys.stderr, flush=True)
    sys.argv = [os.path.join(ROOT, "bench.py")] + argv[cut + 1:]
    runpy.run_path(sys.argv[0], run_name="__main__")


if __name__ == "__main__":
    main()
