#!/usr/bin/env python3
"""Mean per-dispatch PMC values of the kernels whose name contains a filter (default "conv")
from per-pass rocprofv3 --pmc output dirs named <case>_g<pass>."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
pat = sys.argv[2] if len(sys.argv) > 2 else "conv"   # kernel-name filter
for d in sorted(glob.glob(os.path.join(root, "*_g1"))):
    base = d[:-3]
    vals = collections.defaultdict(list)
    for g in sorted(glob.glob(base + "_g*")):
        for f in glob.glob(os.path.join(g, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if pat not in r.get("Kernel_Name", ""):
                    continue
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    line = " ".join(f"{k}={sum(v) / len(v):.3g}" for k, v in sorted(vals.items()))
    print(os.path.basename(base), line)
