#!/usr/bin/env python3
"""Render tools/drift.py's JSON (per-iteration EPE of the native engine vs the
fp32 golden model at 440x1024, 32 iterations) as the markdown table of
profiles/r5_drift.md.

    python tools/drift_report.py gpurun_out/r5_drift/drift.json > /tmp/table.md   # -> profiles/r5_drift.md
"""
import json
import sys


def main():
    recs = json.load(open(sys.argv[1]))
    its = (1, 2, 4, 8, 12, 16, 24, 32)
    print("| arch | variant | " + " | ".join(f"it {i}" for i in its) + " | rel. EPE it 32 | |golden flow| it 32 | "
          "final EPE vs fixture |")
    print("|---|---|" + "---|" * len(its) + "---|---|---|")
    for r in recs:
        cells = " | ".join(f"{r['epe'][i - 1]:.4f}" for i in its)
        print(f"| {r['arch']} | {r['variant']} | {cells} | {r['rel'][-1]:.2e} | {r['mean_mag'][-1]:.2f} | "
              f"{r['final_epe_vs_fixture']:.4f} |")
    print()
    print("Relative EPE (EPE / mean |golden flow|) per iteration:")
    print()
    print("| arch | variant | " + " | ".join(f"it {i}" for i in its) + " |")
    print("|---|---|" + "---|" * len(its))
    for r in recs:
        print(f"| {r['arch']} | {r['variant']} | " + " | ".join(f"{r['rel'][i - 1]:.2e}" for i in its) + " |")


if __name__ == "__main__":
    main()
