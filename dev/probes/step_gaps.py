#!/usr/bin/env python3
"""GPU busy / idle split of one training step from a rocprofv3 kernel trace
(steps delimited by a marker kernel), with the largest idle gaps and the
kernel that ended each one."""
import argparse

from kernel_breakdown import _load


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="seq_loss_kernel")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in _load(a.trace)),
                  key=lambda r: r[1])
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    seg = rows[marks[-3]:marks[-2]]
    busy = idle = 0
    cs, ce = seg[0][1], seg[0][2]
    gaps = []
    for n, s, e in seg[1:]:
        if s > ce:
            busy += ce - cs
            idle += s - ce
            gaps.append((s - ce, n))
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print(f"step wall {(seg[-1][2] - seg[0][1]) / 1e6:.2f} ms  busy {busy / 1e6:.2f}  idle {idle / 1e6:.2f}  "
          f"kernels {len(seg)}")
    for g, n in sorted(gaps, reverse=True)[: a.top]:
        print(f"{g / 1e3:8.1f} us idle before {n[:100]}")


if __name__ == "__main__":
    main()
