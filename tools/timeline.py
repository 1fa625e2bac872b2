#!/usr/bin/env python3
"""Iteration timeline from a rocprofv3 kernel trace (rocpd .db or CSV): the
kernels of one refinement iteration of the last forward (between two
corr_lookup starts) with start/end relative to the iteration start, plus the
GPU busy/idle split of the whole last forward."""
import argparse
import re

from kernel_breakdown import _load


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\(.*", "", n)
    n = n.replace("void ", "")
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)(\w+)", n)
    if m:
        n = m.group(2)[: int(m.group(1))]
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--iter", type=int, default=10)
    ap.add_argument("--prologue", action="store_true", help="list the prologue kernels instead")
    a = ap.parse_args()
    rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in _load(a.trace)),
                  key=lambda r: r[1])
    preps = [i for i, r in enumerate(rows) if "prep_images" in r[0]]
    seg = rows[preps[-1]:]
    busy = idle = 0
    cs, ce = seg[0][1], seg[0][2]
    for _, s, e in seg[1:]:
        if s > ce:
            busy += ce - cs
            idle += s - ce
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print(f"forward wall {(seg[-1][2] - seg[0][1]) / 1e6:.3f} ms  busy {busy / 1e6:.3f}  idle {idle / 1e6:.3f}")
    lk = [i for i, r in enumerate(seg) if "corr_lookup" in r[0]]
    print(f"prologue {(seg[lk[0]][1] - seg[0][1]) / 1e6:.3f} ms; loop {(seg[-1][2] - seg[lk[0]][1]) / 1e6:.3f} ms; "
          f"per iteration {(seg[lk[-1]][1] - seg[lk[0]][1]) / 1e3 / (len(lk) - 1):.1f} us")
    it = seg[:lk[0] + 1] if a.prologue else seg[lk[a.iter]:lk[a.iter + 1] + 1]
    t0 = it[0][1]
    for n, s, e in it:
        print(f"{(s - t0) / 1e3:7.1f} {(e - t0) / 1e3:7.1f} {(e - s) / 1e3:6.1f}  {short(n)}")


if __name__ == "__main__":
    main()
