#!/usr/bin/env python3
"""Prologue timeline of the last forward in a rocprofv3 kernel trace (CSV):
every kernel from the last ``prep_images`` to the first correlation lookup
after it, with start / end relative to the prep start and its hardware queue
(one per plan lane), plus per-queue busy time and the critical chain's end
(the correlation pyramid)."""
import argparse
import csv
import re
from collections import defaultdict


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\(.*", "", n).replace("void ", "")
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)(\w+)", n)
    if m:
        n = m.group(2)[: int(m.group(1))]
    return n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
                         int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))))
    rows.sort(key=lambda r: r[1])
    preps = [i for i, r in enumerate(rows) if "prep_images" in r[0]]
    i0 = preps[-2] if len(preps) > 1 else preps[-1]   # the last complete forward
    seg = []
    for r in rows[i0:]:
        if "lookup" in r[0]:
            break
        seg.append(r)
    t0 = seg[0][1]
    busy = defaultdict(float)
    for name, s, e, q, wg in seg:
        busy[q] += (e - s) / 1e3
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} us  q{q:>3} wg={wg:<7} {short(name)}")
    end = max(e for _, _, e, _, _ in seg)
    print(f"\nprologue span {(end - t0) / 1e3:.1f} us; kernels {len(seg)}")
    for q, b in sorted(busy.items()):
        print(f"  queue {q}: busy {b:.1f} us")


if __name__ == "__main__":
    main()
