#!/usr/bin/env python3
"""Compare two rocprofv3 kernel traces of the same forward (e.g. dev/probes/gate_trace.py with the
host gate on and off): per forward, the span, the busy time (union of kernel intervals), the idle
time and the summed kernel time; then the mean duration of the most expensive kernels in both.

    python dev/probes/trace_compare.py A_results.db B_results.db [--marker prep_images] [--skip 4]
"""
import argparse
import collections
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))

from kernel_breakdown import _load  # noqa: E402


def _name(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\(.*", "", n)
    return n[5:] if n.startswith("void ") else n


def analyse(path, marker, skip):
    rows = sorted(_load(path), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    fwd = []
    per_kernel = collections.defaultdict(list)
    for a, b in zip(starts[skip:], starts[skip + 1:]):
        ks = rows[a:b]
        t0, t1 = int(ks[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
        busy, cur_s, cur_e, total = 0, None, None, 0
        for r in ks:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            total += e - s
            per_kernel[_name(r["Kernel_Name"])].append(e - s)
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        fwd.append((t1 - t0, busy, total, len(ks)))
    return fwd, per_kernel


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--marker", default="prep_images")
    ap.add_argument("--skip", type=int, default=4, help="forwards skipped at the start (warm-up)")
    ap.add_argument("--top", type=int, default=16)
    o = ap.parse_args()
    res = {}
    for tag, p in (("A", o.a), ("B", o.b)):
        fwd, pk = analyse(p, o.marker, o.skip)
        res[tag] = pk
        n = max(1, len(fwd))
        span = sum(f[0] for f in fwd) / n / 1e3
        busy = sum(f[1] for f in fwd) / n / 1e3
        ksum = sum(f[2] for f in fwd) / n / 1e3
        print(f"{tag} ({os.path.basename(p)}): {len(fwd)} forwards, {fwd[0][3] if fwd else 0} kernels each; "
              f"span {span:.1f} us, busy {busy:.1f} us, idle {span - busy:.1f} us, kernel sum {ksum:.1f} us")
    tot = {k: sum(v) / len(v) for k, v in res["A"].items()}
    print(f"\n{'kernel':70s} {'A us':>8s} {'B us':>8s} {'B/A':>6s} {'calls':>6s}")
    for k in sorted(tot, key=lambda k: -sum(res["A"][k]))[:o.top]:
        a = tot[k]
        b = sum(res["B"].get(k, [0])) / max(1, len(res["B"].get(k, [])))
        print(f"{k[:70]:70s} {a / 1e3:8.2f} {b / 1e3:8.2f} {b / a if a else 0:6.2f} {len(res['A'][k]):6d}")


if __name__ == "__main__":
    main()
