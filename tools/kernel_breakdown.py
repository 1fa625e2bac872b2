#!/usr/bin/env python3
"""Per-kernel time breakdown of the timed bench steps from a rocprofv3
kernel trace: the ``*_kernel_trace.csv`` or the rocpd SQLite database
(``*_results.db``, rocprofv3's default output format on ROCm 7).
Only dispatches after the autotune/warm-up phase are kept: the last
``--steps`` forwards are located by their prep_images launches."""
import argparse
import collections
import csv
import re


def _load(path):
    if path.endswith(".db"):
        import sqlite3

        con = sqlite3.connect(path)
        cur = con.execute("select name, start, end, grid_x, grid_y from kernels")
        return [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e, "Grid_Size_X": gx, "Grid_Size_Y": gy}
                for n, s, e, gx, gy in cur]
    return list(csv.DictReader(open(path)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--marker", default="prep_images", help="kernel that starts a step ('' = whole trace / steps)")
    ap.add_argument("--between", action="store_true",
                    help="count the --steps whole cycles between the last --steps + 1 markers (a marker "
                         "in the middle of a step, e.g. the training loss kernel)")
    a = ap.parse_args()
    rows = sorted(_load(a.trace), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if a.marker and a.marker in r["Kernel_Name"]]
    if a.between:
        assert len(starts) > a.steps, f"{len(starts)} markers for {a.steps} cycles"
        rows = rows[starts[-a.steps - 1]:starts[-1]]
    else:
        first = starts[-a.steps] if len(starts) >= a.steps else 0
        rows = rows[first:]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        n = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
        n = re.sub(r"\(.*", "", n)
        if n.startswith("void "):
            n = n[5:]
        key = f"{n} grid=({r['Grid_Size_X']},{r['Grid_Size_Y']})" if "conv" in n else n
        agg[key][0] += 1
        agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot = sum(v[1] for v in agg.values())
    wall = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
    print(f"steps={a.steps} kernel-sum={tot / 1e3 / a.steps:.3f} ms/step  wall={wall / 1e3 / a.steps:.3f} ms/step")
    for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f"{d / 1e3 / a.steps:8.3f} ms/step {100 * d / tot:5.1f}% {c // a.steps:5d}/step  {d / c:8.1f} us  {n[:110]}")


if __name__ == "__main__":
    main()
