#!/usr/bin/env python3
"""How much of a pipelined step runs concurrently: from a rocprofv3 rocpd database, the
kernels of one step (between two consecutive ``--marker`` launches) grouped by HIP stream /
HW queue, the busy time of each group, their union and the time two or more groups overlap.

  python tools/overlap.py run_results.db [--step -2] [--list 60]
"""
import argparse
import collections
import sqlite3

from timeline import short


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="prep_images")
    ap.add_argument("--step", type=int, default=-2, help="which marker-delimited window (python index)")
    ap.add_argument("--list", type=int, default=0, help="print the first N kernels of the window")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    key = next((c for c in ("stream_id", "queue_id", "stream", "queue") if c in cols), None)
    print("grouping by", key, "| columns:", ",".join(cols))
    q = f"select name, start, end, {key or 0} from kernels order by start"
    rows = [(n, int(s), int(e), g) for n, s, e, g in con.execute(q)]
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    i0 = marks[a.step]
    i1 = marks[a.step + 1] if a.step + 1 < len(marks) and a.step != -1 else len(rows)
    win = rows[i0:i1]
    t0, t1 = win[0][1], max(r[2] for r in win)
    groups = collections.defaultdict(list)
    for n, s, e, g in win:
        groups[g].append((s, e, n))

    def union(iv):
        tot, cs, ce = 0, None, None
        for s, e in sorted(iv):
            if ce is None or s > ce:
                if ce is not None:
                    tot += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        return tot + (ce - cs if ce is not None else 0)

    allv = [(s, e) for s, e, _ in sum(groups.values(), [])]
    # time covered by >= 2 kernels at once (sweep)
    ev = sorted([(s, 1) for s, _ in allv] + [(e, -1) for _, e in allv])
    depth, last, multi = 0, None, 0
    for t, d in ev:
        if depth >= 2:
            multi += t - last
        depth += d
        last = t
    print(f"window {(t1 - t0) / 1e3:.1f} us, {len(win)} kernels, kernel-sum {sum(e - s for s, e in allv) / 1e3:.1f} us, "
          f"busy (union) {union(allv) / 1e3:.1f} us, >=2 concurrent {multi / 1e3:.1f} us")
    for g, iv in sorted(groups.items(), key=lambda x: x[0] or 0):
        names = collections.Counter(short(n) for _, _, n in iv).most_common(3)
        print(f"  group {g}: {len(iv)} kernels, busy {union([(s, e) for s, e, _ in iv]) / 1e3:.1f} us, "
              f"span {(min(s for s, _, _ in iv) - t0) / 1e3:.1f}..{(max(e for _, e, _ in iv) - t0) / 1e3:.1f} us; {names}")
    for n, s, e, g in win[:a.list]:
        print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f}  g{g}  {short(n)}")


if __name__ == "__main__":
    main()
