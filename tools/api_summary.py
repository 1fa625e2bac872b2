#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database: kernel vs HIP-API activity over the
last forwards of a bench run (which API calls block the host, and for how
long), plus the GPU idle gaps between consecutive kernels."""
import sqlite3
import sys


def main():
    con = sqlite3.connect(sys.argv[1])
    views = [r[0] for r in con.execute("select name from sqlite_master where type in ('view','table')")]
    print("views:", ", ".join(v for v in views if not v.startswith("rocpd_info")))
    ks = sorted(con.execute("select start, end, name from kernels"))
    t_end = ks[-1][1]
    t0 = t_end - int(float(sys.argv[2] if len(sys.argv) > 2 else 0.08) * 1e9)  # last 80 ms
    kw = [k for k in ks if k[0] >= t0]
    busy, last = 0, None
    gaps = []
    for s, e, n in kw:
        if last is not None and s > last:
            gaps.append((s - last, n))
        busy += max(0, e - max(s, last or s))
        last = max(last or e, e)
    print(f"window {(t_end - t0) / 1e6:.1f} ms: kernels {len(kw)}, busy {busy / 1e6:.2f} ms")
    gaps.sort(reverse=True)
    print("largest GPU idle gaps (us, next kernel):", [(round(g / 1e3, 1), n[:40]) for g, n in gaps[:8]])
    for v in views:
        if v in ("kernels",) or v.startswith("rocpd"):
            continue
        cols = [r[1] for r in con.execute(f"pragma table_info('{v}')")]
        if not {"name", "start", "end"} <= set(cols):
            continue
        agg = {}
        for n, s, e in con.execute(f"select name, start, end from {v}"):
            if s is None or s < t0:
                continue
            a = agg.setdefault(n, [0, 0])
            a[0] += 1
            a[1] += e - s
        if agg:
            print(f"-- {v}: top host time in window")
            for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:12]:
                print(f"   {n[:48]:48s} n={c:6d} total={d / 1e6:8.2f} ms")


if __name__ == "__main__":
    main()
