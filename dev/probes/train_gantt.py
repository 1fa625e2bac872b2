#!/usr/bin/env python3
"""Text Gantt chart of one training step per hardware queue from a rocprofv3 kernel trace:
one character per bucket (default 200 us) = the kernel category busiest in it ('.' idle).
Categories: E forward encoder norm/stats, L forward lookup, G forward ConvGRU, S loss,
U upsample adjoint, B lookup backward, P pyramid backward, N encoder norm backward,
W weight gradient, O optimizer / grad-norm, K weight repack, c conv, o other."""
import argparse
import collections

from kernel_breakdown import _load

CATS = [("FusedAdam", "O"), ("multi_tensor", "O"), ("LpNorm", "O"), ("wgrad", "W"), ("norm_bwd", "N"),
        ("gru_halo", "G"), ("gru_fused", "G"), ("corr_lookup_wide", "L"), ("corr_lookup_bwd", "B"),
        ("upsample_convex_bwd", "U"), ("pyr_bwd", "P"), ("channel_stats", "E"), ("norm_act", "E"),
        ("seq_loss", "S"), ("pack_pieces", "K"), ("conv", "c")]


def cat(n):
    for k, c in CATS:
        if k in n:
            return c
    return "o"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="seq_loss_kernel")
    ap.add_argument("--bucket", type=float, default=200.0, help="us per character")
    a = ap.parse_args()
    rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "0"))
                   for r in _load(a.trace)), key=lambda r: r[1])
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    seg = rows[marks[-3]:marks[-2]]
    t0, t1 = seg[0][1], max(r[2] for r in seg)
    nb = int((t1 - t0) / 1e3 / a.bucket) + 1
    queues = collections.OrderedDict()
    for n, s, e, q in seg:
        b = queues.setdefault(q, [collections.Counter() for _ in range(nb)])
        # spread the kernel's time over the buckets it covers
        x = s
        while x < e:
            i = int((x - t0) / 1e3 / a.bucket)
            end = min(e, t0 + int((i + 1) * a.bucket * 1e3))
            b[i][cat(n)] += end - x
            x = end
    print(f"step {(t1 - t0) / 1e3:.0f} us from the loss kernel, {a.bucket:.0f} us per char; {__doc__.splitlines()[2]}")
    for q, b in queues.items():
        busy = sum(sum(c.values()) for c in b) / 1e3
        line = "".join(c.most_common(1)[0][0] if c and sum(c.values()) > 0.2 * a.bucket * 1e3 else
                       ("," if c else ".") for c in b)
        print(f"queue {q:>3} busy {busy:8.0f} us |{line}|")


if __name__ == "__main__":
    main()
