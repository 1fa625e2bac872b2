#!/usr/bin/env python3
"""Per-kernel PMC table from one or more ``rocprofv3 --pmc ... --output-format csv`` passes.

Each pass dir holds a ``*counter_collection.csv`` (one row per dispatch and counter).  Rows are
grouped by (kernel name without arguments, grid size); the mean value per dispatch of every
counter is merged over the passes, then derived columns are printed:

* ``mfma%``  = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES * 4 SIMDs ... ) is not comparable across
  gfx94x formulas, so the table reports raw per-dispatch MFMA busy cycles and the ratio
  ``mfma_busy / (GRBM_GUI_ACTIVE * CUs * 4)`` -- the share of all SIMD-cycles of the dispatch the
  matrix pipes were busy (GRBM_GUI_ACTIVE counts per XCD: divided by 8 here);
* ``valu/mfma`` = SQ_INSTS_VALU / SQ_INSTS_MFMA;
* ``lds_conf%`` = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE;
* ``lds%`` = SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE * CUs): the share of the dispatch's CU-cycles
  the LDS array was busy (256 B/clk/CU for ds_read_b128; compare with ``mfma%``: a kernel whose
  lds% reaches its mfma% feeds its MFMAs from LDS at the array's rate);
* ``fetch_MB`` = FETCH_SIZE (KB) / 1024 x 2 (gfx950 tallies wide streaming reads at half their
  bytes, MI355X_MICROARCH.md "HBM"), ``write_MB`` = WRITE_SIZE / 1024;
* ``wait%`` = SQ_WAIT_ANY / SQ_WAVE_CYCLES, ``stall%`` = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES.

Usage: ``python tools/pmc_table.py <pass_dir> [<pass_dir> ...] [--filter substr] [--min-n N]``
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import re

NUM_CUS = 256


def _short(name: str) -> str:
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", n)
    n = re.sub(r"\(.*", "", n)
    return n[5:] if n.startswith("void ") else n


def load(dirs):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    count = collections.Counter()
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            seen = set()
            for r in csv.DictReader(open(f)):
                key = (_short(r.get("Kernel_Name", "?")), r.get("Grid_Size", r.get("Grid_Size_X", "?")))
                per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
                did = (f, r.get("Dispatch_Id"))
                if did not in seen:
                    seen.add(did)
                    count[(key, f)] += 1
    n = collections.Counter()
    for (key, _), c in count.items():
        n[key] = max(n[key], c)
    return per, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--filter", default="")
    ap.add_argument("--min-n", type=int, default=1)
    a = ap.parse_args()
    per, n = load(a.dirs)

    def m(v, k):
        x = v.get(k)
        return sum(x) / len(x) if x else None

    rows = []
    for key, v in per.items():
        if a.filter and a.filter not in key[0]:
            continue
        if n[key] < a.min_n:
            continue
        gui = m(v, "GRBM_GUI_ACTIVE")
        busy = m(v, "SQ_VALU_MFMA_BUSY_CYCLES")
        imf, iva = m(v, "SQ_INSTS_MFMA"), m(v, "SQ_INSTS_VALU")
        conf, lact = m(v, "SQ_LDS_BANK_CONFLICT"), m(v, "SQ_LDS_IDX_ACTIVE")
        wc, wa, wi = m(v, "SQ_WAVE_CYCLES"), m(v, "SQ_WAIT_ANY"), m(v, "SQ_WAIT_INST_ANY")
        fe, wr = m(v, "FETCH_SIZE"), m(v, "WRITE_SIZE")
        us = gui / 8 / 2100.0 if gui else None   # ~clock under load; wall estimate only
        rows.append(dict(
            kernel=key[0][:60], grid=key[1], n=n[key], us=us,
            mfma=(busy / (gui / 8 * NUM_CUS * 4) * 100) if busy and gui else None,
            vpm=(iva / imf) if iva and imf else None,
            conf=(conf / lact * 100) if conf is not None and lact else None,
            lds=(lact / (gui / 8 * NUM_CUS) * 100) if lact is not None and gui else None,
            fetch=(fe / 1024 * 2) if fe is not None else None,
            write=(wr / 1024) if wr is not None else None,
            wait=(wa / wc * 100) if wa is not None and wc else None,
            stall=(wi / wc * 100) if wi is not None and wc else None,
        ))
    rows.sort(key=lambda r: -(r["us"] or 0) * r["n"])
    hdr = f"{'kernel':60s} {'grid':>8s} {'n':>5s} {'~us':>7s} {'mfma%':>6s} {'valu/mfma':>9s} {'ldsconf%':>8s} {'lds%':>6s} " \
          f"{'fetchMB':>8s} {'writeMB':>8s} {'wait%':>6s} {'stall%':>6s}"
    print(hdr)

    def f(x, w, p=1):
        return f"{x:{w}.{p}f}" if x is not None else " " * (w - 1) + "-"

    for r in rows:
        print(f"{r['kernel']:60s} {r['grid']:>8s} {r['n']:5d} {f(r['us'], 7)} {f(r['mfma'], 6)} {f(r['vpm'], 9, 2)} "
              f"{f(r['conf'], 8)} {f(r['lds'], 6)} {f(r['fetch'], 8, 2)} {f(r['write'], 8, 2)} {f(r['wait'], 6)} {f(r['stall'], 6)}")


if __name__ == "__main__":
    main()
