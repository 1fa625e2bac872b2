"""Persistent tile-config decisions of the implicit-GEMM conv autotuner.

Every conv problem (pixels, channels, kernel, strides, channel strides,
epilogue) picks one of the precompiled tile configs of ``conv_igemm.hip``.
Timing ~25 configs per conv at plan build costs seconds per process -- on
every rank of a multi-GPU job -- and a near-tie can flip between runs, so
run-to-run results differ.  The decisions are therefore kept in a JSON file
per GPU architecture shipped with the package (``tuned/<gfx>.json``),
produced on the target hardware by ``tools/autotune_db.py``:

* a hit returns the stored config (no timing);
* a miss is timed once in-process (the caller's tuner) and remembered for
  the process; ``save()`` writes the merged table back.

``JR_TUNE=fresh`` ignores the file (re-times every problem, e.g. to refresh
it); ``JR_TUNE=db`` (default) uses it; ``JR_TUNE_DB=<file>`` reads another table.

The file records the ``kernel_set`` it was tuned against: when the compiled tile
configs are renumbered or removed, :data:`KERNEL_SET` is bumped and an old file is
ignored (re-timed) instead of handing out ids that no longer exist; and a caller
passing ``valid=`` to :func:`lookup` gets a miss for a stored id outside its
candidate set (e.g. an id from a retired config range).
"""
from __future__ import annotations

import json
import os
import threading
from pathlib import Path
from typing import Dict, Optional

from .. import knobs

DB_DIR = Path(__file__).resolve().parent.parent / "tuned"
KERNEL_SET = 1    # bump when tile-config ids are renumbered / removed (csrc/kernels/conv_igemm.hip)
_lock = threading.Lock()
_tables: Dict[str, Dict[str, int]] = {}
_stats = {"hits": 0, "misses": 0}


def gpu_arch(device=None) -> str:
    """'gfx950' for an MI355X (the gcnArchName without feature suffixes)."""
    import torch

    props = torch.cuda.get_device_properties(device if device is not None else torch.cuda.current_device())
    return str(getattr(props, "gcnArchName", "unknown")).split(":")[0]


def path(arch: str) -> Path:
    """The table file: the packaged ``tuned/<arch>.json``, or ``JR_TUNE_DB`` (a table another
    process saved: e.g. tools/race_check.py hands its decisions to its child processes so that
    they compare kernels, not autotune outcomes)."""
    o = knobs.get("JR_TUNE_DB")
    return Path(o) if o else DB_DIR / f"{arch}.json"


def _key(key) -> str:
    return json.dumps([k if isinstance(k, (int, float, str, bool)) or k is None else str(k) for k in key],
                      separators=(",", ":"))


def _table(arch: str) -> Dict[str, int]:
    with _lock:
        t = _tables.get(arch)
        if t is None:
            t = {}
            p = path(arch)
            if knobs.get("JR_TUNE", "db") != "fresh" and p.exists():
                with open(p) as f:
                    d = json.load(f)
                if int(d.get("kernel_set", 1)) == KERNEL_SET:
                    t = {k: int(v) for k, v in d.get("entries", {}).items()}
            _tables[arch] = t
        return t


def lookup(arch: str, key, valid=None) -> Optional[int]:
    """The stored decision for ``key`` (None: a miss).  ``valid``: the caller's candidate
    ids; a stored id outside them is a miss (stale entry), not a launch failure."""
    cfg = _table(arch).get(_key(key))
    if cfg is not None and valid is not None and cfg not in valid:
        cfg = None
    _stats["hits" if cfg is not None else "misses"] += 1
    return cfg


def peek(arch: str, key) -> Optional[int]:
    """A persisted decision without counting a hit / miss (optional entries, e.g. the
    tile config of a grouped two-conv launch, runtime/engine.py:_conv_group)."""
    return _table(arch).get(_key(key))


def record(arch: str, key, cfg: int) -> None:
    _table(arch)[_key(key)] = int(cfg)


def stats() -> Dict[str, int]:
    return dict(_stats)


def save(arch: str, target=None) -> Path:
    """Write this process's table (file entries + new decisions) for ``arch`` to
    ``target`` (default: the packaged ``tuned/<arch>.json``)."""
    t = _table(arch)
    p = Path(target) if target is not None else path(arch)
    p.parent.mkdir(parents=True, exist_ok=True)
    tmp = p.with_name(p.name + ".tmp")
    with open(tmp, "w") as f:
        json.dump({"version": 1, "kernel_set": KERNEL_SET, "arch": arch, "entries": dict(sorted(t.items()))}, f,
                  indent=0)
    os.replace(tmp, p)
    return p
