#!/usr/bin/env python3
"""Re-time the training plans' tile configs of the ConvGRU convs (1x5 / 5x1 keys of the tuned DB)
in situ, then run the config-5 training bench with the new decisions and print them.
Usage: train_retune.py [--steps K] (the rest goes to tools/train_bench.py)."""
import json
import os
import sys
import tempfile

root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, root)
sys.path.insert(0, os.path.join(root, "tools"))

src = os.path.join(root, "jax_raft_amd", "tuned", "gfx950.json")
d = json.load(open(src))
drop = [k for k in d["entries"] if k.startswith('["train"') and tuple(json.loads(k)[6:8]) in ((1, 5), (5, 1))]
setcfg = None
if "--set" in sys.argv:   # --set C: pin the 256-output-channel data-gradient keys to config C instead
    i = sys.argv.index("--set")
    setcfg = int(sys.argv[i + 1])
    del sys.argv[i:i + 2]
    drop = [k for k in drop if json.loads(k)[13] == 256]
for k in drop:
    if setcfg is None:
        del d["entries"][k]
    else:
        d["entries"][k] = setcfg
tmp = os.path.join(tempfile.mkdtemp(), "db.json")
json.dump(d, open(tmp, "w"))
os.environ["JR_TUNE_DB"] = tmp

import train_bench  # noqa: E402
from jax_raft_amd.runtime import tunedb  # noqa: E402

sys.argv = [sys.argv[0]] + sys.argv[1:]
train_bench.main()
t = tunedb._table("gfx950")
for k in drop:
    print(k, "->", t.get(k), flush=True)
