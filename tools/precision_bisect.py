#!/usr/bin/env python3
"""Where does the bf16 engine's drift come from?  CPU bisection on the fp32 golden model.

The bf16 engine stores activations in bf16 and feeds bf16 operands to fp32-accumulating MFMAs;
the ConvGRU hidden state, flow, coordinates and outputs stay fp32 (runtime/engine.py).  This tool
emulates that on the golden model (models/reference.py) one module group at a time: a patched
``Conv.forward`` rounds its input and kernel to bf16 (products exact in fp32, fp32 sums), and
rounds its output to bf16 unless the conv produces fp32 state; the correlation pyramid can be
rounded too.  Each variant's per-iteration EPE against the pure fp32 forward (same weights, same
input pair as tools/drift.py) shows which layers set the drift.

    python tools/precision_bisect.py raft_small [--iters 32] [--variants all,fe,ce,update,...]
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from jax_raft_amd.models import layers as L  # noqa: E402
from jax_raft_amd.models import reference as R  # noqa: E402

BF = torch.bfloat16


def rb(x: torch.Tensor) -> torch.Tensor:
    return x.to(BF).to(torch.float32)


# conv name groups (module paths of the golden model)
GROUPS = {
    "fe": lambda n: n.startswith("feature_encoder."),
    "fe_stem": lambda n: n.startswith("feature_encoder.convnormrelu."),
    "fe_l1": lambda n: n.startswith("feature_encoder.layer1."),
    "fe_l2": lambda n: n.startswith("feature_encoder.layer2."),
    "fe_l3": lambda n: n.startswith("feature_encoder.layer3."),
    "fe_head": lambda n: n == "feature_encoder.conv",
    "ce": lambda n: n.startswith("context_encoder."),
    "ce_head": lambda n: n == "context_encoder.conv",
    "motion": lambda n: n.startswith("update_block.motion_encoder."),
    "gru": lambda n: n.startswith("update_block.recurrent_block."),
    "flowhead": lambda n: n.startswith("update_block.flow_head."),
    "mask": lambda n: n.startswith("mask_predictor."),
}
GROUPS["fe_hi"] = lambda n: GROUPS["fe_stem"](n) or GROUPS["fe_l1"](n)
GROUPS["update"] = lambda n: any(GROUPS[g](n) for g in ("motion", "gru", "flowhead", "mask"))
GROUPS["all"] = lambda n: True
GROUPS["none"] = lambda n: False


@contextlib.contextmanager
def emulate(model, pred, corr_bf16: bool, parts="xwy"):
    """parts: which operands of the selected convs are bf16 -- x (input), w (kernel), y (output);
    a callable name -> parts string gives per-conv choices."""
    names = {id(m): n for n, m in model.named_modules()}
    orig_conv = L.Conv.forward
    parts_of = parts if callable(parts) else (lambda n, _p=parts: _p)

    def fwd(self, x):
        n = names.get(id(self), "")
        if not pred(n):
            return orig_conv(self, x)
        parts = parts_of(n)
        y = R.conv2d_nhwc(rb(x) if "x" in parts else x, rb(self.kernel) if "w" in parts else self.kernel, self.bias,
                          self.stride, self.padding)
        # the GRU gates / flow-head output feed fp32 state in the engine: keep those fp32
        if ".recurrent_block." in n or n.endswith("flow_head.conv2") or "y" not in parts:
            return y
        return rb(y)

    L.Conv.forward = fwd
    patched = []
    if corr_bf16:
        cb = L.CorrBlock
        orig_build = cb.build_pyramid

        def build(self, *a, **k):
            return [rb(t) for t in orig_build(self, *a, **k)]

        cb.build_pyramid = build
        patched.append((cb, "build_pyramid", orig_build))
    try:
        yield
    finally:
        L.Conv.forward = orig_conv
        for obj, attr, f in patched:
            setattr(obj, attr, f)


def main():
    import drift

    ap = argparse.ArgumentParser()
    ap.add_argument("arch", choices=["raft_small", "raft_large"])
    ap.add_argument("--iters", type=int, default=32)
    ap.add_argument("--size", type=int, nargs=2, default=[440, 1024])
    ap.add_argument("--variants", default="none+corr,all+corr,all,fe,ce,update,motion,gru,flowhead")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    torch.set_num_threads(min(8, os.cpu_count() or 8))
    model = drift.model_for(a.arch)
    i1, i2 = drift.inputs(1, *a.size)
    with torch.no_grad():
        t = time.time()
        ref = model(i1, i2, num_flow_updates=a.iters)
        print(f"fp32 golden in {time.time() - t:.1f} s", flush=True)
        mags = ref.norm(dim=-1).mean(dim=(1, 2, 3))
        out = {}
        for v in a.variants.split(","):
            # variant: groups joined by '&' (a '!' prefix: everything BUT that group), then optional
            # '+corr' (bf16 pyramid) and '+parts=xw' (only those operands rounded)
            if ";" in v:   # per-group parts: "fe=xy;!fe=xwy[+corr]"
                corr = v.endswith("+corr")
                specs = []
                for tok in v.replace("+corr", "").split(";"):
                    g, pp = tok.split("=")
                    neg = g.startswith("!")
                    specs.append((GROUPS[g.lstrip("!")], neg, pp))

                def parts_of(n, specs=specs):
                    for f, neg, pp in specs:
                        if f(n) != neg:
                            return pp
                    return ""

                with emulate(model, lambda n: True, corr, parts_of):
                    t = time.time()
                    o = model(i1, i2, num_flow_updates=a.iters)
                rel = [drift.epe(o[k], ref[k]) / mags[k].item() for k in range(a.iters)]
                out[v] = rel
                pick = [0, 1, 3, 7, 11, 15, 23, 31]
                print(f"{v:24s} rel EPE " + " ".join(f"it{k + 1}={rel[k]:.2e}" for k in pick if k < a.iters)
                      + f"  ({time.time() - t:.1f} s)", flush=True)
                continue
            toks = v.split("+")
            groups, corr = toks[0], "corr" in toks[1:]
            parts = next((t.split("=")[1] for t in toks[1:] if t.startswith("parts=")), "xwy")
            preds = [GROUPS[g] for g in groups.split("&") if not g.startswith("!")]
            negs = [GROUPS[g[1:]] for g in groups.split("&") if g.startswith("!")]
            sel = (lambda n: any(p(n) for p in preds)) if preds else (lambda n: not any(q(n) for q in negs))
            if preds and negs:
                sel = lambda n: any(p(n) for p in preds) and not any(q(n) for q in negs)  # noqa: E731
            with emulate(model, sel, corr, parts):
                t = time.time()
                o = model(i1, i2, num_flow_updates=a.iters)
            rel = [drift.epe(o[k], ref[k]) / mags[k].item() for k in range(a.iters)]
            out[v] = rel
            pick = [0, 1, 3, 7, 11, 15, 23, 31]
            print(f"{v:24s} rel EPE " + " ".join(f"it{k + 1}={rel[k]:.2e}" for k in pick if k < a.iters)
                  + f"  ({time.time() - t:.1f} s)", flush=True)
    if a.json:
        json.dump(dict(arch=a.arch, iters=a.iters, size=a.size, rel_epe=out, mags=mags.tolist()), open(a.json, "w"))


if __name__ == "__main__":
    main()
