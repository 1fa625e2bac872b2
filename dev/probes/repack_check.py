#!/usr/bin/env python3
"""Which packed weight buffers of the fused training plans does the per-step table repack
(train/fused.py:Packer, train.hip:pack_pieces_kernel) leave stale?  Builds the plans, changes
every parameter in place (as an optimizer step does), runs the persistent plans' forward (whose
first op is the table repack) and compares every packed buffer with the Python packing of the
current parameters.

    python dev/probes/repack_check.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from jax_raft_amd import raft_large  # noqa: E402
from jax_raft_amd.ops import native as nat  # noqa: E402
from jax_raft_amd.ops.native import round_up  # noqa: E402
from jax_raft_amd.train import fused as F  # noqa: E402
from jax_raft_amd.train.data import SyntheticFlow  # noqa: E402


def diff(a, b):
    return (a.float() - b.float()).abs().max().item()


def main():
    torch.manual_seed(0)
    model = raft_large()[0].cuda().train()
    data = SyntheticFlow(size=(192, 256), seed=0, device=torch.device("cuda"))
    img1, img2, flow, valid = data.batch([0, 1])
    F._LOOPS.clear()
    with torch.no_grad():
        model(img1, img2, train=True, num_flow_updates=3, fused=True)
        for p in model.parameters():
            p.add_(torch.randn_like(p) * 0.01 * (p.abs().mean() + 1e-3))
        model(img1, img2, train=True, num_flow_updates=3, fused=True)
    torch.cuda.synchronize()
    fm = next(iter(F._LOOPS[model].values()))
    bad = []
    for tag, enc in (("fe", fm.fe), ("ce", fm.ce)):
        for c in enc._convs():
            k, b = c.kernel.detach().float(), c.bias.detach().float()
            kh, kw, cin, cout = k.shape
            sp, tp = enc._specs[id(c)], enc._tspecs[id(c)]
            kt = torch.flip(k, dims=(0, 1)).permute(0, 1, 3, 2)
            checks = [("w", sp.w, nat.pack_weight(k, sp.cin8)), ("b", sp.b[:cout], b)]
            if sp.wh is not None:
                checks.append(("wh", sp.wh, nat.pack_halo_conv(k, sp.cin8)))
            ktp = kt if sp.cin8 == cin else torch.cat([kt, kt.new_zeros(kh, kw, cout, sp.cin8 - cin)], dim=3)
            checks.append(("wT", tp.w, nat.pack_weight(ktp, tp.cin8)))
            if tp.wh is not None and c.stride == (1, 1):
                checks.append(("whT", tp.wh, nat.pack_halo_conv(ktp, tp.cin8)))
            for nm, got, ref in checks:
                d = diff(got, ref)
                if d > 1e-2:
                    bad.append((f"{tag}:{nm}", tuple(k.shape), c.stride, round(d, 4)))
    loop = fm.loop
    for name, fn in loop._src.items():
        k, b, pad, cin8 = fn()
        sp = loop._specs[name]
        d = diff(sp.w, nat.pack_weight(k.to(sp.w.device), sp.cin8))
        if d > 1e-2:
            bad.append((f"loop:{name}.w", tuple(k.shape), None, round(d, 4)))
        if sp.wh is not None:
            gru = name[:2] in ("gA", "gB") and name[2:].isdigit()
            ref = (nat.pack_gru_halo if gru else nat.pack_halo_conv)(k.to(sp.w.device), sp.cin8)
            d = diff(sp.wh, ref)
            if d > 1e-2:
                bad.append((f"loop:{name}.wh", tuple(k.shape), None, round(d, 4)))
        d = diff(sp.b[:b.numel()], b.to(sp.b.device))
        if d > 1e-3:
            bad.append((f"loop:{name}.b", tuple(k.shape), None, round(d, 5)))
    print(f"stale packed buffers after an in-place update + one persistent forward: {len(bad)}")
    for r in bad:
        print("  ", r)


if __name__ == "__main__":
    main()
