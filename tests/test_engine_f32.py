"""fp32 parity mode (``RaftEngine(precision="fp32")``, runtime/engine_f32.py).

CPU: the recorded plan is executed by a PyTorch interpreter of every fp32 op
(the documented semantics of csrc/kernels/conv_f32.hip and f32.hip) and must
reproduce the fp32 golden forward -- this checks the lowering (buffer layout,
channel offsets, the folded context share of the ConvGRU gates, iteration
order) without a GPU.  GPU: the kernels against the same interpreter / the
golden ops, and the engine end to end against the golden forward."""
import math

import pytest
import torch
import torch.nn.functional as F

from jax_raft_amd import raft_large, raft_small
from jax_raft_amd.models import reference as R
from jax_raft_amd.ops import native as nat
from jax_raft_amd.runtime import engine as E
from jax_raft_amd.runtime import tunedb

ACT = {0: lambda v: v, 1: torch.relu, 2: torch.sigmoid, 3: torch.tanh}


def _rows(t, M):
    return t.view(M, t.shape[-1]) if t.dim() != 2 or t.shape[0] != M else t


def conv_f32_ref(t, i, alpha):
    """PyTorch semantics of the conv_f32 op (kernels.h: ConvF32Params)."""
    x, w, bias, y, y2, res, h32, zbuf, bmap = t
    (N, H, W, x_coff, cin4, KH, KW, SH, SW, PH, PW, cout, act, split, y_coff, y2_coff, res_coff, res_post,
     hidden, bmap_coff, epi, _ksplit) = i
    xin = x.reshape(N, H, W, x.shape[-1])[..., x_coff:x_coff + cin4].permute(0, 3, 1, 2)
    k = w.reshape(cout, KH, KW, cin4).permute(0, 3, 1, 2)
    v = F.conv2d(xin, k, None, stride=(SH, SW), padding=(PH, PW)).permute(0, 2, 3, 1)
    M = v.shape[0] * v.shape[1] * v.shape[2]
    v = v.reshape(M, cout) + bias[:cout]
    if bmap is not None:
        v = v + _rows(bmap, M)[:, bmap_coff:bmap_coff + cout]

    def a(u):
        if act == 4:
            return torch.cat([torch.tanh(u[:, :split]), torch.relu(u[:, split:])], 1)
        return ACT[act](u)

    Y = _rows(y, M)
    if epi == 0:
        if res is not None:
            r = _rows(res, M)[:, res_coff:res_coff + cout]
            v = torch.relu(a(v) + r) if res_post else a(v + r)
        else:
            v = a(v)
        v = v * alpha
        Y[:, y_coff:y_coff + cout] = v
        if y2 is not None:
            _rows(y2, M)[:, y2_coff:y2_coff + cout] = v
        if h32 is not None:
            _rows(h32, M)[:, :split] = v[:, :split]
    elif epi == 1:
        g = torch.sigmoid(v)
        _rows(zbuf, M)[:] = g[:, :hidden]
        Y[:, y_coff:y_coff + hidden] = g[:, hidden:] * _rows(h32, M)
    else:
        z = _rows(zbuf, M)
        hn = (1 - z) * _rows(h32, M) + z * torch.tanh(v)
        _rows(h32, M)[:] = hn
        Y[:, y_coff:y_coff + hidden] = hn
        if y2 is not None:
            _rows(y2, M)[:, y2_coff:y2_coff + hidden] = hn


class F32Interp:
    """Records a plan like the native Plan and executes it with PyTorch ops."""

    def __init__(self):
        self.segs = {0: [], 1: [], 2: [], 3: []}
        self.seg = 0

    def set_segment(self, s):
        self.seg = s

    def set_lane(self, l):
        assert l == 0

    def __getattr__(self, name):
        if not name.startswith("add_"):
            raise AttributeError(name)
        op = name[4:]

        def rec(*args):
            self.segs[self.seg].append((op, args))
        return rec

    def names(self, seg):
        return [op for op, _ in self.segs[seg]]

    def run(self, n_iters):
        for op, a in self.segs[0]:
            self._exec(op, a, 0)
        for it in range(n_iters):
            for op, a in self.segs[1] + self.segs[3]:
                self._exec(op, a, it)
        for op, a in self.segs[2]:
            self._exec(op, a, n_iters)

    def run_segment(self, seg, it):
        for op, a in self.segs[seg]:
            self._exec(op, a, it)

    @staticmethod
    def _exec(op, a, it):
        if op == "memset":
            a[0][0].zero_()
        elif op == "prep_f32":
            (i1, i2, out), (B, H, W) = a
            out.zero_()
            out[:B, ..., :3] = i1
            out[B:, ..., :3] = i2
        elif op == "conv_f32":
            conv_f32_ref(*a)
        elif op == "stats_f32":
            (x, st), (N, HW, C) = a
            xf = x.reshape(N, HW, C)
            st[..., 0] = xf.sum(1)
            st[..., 1] = (xf * xf).sum(1)
        elif op == "norm_act_f32":
            (x, sx, r, sr, y), (mx, mr, N, HW, C, relu), eps = a

            def norm(v, s, mode):
                v = v.reshape(N, HW, C)
                if mode == 0:
                    return v
                mean = s[..., 0:1].transpose(1, 2) / HW
                var = (s[..., 1:2].transpose(1, 2) / HW - mean * mean).clamp_min(0)
                return (v - mean) / torch.sqrt(var + eps)
            u = norm(x, sx, mx)
            if relu & 1:
                u = torch.relu(u)
            if r is not None:
                u = u + norm(r, sr, mr)
            if relu & 2:
                u = torch.relu(u)
            y.copy_(u.reshape(y.shape))
        elif op == "copy_channels_f32":
            (s, d), (so, do, M, C) = a
            _rows(d, M)[:, do:do + C] = _rows(s, M)[:, so:so + C]
        elif op == "init_coords":
            (c,), (B, h, w) = a
            g = R.make_coords_grid(B, h, w)
            c.copy_(g.reshape(c.shape))
        elif op == "corr_pool_f32":
            (s, d), (M, hl, wl) = a
            ho, wo = hl // 2, wl // 2
            d.copy_(s[:, :2 * ho, :2 * wo].reshape(M, ho, 2, wo, 2).mean(dim=(2, 4)))
        elif op == "lookup_f32":
            t, i = a
            L, B, h, w, r = i[:5]
            nq = i[5] if len(i) > 5 else h * w
            coords, out = t[0], t[1]
            lv = [v for v in t[2:2 + L]]
            c = coords.reshape(B, nq, 1, 2)
            o = R.index_pyramid(lv, c, r).reshape(B * nq, -1)
            out.view(-1, out.shape[-1])[:B * nq, :o.shape[1]] = o
        elif op == "flow_update_f32":
            (d, coords, f32, hx, qx, f4), (N, h, w, hx_off, qx_off) = a
            M = N * h * w
            coords += d[:, :2]
            g = R.make_coords_grid(N, h, w).reshape(M, 2)
            f = coords - g
            f32.copy_(f)
            hx[:, hx_off:hx_off + 2] = f
            qx[:, qx_off:qx_off + 2] = f
            f4.zero_()
            f4[:, :2] = f
        elif op == "upsample_convex_f32":
            (mask, flow, out, _slot), (B, h, w, stride, _off) = a
            up = R.upsample_flow(flow.reshape(B, h, w, 2), mask[:, :576].reshape(B, h, w, 576))
            out.view(-1)[stride * it: stride * it + up.numel()] = up.reshape(-1)
        elif op == "upsample_bilinear":
            (flow, out, _slot), (B, h, w, stride, _off) = a
            up = R.upsample_flow(flow.reshape(B, h, w, 2))
            out.view(-1)[stride * it: stride * it + up.numel()] = up.reshape(-1)
        else:
            raise NotImplementedError(op)


@pytest.fixture
def interp(monkeypatch):
    monkeypatch.setattr(nat, "require", lambda: None)
    monkeypatch.setattr(nat, "new_plan", F32Interp)
    monkeypatch.setattr(tunedb, "gpu_arch", lambda device=None: "cpu")


def _inputs(B, H, W, seed=0):
    g = torch.Generator().manual_seed(seed)
    base = torch.rand(B, H + 8, W + 8, 3, generator=g) * 2 - 1
    return base[:, 4:4 + H, 4:4 + W].contiguous(), base[:, 2:2 + H, 6:6 + W].contiguous()


@pytest.mark.parametrize("factory", [raft_small, raft_large])
@pytest.mark.parametrize("all_iters", [True, False])
def test_fp32_lowering_reproduces_golden(factory, all_iters, interp):
    torch.manual_seed(0)
    model = factory(seed=0)[0].eval()
    B, H, W, n = 2, 128, 160, 3
    i1, i2 = _inputs(B, H, W)
    with torch.no_grad():
        ref = model(i1, i2, num_flow_updates=n)
        eng = E.RaftEngine(model, "cpu", precision="fp32")
        assert type(eng).__name__ == "RaftEngineF32" and eng.precision == "fp32"
        st = eng._build(B, H, W, n, all_iters)
        plan = st.plan
        # one lane; every loop op is an fp32 op
        assert all(op.endswith("_f32") for op in plan.names(1) if op != "upsample_bilinear")
        st.inp1.copy_(i1)
        st.inp2.copy_(i2)
        plan.run(n)
    out = st.out
    want = ref if all_iters else ref[-1:]
    assert out.shape == want.shape
    err = (out - want).abs().max().item()
    assert err < 2e-3 * (1 + want.abs().max().item()), err


def test_precision_argument_is_validated():
    with pytest.raises(ValueError):
        E.RaftEngine(None, "cpu", precision="fp16")


# ------------------------------------------------------------------ GPU


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [
    # N, H, W, cin, cout, k, stride, pad, xcs, xoff
    (2, 24, 40, 4, 64, 7, 2, 3, 4, 0),        # stem
    (2, 16, 20, 64, 96, 3, 1, 1, 64, 0),
    (1, 16, 24, 324, 256, 1, 1, 0, 324, 0),   # convcorr1
    (2, 10, 12, 128, 2, 3, 1, 1, 128, 0),     # FlowHead conv2 (channel tail)
    (1, 12, 16, 128, 126, 3, 1, 1, 256, 128),  # motion conv (tail), input channel slice
    (2, 12, 16, 256, 256, 1, 5, 0, 256, 0),   # (1, 5) GRU-shaped, pad (0, 2) below
])
@pytest.mark.parametrize("act", [0, 1, 4])
@pytest.mark.parametrize("ksplit", [0, 1, 3])
def test_conv_f32_kernel(shape, act, ksplit):
    """vs the interpreter; ksplit: the automatic split-K choice (0), forced off, forced 3-way."""
    N, H, W, cin, cout, k, s, p, xcs, xoff = shape
    kh, kw = (k, k) if k != 1 or s != 5 else (1, 5)
    sh, sw = (s, s) if s != 5 else (1, 1)
    ph, pw = (p, p) if s != 5 else (0, 2)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, H, W, xcs, generator=g)
    kern = torch.randn(kh, kw, cin, cout, generator=g) / math.sqrt(kh * kw * cin)
    b = torch.randn(cout, generator=g)
    spec = nat.make_spec_f32(kern, b, (sh, sw), (ph, pw))
    OH, OW = spec.out_hw(H, W)
    res = torch.randn(N, OH, OW, cout, generator=g) if cout % 4 == 0 else None
    ycs = nat.round_up(cout, 4)   # fp32 rows in 16-byte chunks (a channel tail stays inside the row)
    yr = torch.zeros(N, OH, OW, ycs)
    args = nat.conv_f32_args(spec, x, N, H, W, yr, x_coff=xoff, act=act, split=cout // 2, alpha=0.5, res=res)
    conv_f32_ref(*args)
    dev = torch.device("cuda")
    sg = nat.make_spec_f32(kern, b, (sh, sw), (ph, pw), device=dev)
    yg = torch.zeros(N, OH, OW, ycs, device=dev)
    nat.ops().conv_f32(*nat.conv_f32_args(sg, x.to(dev), N, H, W, yg, x_coff=xoff, act=act, split=cout // 2,
                                          alpha=0.5, res=None if res is None else res.to(dev), ksplit=ksplit))
    torch.cuda.synchronize()
    assert (yg.cpu() - yr).abs().max().item() < 1e-4 * (1 + yr.abs().max().item())
    assert not yg[..., cout:].any()


@pytest.mark.gpu
@pytest.mark.parametrize("ksplit", [1, 4])
def test_conv_f32_gru_epilogues(ksplit):
    """GRU-A (z, r*h) and GRU-B (blend) epilogues with a bias map, vs the interpreter
    (without / with split-K: the epilogue then runs in the reduction kernel)."""
    g = torch.Generator().manual_seed(2)
    N, H, W, hd, cs = 2, 8, 12, 64, 132
    M = N * H * W
    x = torch.randn(M, cs, generator=g)
    spec_a = nat.make_spec_f32(torch.randn(1, 5, cs, 2 * hd, generator=g) * 0.05, torch.zeros(2 * hd), (1, 1), (0, 2))
    spec_b = nat.make_spec_f32(torch.randn(5, 1, cs, hd, generator=g) * 0.05, torch.zeros(hd), (1, 1), (2, 0))
    bmap = torch.randn(M, 3 * hd + 4, generator=g)
    h32 = torch.randn(M, hd, generator=g)
    res = {}
    for devname in ("cpu", "cuda"):
        d = torch.device(devname)
        sa = nat.make_spec_f32(spec_a.w.reshape(2 * hd, 1, 5, cs).permute(1, 2, 3, 0), spec_a.b, (1, 1), (0, 2), device=d)
        sb = nat.make_spec_f32(spec_b.w.reshape(hd, 5, 1, cs).permute(1, 2, 3, 0), spec_b.b, (1, 1), (2, 0), device=d)
        xx, hh, bm = x.to(d).clone(), h32.to(d).clone(), bmap.to(d)
        z = torch.zeros(M, hd, device=d)
        q = torch.zeros(M, cs, device=d)
        y = torch.zeros(M, cs, device=d)
        a1 = nat.conv_f32_args(sa, xx, N, H, W, q, zbuf=z, h32=hh, hidden=hd, epi=nat.EPI_GRU_A, bmap=bm,
                               ksplit=ksplit)
        a2 = nat.conv_f32_args(sb, xx, N, H, W, y, zbuf=z, h32=hh, hidden=hd, epi=nat.EPI_GRU_B, bmap=bm,
                               bmap_coff=2 * hd, ksplit=ksplit)
        for a in (a1, a2):
            if devname == "cpu":
                conv_f32_ref(*a)
            else:
                nat.ops().conv_f32(*a)
        res[devname] = (q.cpu(), y.cpu(), hh.cpu(), z.cpu())
    torch.cuda.synchronize()
    for u, v in zip(res["cpu"], res["cuda"]):
        assert (u - v).abs().max().item() < 1e-4


@pytest.mark.gpu
def test_lookup_pool_f32_kernels():
    g = torch.Generator().manual_seed(3)
    B, h, w, r, L = 2, 16, 20, 4, 4
    M = B * h * w
    l0 = torch.randn(M, h, w, generator=g)
    coords = (R.make_coords_grid(B, h, w) + torch.randn(B, h, w, 2, generator=g) * 3).reshape(M, 2)
    dev = torch.device("cuda")
    lv_g = [l0.to(dev)]
    hl, wl = h, w
    for _ in range(1, L):
        t = torch.empty(M, hl // 2, wl // 2, device=dev)
        nat.ops().corr_pool_f32([lv_g[-1], t], [M, hl, wl])
        lv_g.append(t)
        hl //= 2
        wl //= 2
    pyr = [l0]
    for _ in range(1, L):
        v = pyr[-1]
        ho, wo = v.shape[1] // 2, v.shape[2] // 2
        pyr.append(v[:, :2 * ho, :2 * wo].reshape(M, ho, 2, wo, 2).mean(dim=(2, 4)))
    out = torch.zeros(M, L * (2 * r + 1) ** 2, device=dev)
    nat.ops().lookup_f32([coords.to(dev), out] + lv_g, [L, B, h, w, r])
    torch.cuda.synchronize()
    for a, b in zip(lv_g, pyr):
        assert (a.cpu() - b).abs().max().item() < 1e-5
    ref = R.index_pyramid(pyr, coords.reshape(B, h, w, 2), r).reshape(M, -1)
    assert (out.cpu() - ref).abs().max().item() < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("factory", [raft_small, raft_large])
@pytest.mark.parametrize("use_graph", [False, True])
def test_fp32_engine_matches_golden(factory, use_graph):
    """fp32 engine vs the fp32 golden forward: agreement to fp32 rounding, a
    bound ~100x tighter than the bf16 engine's (tests/test_engine_gpu.py)."""
    torch.manual_seed(0)
    model = factory(seed=0)[0].eval()
    i1, i2 = _inputs(2, 128, 256)
    n = 4
    with torch.no_grad():
        ref = model(i1, i2, num_flow_updates=n)
        eng = E.RaftEngine(model.cuda(), torch.device("cuda", 0), precision="fp32", use_graph=use_graph)
        out = eng.forward(i1.cuda(), i2.cuda(), n).cpu()
    torch.cuda.synchronize()
    assert out.shape == ref.shape
    err = (out - ref).norm(dim=-1).mean().item()
    assert err < 1e-3 * (1 + ref.norm(dim=-1).mean().item()), err


@pytest.mark.gpu
def test_fp32_engine_pipelined_equals_forward():
    """Graph-pipelined steps (bench.py's batch-1 path) give forward()'s flows, bitwise."""
    model = raft_small(seed=0)[0].eval().cuda()
    eng = E.RaftEngine(model, torch.device("cuda", 0), precision="fp32")
    ins = [_inputs(1, 128, 256, seed=s) for s in (5, 6, 7)]
    with torch.no_grad():
        ref = [eng.forward(a.cuda(), b.cuda(), 3) for a, b in ins]
        outs = [eng.pipelined(a.cuda(), b.cuda(), 3) for a, b in ins]
        outs.append(eng.flush())
    torch.cuda.synchronize()
    assert outs[0] is None
    for r, o in zip(ref, outs[1:]):
        assert torch.equal(r, o)


def _cp_worker(rank, world, port, arch, out):
    import os

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(2)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    nat.require = lambda: None
    nat.new_plan = F32Interp
    tunedb.gpu_arch = lambda device=None: "cpu"
    model = (raft_large if arch == "raft_large" else raft_small)(seed=0)[0].eval()
    i1, i2 = _inputs(2, 128, 160, seed=7)
    with torch.no_grad():
        eng = E.RaftEngine(model, "cpu", precision="fp32", cp_group=True, copy_output=False)
        flows = eng.forward(i1, i2, 2).clone()
        st = next(iter(eng._states.values()))
        assert st.cp is not None and st.plan.names(1) == ["lookup_f32"] * 2
    parts = [torch.empty_like(flows) for _ in range(world)]
    torch.distributed.all_gather(parts, flows)
    if rank == 0:
        torch.save(torch.stack(parts), out)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("arch,world", [("raft_small", 2), ("raft_small", 3), ("raft_large", 2)])
def test_engine_context_parallel_gloo(tmp_path, arch, world):
    """Context parallelism on the native engine (cp_group): 16 query rows over 2 / 3
    gloo ranks (3: uneven slabs), each rank's plan holding its slab's pyramid, the
    looked-up features all-gathered between the two halves of every iteration; the
    fp32 plans run by the interpreter reproduce the single-process golden forward."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "cp.pt")
    mp.spawn(_cp_worker, args=(world, port, arch, out), nprocs=world, join=True)
    got = torch.load(out, weights_only=True)
    for r in range(1, world):
        assert torch.equal(got[r], got[0])
    model = (raft_large if arch == "raft_large" else raft_small)(seed=0)[0].eval()
    i1, i2 = _inputs(2, 128, 160, seed=7)
    with torch.no_grad():
        ref = model(i1, i2, num_flow_updates=2)
    err = (got[0] - ref).abs().max().item()
    assert err < 2e-3 * (1 + ref.abs().max().item()), err
