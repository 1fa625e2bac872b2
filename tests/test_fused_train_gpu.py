"""Fused native training path of the refinement loop (jax_raft_amd/train/fused.py)
against the unfused native autograd path and fp32 CPU autograd of the golden
model, plus the training-only kernels (upsampling adjoints) against torch
autograd of the reference ops."""
import pytest
import torch

from jax_raft_amd import raft_large, raft_small
from jax_raft_amd.models import reference as R

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float().cpu() - b.float().cpu()).norm() / (b.float().cpu().norm() + 1e-8)).item()


def _cos(a, b):
    a, b = a.float().cpu().flatten(), b.float().cpu().flatten()
    return (torch.dot(a, b) / (a.norm() * b.norm() + 1e-12)).item()


@pytest.mark.parametrize("B,h,w", [(2, 5, 7), (1, 5, 7), (3, 6, 16)])   # odd pixel counts: a half-idle last wave
def test_upsample_convex_bwd_kernel(B, h, w):
    from jax_raft_amd.ops import native as nat

    torch.manual_seed(0)
    M = B * h * w
    mask = (torch.randn(B, h, w, 576) * 2).to(torch.bfloat16).float()
    flow = torch.randn(B, h, w, 2) * 3
    g = torch.randn(B, 8 * h, 8 * w, 2)
    a = 0.25
    m_ = (mask / a).requires_grad_(True)   # conv output before the multiplier
    f_ = flow.clone().requires_grad_(True)
    up = R.upsample_flow(f_, m_ * a)
    (up * g).sum().backward()
    dm = torch.empty(M, 576, dtype=torch.bfloat16, device="cuda")
    taps = torch.empty(M, 18, device="cuda")
    nat.ops().upsample_convex_bwd([mask.reshape(M, 576).to(torch.bfloat16).cuda(), flow.reshape(M, 2).cuda(),
                                   g.cuda(), dm, taps], [B, h, w], a)
    dflow = torch.empty(M, 8, dtype=torch.bfloat16, device="cuda")
    nat.ops().flow_gather_bwd([taps, dflow], [B, h, w])
    torch.cuda.synchronize()
    assert _rel(dm, m_.grad.reshape(M, 576)) < 1e-2
    assert _rel(dflow[:, :2], f_.grad.reshape(M, 2)) < 1e-2
    assert dflow[:, 2:].abs().max().item() == 0


def test_upsample_bilinear_bwd_kernel():
    from jax_raft_amd.ops import native as nat

    torch.manual_seed(1)
    B, h, w = 2, 16, 20
    M = B * h * w
    flow = torch.randn(B, h, w, 2).requires_grad_(True)
    g = torch.randn(B, 8 * h, 8 * w, 2)
    (R.upsample_flow(flow, None) * g).sum().backward()
    d = torch.empty(M, 8, dtype=torch.bfloat16, device="cuda")
    nat.ops().upsample_bilinear_bwd([g.cuda(), d], [B, h, w])
    torch.cuda.synchronize()
    assert _rel(d[:, :2], flow.grad.reshape(M, 2)) < 1e-2


def _setup(factory, B=2, H=128, W=160, seed=3):
    torch.manual_seed(seed)
    model, _ = factory()
    model = model.cuda().train()
    g = torch.Generator().manual_seed(seed)
    i1 = torch.rand(B, H, W, 3, generator=g) * 2 - 1
    i2 = torch.rand(B, H, W, 3, generator=g) * 2 - 1
    target = torch.randn(B, H, W, 2, generator=g) * 4
    return model, i1, i2, target


def _run(model, i1, i2, target, iters, fused):
    model.zero_grad(set_to_none=True)
    out = model(i1.cuda(), i2.cuda(), train=True, num_flow_updates=iters, fused=fused)
    w = torch.tensor([0.8 ** (iters - k - 1) for k in range(iters)], device="cuda").view(-1, 1, 1, 1, 1)
    (w * (out.float() - target.cuda()).abs()).mean().backward()
    torch.cuda.synchronize()
    return out.detach(), {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("encoders", [True, False], ids=["whole-model", "loop-only"])
@pytest.mark.parametrize("factory", [raft_large, raft_small])
def test_fused_matches_unfused(factory, encoders, monkeypatch):
    """Both GPU paths against fp32 CPU autograd of the golden model: the fused
    gradients are at least as close to the fp32 reference as the unfused
    path's (two bf16 paths differ from each other by ~the bf16 noise of the
    early encoder layers, cos ~0.97, so they are not compared directly)."""
    from jax_raft_amd.train import fused as F

    monkeypatch.setattr(F, "FUSED_ENCODERS", encoders)
    F._LOOPS.clear()
    model, i1, i2, target = _setup(factory)
    state = {k: v.clone() for k, v in model.state_dict().items()}
    mc = factory()[0]
    mc.load_state_dict({k: v.cpu() for k, v in state.items()})
    mc.train()
    iters = 3
    out_r = mc(i1, i2, train=True, num_flow_updates=iters)
    w = torch.tensor([0.8 ** (iters - k - 1) for k in range(iters)]).view(-1, 1, 1, 1, 1)
    (w * (out_r - target).abs()).mean().backward()
    g_r = {n: p.grad for n, p in mc.named_parameters() if p.grad is not None}
    out_u, g_u = _run(model, i1, i2, target, iters, fused=False)
    bufs_u = {k: v.clone() for k, v in model.state_dict().items() if k.endswith(".mean") or k.endswith(".var")}
    model.load_state_dict(state)
    out_f, g_f = _run(model, i1, i2, target, iters, fused=True)
    for k, v in model.state_dict().items():   # BatchNorm running statistics updated alike
        if k in bufs_u:
            assert _rel(v, bufs_u[k]) < 1e-2, k
    assert out_f.shape == out_u.shape
    ef, eu = _rel(out_f, out_r), _rel(out_u, out_r)
    assert ef < max(2e-2, 1.5 * eu), (ef, eu)
    assert set(g_f) == set(g_u) == set(g_r)
    _assert_as_accurate(g_f, g_u, g_r)


def _assert_as_accurate(g_f, g_u, g_r):
    """Per parameter, the fused gradient's relative error against fp32 autograd is within 1.3x
    (+ 0.03) of the unfused path's, and the median error within 1.1x (+ 0.005).  (The whole-model
    errors themselves are large -- median ~0.2 for raft_large -- because the early encoder layers'
    weight gradients cancel through the instance norms and carry the bf16 noise of both paths;
    measured: dev/probes/fused_rel_errors.py.  The loop alone is held to tighter absolute bounds by
    test_fused_loop_gradient_oracle.)"""
    scale = max(v.norm().item() for v in g_r.values())
    bad, efs, eus = [], [], []
    for n in g_r:
        if g_r[n].norm().item() < 1e-4 * scale:
            continue  # e.g. biases feeding an InstanceNorm: exactly-zero true gradient, rounding noise
        ef, eu = _rel(g_f[n], g_r[n]), _rel(g_u[n], g_r[n])
        efs.append(ef)
        eus.append(eu)
        if ef > 1.3 * eu + 0.03:
            bad.append((n, round(ef, 4), round(eu, 4)))
    assert not bad, bad
    assert sorted(efs)[len(efs) // 2] <= 1.1 * sorted(eus)[len(eus) // 2] + 0.005, (efs, eus)


@pytest.mark.parametrize("factory", [raft_large, raft_small])
def test_fused_matches_cpu_fp32(factory):
    model, i1, i2, target = _setup(factory, seed=5)
    mc = factory()[0]
    mc.load_state_dict(model.state_dict())
    mc.train()
    out = mc(i1, i2, train=True, num_flow_updates=2)
    w = torch.tensor([0.8, 1.0]).view(-1, 1, 1, 1, 1)
    (w * (out - target).abs()).mean().backward()
    ref = {n: p.grad for n, p in mc.named_parameters() if p.grad is not None}
    state = {k: v.clone() for k, v in model.state_dict().items()}
    outg, gg = _run(model, i1, i2, target, 2, fused=True)
    assert _rel(outg, out) < 5e-2  # bf16 convs vs the fp32 golden model (random-init raft_small: ~3 %)
    model.load_state_dict(state)
    _, gu = _run(model, i1, i2, target, 2, fused=False)
    _assert_as_accurate(gg, gu, ref)


def test_fused_graph_equals_eager(monkeypatch):
    from jax_raft_amd.train import fused as F

    model, i1, i2, target = _setup(raft_large, seed=7)
    state = {k: v.clone() for k, v in model.state_dict().items()}
    monkeypatch.setattr(F, "FUSED_GRAPH", False)
    F._LOOPS.clear()
    out_e, g_e = _run(model, i1, i2, target, 2, fused=True)
    monkeypatch.setattr(F, "FUSED_GRAPH", True)
    F._LOOPS.clear()
    model.load_state_dict(state)
    out_g, g_g = _run(model, i1, i2, target, 2, fused=True)
    assert torch.equal(out_e, out_g)
    for n in g_e:
        assert torch.equal(g_e[n], g_g[n]), n


def test_fused_repeated_steps_and_guard():
    """Weights repacked per step (an optimizer step changes the result), and a
    second forward before the first backward is refused."""
    model, i1, i2, target = _setup(raft_large, seed=9)
    opt = torch.optim.SGD(model.parameters(), lr=1e-2)
    losses = []
    for _ in range(3):
        opt.zero_grad()
        out = model(i1.cuda(), i2.cuda(), train=True, num_flow_updates=2, fused=True)
        loss = (out - target.cuda()).abs().mean()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[0] != losses[1] != losses[2]
    a = model(i1.cuda(), i2.cuda(), train=True, num_flow_updates=2, fused=True)
    b = model(i1.cuda(), i2.cuda(), train=True, num_flow_updates=2, fused=True)
    b.sum().backward()
    with pytest.raises(RuntimeError, match="overwritten"):
        a.sum().backward()


@pytest.mark.parametrize("with_valid", [False, True])
def test_native_sequence_loss(with_valid):
    from jax_raft_amd.train.loss import sequence_loss, sequence_loss_reference

    torch.manual_seed(11)
    N, B, H, W = 5, 2, 24, 40
    preds = torch.randn(N, B, H, W, 2) * 3
    gt = torch.randn(B, H, W, 2) * 3
    gt[0, 0, :4] = 500.0  # beyond max_flow: excluded
    valid = (torch.rand(B, H, W) > 0.3).float() if with_valid else None
    pr = preds.clone().requires_grad_(True)
    lr, mr = sequence_loss_reference(pr, gt, valid)
    lr.backward()
    pg = preds.cuda().requires_grad_(True)
    lg, mg = sequence_loss(pg, gt.cuda(), None if valid is None else valid.cuda())
    lg.backward()
    torch.cuda.synchronize()
    assert abs(lg.item() - lr.item()) < 1e-4 * abs(lr.item())
    for k in mr:
        assert abs(mg[k].item() - mr[k].item()) < 1e-4, k
    assert _rel(pg.grad, pr.grad) < 1e-5


def test_fused_plans_follow_swapped_parameters():
    """``RAFT.apply`` with foreign variables (``torch.func.functional_call``) on
    the fused training path runs and differentiates THOSE leaves, not the
    plans cached for the module's own weights; an ordinary step afterwards
    runs the module's own weights again (fused.py:_tensor_sig)."""
    from jax_raft_amd.train import fused as F
    from jax_raft_amd.utils import checkpoint as ckpt

    F._LOOPS.clear()
    model, i1, i2, target = _setup(raft_small, B=1, seed=21)
    i1, i2, tg = i1.cuda(), i2.cuda(), target.cuda()

    def step(fn):
        out = fn()
        (out.float() - tg).abs().mean().backward()
        torch.cuda.synchronize()
        return out.detach().clone()

    model.zero_grad(set_to_none=True)
    o_own = step(lambda: model(i1, i2, train=True, num_flow_updates=2))
    g_own = {n: p.grad.clone() for n, p in model.named_parameters()}
    other = raft_small(seed=1)[0].cuda().train()
    fv = ckpt.variables_from_module(other)          # differentiable CUDA leaves of another init
    o_app = step(lambda: model.apply(fv, i1, i2, train=True, num_flow_updates=2))
    g_app = {n: p.grad.clone() for n, p in other.named_parameters()}
    other.zero_grad(set_to_none=True)
    o_oth = step(lambda: other(i1, i2, train=True, num_flow_updates=2))
    assert torch.equal(o_app, o_oth) and not torch.equal(o_app, o_own)
    for n, p in other.named_parameters():
        assert torch.equal(g_app[n], p.grad), n
    model.zero_grad(set_to_none=True)
    o_again = step(lambda: model(i1, i2, train=True, num_flow_updates=2))
    assert torch.equal(o_again, o_own)
    for n, p in model.named_parameters():
        assert torch.equal(g_own[n], p.grad), n


@pytest.mark.parametrize("where", ["valid", "invalid"])
def test_native_sequence_loss_nonfinite(where):
    """A NaN prediction poisons the native loss as it does the PyTorch
    oracle's -- also at a pixel the valid mask excludes (0 * NaN = NaN), so the
    trainer's non-finite step guard sees it -- and the gradients agree (the
    oracle's abs backward uses sign(NaN) = 0)."""
    from jax_raft_amd.train.loss import sequence_loss, sequence_loss_reference

    torch.manual_seed(12)
    N, B, H, W = 3, 1, 16, 24
    preds = torch.randn(N, B, H, W, 2)
    gt = torch.randn(B, H, W, 2)
    valid = torch.ones(B, H, W)
    valid[0, 3, 5] = 0.0
    y, x = (3, 5) if where == "invalid" else (7, 9)
    preds[1, 0, y, x, 0] = float("nan")
    pr = preds.clone().requires_grad_(True)
    lr, _ = sequence_loss_reference(pr, gt, valid)
    lr.backward()
    pg = preds.cuda().requires_grad_(True)
    lg, _ = sequence_loss(pg, gt.cuda(), valid.cuda())
    lg.backward()
    torch.cuda.synchronize()
    assert torch.isnan(lr) and torch.isnan(lg.cpu())
    gg = pg.grad.cpu()
    assert torch.equal(torch.isnan(gg), torch.isnan(pr.grad))
    fin = ~torch.isnan(pr.grad)
    assert torch.allclose(gg[fin], pr.grad[fin], rtol=1e-5, atol=1e-12)


@pytest.mark.parametrize("factory", [raft_large, raft_small])
def test_native_pack_table_matches_python_packing(factory):
    """The one-launch weight repack of the training plans reproduces the
    PyTorch packing (ops/native.py:pack_weight of the flipped / sliced /
    concatenated kernels) of every forward, data-gradient and tap spec."""
    from jax_raft_amd.train.fused import FusedModel

    torch.manual_seed(13)
    model, _ = factory()
    model = model.cuda().train()
    fm = FusedModel(model, 1, 128, 128, 2, "cuda", use_graph=False)
    specs = list(fm.loop._specs.items())
    for tag, enc in (("fe", fm.fe), ("ce", fm.ce)):
        specs += [(f"{tag}{k}", v) for k, v in enc._specs.items()] + [(f"{tag}T{k}", v) for k, v in enc._tspecs.items()]
    want = {n: (s.w.clone(), s.b.clone()) for n, s in specs}
    fb = fm.loop._fh2_bias.clone()
    for n, s in specs:
        s.w.zero_()
        s.b.zero_()
    fm.loop._fh2_bias.zero_()
    for pk in (fm.loop.packer, fm.fe.packer, fm.ce.packer):
        pk.record(None)
    torch.cuda.synchronize()
    for n, s in specs:
        assert torch.equal(s.w, want[n][0]), n
        assert torch.equal(s.b, want[n][1]), n
    assert torch.equal(fm.loop._fh2_bias, fb)


WG_CASES = [
    # N, H, W, xcs, xoff, cin, cin8, cout, ycs, yoff, kh, kw, stride, pad
    (2, 12, 16, 64, 0, 64, 64, 64, 64, 0, 3, 3, 1, (1, 1)),
    (2, 12, 16, 64, 0, 64, 64, 96, 96, 0, 3, 3, 2, (1, 1)),
    (2, 13, 17, 32, 0, 32, 32, 64, 64, 0, 1, 1, 2, (0, 0)),
    (1, 24, 32, 8, 0, 3, 8, 64, 64, 0, 7, 7, 2, (3, 3)),
    (2, 9, 11, 264, 8, 256, 256, 256, 256, 0, 1, 5, 1, (0, 2)),
    (1, 10, 12, 512, 0, 256, 256, 2, 8, 0, 3, 3, 1, (1, 1)),
    (1, 10, 12, 8, 0, 2, 8, 128, 128, 0, 7, 7, 1, (3, 3)),
    (1, 10, 12, 328, 0, 324, 328, 256, 256, 0, 1, 1, 1, (0, 0)),
    (2, 11, 9, 256, 0, 256, 256, 126, 128, 0, 3, 3, 1, (1, 1)),
    (2, 11, 9, 512, 256, 256, 256, 64, 256, 192, 3, 3, 1, (1, 1)),
    (3, 16, 20, 96, 0, 96, 96, 80, 88, 0, 3, 3, 1, (1, 1)),
    # 256 x 256 tiles (cout >= 192, K >= 1024): a partial cout tile, gradient slices at an offset
    (2, 7, 9, 256, 0, 256, 256, 192, 200, 8, 3, 3, 1, (1, 1)),
    (2, 10, 13, 128, 0, 128, 128, 320, 320, 0, 3, 3, 1, (1, 1)),
    (3, 5, 66, 264, 8, 256, 256, 256, 256, 0, 5, 1, 1, (2, 0)),
]


@pytest.mark.parametrize("case", WG_CASES)
def test_native_wgrad(case):
    """Implicit-GEMM weight / bias gradient (csrc/kernels/wgrad.hip) against
    fp32 autograd of the conv on the same bf16 operands."""
    from jax_raft_amd.ops import native as nat

    N, H, W, xcs, xoff, cin, cin8, cout, ycs, yoff, kh, kw, s, pad = case
    torch.manual_seed(17)
    OH = (H + 2 * pad[0] - kh) // s + 1
    OW = (W + 2 * pad[1] - kw) // s + 1
    x = torch.randn(N, H, W, xcs).to(torch.bfloat16)
    dy = torch.randn(N, OH, OW, ycs).to(torch.bfloat16)
    xr = x[..., xoff:xoff + cin].float().requires_grad_(False)
    k = torch.zeros(kh, kw, cin, cout, requires_grad=True)
    b = torch.zeros(cout, requires_grad=True)
    y = R.conv2d_nhwc(xr, k, b, (s, s), pad)
    y.backward(dy[..., yoff:yoff + cout].float())
    dw = torch.empty(kh, kw, cin, cout, device="cuda")
    db = torch.empty(cout, device="cuda")
    nat.ops().wgrad([x.cuda(), dy.cuda(), dw, db],
                    [N, H, W, xoff, cin8, kh, kw, s, s, pad[0], pad[1], yoff, OH, OW, cout, cin])
    torch.cuda.synchronize()
    assert _rel(dw, k.grad) < 1e-3, _rel(dw, k.grad)
    assert _rel(db, b.grad) < 1e-3


def test_race_check_tool():
    """tools/race_check.py: inference (graph / eager) and a fused training step
    are bitwise reproducible, and equal under serialised kernel launches
    (AMD_SERIALIZE_KERNEL=3) and per-op checked plans (JR_PLAN_CHECK=1)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "race_check.py"), "--size", "128", "128",
                        "--iters", "2"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "race check ok" in r.stdout


@pytest.mark.parametrize("halo_norm", [True, False], ids=["fused-norms", "norm-passes"])
def test_fused_encoder_norms_on_halo_convs(halo_norm, monkeypatch):
    """raft_large's instance-norm feature encoder in the training forward: with HALO_NORM the
    stride-1 3x3 convs write their output statistics partials in the epilogue and normalise
    (+ residual, relu) their raw input while loading it, writing back the activation the backward
    keeps (no statistics / norm_act passes); without it the separate passes.  Both: gradients
    against fp32 CPU autograd of the golden model as in test_fused_matches_cpu_fp32, and the
    forward plan's op list shows which lowering ran."""
    from jax_raft_amd.train import fused as F
    from jax_raft_amd.train import fused_encoder as FE

    monkeypatch.setattr(FE, "HALO_NORM", halo_norm)
    F._LOOPS.clear()
    model, i1, i2, target = _setup(raft_large, seed=6)
    mc = raft_large()[0]
    mc.load_state_dict(model.state_dict())
    mc.train()
    out = mc(i1, i2, train=True, num_flow_updates=2)
    w = torch.tensor([0.8, 1.0]).view(-1, 1, 1, 1, 1)
    (w * (out - target).abs()).mean().backward()
    ref = {n: p.grad for n, p in mc.named_parameters() if p.grad is not None}
    outg, gg = _run(model, i1, i2, target, 2, fused=True)
    assert _rel(outg, out) < 5e-2
    scale = max(v.norm().item() for v in ref.values())
    fe = {n: _cos(gg[n], ref[n]) for n in ref if n.startswith("feature_encoder.") and ref[n].norm().item() > 1e-4 * scale}
    cos = torch.tensor(list(fe.values()))
    assert cos.median() > 0.97 and cos.min() > 0.7, fe
    fm = next(iter(F._LOOPS[model].values()))
    names = fm.fe.plan_f.op_names(0)
    n_norm, n_stats, n_final = names.count("norm_act"), names.count("stats"), names.count("stats_final")
    # 15 normalised convs; the two downsample norms fold into their block's residual norm_act.
    # Fused: the 10 stride-1 3x3 convs (layer 1, and 3 in each of layers 2 / 3) produce their
    # statistics and normalise their input; norm_act passes remain for the inputs of the two
    # stride-2 convs and of the final 1x1 conv
    if halo_norm:
        assert (n_norm, n_stats, n_final) == (3, 5, 10), (n_norm, n_stats, n_final)
    else:
        assert (n_norm, n_stats, n_final) == (13, 15, 0), (n_norm, n_stats, n_final)


def test_plans_follow_optimizer_updates():
    """After optimizer steps the persistent fused plans must compute what freshly built plans
    compute on the updated weights: every packed weight buffer -- the halo kernels' weight
    streams of the loop's 3x3 convs included -- is refreshed by the per-step repack
    (train/fused.py:Packer).  (Round 5 found those streams left at the first step's weights,
    dev/probes/converge_step2.py: 39.8 vs 78.3.)"""
    from jax_raft_amd.train import fused as F
    from jax_raft_amd.train.data import SyntheticFlow
    from jax_raft_amd.train.loss import sequence_loss

    torch.manual_seed(0)
    model = raft_large()[0].cuda().train()
    img1, img2, flow, valid = SyntheticFlow(size=(192, 256), seed=0, device=torch.device("cuda")).batch([0, 1])
    opt = torch.optim.AdamW(model.parameters(), lr=2e-4, weight_decay=1e-4)
    F._LOOPS.clear()
    for _ in range(2):
        opt.zero_grad(set_to_none=True)
        loss, _ = sequence_loss(model(img1, img2, train=True, num_flow_updates=4, fused=True), flow, valid)
        loss.backward()
        opt.step()
    with torch.no_grad():
        a = model(img1, img2, train=True, num_flow_updates=4, fused=True).float()
        F._LOOPS.clear()
        b = model(img1, img2, train=True, num_flow_updates=4, fused=True).float()
    torch.cuda.synchronize()
    assert _rel(a, b) < 1e-3, _rel(a, b)


def _flat_rel(ga, gb, floor_frac=1e-4):
    """(whole-vector relative difference, worst per-tensor relative difference) of two
    gradient dicts; tensors below ``floor_frac`` of the largest norm are skipped."""
    scale = max(v.norm().item() for v in gb.values())
    num = sum(((ga[n].float() - gb[n].float()) ** 2).sum().item() for n in gb)
    den = sum((gb[n].float() ** 2).sum().item() for n in gb)
    worst = max(_rel(ga[n], gb[n]) for n in gb if gb[n].norm().item() >= floor_frac * scale)
    return (num / den) ** 0.5, worst


def test_fused_trajectory_oracle():
    """Sixteen AdamW steps on the fused path with its persistent plans (as Trainer / bench.py
    run it).  At EVERY step, on that step's weights: freshly built fused plans give the same
    loss and gradients (no state carried across steps: stale packed weights, unrewritten
    buffers -- the round-4 stale halo weight streams parted at step 2, 39.8 vs 78.3), and the
    unfused autograd path gives the same loss within bf16 noise.  tools/train_trajectory.py
    is the 30-step version with fp32 golden gradients (profiles/r6_train_trajectory.json)."""
    from jax_raft_amd.train import fused as F
    from jax_raft_amd.train.data import SyntheticFlow
    from jax_raft_amd.train.loss import sequence_loss

    torch.manual_seed(0)
    F._LOOPS.clear()
    traj = raft_large()[0].cuda().train()
    scratch = raft_large()[0].cuda().train()
    img1, img2, flow, valid = SyntheticFlow(size=(192, 256), seed=0, device=torch.device("cuda")).batch([0, 1])
    opt = torch.optim.AdamW(traj.parameters(), lr=2e-4, weight_decay=1e-4)

    def step(model, fused):
        model.zero_grad(set_to_none=True)
        loss, _ = sequence_loss(model(img1, img2, train=True, num_flow_updates=4, fused=fused).float(), flow, valid)
        loss.backward()
        torch.cuda.synchronize()
        return loss.item(), {n: p.grad.detach().clone() for n, p in model.named_parameters()}

    report = []
    for k in range(16):
        snap = {n: t.detach().clone() for n, t in traj.state_dict().items()}
        lp, gp = step(traj, True)
        scratch.load_state_dict(snap)
        F._LOOPS.pop(scratch, None)
        lf, gf = step(scratch, True)
        scratch.load_state_dict(snap)
        lu, _ = step(scratch, False)
        vec, worst = _flat_rel(gp, gf)
        report.append((k + 1, lp, lf, lu, vec, worst))
        assert abs(lp - lf) <= 1e-3 * abs(lf), report
        assert vec < 1e-2, report
        assert abs(lp - lu) <= 5e-3 * abs(lu), report
        for n, p in traj.named_parameters():
            p.grad = gp[n]
        torch.nn.utils.clip_grad_norm_(traj.parameters(), 1.0)
        opt.step()
    print(report)


def _golden_loop(model, f1, f2, ctx, T):
    """models/raft.py:forward_reference after the encoders (model.py:567-605)."""
    B, h, w, _ = f1.shape
    pyr = model.corr_block.build_pyramid(f1, f2)
    hs = model.update_block.hidden_state_size
    hidden, context = torch.tanh(ctx[..., :hs]), torch.relu(ctx[..., hs:])
    c0 = R.make_coords_grid(B, h, w, device=f1.device)
    c1 = c0.clone()
    preds = []
    for _ in range(T):
        c1 = c1.detach()   # model.py:498
        corr = model.corr_block.index_pyramid(pyr, c1)
        hidden, delta = model.update_block(hidden, context, corr, c1 - c0, True)
        c1 = c1 + delta
        m = None if model.mask_predictor is None else model.mask_predictor(hidden, True)
        preds.append(R.upsample_flow(c1 - c0, m))
    return torch.stack(preds, 0)


def test_fused_loop_gradient_oracle():
    """Per-tensor gradient error of the fused refinement-loop node (FusedRefine, 2 iterations)
    against fp32 autograd of the golden ops on the GPU, on bf16-rounded weights / feature maps /
    context -- the loop alone, so the encoders' bf16 cancellation noise is out of the picture.
    Every tensor is at least as accurate as on the per-op autograd path (within 15 % + 1e-3),
    the median is below 5e-3 and every update-block weight below 2.5e-2.  (The largest errors,
    d_fmap ~7 % and the mask head's 3x3 conv ~5 %, are the sensitivity of those gradients to the
    bf16 storage of the correlation volume: rounding only the pyramid and the looked-up features of
    the fp32 golden model moves them by 6 % / 3.5 % -- dev/probes/loop_oracle.py,
    profiles/r6_loop_oracle.txt.)"""
    from jax_raft_amd.ops.functional import golden_ops
    from jax_raft_amd.train import fused as F

    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = raft_large()[0].to(dev).train()
    with torch.no_grad():
        for p in model.parameters():
            p.copy_(p.bfloat16().float())
    B, H, W, T = 2, 192, 256, 2
    g = torch.Generator(device=dev).manual_seed(1)
    f1 = torch.randn(B, H // 8, W // 8, 256, generator=g, device=dev).bfloat16().float()
    f2 = (0.7 * f1 + 0.7 * torch.randn(B, H // 8, W // 8, 256, generator=g, device=dev)).bfloat16().float()
    ctx = torch.randn(B, H // 8, W // 8, 256, generator=g, device=dev).bfloat16().float()
    target = torch.randn(B, H, W, 2, generator=g, device=dev) * 4
    wts = torch.tensor([0.8 ** (T - k - 1) for k in range(T)], device=dev).view(-1, 1, 1, 1, 1)
    res = {}
    for path in ("fused", "unfused", "golden"):
        model.zero_grad(set_to_none=True)
        x1, x2, xc = (t.clone().requires_grad_(True) for t in (f1, f2, ctx))
        if path == "fused":
            F._LOOPS.clear()
            loop = F.get_loop(model, B, H, W, T, dev)
            out = F.FusedRefine.apply(loop, x1, x2, xc, *loop.params)
        elif path == "unfused":
            out = _golden_loop(model, x1, x2, xc, T)
        else:
            with golden_ops():
                out = _golden_loop(model, x1, x2, xc, T)
        (wts * (out.float() - target).abs()).mean().backward()
        gr = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
        gr.update({"d_fmap1": x1.grad, "d_fmap2": x2.grad, "d_ctx": xc.grad})
        res[path] = gr
    gf, gu, gg = res["fused"], res["unfused"], res["golden"]
    assert set(gf) == set(gg)
    scale = max(v.norm().item() for v in gg.values())
    errs, bad = [], []
    for n, r in gg.items():
        if r.norm().item() < 1e-4 * scale:
            continue
        ef, eu = _rel(gf[n], r), _rel(gu[n], r)
        errs.append(ef)
        if ef > 1.15 * eu + 1e-3 or (n.startswith("update_block.") and ef > 2.5e-2):
            bad.append((n, ef, eu))
    assert not bad, bad
    assert sorted(errs)[len(errs) // 2] < 5e-3, sorted(errs)
