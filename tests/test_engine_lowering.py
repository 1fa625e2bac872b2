"""CPU checks of the inference engine's plan lowering (runtime/engine.py): the
op sequence each schedule records, without a GPU (a recording stand-in for
the native Plan; weights packed on the CPU).  The numerics of the same plans
are covered on the MI355X by tests/test_engine_gpu.py."""
import pytest
import torch

from jax_raft_amd import raft_large, raft_small
from jax_raft_amd.ops import native as nat
from jax_raft_amd.runtime import engine as E
from jax_raft_amd.runtime import tunedb


class FakePlan:
    """Records (segment, lane, defer, op) for every add_* call."""

    def __init__(self):
        self.ops = []
        self.seg, self.ln, self.defer = 0, 0, 0

    def set_segment(self, s):
        self.seg = s

    def set_lane(self, l):
        self.ln = l

    def set_defer(self, d):
        self.defer = d

    def __getattr__(self, name):
        if not name.startswith("add_"):
            raise AttributeError(name)

        def rec(*args):
            self.ops.append((self.seg, self.ln, self.defer, name[4:], args))
        return rec

    def names(self, seg):
        return [op for s, _, _, op, _ in self.ops if s == seg]


@pytest.fixture
def fake(monkeypatch):
    monkeypatch.setattr(nat, "require", lambda: None)
    monkeypatch.setattr(nat, "new_plan", FakePlan)
    monkeypatch.setattr(tunedb, "gpu_arch", lambda device=None: "cpu")


def _plan(factory, B, all_iters=True, streams="auto", H=128, W=256):
    model = factory()[0].eval()
    eng = E.RaftEngine(model, "cpu", autotune=False, streams=streams)
    st = eng._build(B, H, W, 3, all_iters)
    return eng, st.plan


@pytest.mark.parametrize("gru", ["unfused", "halo"])
def test_lane_schedule_raft_large(fake, gru, monkeypatch):
    monkeypatch.setattr(E.RaftEngine, "GRU", gru)
    eng, p = _plan(raft_large, 4)
    assert eng.uses_lanes(4) and not eng.uses_lanes(1) and not eng.uses_lanes(4, all_iters=False)
    loop = [(ln, d, op) for s, ln, d, op, _ in p.ops if s == 1]
    ops = [op for _, _, op in loop]
    # critical lane: lookup (+ update) -> cc1 (LDS kernel) -> cc2 -> motion -> 2 x GRU -> FlowHead taps
    assert ops.count("lookup") == 1 and ops.count("flow_taps") == 0
    stages = ["conv"] * 4 if gru == "unfused" else ["gru_halo"] * 2
    assert [op for ln, d, op in loop if ln == 0 and op not in ("record", "wait")] == \
        ["lookup", "conv1x1", "conv", "conv"] + stages + ["conv"]
    # mask lane: deferred flow features + mask conv + convex head of the previous iteration
    side = [op for ln, d, op in loop if ln == 2 and op not in ("record", "wait")]
    assert side == ["conv_direct", "conv", "conv", "convex_head"]
    assert all(d == 1 for ln, d, op in loop if ln == 2 and op not in ("record", "wait"))
    assert p.names(2).count("flow_taps") == 1 and p.names(2).count("convex_head") == 1
    # three cross-lane waits per iteration
    assert ops.count("wait") == 3


def test_lane_schedule_fused_gru_parity(fake, monkeypatch):
    """Default lane schedule with the fused ConvGRU: the last stage writes the mask lane's h
    copy into hm / hm2 by iteration parity, the update writes the flow into flow32 / flow32b,
    the lane's mask conv and convex head read the matching buffer -- and the E_MASK join is
    gone (two waits per iteration: the lane's E_FH fork and the E_FLOW join).  Opt-in
    (RaftEngine.MASK_PARITY = True): measured slower on MI355X."""
    monkeypatch.setattr(E.RaftEngine, "GRU", "fused")
    monkeypatch.setattr(E.RaftEngine, "MASK_PARITY", True)
    eng, p = _plan(raft_large, 4)
    loop = [(ln, d, op, a) for s, ln, d, op, a in p.ops if s == 1]
    main = [op for ln, d, op, _ in loop if ln == 0]
    assert [op for op in main if op not in ("record", "wait")] == \
        ["lookup", "conv1x1", "conv", "conv", "gru_fused", "gru_fused", "conv"]
    assert [op for _, _, op, _ in loop].count("wait") == 2
    i1, i2 = [i for i, op in enumerate(main) if op == "gru_fused"]
    assert main[i1 - 1] != "wait" and main[i2 - 1] != "wait"
    g1, g2 = [a for _, _, op, a in loop if op == "gru_fused"]
    hm, hm2 = g2[0][6], g2[0][8]
    assert g1[0][6] is None and len(g1[0]) == 7 and hm is not None and hm2 is not None and hm2 is not hm
    side = [(d, op, a) for ln, d, op, a in loop if ln == 2]
    alt = [a for d, op, a in side if op == "conv_alt"]
    assert len(alt) == 1 and alt[0][0][0] is hm and alt[0][-1] is hm2   # mask conv: hm (even) / hm2 (odd)
    lk = [a for _, _, op, a in loop if op == "lookup"][0]
    cx = [a for d, op, a in side if op == "convex_head"][0]
    assert lk[0][12] is cx[0][6] and lk[0][8] is cx[0][3]               # flow32 / flow32b pair
    epi = [(op, a) for s, ln, d, op, a in p.ops if s == 2]
    ft = [a for op, a in epi if op == "flow_taps"][0]
    assert ft[0][7] is cx[0][6]


def test_lane_schedule_fused_gru(fake, monkeypatch):
    """raft_large with the fused ConvGRU stages (gru_fused.hip, forced on at this small
    size), the default schedule (no parity buffers): one gru_fused op per stage on the
    critical lane, the mask lane's mask conv reads its own h copy `hm` (written by the last
    stage), and the E_MASK wait moves from the first stage to the last one (three waits per
    iteration)."""
    monkeypatch.setattr(E.RaftEngine, "GRU", "fused")
    eng, p = _plan(raft_large, 4)
    loop = [(ln, d, op, a) for s, ln, d, op, a in p.ops if s == 1]
    main = [op for ln, d, op, _ in loop if ln == 0]
    assert [op for op in main if op not in ("record", "wait")] == \
        ["lookup", "conv1x1", "conv", "conv", "gru_fused", "gru_fused", "conv"]
    i1, i2 = [i for i, op in enumerate(main) if op == "gru_fused"]
    assert main[i2 - 1] == "wait" and main[i1 - 1] != "wait"
    assert [op for _, _, op, _ in loop].count("wait") == 3
    g1, g2 = [a for _, _, op, a in loop if op == "gru_fused"]
    assert g1[0][6] is None and g2[0][6] is not None           # only the last stage writes hm
    assert g1[1][3] == 0 and g2[1][3] == 1                      # 1x5 (rows), then 5x1 (columns)
    hm = g2[0][6]
    mask_convs = [a for ln, d, op, a in loop if ln == 2 and op == "conv"]
    assert any(t[0] is hm for t, *_ in mask_convs)             # the mask conv reads hm
    assert not eng._gru_fused_ok(1, 55, 128) or eng._gru_fused_ok(4, 55, 128)
    monkeypatch.setattr(E.RaftEngine, "GRU", "auto")
    assert eng._gru_fused_ok(4, 55, 128) and not eng._gru_fused_ok(1, 55, 128)
    assert not eng._gru_fused_ok(4, 55, 129)                    # a row wider than a tile


def test_fused_gru_not_for_raft_small(fake, monkeypatch):
    monkeypatch.setattr(E.RaftEngine, "GRU", "fused")
    _, p = _plan(raft_small, 4)
    assert "gru_fused" not in p.names(1)


def test_halo_gru_raft_large_buffers(fake, monkeypatch):
    """gru_halo lowering of raft_large (any batch): stage 1 (1x5 runs) reads [h | x] from hx
    and writes h' into qx; stage 2 (5x1 runs) reads h' from qx, x from hx and writes hx (never
    in place: neighbouring tiles read h); qx's [motion | flow] part is no longer written."""
    monkeypatch.setattr(E.RaftEngine, "GRU", "halo")
    for B, lanes in ((1, False), (4, True)):
        eng, p = _plan(raft_large, B)
        assert eng.gru_path == "halo"
        g = [a for s, ln, d, op, a in p.ops if s == 1 and op == "gru_halo"]
        assert len(g) == 2
        (t1, i1), (t2, i2) = g
        hx, qx = t1[0], t1[6]
        assert t1[1] is hx and t2[0] is qx and t2[1] is hx and t2[6] is hx and t1[6] is not hx
        assert i1[3:5] == [0, 0] and i2[3:5] == [0, 1]                 # 1x5 along W, then 5x1 along H
        assert nat.gru_halo_geom_ok(128, 0, *i1[5:]) and nat.gru_halo_geom_ok(128, 0, *i2[5:])
        assert (t2[7] is not None) == lanes and t1[7] is None          # hm copy only for the mask lane
        mc = [a for s, ln, d, op, a in p.ops if s == 1 and op == "conv" and a[0][0] is not None
              and a[0][4] is not None and a[0][4] is qx]
        assert not mc                                                  # me.conv no longer copies into qx


def test_halo_gru_raft_small_ping_pong(fake, monkeypatch):
    """raft_small's single 3x3 stage ping-pongs h between hx and qx: even iterations read hx
    and write qx, odd ones the reverse, and the FlowHead conv reads the buffer just written."""
    monkeypatch.setattr(E.RaftEngine, "GRU", "auto")
    eng, p = _plan(raft_small, 1)
    assert eng.gru_path == "halo"
    (t, i), = [a for s, ln, d, op, a in p.ops if s == 1 and op == "gru_halo"]
    hx, qx = t[0], t[6]
    assert t[1] is hx and t[8] is qx and t[9] is qx and t[10] is hx and qx is not hx
    assert i[3] == 1 and nat.gru_halo_geom_ok(96, 1, *i[5:])
    (fh,) = [a for s, ln, d, op, a in p.ops if s == 1 and op == "conv_alt"]
    assert fh[0][0] is qx and fh[3] is hx


@pytest.mark.parametrize("merged", ["1", "0"])
@pytest.mark.parametrize("factory", [raft_large, raft_small])
def test_one_lane_schedule(factory, fake, merged, monkeypatch):
    monkeypatch.setattr(E.RaftEngine, "MERGED_UP", merged == "1")
    eng, p = _plan(factory, 1)
    assert not eng.uses_lanes(1)
    loop = [(ln, d, op) for s, ln, d, op, _ in p.ops if s == 1]
    assert {ln for ln, _, _ in loop} == {0} and not any(op in ("record", "wait") for _, _, op in loop)
    ops = [op for _, _, op in loop]
    assert ops[0] == "lookup" and "flow_taps" not in ops   # the update runs inside the lookup
    up = "convex_head" if factory is raft_large else "upsample_bilinear"
    if merged == "1":   # flow conv + the previous iteration's upsampling in one grid (merged.hip)
        assert ops[1] == "flowin_dual" and up not in ops and "conv_direct" not in ops
        assert all(d == 0 for _, d, _ in loop)
        ints = [a for s, ln, d, op, a in p.ops if s == 1 and op == "flowin_dual"][0][1]
        assert ints[11] == (2 if factory is raft_large else 1)
        # raft_large: convcorr1 (the 1x1 LDS-weight conv) runs in the same merged grid
        assert (len(ints) == 21 and "conv1x1" not in ops) if factory is raft_large else len(ints) == 15
    else:
        assert ops.count(up) == 1 and [d for _, d, op in loop if op == up] == [1]
        assert ("conv1x1" in ops) == (factory is raft_large)
    assert "taps_gemm" in ops   # raft_large: fused 128 -> 512 FlowHead/mask conv + taps GEMM
    assert p.names(2) == ["flow_taps", up]


@pytest.mark.parametrize("group", ["1", "0"])
@pytest.mark.parametrize("factory", [raft_large, raft_small])
def test_one_lane_grouped_corr_flow_conv(factory, fake, group, monkeypatch):
    """One-lane schedule: the last correlation conv and convflow2 as one grid in the corr
    conv's tile config (when a grouped launch serves it)."""
    monkeypatch.setattr(E.RaftEngine, "CONV_GROUP", group == "1")
    last = "me.convcorr2" if factory is raft_large else "me.convcorr1"
    model = factory()[0].eval()
    eng = E.RaftEngine(model, "cpu", autotune=False, cfg_override={last: 2})
    p = eng._build(1, 128, 256, 3, True).plan
    ops = p.names(1)
    if group == "1":
        g = [a for s, ln, d, op, a in p.ops if s == 1 and op == "conv_group"]
        assert len(g) == 1 and ops.index("conv_group") > ops.index("flowin_dual")
        t1, i1, _, t2, i2, _ = g[0]
        assert t1[3] is t2[3] and eng.chosen_cfgs["me.convflow2"] == 2   # both write cf; one config
    else:
        assert "conv_group" not in ops
    eng2 = E.RaftEngine(model, "cpu", autotune=False, cfg_override={last: 99})
    assert "conv_group" not in eng2._build(1, 128, 256, 3, True).plan.names(1)   # no grouped variant


@pytest.mark.parametrize("factory", [raft_large, raft_small])
def test_final_only_schedule(factory, fake):
    eng, p = _plan(factory, 4, all_iters=False)
    ops = p.names(1)
    assert "flow_taps" in ops and "convex_head" not in ops and "upsample_bilinear" not in ops
    ep = p.names(2)
    assert ep[-1] == ("convex_head" if factory is raft_large else "upsample_bilinear")


def test_engine_knobs_are_few(fake):
    import inspect

    params = [n for n in inspect.signature(E.RaftEngine.__init__).parameters if n not in ("self", "model", "device")]
    assert len(params) <= 10, params


@pytest.mark.parametrize("factory", [raft_large, raft_small])
def test_context_parallel_schedule(factory, fake):
    """cp_group: the slab lookups (one per image) alone in loop segment 1, the rest
    of the iteration in segment 3 (after the engine's all-gather), per-image slab
    correlation in the prologue, no cross-lane events, no deferred ops."""
    model = factory()[0].eval()
    eng = E.RaftEngine(model, "cpu", autotune=False, cp_group=True)
    st = eng._build(2, 128, 256, 3, True)
    p = st.plan
    assert st.cp is not None and not eng.uses_lanes(2)
    assert p.names(1) == ["lookup", "lookup"]
    seg3 = p.names(3)
    assert "lookup" not in seg3 and seg3.count("flow_taps") == 1
    assert seg3[-1] in ("convex_head", "upsample_bilinear", "upsample_convex")
    assert p.names(0).count("corr") == 2
    assert not any(op in ("record", "wait") for s, _, _, op, _ in p.ops if s in (1, 3))
    assert all(d == 0 for s, _, d, _, _ in p.ops)
    # one slab of every query row without a process group
    assert st.cp["slabs"] == [(0, 16)]


def test_grouped_launch_uses_the_pair_config(fake, monkeypatch):
    """A persisted decision for the PAIR (tuned DB key "group" + both problems) overrides the
    first conv's own tile config in the grouped launch; without one the first conv's stays."""
    model = raft_large()[0].eval()
    seen = []

    def peek(arch, key):
        seen.append(key)
        return 24 if key[0] == "group" else None

    monkeypatch.setattr(tunedb, "peek", peek)
    eng = E.RaftEngine(model, "cpu", autotune=True)
    monkeypatch.setattr(eng, "_conv_kw", lambda spec, x, N, H, W, y, kw: dict(kw, cfg=23))
    p = eng._build(1, 128, 256, 3, True).plan
    g = [a for s, ln, d, op, a in p.ops if s == 1 and op == "conv_group"]
    assert len(g) == 1 and g[0][1][20] == 24 and g[0][4][20] == 24       # ints[20] = cfg
    assert seen and seen[0][:2] == ("group", 16 * 32)
    monkeypatch.setattr(tunedb, "peek", lambda arch, key: None)
    p = eng._build(1, 128, 256, 3, True).plan
    g = [a for s, ln, d, op, a in p.ops if s == 1 and op == "conv_group"]
    assert g[0][1][20] == 23 and g[0][4][20] == 23


@pytest.mark.parametrize("fuse", ["1", "0"])
def test_encoder_instance_norm_fused_into_halo_convs(fake, monkeypatch, fuse):
    """raft_large's feature encoder (instance norm): with RaftEngine.HALO_NORM on, every 3x3 / stride-1
    conv runs on a halo config that writes its statistics partials (one stats_final each, no
    channel_stats pass) and the conv after it normalises on load (the block-internal norm_act
    passes disappear); a block output (or the stem's) is built inside the next block's first
    conv when that is a stride-1 halo conv, which writes it out for the residual; only the
    outputs feeding a stride-2 block or the final 1x1 conv are materialised by norm_act."""
    monkeypatch.setattr(E.RaftEngine, "HALO_NORM", fuse == "1")
    monkeypatch.setattr(E.RaftEngine, "PRO_LANES", "off")   # one feature-encoder pass over both images
    eng, p = _plan(raft_large, 1)
    pro = p.names(0)
    fe_ops = [(op, a) for s, ln, d, op, a in p.ops if s == 0]
    halo_convs = [a for op, a in fe_ops if op == "conv" and a[1][20] >= nat.HALO_CFG0]
    if fuse == "1":
        # per encoder image set: 10 stride-1 3x3 convs (4 in layer 1, 3 in layers 2 and 3)
        assert pro.count("stats_final") == 10 and len(halo_convs) == 10
        with_norm = [a for a in halo_convs if len(a[0]) > 14 and a[0][14] is not None]
        assert len(with_norm) == 10           # every halo conv builds its input
        with_res = [a for a in with_norm if len(a[0]) > 17 and a[0][15] is not None]
        assert len(with_res) == 3 and all(a[0][17] is not None for a in with_res)   # L1B1, L2B1, L3B1 conv1
        ds_res = [a for a in with_res if a[0][16] is not None]
        assert len(ds_res) == 2               # layers 2 / 3 block 1: the residual is block 0's downsample
        assert pro.count("norm_act") == 3     # outputs of L1B1 / L2B1 (before stride-2 blocks), L3B1
    else:
        assert "stats_final" not in pro and pro.count("norm_act") == 1 + 6 + 6


@pytest.mark.parametrize("arch", [raft_large, raft_small])
def test_prologue_lanes_at_batch_one(fake, monkeypatch, arch):
    """At batch 1 ("auto") the context encoder runs on lane 1 and the feature encoder as ONE
    batch-2 chain over both images on lane 0 with the pyramid (measured faster,
    profiles/r6_ce_lane_b1_ab.txt); RaftEngine.PRO_LANES = "on" adds image 2's feature encoder
    on lane 2; "off" keeps the whole forward on lane 0.  The loop stays on one lane."""
    eng, p = _plan(arch, 1)
    pro_lanes = {ln for s, ln, d, op, a in p.ops if s == 0}
    loop_lanes = {ln for s, ln, d, op, a in p.ops if s == 1}
    assert pro_lanes == {0, 1} and loop_lanes == {0}
    monkeypatch.setattr(E.RaftEngine, "PRO_LANES", "on")
    eng, p = _plan(arch, 1)
    assert {ln for s, ln, d, op, a in p.ops if s == 0} == {0, 1, 2}
    monkeypatch.setattr(E.RaftEngine, "PRO_LANES", "off")
    eng, p = _plan(arch, 1)
    assert {ln for s, ln, d, op, a in p.ops} == {0}


@pytest.mark.parametrize("factory", [raft_large, raft_small])
def test_final_only_schedule_batch1(factory, fake):
    """Final-only below batch 4: the all-iterations one-lane order -- the update inside the
    lookup, the 7x7 flow conv in the merged grid whose bilinear half writes the single output
    slot (iteration stride 0), the last update + the one upsampling in the epilogue."""
    eng, p = _plan(factory, 1, all_iters=False)
    ops = p.names(1)
    assert ops[0] == "lookup" and ops[1] == "flowin_dual" and "flow_taps" not in ops
    assert "convex_head" not in ops and "conv_direct" not in ops
    ints = [a for s, ln, d, op, a in p.ops if s == 1 and op == "flowin_dual"][0][1]
    assert len(ints) == 15 and ints[11] == 1 and ints[12] == 0   # bilinear, iteration stride 0
    ep = p.names(2)   # (raft_large: + the mask head's 3x3 conv before the convex head)
    assert ep[0] == "flow_taps" and ep[-1] == ("convex_head" if factory is raft_large else "upsample_bilinear")


def test_stale_check_sees_every_change(fake):
    """The per-forward staleness check (RaftEngine._stale, a flat snapshot walk instead of the
    tuple signature) notices in-place updates, replaced parameters / buffers / submodules and
    new entries -- and nothing else."""
    import torch.nn as nn

    model = raft_small()[0].eval()
    eng = E.RaftEngine(model, "cpu", autotune=False)
    assert not eng._stale()
    p = next(model.parameters())
    with torch.no_grad():
        p.add_(1.0)                                  # optimizer-style in-place update
    assert eng._stale()
    eng._pack()
    assert not eng._stale()
    conv = model.update_block.flow_head.conv2
    conv.kernel = nn.Parameter(conv.kernel.detach().clone())   # replaced parameter
    assert eng._stale()
    eng._pack()
    model.update_block.flow_head.register_buffer("extra", torch.zeros(1))   # a new entry
    assert eng._stale()
    eng._pack()
    import copy
    model.update_block.flow_head.conv2 = copy.deepcopy(model.update_block.flow_head.conv2)   # replaced submodule
    assert eng._stale()
    eng._pack()
    assert not eng._stale()
    model(torch.zeros(1, 128, 128, 3), torch.zeros(1, 128, 128, 3), num_flow_updates=1)   # a CPU forward: no change
    assert not eng._stale()


@pytest.mark.parametrize("factory", [raft_small, raft_large])
def test_mixed_precision_lowering(fake, factory):
    """precision="mixed" (runtime/engine_f32.py:RaftEngineMixed): the bf16 plan has no feature
    encoder (its fmap buffer is filled before each replay) but keeps the context encoder, the
    pyramid and the loop; the fp32 plan holds the feature encoder of both images and its final
    1x1 conv on the fp32 kernels."""
    model = factory()[0].eval()
    eng = E.RaftEngine(model, "cpu", autotune=False, precision="mixed")
    ref = E.RaftEngine(model, "cpu", autotune=False)
    st = eng._build(1, 128, 256, 3)
    st_ref = ref._build(1, 128, 256, 3)
    pro = [op for s, _, _, op, _ in st.plan.ops if s == 0]
    pro_ref = [op for s, _, _, op, _ in st_ref.plan.ops if s == 0]
    assert len(pro) < len(pro_ref) and "corr" in pro and "prep" in pro
    # the loop is the bf16 engine's
    assert st.plan.names(1) == st_ref.plan.names(1)
    fplan = st.fe32[0]
    fops = fplan.names(0)
    assert fops[0] == "prep_f32" and fops.count("conv_f32") == sum(
        1 for n in eng._f32._specs if n.startswith("fe.") and not n.endswith("stem_s2d"))
    assert st.fe32[2].dtype == torch.float32 and st.fe32[3] is st.bufs["p0.fmap"]
