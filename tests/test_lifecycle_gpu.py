"""Native resource lifecycle: engines, their plans (hipGraphs, 64 events and up to 8 lane streams
each, pyramid / loop buffers) and the fused training plans are freed by reference counting when
their owner goes away, and an engine keeps a bounded LRU set of plans.

Round 4 saw a hipGraph capture segfault after ~900 GPU tests in one process, masked then by a
conftest fixture that garbage-collects after every test.  The cause: ``model._engines -> engine ->
model`` and the fused training cache (a module-level dict holding every trained model strongly)
kept every engine's / loop's native state alive until a full collection -- or forever.  These tests
run with the cyclic garbage collector DISABLED, so anything still held by a reference cycle would
accumulate and show up in ``torch.cuda.memory_allocated()``."""
import gc
import weakref

import pytest
import torch

from jax_raft_amd import raft_large, raft_small

pytestmark = pytest.mark.gpu


def _pair(B, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    a = (torch.rand(B, H, W, 3, generator=g) * 2 - 1).cuda()
    b = (torch.rand(B, H, W, 3, generator=g) * 2 - 1).cuda()
    return a, b


def _settle():
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return torch.cuda.memory_allocated()


def test_engines_and_plans_freed_by_refcount():
    """300 plans over varying shapes / iteration counts on 100 directly built engines (LRU of 2
    plans each, so every engine also evicts), then 20 models whose cached engine dies with them,
    all with gc disabled: every engine is unreachable right after its last reference goes, and the
    device memory returns to the baseline."""
    from jax_raft_amd.runtime.engine import RaftEngine

    model, _ = raft_small()
    model = model.cuda()
    dev = torch.device("cuda", 0)
    shapes = [(1, 128, 128), (2, 128, 160), (1, 136, 192), (2, 128, 128)]
    inputs = {s: _pair(*s, seed=i) for i, s in enumerate(shapes)}
    gc.collect()
    base = _settle()
    gc.disable()
    try:
        plans = 0
        dead = []
        for k in range(100):
            shp = shapes[k % len(shapes)]
            eng = RaftEngine(model, dev, autotune=False)
            eng.max_plans = 2
            for n in (2, 3, 4):
                out = eng.forward(*inputs[shp], num_flow_updates=n)
                plans += 1
                assert eng.num_plans() <= 2
            assert out.shape == (4,) + shp + (2,)
            dead.append(weakref.ref(eng))
            del eng, out
            assert dead[-1]() is None, "an engine is held by a reference cycle"
        assert plans >= 300
        assert _settle() <= base, (torch.cuda.memory_allocated(), base)
        # model-owned engines (model(...) -> model.engine, autotuned): no model <-> engine cycle.
        # The first one may leave process-level state behind (autotune trials of configs the
        # persisted table misses); from then on nothing accumulates per model.
        mem = []
        for k in range(20):
            m, _ = raft_small(seed=k)
            m = m.cuda()
            out = m(*inputs[shapes[0]], num_flow_updates=2)
            ref = weakref.ref(m)
            eref = weakref.ref(next(iter(m._engines.values())))
            del m, out
            assert ref() is None and eref() is None, "a model / its engine is held by a reference cycle"
            mem.append(_settle())
        print("memory after each model-owned engine:", mem, "baseline", base)
        assert max(mem[1:]) <= mem[0], (mem, base)
    finally:
        gc.enable()


def test_plan_cache_lru_and_release():
    """The engine keeps at most max_plans key groups (a forward's plan + its pipelined slots are
    one group), evicting the least recently used one; a pending pipelined batch is never evicted;
    release() frees everything."""
    from jax_raft_amd.runtime.engine import RaftEngine

    model, _ = raft_small()
    model = model.cuda()
    eng = RaftEngine(model, torch.device("cuda", 0), autotune=False)
    eng.max_plans = 2
    x = _pair(1, 128, 128, seed=1)
    a = eng.forward(*x, num_flow_updates=2)
    eng.forward(*x, num_flow_updates=3)
    assert eng.num_plans() == 2
    eng.forward(*x, num_flow_updates=2)            # 2 is now the most recently used
    eng.forward(*x, num_flow_updates=4)            # evicts 3
    keys = {k[3] for k in eng._states}
    assert keys == {2, 4}, keys
    assert torch.equal(eng.forward(*x, num_flow_updates=2), a)
    # a pending pipelined batch (two slot plans, one group) survives any number of other shapes
    assert eng.pipelined(*x, num_flow_updates=3) is None
    for n in (5, 6, 7):
        eng.forward(*x, num_flow_updates=n)
    assert any(len(k) > 5 and k[3] == 3 for k in eng._states)
    with pytest.raises(RuntimeError):
        eng.release()
    flushed = eng.flush()
    assert flushed.shape == (3, 1, 128, 128, 2)
    before = _settle()
    eng.release()
    assert eng.num_plans() == 0
    assert _settle() < before
    assert torch.equal(eng.forward(*x, num_flow_updates=2), a)   # rebuilt on demand


def test_fused_training_plans_die_with_the_model():
    """The fused training cache (train/fused.py:_LOOPS) holds its plans per model, weakly: a
    trained model's native forward / backward plans are freed with it."""
    from jax_raft_amd.train import fused as F

    gc.collect()
    base = _settle()
    gc.disable()
    try:
        mem, refs = [], []
        for k in range(4):
            model, _ = raft_large(seed=k)
            model = model.cuda().train()
            i1, i2 = _pair(1, 128, 128, seed=k)
            out = model(i1, i2, train=True, num_flow_updates=2)
            out.abs().mean().backward()
            assert len(F._LOOPS) >= 1
            ref = weakref.ref(model)
            loops = [weakref.ref(o) for o in F._LOOPS[model].values()]
            del model, out
            assert ref() is None, "a trained model is held by the training plan cache"
            assert all(r() is None for r in loops), "a training plan set is held by a reference cycle"
            mem.append(_settle())
        assert len(F._LOOPS) == 0
        # the first step leaves process-level state (the GEMM library's workspace); nothing
        # accumulates per model after it
        print("memory after each trained model:", mem, "baseline", base)
        assert max(mem[1:]) <= mem[0], (mem, base)
    finally:
        gc.enable()
