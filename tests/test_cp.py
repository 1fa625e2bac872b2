"""Context parallelism of the correlation volume (parallel/cp.py) on CPU:
query-row slabs over gloo ranks reproduce the single-process reference forward
(``RAFT.forward_reference`` = jax_raft/model.py:557-605 semantics)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from jax_raft_amd import raft_large, raft_small
from jax_raft_amd.models import reference as R
from jax_raft_amd.parallel.cp import ContextParallelRAFT, pyramid_bytes, row_slabs


def test_row_slabs_partition():
    assert row_slabs(16, 1) == [(0, 16)]
    assert row_slabs(16, 3) == [(0, 6), (6, 11), (11, 16)]
    assert row_slabs(55, 8)[-1] == (49, 55)
    for h, wd in [(55, 8), (17, 4), (16, 16)]:
        s = row_slabs(h, wd)
        assert s[0][0] == 0 and s[-1][1] == h and all(a[1] == b[0] for a, b in zip(s, s[1:]))
        assert max(b - a for a, b in s) - min(b - a for a, b in s) <= 1
    with pytest.raises(AssertionError):
        row_slabs(4, 5)


def test_pyramid_bytes_matches_survey():
    # 440x1024 -> 65.3 M elements, 125 MiB bf16 per pair
    n = pyramid_bytes(1, 440, 1024)
    assert abs(n / 2 - 65.3e6) / 65.3e6 < 0.01
    # 8 slabs of 55 rows: the rank with 7 rows holds 7/55 of it
    assert pyramid_bytes(1, 440, 1024, query_rows=7) * 55 == n * 7


def test_build_pyramid_queries_rows_of_full():
    torch.manual_seed(0)
    f1, f2 = torch.randn(2, 17, 20, 8), torch.randn(2, 17, 20, 8)
    full = R.build_pyramid(f1, f2, 4)
    part = R.build_pyramid_queries(f1[:, 5:11], f2, 4)
    for a, b in zip(full, part):
        ref = a.reshape(2, 17, 20, *a.shape[1:])[:, 5:11].reshape(-1, *a.shape[1:])
        assert torch.allclose(b, ref, atol=1e-5)


def test_cp_single_process_equals_reference():
    model, variables = raft_small(seed=0)
    g = torch.Generator().manual_seed(2)
    i1 = torch.rand(1, 128, 136, 3, generator=g) * 2 - 1
    i2 = torch.rand(1, 128, 136, 3, generator=g) * 2 - 1
    ref = model.apply(variables, i1, i2, num_flow_updates=2)
    out = ContextParallelRAFT(model)(i1, i2, num_flow_updates=2)
    assert torch.allclose(out, ref, atol=1e-4, rtol=1e-4)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs():
    g = torch.Generator().manual_seed(7)
    i1 = torch.rand(2, 128, 160, 3, generator=g) * 2 - 1
    i2 = torch.rand(2, 128, 160, 3, generator=g) * 2 - 1
    return i1, i2


def _cp_worker(rank, world, port, arch, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(2)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    model, _ = (raft_large if arch == "raft_large" else raft_small)(seed=0)
    i1, i2 = _inputs()
    flows = ContextParallelRAFT(model)(i1, i2, num_flow_updates=2)
    parts = [torch.empty_like(flows) for _ in range(world)]
    torch.distributed.all_gather(parts, flows)
    if rank == 0:
        torch.save(torch.stack(parts), out)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("arch,world", [("raft_small", 2), ("raft_small", 3), ("raft_large", 2)])
def test_cp_gloo_matches_reference(tmp_path, arch, world):
    """16 feature rows over 2 / 3 ranks (3: uneven 6/5/5 slabs)."""
    out = str(tmp_path / "cp.pt")
    mp.spawn(_cp_worker, args=(world, _free_port(), arch, out), nprocs=world, join=True)
    got = torch.load(out, weights_only=True)
    for r in range(1, world):  # replicated update block: every rank holds the same flows
        assert torch.equal(got[r], got[0])
    model, variables = (raft_large if arch == "raft_large" else raft_small)(seed=0)
    i1, i2 = _inputs()
    ref = model.apply(variables, i1, i2, num_flow_updates=2)
    err = (got[0] - ref).abs().max().item()
    assert err < 1e-3 * max(1.0, ref.abs().max().item()), err
