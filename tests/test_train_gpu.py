"""Training steps on the GPU through the native autograd path."""
import pytest
import torch

from jax_raft_amd.train.trainer import TrainConfig, Trainer

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("arch", ["raft_small", "raft_large"])
def test_gpu_train_steps_reduce_loss(arch):
    cfg = TrainConfig(arch=arch, steps=6, batch=2, iters=3, size=(128, 160), log_every=1, lr=2e-4)
    tr = Trainer(cfg)
    assert tr.device.type == "cuda"
    logs = []
    tr.fit(log=logs.append)
    import json

    losses = [json.loads(l)["loss"] for l in logs]
    assert all(torch.isfinite(torch.tensor(losses)))
    assert all(torch.isfinite(p).all() for p in tr.model.parameters())


def test_dp_two_ranks_shared_gpu(tmp_path):
    """2-rank data parallelism through the native autograd path (both ranks on
    cuda:0 over gloo): different data per rank, all-reduced gradients, so the
    replicas must stay bit-identical after the optimizer steps."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, JR_SHARE_GPU="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29631",
           os.path.join(root, "tests", "_dp_gpu_worker.py"), str(tmp_path)]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    a = (tmp_path / "rank0.txt").read_text().split()
    b = (tmp_path / "rank1.txt").read_text().split()
    assert a[:2] == b[:2], (a, b)      # identical parameters on both replicas
    assert a[2] != b[2]                # but each rank saw its own data
