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
