"""Worker for test_train_gpu.py::test_dp_grads_equal_full_batch: two DP ranks on
one GPU (gloo, JR_SHARE_GPU=1) each run the fused native training forward /
backward of raft_small on ITS sample, the Trainer's gradient communication
averages the gradients (flat-arena all-reduce overlapped with the backward +
the bucketed hook reducer), and each rank saves the result."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from jax_raft_amd.train.loss import sequence_loss  # noqa: E402
from jax_raft_amd.train.trainer import Trainer, TrainConfig  # noqa: E402

out = sys.argv[1]
cfg = TrainConfig(arch="raft_small", steps=2, batch=1, iters=2, size=(128, 160), log_every=10 ** 9)
tr = Trainer(cfg)
img1, img2, flow, valid = tr.data.batch([tr.rank])
tr.opt.zero_grad(set_to_none=True)
preds = tr.model(img1, img2, train=True, num_flow_updates=cfg.iters, autograd=True)
loss, _ = sequence_loss(preds, flow, valid, cfg.gamma, cfg.max_flow)
with tr._comm():
    loss.backward()
tr.sync.finish()
torch.save({n: p.grad.detach().float().cpu() for n, p in tr.model.named_parameters()},
           os.path.join(out, f"rank{tr.rank}.pt"))
with open(os.path.join(out, f"rank{tr.rank}.txt"), "w") as f:
    f.write(f"{float(loss):.6f}\n")
torch.distributed.destroy_process_group()
