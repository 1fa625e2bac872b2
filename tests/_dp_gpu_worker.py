"""Worker for test_train_gpu.py::test_dp_two_ranks_shared_gpu: two DP ranks on
one GPU (gloo, JR_SHARE_GPU=1) run native-autograd training steps and write a
parameter checksum per rank."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from jax_raft_amd.train.trainer import Trainer, TrainConfig  # noqa: E402

out = sys.argv[1]
tr = Trainer(TrainConfig(arch="raft_small", steps=2, batch=1, iters=2, size=(128, 160), log_every=10 ** 9))
for i in range(2):
    m = tr.train_step(tr.batch_for(i))
flat = torch.cat([p.detach().float().reshape(-1) for p in tr.model.parameters()])
with open(os.path.join(out, f"rank{tr.rank}.txt"), "w") as f:
    f.write(f"{flat.double().sum().item():.10e} {flat.double().abs().sum().item():.10e} {float(m['loss']):.6f}\n")
torch.distributed.destroy_process_group()
