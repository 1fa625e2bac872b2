"""MPI-Sintel validation: EPE / 1px / 3px / 5px and FPS.

Re-implements the reference methodology of ``scripts/validate_sintel.py``:

* dataset: consecutive frame pairs per scene with the ``.flo`` ground truth
  (``MpiSintel``, ``validate_sintel.py:145-161``);
* per pair: normalise to [-1, 1], replicate-pad to /8 ('sintel' mode),
  run ``num_flow_updates`` (default 32) iterations, take the last prediction,
  unpad, per-pixel EPE = ||flow - gt||_2 over ALL pixels (no valid mask)
  (``validate_sintel.py:175-198``);
* FPS = 1 / mean per-pair latency, excluding the first (compile/plan-build)
  pair, with the latency covering H2D of the inputs and a device sync on the
  prediction (``validate_sintel.py:185-188,201-203``).

MI355X additions: batched evaluation (``batch_size``) and data-parallel
evaluation over ranks (``torch.distributed``; each rank takes a strided shard,
EPE sums are all-reduced).
"""
from __future__ import annotations

import os
import os.path as osp
import time
from glob import glob
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..utils.flow_io import InputPadder, normalize_image, read_flo, read_image


class MpiSintel:
    """Frame pairs of MPI-Sintel ``<root>/<split>/<dstype>/<scene>/*.png``."""

    def __init__(self, root: str, split: str = "training", dstype: str = "clean"):
        self.is_test = split == "test"
        self.image_list: List[Tuple[str, str]] = []
        self.flow_list: List[str] = []
        self.extra_info: List[Tuple[str, int]] = []
        image_root = osp.join(root, split, dstype)
        flow_root = osp.join(root, split, "flow")
        if not osp.isdir(image_root):
            raise FileNotFoundError(f"Sintel images not found at {image_root}")
        for scene in sorted(os.listdir(image_root)):
            imgs = sorted(glob(osp.join(image_root, scene, "*.png")))
            for i in range(len(imgs) - 1):
                self.image_list.append((imgs[i], imgs[i + 1]))
                self.extra_info.append((scene, i))
            if not self.is_test:
                self.flow_list += sorted(glob(osp.join(flow_root, scene, "*.flo")))
        if not self.is_test and len(self.flow_list) != len(self.image_list):
            raise ValueError(f"{len(self.image_list)} pairs but {len(self.flow_list)} flow files")

    def __len__(self):
        return len(self.image_list)

    def __getitem__(self, i):
        a = read_image(self.image_list[i][0])
        b = read_image(self.image_list[i][1])
        flow = None if self.is_test else read_flo(self.flow_list[i])
        return a, b, flow



def _finite_mean(rates) -> float:
    ok = [r for r in rates if np.isfinite(r)]
    return float(np.mean(ok)) if ok else float("nan")

def epe_metrics(epe_all: np.ndarray) -> Dict[str, float]:
    return {
        "epe": float(np.mean(epe_all)),
        "1px": float(np.mean(epe_all < 1)),
        "3px": float(np.mean(epe_all < 3)),
        "5px": float(np.mean(epe_all < 5)),
    }


@torch.no_grad()
def validate_sintel(model, data_root: str, iters: int = 32, dstypes: Sequence[str] = ("clean", "final"),
                    device: Optional[torch.device] = None, max_pairs: Optional[int] = None, verbose: bool = True,
                    batch_size: int = 1, device_prep: Optional[bool] = None,
                    **engine_kw) -> Dict[str, Dict[str, float]]:
    """Reference-methodology Sintel validation of a RAFT model.

    ``batch_size`` pairs (consecutive pairs of this rank's shard; all Sintel
    frames share one size) run as one batched forward; FPS is then pairs per
    second of the timed batches.  The first batch of every batch SHAPE (the
    first one, and a smaller tail batch: a new plan build, autotune, graph
    capture) is excluded, as the reference excludes its JIT compile.
    ``batch_size=1`` is exactly the reference's per-pair protocol.

    ``device_prep`` (default: on for a GPU device) hands the model the raw uint8 frames: the
    normalisation and the replicate padding run on the device (the engine's prep kernel) and the
    model returns unpadded flows; off, they run on the host as in the reference script.

    Data parallel (an initialised process group): each rank takes every
    world-th pair; ``fps`` is the mean per-GPU rate (comparable to the
    reference's single-GPU FPS) and ``fps_aggregate`` the job's total pairs/s
    (the sum of the per-rank rates)."""
    dist = torch.distributed if torch.distributed.is_available() and torch.distributed.is_initialized() else None
    rank, world = (dist.get_rank(), dist.get_world_size()) if dist else (0, 1)
    device = device or (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
    model = model.to(device).eval()
    bs = max(1, int(batch_size))
    # on the GPU the engine takes the raw uint8 frames (device-side normalise + pad)
    u8 = device.type == "cuda" if device_prep is None else bool(device_prep)
    results = {}
    for dstype in dstypes:
        ds = MpiSintel(data_root, "training", dstype)
        n = len(ds) if max_pairs is None else min(len(ds), max_pairs)
        idx = list(range(rank, n, world))
        sums = np.zeros(5, dtype=np.float64)  # epe_sum, <1, <3, <5, count
        t_sum, t_pairs = 0.0, 0
        seen_shapes = set()
        for k in range(0, len(idx), bs):
            items = [ds[i] for i in idx[k:k + bs]]
            if u8:
                # raw uint8 frames: x / 255 * 2 - 1 and the 'sintel' replicate padding run in the
                # engine's prep kernel, the flows come back unpadded (models/raft.py:_forward_u8);
                # the timed H2D moves 1 byte per channel instead of 4
                i1 = torch.from_numpy(np.stack([a for a, _, _ in items]))
                i2 = torch.from_numpy(np.stack([b for _, b, _ in items]))
                padder = None
            else:
                i1 = torch.cat([normalize_image(a) for a, _, _ in items])
                i2 = torch.cat([normalize_image(b) for _, b, _ in items])
                padder = InputPadder(i1.shape, channels_last=True)
                i1, i2 = padder.pad(i1, i2)
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            pred = model(i1.to(device), i2.to(device), num_flow_updates=iters, **engine_kw)[-1]
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            if tuple(i1.shape) in seen_shapes:   # a new batch shape builds a new plan: untimed
                t_sum += time.perf_counter() - t0
                t_pairs += len(items)
            seen_shapes.add(tuple(i1.shape))
            pred = pred.float().cpu()
            flows = (pred if padder is None else padder.unpad(pred)).numpy()
            for f, (_, _, gt) in zip(flows, items):
                epe = np.sqrt(((f - gt) ** 2).sum(-1)).reshape(-1)
                sums += [epe.sum(), (epe < 1).sum(), (epe < 3).sum(), (epe < 5).sum(), epe.size]
        rate = t_pairs / t_sum if t_sum > 0 else float("nan")   # this rank's pairs / s
        rates = [rate]
        if dist:
            st = torch.tensor(sums, dtype=torch.float64, device=device)
            dist.all_reduce(st)
            sums = st.cpu().numpy()
            rt = [torch.zeros(1, dtype=torch.float64, device=device) for _ in range(world)]
            dist.all_gather(rt, torch.tensor([rate], dtype=torch.float64, device=device))
            rates = [float(r.item()) for r in rt]
        cnt = max(sums[4], 1)
        res = {"epe": sums[0] / cnt, "1px": sums[1] / cnt, "3px": sums[2] / cnt, "5px": sums[3] / cnt,
               # ranks without a timed batch (a short shard: every batch the first of its shape) report nan
               # and are left out, so one such rank cannot turn the job's rate into nan
               "fps": _finite_mean(rates), "fps_aggregate": float(np.sum([r for r in rates if np.isfinite(r)])),
               "world": world,
               "pairs": int(n), "batch_size": bs}
        results[dstype] = res
        if verbose and rank == 0:
            print("Validation (%s) EPE: %f, 1px: %f, 3px: %f, 5px: %f, fps: %f" % (
                dstype, res["epe"], res["1px"], res["3px"], res["5px"], res["fps"])
                + (" per GPU, %f aggregate over %d GPUs" % (res["fps_aggregate"], world) if world > 1 else ""))
    return results
