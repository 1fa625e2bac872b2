"""The environment variables jax_raft_amd reads -- all of them, in one place.

They are operational settings (which library to load, where the tuned-config table lives,
debugging aids, the rank layout of a rehearsal); none of them changes what a kernel computes.
Lowering / schedule choices are not environment switches: each is fixed to the winner of its
A/B (the profile is cited where the choice is made) and the ones tests flip to cover the
alternative are class or module attributes -- ``RaftEngine.GRU``, ``.PRO_LANES``,
``.HALO_NORM``, ``.MERGED_UP``, ``.CONV_GROUP``, ``.MASK_PARITY``, ``.HOST_GATE``,
``.AUTO_STREAMS_MIN_BATCH``, ``.GATE_MIN_ITERS``, ``.max_plans`` (runtime/engine.py) and
``FUSED_ENCODERS``, ``FUSED_GRAPH``, ``FUSED_TRAIN``, ``FusedModel.SIDE_ENCODER``,
``FusedModel.EARLY_CE``, ``FusedLoop.LANES`` / ``.FWD_LANES`` (train/fused.py), ``HALO_NORM``
(train/fused_encoder.py), ``Trainer.SETTLE_LAG`` (train/trainer.py) -- and per-kernel variants
are op arguments (``conv_f32_args(ksplit=)``, ``gru_fused``'s fifth int, conv cfg bits 10 / 11).

===================  =====================================================================
JR_NATIVE_SO         path of another build of the native library (e.g. the host-sanitizer
                     build ``python -m jax_raft_amd._build --sanitize``); default: in-tree _C.so
JR_OFFLOAD_ARCH      offload target of ``jax_raft_amd._build`` (default gfx950)
JR_TUNE_DB           path of a tuned-config table to use instead of the packaged
                     ``jax_raft_amd/tuned/<arch>.json`` (tools/race_check.py hands its table to its
                     child processes this way)
JR_TUNE              ``fresh``: ignore the persisted table, time every conv's candidates again
                     (tools/autotune_db.py)
JR_CFG_OVERRIDE      ``name=cfg,...``: fixed tile configs per conv spec, merged into the
                     engine's ``cfg_override`` (tools/schedule_tune.py output)
JR_PLAN_CHECK        ``1``: eager plans synchronise after every launch and name the op that
                     faulted (fault localisation; also makes the fused training path eager)
JR_PLAN_DEBUG        ``1``: log plan capture / instantiate steps to stderr
JR_DIST_BACKEND      torch.distributed backend (default: nccl = RCCL on GPUs, gloo on CPU)
JR_SHARE_GPU         ``1``: ranks share the visible GPU(s) over gloo -- a multi-rank rehearsal
                     on a one-GPU box (RCCL refuses two ranks on one GPU)
JAX_RAFT_AMD_WEIGHTS directory searched for released checkpoints (utils/checkpoint.py)
===================  =====================================================================

``WORLD_SIZE`` / ``RANK`` / ``LOCAL_RANK`` / ``MASTER_ADDR`` / ``MASTER_PORT`` are the usual
torch.distributed launcher variables.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

DOCUMENTED = ("JR_NATIVE_SO", "JR_OFFLOAD_ARCH", "JR_TUNE_DB", "JR_TUNE", "JR_CFG_OVERRIDE", "JR_PLAN_CHECK",
              "JR_PLAN_DEBUG", "JR_DIST_BACKEND", "JR_SHARE_GPU", "JAX_RAFT_AMD_WEIGHTS")


def get(name: str, default: Optional[str] = None) -> Optional[str]:
    """The value of one of the documented variables (an undocumented name is a bug)."""
    assert name in DOCUMENTED, f"{name} is not a documented jax_raft_amd environment variable"
    v = os.environ.get(name)
    return default if v is None or v == "" else v


def flag(name: str) -> bool:
    return get(name, "0") == "1"


def cfg_override() -> Dict[str, int]:
    """JR_CFG_OVERRIDE parsed: {conv spec name: tile config}."""
    out: Dict[str, int] = {}
    for item in filter(None, (get("JR_CFG_OVERRIDE") or "").split(",")):
        k, v = item.split("=")
        out[k.strip()] = int(v)
    return out
