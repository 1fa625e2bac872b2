"""Checkpoint I/O: the Flax msgpack format of jax-raft, without Flax.

The reference restores weights with ``flax.serialization.from_bytes`` onto the
``init``-ed variable template (``jax_raft/model.py:684-689``) and writes them
with ``flax.serialization.to_bytes`` in its converter
(``scripts/convert_checkpoint.py:53-56``).  The on-disk encoding is
``msgpack.packb(state_dict)`` where every array leaf is a msgpack ExtType
(code 1) whose payload is ``msgpack.packb((shape, dtype_name, raw_bytes))``;
arrays above 2**30 bytes are split into a ``{'__msgpack_chunked_array__': ...}``
dict.  Both directions are implemented here with the ``msgpack`` package and
numpy only; nothing executable is ever deserialised.

Also implemented: the torchvision ``state_dict`` -> Flax tree conversion of
``scripts/convert_checkpoint.py:11-52`` (BN running stats moved to
``batch_stats``, OIHW -> HWIO, 1-D ``weight`` -> ``scale``, numeric Sequential
indices -> ``layers_N``).
"""
from __future__ import annotations

import os
from typing import Any, Dict, Mapping, Optional

import msgpack
import numpy as np
import torch

from .. import knobs

_EXT_NDARRAY = 1
_EXT_NATIVE_COMPLEX = 2
_EXT_NPSCALAR = 3
_MAX_CHUNK = 2 ** 30
_CHUNK_KEY = "__msgpack_chunked_array__"

_DTYPES = {
    "float32": np.float32, "float64": np.float64, "float16": np.float16, "int32": np.int32, "int64": np.int64,
    "int8": np.int8, "uint8": np.uint8, "uint32": np.uint32, "bool": np.bool_,
}


def _dtype_from_name(name: str):
    if name == "bfloat16":
        return "bfloat16"
    if name not in _DTYPES:
        raise ValueError(f"unsupported dtype in checkpoint: {name}")
    return np.dtype(_DTYPES[name])


def _ndarray_from_bytes(data: bytes):
    shape, dtype_name, buf = msgpack.unpackb(data, raw=True)
    if isinstance(dtype_name, bytes):
        dtype_name = dtype_name.decode()
    dt = _dtype_from_name(dtype_name)
    if dt == "bfloat16":
        raw = np.frombuffer(buf, dtype=np.uint16).reshape(shape)
        return torch.from_numpy(raw.astype(np.int32) << 16).view(torch.float32).numpy()
    return np.frombuffer(buf, dtype=dt).reshape(tuple(shape)).copy()


def _ext_hook(code: int, data: bytes):
    if code == _EXT_NDARRAY:
        return _ndarray_from_bytes(data)
    if code == _EXT_NATIVE_COMPLEX:
        re, im = msgpack.unpackb(data)
        return complex(re, im)
    if code == _EXT_NPSCALAR:
        shape, dtype_name, buf = msgpack.unpackb(data, raw=True)
        if isinstance(dtype_name, bytes):
            dtype_name = dtype_name.decode()
        return np.frombuffer(buf, dtype=_dtype_from_name(dtype_name))[0]
    return msgpack.ExtType(code, data)


def _unchunk(tree):
    if isinstance(tree, dict):
        if tree.get(_CHUNK_KEY):
            # Flax stores the shape and the chunk list via _tuple_to_dict: {'0': .., '1': ..}
            shp = tree["shape"]
            shape = tuple(int(shp[str(i)]) for i in range(len(shp))) if isinstance(shp, Mapping) else tuple(shp)
            chunks = tree["chunks"]
            flat = np.concatenate([chunks[str(i)].reshape(-1) for i in range(len(chunks))])
            return flat.reshape(shape)
        return {k: _unchunk(v) for k, v in tree.items()}
    return tree


def msgpack_restore(data: bytes) -> Dict[str, Any]:
    """Decode Flax msgpack bytes into a nested dict of numpy arrays."""
    tree = msgpack.unpackb(data, ext_hook=_ext_hook, raw=False, strict_map_key=False)
    return _unchunk(tree)


def _ndarray_to_bytes(arr: np.ndarray) -> bytes:
    arr = np.ascontiguousarray(arr)
    return msgpack.packb((arr.shape, arr.dtype.name, arr.tobytes("C")), use_bin_type=True)


def _ext_pack(x):
    if isinstance(x, np.ndarray):
        return msgpack.ExtType(_EXT_NDARRAY, _ndarray_to_bytes(x))
    if isinstance(x, np.generic):
        return msgpack.ExtType(_EXT_NPSCALAR, _ndarray_to_bytes(np.asarray(x)))
    if isinstance(x, complex):
        return msgpack.ExtType(_EXT_NATIVE_COMPLEX, msgpack.packb((x.real, x.imag)))
    raise TypeError(f"cannot serialise {type(x)}")


def _chunk(tree):
    if isinstance(tree, dict):
        return {k: _chunk(v) for k, v in tree.items()}
    if isinstance(tree, np.ndarray) and tree.nbytes > _MAX_CHUNK:
        flat = tree.reshape(-1)
        per = max(1, _MAX_CHUNK // tree.itemsize)
        chunks = {str(i): flat[j:j + per] for i, j in enumerate(range(0, flat.size, per))}
        return {_CHUNK_KEY: True, "shape": {str(i): int(d) for i, d in enumerate(tree.shape)}, "chunks": chunks}
    return tree


def _to_numpy_tree(tree):
    if isinstance(tree, Mapping):
        return {str(k): _to_numpy_tree(v) for k, v in tree.items()}
    if isinstance(tree, torch.Tensor):
        return tree.detach().to("cpu", torch.float32).contiguous().numpy()
    if isinstance(tree, np.ndarray):
        return tree
    return tree


def msgpack_serialize(tree: Mapping[str, Any]) -> bytes:
    """Encode a nested dict of arrays/tensors as Flax msgpack bytes."""
    return msgpack.packb(_chunk(_to_numpy_tree(tree)), default=_ext_pack, strict_types=True)


# ----------------------------------------------------------------- tree helpers

def flatten_tree(tree: Mapping[str, Any], prefix: str = "", sep: str = ".") -> Dict[str, Any]:
    out = {}
    for k, v in tree.items():
        key = f"{prefix}{sep}{k}" if prefix else str(k)
        if isinstance(v, Mapping):
            out.update(flatten_tree(v, key, sep))
        else:
            out[key] = v
    return out


def unflatten_tree(flat: Mapping[str, Any], sep: str = ".") -> Dict[str, Any]:
    out: Dict[str, Any] = {}
    for k, v in flat.items():
        parts = k.split(sep)
        d = out
        for p in parts[:-1]:
            d = d.setdefault(p, {})
        d[parts[-1]] = v
    return out


def variables_from_module(model: torch.nn.Module) -> Dict[str, Dict[str, Any]]:
    """``{'params': ..., 'batch_stats': ...}`` nested dicts whose leaves ARE the
    module's parameter / buffer tensors (shared storage)."""
    params = {k: v for k, v in model.named_parameters()}
    stats = {k: v for k, v in model.named_buffers() if k.endswith(".mean") or k.endswith(".var")}
    return {"params": unflatten_tree(params), "batch_stats": unflatten_tree(stats)}


def load_variables_into(model: torch.nn.Module, variables: Mapping[str, Any], strict: bool = True) -> None:
    """Copy a Flax-style variable tree (numpy or torch leaves) into the module,
    validating the structure like ``flax.serialization.from_state_dict``."""
    target = {k: v for k, v in model.named_parameters()}
    target.update({k: v for k, v in model.named_buffers() if k.endswith(".mean") or k.endswith(".var")})
    src = {}
    for coll in ("params", "batch_stats"):
        if coll in variables and variables[coll]:
            src.update(flatten_tree(variables[coll]))
    missing = sorted(set(target) - set(src))
    extra = sorted(set(src) - set(target))
    if strict and (missing or extra):
        raise KeyError(f"checkpoint tree mismatch: missing={missing[:8]}{'...' if len(missing) > 8 else ''} "
                       f"unexpected={extra[:8]}{'...' if len(extra) > 8 else ''}")
    with torch.no_grad():
        for k, t in target.items():
            if k not in src:
                continue
            v = src[k]
            v = torch.as_tensor(np.asarray(v)) if not isinstance(v, torch.Tensor) else v
            if tuple(v.shape) != tuple(t.shape):
                raise ValueError(f"shape mismatch for {k}: checkpoint {tuple(v.shape)} vs model {tuple(t.shape)}")
            t.copy_(v.to(t.dtype))


def variables_as_tensors(model: torch.nn.Module, variables: Mapping[str, Any]) -> Dict[str, torch.Tensor]:
    """Validate a foreign variable tree against ``model`` and return its leaves
    as fresh tensors (the module's device and dtypes), keyed by the module's
    parameter / buffer names, for ``torch.func.functional_call``.

    Strict like Flax's ``apply``: a missing or unexpected ``params`` leaf or a
    shape mismatch raises.  The ``batch_stats`` collection may be absent as a
    whole (the module's own statistics are used); when it is given it must be
    complete."""
    if not isinstance(variables, Mapping) or "params" not in variables:
        raise KeyError("variables must be a mapping with a 'params' collection")
    params = {k: v for k, v in model.named_parameters()}
    stats = {k: v for k, v in model.named_buffers() if k.endswith(".mean") or k.endswith(".var")}
    out: Dict[str, torch.Tensor] = {}
    for coll, target in (("params", params), ("batch_stats", stats)):
        given = variables.get(coll)
        if coll == "batch_stats" and not given:
            continue
        src = flatten_tree(given or {})
        missing = sorted(set(target) - set(src))
        extra = sorted(set(src) - set(target))
        if missing or extra:
            raise KeyError(f"variable tree mismatch in '{coll}': missing={missing[:8]}"
                           f"{'...' if len(missing) > 8 else ''} unexpected={extra[:8]}"
                           f"{'...' if len(extra) > 8 else ''}")
        for k, t in target.items():
            v = src[k]
            v = v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v))
            if tuple(v.shape) != tuple(t.shape):
                raise ValueError(f"shape mismatch for {coll}/{k}: given {tuple(v.shape)} vs model {tuple(t.shape)}")
            if v.requires_grad and v.device == t.device and v.dtype == t.dtype:
                out[k] = v   # differentiable w.r.t. the given leaf (jax.grad over variables)
            else:
                out[k] = v.detach().to(device=t.device, dtype=t.dtype, copy=True)
    return out


def save_msgpack(model_or_vars, path: str) -> None:
    """Write ``{'params', 'batch_stats'}`` as a Flax msgpack file."""
    if isinstance(model_or_vars, torch.nn.Module):
        variables = variables_from_module(model_or_vars)
    else:
        variables = model_or_vars
    tree = {"params": variables.get("params", {}), "batch_stats": variables.get("batch_stats", {})}
    with open(path, "wb") as f:
        f.write(msgpack_serialize(tree))


def load_msgpack(path: str) -> Dict[str, Any]:
    with open(path, "rb") as f:
        return msgpack_restore(f.read())


# ---------------------------------------------------------- torchvision import

def _convert_torchvision(in_dict: Mapping[str, Any]) -> Dict[str, Any]:
    """Recursive rename of ``scripts/convert_checkpoint.py:11-32``."""
    top_keys = {k.split(".")[0] for k in in_dict}
    leaves = {k for k in in_dict if "." not in k}
    out: Dict[str, Any] = {}
    for l in leaves:
        v = np.asarray(in_dict[l])
        if l == "weight" and v.ndim == 4:
            out["kernel"] = v.transpose(2, 3, 1, 0)
        elif l == "weight" and v.ndim == 1:
            out["scale"] = v
        else:
            out[l] = v
    for tk in top_keys - leaves:
        nk = "layers_" + tk if tk.isdigit() else tk
        out[nk] = _convert_torchvision({k[len(tk) + 1:]: v for k, v in in_dict.items() if k.startswith(tk + ".")})
    return out


def convert_torchvision_state_dict(state_dict: Mapping[str, Any]) -> Dict[str, Any]:
    """torchvision RAFT ``state_dict`` -> ``{'params', 'batch_stats'}`` Flax tree
    (``scripts/convert_checkpoint.py:35-52``)."""
    params, stats = {}, {}
    for k, v in state_dict.items():
        v = v.detach().cpu().float().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)
        if k.endswith(".running_mean"):
            stats[k.replace(".running_mean", ".mean")] = v
        elif k.endswith(".running_var"):
            stats[k.replace(".running_var", ".var")] = v
        elif k.endswith(".num_batches_tracked"):
            continue
        else:
            params[k] = v
    return {"params": _convert_torchvision(params), "batch_stats": _convert_torchvision(stats)}


def convert_checkpoint(torch_checkpoint: str, output_file: str) -> None:
    """CLI-equivalent of ``scripts/convert_checkpoint.py:35-56``.  Loads the
    ``.pth`` with ``weights_only=True`` (no unpickling of code)."""
    sd = torch.load(torch_checkpoint, map_location="cpu", weights_only=True)
    tree = convert_torchvision_state_dict(sd)
    with open(output_file, "wb") as f:
        f.write(msgpack_serialize(tree))


def count_params(variables: Mapping[str, Any]) -> int:
    return int(sum(np.prod(np.shape(v)) for v in flatten_tree(variables.get("params", {})).values()))


def resolve_pretrained(arch: str, url: str, weights: Optional[str] = None) -> bytes:
    """Return checkpoint bytes from an explicit path, the weights cache
    directory (``$JAX_RAFT_AMD_WEIGHTS``, ``~/.cache/jax_raft_amd``) or, as a
    last resort, the reference release URL (``model.py:17-21,684-689``)."""
    if weights is not None:
        with open(weights, "rb") as f:
            return f.read()
    fname = url.rsplit("/", 1)[-1]
    for d in (knobs.get("JAX_RAFT_AMD_WEIGHTS"), os.path.expanduser("~/.cache/jax_raft_amd")):
        if d and os.path.exists(os.path.join(d, fname)):
            with open(os.path.join(d, fname), "rb") as f:
                return f.read()
    import urllib.request

    try:
        with urllib.request.urlopen(url, timeout=30) as resp:
            return resp.read()
    except Exception as e:  # no network in this environment
        raise RuntimeError(
            f"pretrained weights for {arch} not found locally and download failed ({e}). "
            f"Place {fname} in $JAX_RAFT_AMD_WEIGHTS or pass weights=<path>."
        ) from e
