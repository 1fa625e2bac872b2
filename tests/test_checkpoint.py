"""Flax-msgpack checkpoint format and the
torchvision converter (reference scripts/convert_checkpoint.py).

No real jax-raft checkpoint is reachable offline, so the files are synthesised
with the exact Flax encoding (ExtType 1 = msgpack((shape, dtype, bytes)));
parity with an actual released file is unpinned."""
import msgpack
import numpy as np
import pytest
import torch

from jax_raft_amd import raft_large, raft_small
from jax_raft_amd.utils import checkpoint as C


def _flax_bytes(tree):
    """Independent re-implementation of flax.serialization.to_bytes."""

    def ext(x):
        if isinstance(x, np.ndarray):
            return msgpack.ExtType(1, msgpack.packb((x.shape, x.dtype.name, x.tobytes("C")), use_bin_type=True))
        raise TypeError(type(x))

    def tonp(t):
        if isinstance(t, dict):
            return {k: tonp(v) for k, v in t.items()}
        return t.detach().numpy() if isinstance(t, torch.Tensor) else t

    return msgpack.packb(tonp(tree), default=ext, strict_types=True)


def test_param_counts_and_tree():
    m, v = raft_large()
    assert C.count_params(v) == 5_257_536
    assert len(C.flatten_tree(v["params"])) == 124
    bs = C.flatten_tree(v["batch_stats"])
    assert sum(x.numel() for x in bs.values()) == 2880
    p = v["params"]
    assert tuple(p["feature_encoder"]["convnormrelu"]["layers_0"]["kernel"].shape) == (7, 7, 3, 64)
    assert tuple(p["update_block"]["recurrent_block"]["convgru1"]["convz"]["kernel"].shape) == (1, 5, 384, 128)
    assert tuple(p["update_block"]["recurrent_block"]["convgru2"]["convq"]["kernel"].shape) == (5, 1, 384, 128)
    assert tuple(p["mask_predictor"]["conv"]["kernel"].shape) == (1, 1, 256, 576)
    assert tuple(p["context_encoder"]["layer2"]["layers_0"]["downsample"]["layers_1"]["scale"].shape) == (96,)
    assert "layers_1" not in p["feature_encoder"]["convnormrelu"]  # InstanceNorm has no params
    ms, vs = raft_small()
    assert C.count_params(vs) == 990_162
    assert len(C.flatten_tree(vs["params"])) == 106
    assert not vs["batch_stats"]
    assert tuple(vs["params"]["update_block"]["recurrent_block"]["convgru1"]["convz"]["kernel"].shape) == (3, 3, 242, 96)
    assert tuple(vs["params"]["context_encoder"]["conv"]["kernel"].shape) == (1, 1, 96, 160)


def test_variables_share_storage():
    m, v = raft_small()
    k = v["params"]["update_block"]["flow_head"]["conv2"]["bias"]
    assert k is m.update_block.flow_head.conv2.bias


@pytest.mark.parametrize("factory", [raft_small, raft_large])
def test_flax_msgpack_roundtrip(tmp_path, factory):
    m1, v1 = factory(seed=1)
    data = _flax_bytes({"params": v1["params"], "batch_stats": v1["batch_stats"]})
    f = tmp_path / "w.msgpack"
    f.write_bytes(data)
    m2, v2 = factory(seed=2, weights=str(f))
    for (k1, a), (k2, b) in zip(sorted(C.flatten_tree(v1["params"]).items()), sorted(C.flatten_tree(v2["params"]).items())):
        assert k1 == k2 and torch.equal(a, b)
    # our own writer produces the same bytes-level tree
    f2 = tmp_path / "w2.msgpack"
    C.save_msgpack(m2, str(f2))
    t = C.load_msgpack(str(f2))
    assert set(C.flatten_tree(t["params"])) == set(C.flatten_tree(v1["params"]))
    assert C.msgpack_restore(data).keys() == t.keys()


def test_small_checkpoint_without_batch_stats(tmp_path):
    m1, v1 = raft_small(seed=3)
    f = tmp_path / "s.msgpack"
    f.write_bytes(_flax_bytes({"params": v1["params"]}))  # template of raft_small has only params
    m2, v2 = raft_small(weights=str(f))
    assert torch.equal(v2["params"]["context_encoder"]["conv"]["bias"], v1["params"]["context_encoder"]["conv"]["bias"])


def test_strict_mismatch_raises(tmp_path):
    _, v = raft_small()
    tree = {"params": dict(v["params"])}
    tree["params"].pop("update_block")
    f = tmp_path / "bad.msgpack"
    f.write_bytes(_flax_bytes(tree))
    with pytest.raises(KeyError):
        raft_small(weights=str(f))


def test_bfloat16_leaf_decodes():
    x = torch.randn(3, 4)
    raw = x.to(torch.bfloat16).view(torch.int16).numpy().astype(np.uint16)
    payload = msgpack.packb(((3, 4), "bfloat16", raw.tobytes()), use_bin_type=True)
    data = msgpack.packb({"a": msgpack.ExtType(1, payload)})
    out = C.msgpack_restore(data)["a"]
    assert np.allclose(out, x.to(torch.bfloat16).float().numpy())


def _to_torchvision(v):
    """Inverse of convert_checkpoint._convert: our Flax tree -> torchvision state_dict."""
    sd = {}
    for k, t in C.flatten_tree(v["params"]).items():
        parts = [p[len("layers_"):] if p.startswith("layers_") else p for p in k.split(".")]
        if parts[-1] == "kernel":
            parts[-1] = "weight"
            t = t.permute(3, 2, 0, 1)
        elif parts[-1] == "scale":
            parts[-1] = "weight"
        sd[".".join(parts)] = t.detach().clone()
    for k, t in C.flatten_tree(v["batch_stats"]).items():
        parts = [p[len("layers_"):] if p.startswith("layers_") else p for p in k.split(".")]
        parts[-1] = {"mean": "running_mean", "var": "running_var"}[parts[-1]]
        sd[".".join(parts)] = t.detach().clone()
        sd[".".join(parts[:-1] + ["num_batches_tracked"])] = torch.tensor(5)
    return sd


def test_torchvision_conversion_roundtrip(tmp_path):
    m1, v1 = raft_large(seed=4)
    sd = _to_torchvision(v1)
    assert "feature_encoder.layer1.0.convnormrelu1.0.weight" in sd
    assert "context_encoder.layer1.0.convnormrelu1.1.running_mean" in sd
    pth = tmp_path / "tv.pth"
    torch.save(sd, pth)
    out = tmp_path / "tv.msgpack"
    C.convert_checkpoint(str(pth), str(out))
    m2, v2 = raft_large(weights=str(out))
    for coll in ("params", "batch_stats"):
        a, b = C.flatten_tree(v1[coll]), C.flatten_tree(v2[coll])
        assert set(a) == set(b)
        for k in a:
            assert torch.equal(a[k], b[k]), k


def test_chunked_array_flax_encoding(monkeypatch):
    """Arrays above the chunk limit use Flax's {'0': .., '1': ..} encoding for
    both 'shape' and 'chunks' (flax.serialization._tuple_to_dict)."""
    monkeypatch.setattr(C, "_MAX_CHUNK", 64)
    big = np.arange(3 * 7 * 5, dtype=np.float32).reshape(3, 7, 5)
    raw = C.msgpack_serialize({"params": {"w": big, "b": np.ones(2, np.float32)}})
    tree = msgpack.unpackb(raw, ext_hook=C._ext_hook, raw=False, strict_map_key=False)
    enc = tree["params"]["w"]
    assert enc[C._CHUNK_KEY] is True
    assert enc["shape"] == {"0": 3, "1": 7, "2": 5}
    assert set(enc["chunks"]) == {str(i) for i in range(len(enc["chunks"]))} and len(enc["chunks"]) > 1
    back = C.msgpack_restore(raw)
    assert np.array_equal(back["params"]["w"], big)
    # a file written by Flax itself (shape dict) and a legacy list shape both decode
    legacy = dict(enc, shape=[3, 7, 5])
    assert np.array_equal(C._unchunk(legacy), big)
