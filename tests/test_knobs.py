"""Every environment variable the framework reads is one of the few documented in
jax_raft_amd/knobs.py (schedule / lowering A/B choices are not environment switches)."""
import re
from pathlib import Path

import pytest

from jax_raft_amd import knobs

ROOT = Path(__file__).resolve().parent.parent


def _sources():
    for d, pats in (("jax_raft_amd", ("*.py",)), ("csrc", ("*.cpp", "*.hip", "*.h"))):
        for pat in pats:
            yield from (ROOT / d).rglob(pat)


def test_every_env_read_is_documented():
    reads = set()
    py = re.compile(r"""(?:os\.environ(?:\.get)?\s*[\[(]\s*|knobs\.(?:get|flag)\(\s*)["']([A-Z_0-9]+)["']""")
    cc = re.compile(r"""getenv\(\s*"([A-Z_0-9]+)"\s*\)""")
    for f in _sources():
        text = f.read_text()
        for m in (cc if f.suffix in (".cpp", ".hip", ".h") else py).finditer(text):
            reads.add(m.group(1))
    ours = {n for n in reads if n.startswith("JR_") or n.startswith("JAX_RAFT")}
    assert ours <= set(knobs.DOCUMENTED), sorted(ours - set(knobs.DOCUMENTED))
    assert len(knobs.DOCUMENTED) <= 10
    for n in knobs.DOCUMENTED:   # each one is described in the module docstring table
        assert re.search(rf"^{n}\s", knobs.__doc__, re.M), n


def test_undocumented_name_is_refused():
    with pytest.raises(AssertionError):
        knobs.get("JR_SOMETHING_ELSE")


def test_cfg_override_parse(monkeypatch):
    monkeypatch.setenv("JR_CFG_OVERRIDE", "gru0.b=27, me.convflow2=4")
    assert knobs.cfg_override() == {"gru0.b": 27, "me.convflow2": 4}
    monkeypatch.setenv("JR_CFG_OVERRIDE", "")
    assert knobs.cfg_override() == {}
