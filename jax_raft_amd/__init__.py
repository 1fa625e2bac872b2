"""jax_raft_amd: an MI355X (gfx950)-native RAFT optical-flow framework with the
API of alebeck/jax-raft (``RAFT``, ``raft_large``, ``raft_small``)."""
from .models.raft import RAFT, raft_large, raft_small

__version__ = "0.1.0"
__all__ = ("RAFT", "raft_large", "raft_small")
