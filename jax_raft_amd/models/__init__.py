from .raft import RAFT, raft_large, raft_small  # noqa: F401
