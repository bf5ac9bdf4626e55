"""Decomposition and process groups (torch.distributed + native RCCL)."""
from . import decomposition  # noqa: F401
