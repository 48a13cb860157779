"""Decomposition and communication (row partition, torch.distributed/RCCL communicators)."""
from .partition import Block, block_partition, row_partition  # noqa: F401
