"""Row (pixel) partition of the ray-transfer matrix across ranks.

Same balanced 1-D block partition as the reference (reference main.cpp:67-68): the first
``npixel % nproc`` ranks get one extra row; every rank holds all voxels. Forward projection is then
rank-local and the back-projection yields voxel partial sums that are all-reduced once per iteration.
``col_partition`` gives the optional voxel-sharded layout (every rank holds all pixel rows of a
block of voxels; the per-iteration all-reduce then carries the pixel vector A.x instead).
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class Block:
    offset: int
    size: int

    @property
    def stop(self) -> int:
        return self.offset + self.size


def block_partition(n: int, nparts: int, part: int) -> Block:
    if nparts <= 0 or not 0 <= part < nparts:
        raise ValueError(f"invalid partition request part={part} nparts={nparts}")
    base, rem = divmod(n, nparts)
    offset = part * base + min(part, rem)
    size = base + (1 if part < rem else 0)
    return Block(offset, size)


def row_partition(npixel: int, world_size: int, rank: int) -> Block:
    """Pixel rows owned by ``rank`` (reference main.cpp:67-68)."""
    return block_partition(npixel, world_size, rank)


def col_partition(nvoxel: int, world_size: int, rank: int) -> Block:
    """Voxel columns owned by ``rank`` in the column-shard layout (EngineConfig::column_shard)."""
    return block_partition(nvoxel, world_size, rank)


def all_blocks(n: int, nparts: int) -> list[Block]:
    return [block_partition(n, nparts, p) for p in range(nparts)]


def round_up(n: int, m: int) -> int:
    return (n + m - 1) // m * m
