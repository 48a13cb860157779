"""Partition helpers (row / column shards) and the bench.py configuration presets (CPU only)."""
import importlib.util
import os

import pytest

from mpi_cuda_sartsolver_amd.parallel.partition import all_blocks, col_partition, row_partition

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n,parts", [(10, 3), (65536, 8), (7, 7), (5, 8), (1000003, 6)])
def test_block_partitions_tile_the_range(n, parts):
    for fn in (row_partition, col_partition):
        blocks = [fn(n, parts, r) for r in range(parts)]
        assert blocks[0].offset == 0 and blocks[-1].stop == n
        assert all(a.stop == b.offset for a, b in zip(blocks, blocks[1:]))
        sizes = [b.size for b in blocks]
        assert max(sizes) - min(sizes) <= 1 and sizes == sorted(sizes, reverse=True)  # extra rows go first
    assert all_blocks(n, parts) == [row_partition(n, parts, r) for r in range(parts)]


def test_partition_rejects_bad_rank():
    with pytest.raises(ValueError):
        row_partition(10, 2, 2)
    with pytest.raises(ValueError):
        col_partition(10, 0, 0)


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_bench_presets_match_baseline_configs():
    b = _bench()
    p = b.PRESETS
    # 64k x 64k on one GPU, 100 iterations (BASELINE.json config 2)
    assert (p["64k"]["npix"], p["64k"]["nvox"], p["64k"]["iters"]) == (65536, 65536, 100)
    # 256k x 256k fp32 fills one 288 GB GPU (config 3)
    assert p["256k"]["npix"] * p["256k"]["nvox"] * 4 / 1e9 == pytest.approx(274.9, abs=0.1)
    # 512k x 256k row-partitioned over 8 GPUs (config 4): weak preset, 8 shards
    assert (8 * p["512kx256k"]["npix"], p["512kx256k"]["nvox"]) == (524288, 262144)
    # ~2 TB over 8 x 288 GB with the Laplacian and a multi-frame batch (config 5)
    two = p["2tb"]
    assert 8 * two["npix"] * two["nvox"] * 4 / 1e12 == pytest.approx(2.06, abs=0.01)
    assert two["laplacian"] and two["frames"] > 1
    assert two["npix"] * two["nvox"] * 4 < 288e9 * 0.95  # shard + workspaces fit one GPU


@pytest.mark.parametrize("n", [4096, 65536, 262144, 1000, 17])
def test_grid_dims_factorise(n):
    nx, ny, nz = _bench().grid_dims(n)
    assert nx * ny * nz == n and nx >= ny >= nz >= 1
