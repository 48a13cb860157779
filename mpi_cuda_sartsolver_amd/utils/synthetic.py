"""Synthetic dense problems generated on the device (benchmarks, smoke tests, invariance tests).

The RTM element (p, v) and the phantom x_true[v] are pure functions of (seed, global index), so the
same global problem is reproduced exactly for any number of ranks / row shards.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from ..models.rtm import DenseRTM
from ..ops import hip


@dataclass
class SyntheticProblem:
    rtm: DenseRTM
    measurement: torch.Tensor  # fp64 on device, local rows
    x_true: torch.Tensor       # fp64 on device, all voxels


def make_problem(npixel_local: int, nvoxel: int, row_offset: int = 0, seed: int = 1234, device=None,
                 saturate_fraction: float = 0.0, ld=None, storage: str = "fp32") -> SyntheticProblem:
    """storage "bf16": the shard is stored in bf16 and g = A x_true is taken over the stored matrix."""
    k = hip()
    dev = device or torch.device("cuda", torch.cuda.current_device())
    rtm = DenseRTM.synthetic(npixel_local, nvoxel, row_offset, seed=seed, device=dev, ld=ld, storage=storage)
    s = torch.cuda.current_stream(dev).cuda_stream
    x_true = torch.empty(nvoxel, dtype=torch.float64, device=dev)
    k.synth_vector(x_true.data_ptr(), nvoxel, 0, int(seed) + 17, 0.0, 1.0, s)
    xx = torch.zeros(rtm.ld, dtype=torch.float32, device=dev)
    xx[:nvoxel] = x_true.to(torch.float32)
    f = torch.zeros(rtm.nrows_pad, dtype=torch.float32, device=dev)
    k.forward(0, rtm.A.data_ptr(), rtm.ld, rtm.npixel, rtm.nrows_pad, xx.data_ptr(), 0, 0, f.data_ptr(), 0, 0, 0, s,
              rtm.is_bf16)
    g = f[:npixel_local].to(torch.float64)
    if saturate_fraction > 0:
        u = torch.empty(npixel_local, dtype=torch.float64, device=dev)
        k.synth_vector(u.data_ptr(), npixel_local, row_offset, int(seed) + 29, 0.0, 1.0, s)
        g = torch.where(u < saturate_fraction, -torch.ones_like(g), g)
    return SyntheticProblem(rtm=rtm, measurement=g, x_true=x_true)


def make_column_problem(npixel: int, nvoxel_local: int, col_offset: int, nvoxel_total: int, comm=None,
                        seed: int = 1234, device=None) -> SyntheticProblem:
    """Column shard [0, npixel) x [col_offset, +nvoxel_local) of the global synthetic problem, with the
    FULL measurement g = A x_true (partial products all-reduced over ``comm``); x_true is this shard's
    slice. Same global matrix and phantom as ``make_problem`` for the same seed."""
    k = hip()
    dev = device or torch.device("cuda", torch.cuda.current_device())
    rtm = DenseRTM.synthetic(npixel, nvoxel_local, 0, seed=seed, device=dev, col_offset=col_offset,
                             nvoxel_total=nvoxel_total)
    s = torch.cuda.current_stream(dev).cuda_stream
    x_true = torch.empty(nvoxel_local, dtype=torch.float64, device=dev)
    k.synth_vector(x_true.data_ptr(), nvoxel_local, col_offset, int(seed) + 17, 0.0, 1.0, s)
    xx = torch.zeros(rtm.ld, dtype=torch.float32, device=dev)
    xx[:nvoxel_local] = x_true.to(torch.float32)
    f = torch.zeros(rtm.nrows_pad, dtype=torch.float32, device=dev)
    k.forward(0, rtm.A.data_ptr(), rtm.ld, rtm.npixel, rtm.nrows_pad, xx.data_ptr(), 0, 0, f.data_ptr(), 0, 0, 0, s)
    g = f[:npixel].to(torch.float64)
    if comm is not None and comm.world_size > 1:
        on_cpu = getattr(comm, "backend", "gloo") != "nccl"
        t = g.cpu() if on_cpu else g
        comm.all_reduce_(t)
        g = t.to(dev)
    return SyntheticProblem(rtm=rtm, measurement=g, x_true=x_true)


def host_problem(npixel: int, nvoxel: int, seed: int = 7, saturate_fraction: float = 0.0):
    """Small CPU-side problem (numpy) for tests that do not need the device generator."""
    rng = np.random.default_rng(seed)
    A = rng.random((npixel, nvoxel), dtype=np.float32)
    x = rng.random(nvoxel)
    g = A.astype(np.float64) @ x
    if saturate_fraction > 0:
        g[rng.random(npixel) < saturate_fraction] = -1.0
    return A, g, x
