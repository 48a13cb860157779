"""Multi-frame SART: up to 128 independent frames solved together on the matrix cores (fp32, or bf16 shards).

The reference solves the time series strictly frame by frame (reference main.cpp:131-140), streaming
the RTM twice per iteration per frame. For throughput on long time series (BASELINE.json config 5),
frames can be batched: the forward and back projections become skinny GEMMs ``A.X`` / ``A^T.W`` with
16, 32, 64 or 128 right-hand sides (csrc/kernels/multiframe.hip, ``v_mfma_f32_16x16x4_f32`` on 1, 2 or 4
column groups; from 32 frames on A is split in registers into two f16 pieces of A scaled per row (forward) / per
column (back-projection) for the 16-bit matrix cores, csrc/kernels/multiframe_bf16.hip, which also take 128 frames
on 8 column groups), reading A twice per iteration for the whole batch. Every frame keeps its own normalisation,
saturation mask, convergence history, iteration count and status. The batch's columns are slots refilled on the
device: frames are staged into a device queue ahead of the sweeps, and the sweep in which a frame finishes retires
it (into an output ring the host drains) and admits the next queued frame into its slot, so no sweep is spent on
finished frames while frames wait and the host never sits between a slot and its next frame. Frames are
cold-started (``--no_guess``), or started as a time series: each frame from the current iterate of the newest
frame in flight (or finished), rescaled to its own normalisation (``SolveResult.warm_from`` / ``warm_iter``; the
reference warm-starts frame k from frame k-1's converged solution, main.cpp:127-139 -- here the chain is
pipelined), the first ones from ``x0`` (or cold). A frame whose iterate turns non-finite returns its last finite
iterate.

The solver runs in the native engine (csrc/engine/multiframe.cpp, ``sart::MultiFrameEngine``; glue
kernels in csrc/kernels/multiframe_glue.hip); this class is its Python face.
"""
from __future__ import annotations

import os
from typing import List, Optional

import numpy as np

from ..ops import hip
from ..ops.state import MAX_ITERATIONS_EXCEEDED, SUCCESS
from ..parallel.comm import Communicator, SingleProcessComm, native_communicator
from .laplacian import LaplacianCSR
from .rtm import DenseRTM
from .sart import SolveResult, SolverParams, _host_f64

NF = 16        # MFMA column group (frames per 16-wide N tile)
MAX_BATCH = 128  # widest batch: 8 column groups (bf16 storage and split-A with f16 pairs; the fp32 MFMA and bf16
                 # six-product back-projection paths take 64)


class MultiFrameSARTSolver:
    def __init__(self, rtm, laplacian: Optional[LaplacianCSR] = None, comm: Optional[Communicator] = None,
                 params: Optional[SolverParams] = None, logarithmic: bool = False, batch: int = NF,
                 check_interval: int = 16, allow_zero_tolerance: bool = False, split_a: Optional[bool] = None):
        if getattr(rtm, "is_column_shard", False):
            raise NotImplementedError("the multi-frame engine runs on row shards (use SARTSolver for column shards)")
        self.k = hip()
        self.rtm = rtm
        self.dev = rtm.device
        self.comm = comm or SingleProcessComm()
        self.params = params or SolverParams()
        self.params.validate(allow_zero_tolerance)
        self.log = bool(logarithmic)
        self.batch = max(1, min(int(batch), MAX_BATCH))
        self.L = laplacian if (laplacian is not None and laplacian.nnz > 0 and self.params.beta_laplace > 0) else None
        if self.L is not None and self.L.n != rtm.nvoxel:
            raise ValueError("Laplacian and ray-transfer matrices have different number of voxels.")
        p = self.params
        cfg = self.k.EngineConfig()
        cfg.logarithmic = self.log
        cfg.ray_density_threshold = float(p.ray_density_threshold)
        cfg.ray_length_threshold = float(p.ray_length_threshold)
        cfg.conv_tolerance = float(p.conv_tolerance)
        cfg.beta_laplace = float(p.beta_laplace)
        cfg.relaxation = float(p.relaxation)
        cfg.max_iterations = int(p.max_iterations)
        cfg.allow_zero_tolerance = bool(allow_zero_tolerance)
        cfg.check_interval = max(1, int(check_interval))
        cfg.mf_frames = self.batch
        cfg.rtm_bf16 = bool(getattr(rtm, "is_bf16", False))  # bf16 storage: bf16 MFMA projections
        # fp32 storage: fp32 MFMA, or A split into hi + lo bf16 on the bf16 matrix cores (None: the engine's
        # default, on for batches of 32 / 64 frames, env SART_MF_X3)
        cfg.mf_split_a = -1 if split_a is None else int(bool(split_a))
        device = self.dev.index if self.dev.index is not None else 0
        self.native_comm = native_communicator(self.comm, device)
        if getattr(rtm, "nnz", None) is not None:  # SparseRTM: fp32 SpMM projections (csrc/kernels/sparse.hip)
            self.engine = self.k.MultiFrameEngine.from_sparse(device, *rtm.pointers(), rtm.nnz, rtm.npixel,
                                                              rtm.nvoxel, self.native_comm, cfg)
        else:
            self.engine = self.k.MultiFrameEngine(device, rtm.A.data_ptr(), rtm.npixel, rtm.nrows_pad, rtm.nvoxel,
                                                  rtm.ld, self.native_comm, cfg)
        if self.L is not None:
            self.engine.set_laplacian(self.L.row_ptr_host, self.L.col_host, self.L.val_host)
        self.P, self.Pp, self.V, self.ld = rtm.npixel, rtm.nrows_pad, rtm.nvoxel, rtm.ld
        self.batch_width = int(self.engine.batch_frames)  # 16, 32, 64 or 128 columns on the matrix cores
        self.split_a = bool(self.engine.split_a)
        # operand pieces of the projections: "f16x2" (split-A default: range-safe f16 pairs, per-row scales in the
        # forward, per-column in the back-projection), "bf16x2" / "bf16x3" (SART_MF_FWD16=0 / SART_MF_BWD16=0),
        # "fp32" (fp32 MFMA) or "bf16-storage"
        self.forward_split = str(self.engine.forward_split)
        self.backproject_split = str(self.engine.backproject_split)

    def solve_batch(self, measurements, x0=None, chain: bool = False, record_starts: bool = False) -> List[SolveResult]:
        """Frames [nframes, local pixels] through ``batch_width`` slots refilled on the device. ``x0`` (nvoxel,
        optional): with ``chain`` the start value while no frame is in flight yet, else of the first
        ``batch_width`` frames (None: cold). ``chain``: a time series -- every frame starts from the current
        iterate of the newest frame in flight or finished (``SolveResult.warm_from`` / ``warm_iter``); otherwise
        frames cold-start. ``record_starts``: keep every frame's start value (de-normalised) in ``self.starts``
        (tests of the chain). ``self.series_stats``: sweeps, slot utilisation, mean iterations of the run."""
        g_all = np.ascontiguousarray(np.asarray(measurements, dtype=np.float64))
        if g_all.ndim == 1:
            g_all = g_all[None]
        warm = None if x0 is None else _host_f64(x0)
        ret = self.engine.solve_batch(g_all, warm, bool(chain), bool(record_starts))
        x, infos = ret[0], ret[1]
        self.starts = ret[2] if record_starts else None
        self.series_stats = dict(self.engine.series_stats)
        out: List[SolveResult] = []
        for f, info in enumerate(infos):
            status = SUCCESS if info["status"] == SUCCESS else MAX_ITERATIONS_EXCEEDED
            r = SolveResult(solution=x[f], status=status, iterations=int(info["iterations"]),
                            convergence=float(info["convergence"]), used_fused=False,
                            elapsed_ms=float(info["ms"]), nonfinite=bool(info["nonfinite"]),
                            comm_fallbacks=int(info["comm_fallbacks"]), comm=str(info["comm"]))
            r.warm_from = int(info["warm_from"])
            r.warm_iter = int(info["warm_iter"])
            r.warm_live = bool(info["warm_live"])
            out.append(r)
        return out

    def solve(self, measurement, solution=None) -> SolveResult:
        return self.solve_batch(_host_f64(measurement)[None], x0=solution)[0]
