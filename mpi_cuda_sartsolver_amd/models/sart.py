"""GPU SART solvers (linear and logarithmic, optional Laplacian regulariser) on MI355X.

Functional parity with the reference GPU solvers ``SARTSolverMPICuda`` / ``LogSARTSolverMPICuda``
(reference sartsolver_cuda.cpp:197-354, math in manual.pdf p.2 eqs. 1-6), re-designed for gfx950.
The solver runs in the native C++ engine (csrc/engine/engine.cpp, class ``sart::Engine``); this module
is its Python face (parameters, communicator hand-over, results):

* ray density / ray length: device fp64 column/row sums (reference: CPU loops, sartsolver.cpp:38-56);
* per iteration ONE fused sweep over the local RTM shard (forward projection + SART weight +
  back-projection from a single HBM read, csrc/kernels/fused_sweep.hip), or the two-pass
  kernels (forward with fused epilogue + deterministic split-K back-projection) as fallback;
* the penalty ``beta L x`` (or ``beta L log x``) is applied after the reduction on every rank --
  equivalent to the reference's rank-0-only penalty added before the reduction (main.cpp:73-74,
  sart_kernels.cu:106-109) and identical for the logarithmic variant (sart_kernels.cu:219-220);
* logarithmic SART: the observed back-projection ``O = A^T(a g)`` depends only on the frame, so it is
  computed and reduced once per frame; the reference recomputes and all-reduces it every iteration
  (sart_kernels.cu:113-176, sartsolver_cuda.cpp:322-324);
* one collective per iteration (correction + ||A x||^2 piggybacked) on device buffers;
* convergence test, iteration counter and status are device-resident (``SartState``); the host
  checks them every ``check_interval`` iterations, never per iteration.

Iteration semantics are those of the reference loop: sweep ``s`` computes ``f = A x_s``; for ``s >= 1``
it yields the reference's ``conv_{s-1}``; the solve stops when ``s >= 2`` and
``|conv_{s-1} - conv_{s-2}| < tol`` (SUCCESS, 0) or after ``max_iterations`` updates
(MAX_ITERATIONS_EXCEEDED, -1), returning ``x_s`` de-normalised in fp64.
"""
from __future__ import annotations

import logging
import math
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from ..ops import hip
from ..ops.state import MAX_ITERATIONS_EXCEEDED, SUCCESS
from ..parallel.comm import Communicator, SingleProcessComm, native_communicator
from .laplacian import LaplacianCSR
from .rtm import DenseRTM

log = logging.getLogger(__name__)

EPI_PLAIN, EPI_LINEAR, EPI_LOG = 0, 1, 2


@dataclass
class SolverParams:
    """Solver parameters with the reference defaults (sartsolver.hpp:64-66, arguments.cpp:101-133)."""

    ray_density_threshold: float = 1e-6
    ray_length_threshold: float = 1e-6
    conv_tolerance: float = 1e-5
    beta_laplace: float = 1e-2
    relaxation: float = 1.0
    max_iterations: int = 2000

    def validate(self, allow_zero_tolerance: bool = False) -> None:
        # Same checks as the reference setters (sartsolver.cpp:61-123).
        if self.ray_density_threshold < 0:
            raise ValueError("Ray density threshold must be non-negative.")
        if self.ray_length_threshold < 0:
            raise ValueError("Ray length threshold must be non-negative.")
        if self.conv_tolerance < 0 or (self.conv_tolerance == 0 and not allow_zero_tolerance):
            raise ValueError("Convolution tolerance must be positive.")
        if self.beta_laplace < 0:
            raise ValueError("Attribute beta_laplace must be non-negative.")
        if not (0 < self.relaxation <= 1.0):
            raise ValueError("Attribute relaxation must be within (0, 1] interval.")
        if self.max_iterations <= 0:
            raise ValueError("Attribute max_iterations must be positive.")


@dataclass
class SolveResult:
    solution: np.ndarray  # fp64, de-normalised (reference sartsolver_cuda.cpp:264-265)
    status: int
    iterations: int
    convergence: float
    used_fused: bool
    elapsed_ms: float = 0.0
    comm_ms: float = -1.0  # GPU time in the per-sweep all-reduces (time_collectives=True), else -1
    fallbacks: int = 0      # persistent-sweep timeouts recovered in this solve (identical on every rank)
    comm_fallbacks: int = 0  # device all-reduce timeouts recovered (re-solved on the base communicator)
    comm: str = ""           # device communicator that produced the result (p2p / rccl / staged / local)
    fused_variant: int = -1  # fused sweep variant that produced the result (-1: two-pass kernels)
    nonfinite: bool = False  # stopped by the NaN/Inf guard: ``solution`` is the last finite iterate
    warm_from: int = -1      # multi-frame time series: frame whose iterate started this one (-1: x0 / cold)
    warm_iter: int = -1      # ... and that iterate's update count (its final count when it had finished)
    warm_live: bool = False  # ... which was still in flight (extrapolated along its last update)


def _host_f64(v) -> np.ndarray:
    if isinstance(v, torch.Tensor):
        v = v.detach().to("cpu", torch.float64).numpy()
    return np.ascontiguousarray(np.asarray(v, dtype=np.float64).ravel())


class SARTSolver:
    """Per-GPU SART solver over a device-resident row shard (one instance per rank).

    Thin wrapper of ``sart::Engine``: all device work, the per-iteration all-reduce (RCCL for the
    ``nccl`` process group, host TCP otherwise) and the convergence loop run in C++.
    """

    def __init__(self, rtm, laplacian: Optional[LaplacianCSR] = None,
                 comm: Optional[Communicator] = None, params: Optional[SolverParams] = None,
                 logarithmic: bool = False, use_fused: bool = True, check_interval: int = 16,
                 allow_zero_tolerance: bool = False, fused_variant: Optional[int] = None,
                 fused_rows_per_tile: Optional[int] = None, use_graph: Optional[bool] = None,
                 fused_min_bytes: float = 0.0, partition: Optional[str] = None, time_collectives: bool = False):
        self.k = hip()
        self.rtm = rtm
        self.dev = rtm.device
        self.comm = comm or SingleProcessComm()
        self.params = params or SolverParams()
        self.params.validate(allow_zero_tolerance)
        self.log = bool(logarithmic)
        self.L = laplacian if (laplacian is not None and laplacian.nnz > 0 and self.params.beta_laplace > 0) else None
        # "rows" (reference layout) or "cols" (voxel shard); default: from the shard
        if partition not in (None, "rows", "cols"):
            raise ValueError("partition must be 'rows' or 'cols'")
        self.column_shard = partition == "cols" or (partition is None and bool(getattr(rtm, "is_column_shard", False)))
        if self.L is not None and self.L.n != getattr(rtm, "nvoxel_total", rtm.nvoxel):
            raise ValueError("Laplacian and ray-transfer matrices have different number of voxels.")
        if fused_variant is None:
            fused_variant = int(os.environ.get("SART_FUSED_VARIANT", "6"))
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
        cfg.use_fused = bool(use_fused)
        cfg.fused_variant = int(fused_variant)
        cfg.rows_per_tile = int(fused_rows_per_tile or 0)
        cfg.fused_schedule = int(os.environ.get("SART_FUSED_SCHEDULE", "-1"))
        if use_graph is None:
            use_graph = os.environ.get("SART_GRAPH", "0") == "1"
        cfg.use_graph = bool(use_graph)
        cfg.fused_min_bytes = float(fused_min_bytes)  # smaller shards use the two-pass kernels
        cfg.time_collectives = bool(time_collectives)
        cfg.rtm_bf16 = bool(getattr(rtm, "is_bf16", False))  # bf16-stored shard: two-pass kernels  # SolveResult.comm_ms (events around each all-reduce)
        if self.column_shard:  # all pixel rows of voxels [col_offset, +nvoxel): two-pass, pixel all-reduce
            cfg.column_shard = True
            cfg.col_offset = int(getattr(rtm, "col_offset", 0))
            cfg.nvoxel_total = int(getattr(rtm, "nvoxel_total", rtm.nvoxel))
        device = self.dev.index if self.dev.index is not None else 0
        self.native_comm = native_communicator(self.comm, device)
        if getattr(rtm, "nnz", None) is not None:  # SparseRTM: CSR / CSC kernels, two-pass sweep
            if self.column_shard:
                raise ValueError("a sparse RTM shard is a row shard")
            self.engine = self.k.Engine.from_sparse(device, *rtm.pointers(), rtm.nnz, rtm.npixel, rtm.nvoxel,
                                               self.native_comm, cfg)
        else:
            self.engine = self.k.Engine(device, rtm.A.data_ptr(), rtm.npixel, rtm.nrows_pad, rtm.nvoxel, rtm.ld,
                                        self.native_comm, cfg)
        if self.L is not None:
            self.engine.set_laplacian(self.L.row_ptr_host, self.L.col_host, self.L.val_host)
        self.P, self.Pp, self.V, self.ld = rtm.npixel, rtm.nrows_pad, rtm.nvoxel, rtm.ld
        self.num_cus = self.engine.num_cus

    @property
    def use_fused(self) -> bool:
        return self.engine.use_fused

    @property
    def shared_device(self) -> bool:
        """Another rank of the group drives the same physical GPU (two-pass kernels, or the fused sweep on a
        share of the CUs with SART_FUSED_SHARED=1)."""
        return self.engine.shared_device

    @property
    def ranks_per_device(self) -> int:
        return self.engine.ranks_per_device

    @property
    def plan_cus(self) -> int:
        """CUs the fused geometry was planned for (all of them, or a share when ranks share the GPU)."""
        return self.engine.plan_cus

    @property
    def geom(self):
        return self.engine.geometry if self.engine.use_fused else None

    @property
    def ray_density64(self) -> np.ndarray:
        return self.engine.ray_density()

    @property
    def ray_length64(self) -> np.ndarray:
        return self.engine.ray_length()

    def solve(self, measurement, solution=None) -> SolveResult:
        """Solve one frame. ``measurement``: this rank's pixel slice (fp64; ALL pixels for a column shard);
        ``solution``: warm start (fp64, this shard's voxels) or None for the default initial guess. The
        solution holds this shard's voxels (all of them for a row shard; see ``gather_solution``)."""
        g = _host_f64(measurement)
        x0 = None if solution is None else _host_f64(solution)
        x, info = self.engine.solve(g, x0)
        if info["fallbacks"]:
            log.warning("fused sweep fell back %d time(s); now %s", info["fallbacks"],
                        f"variant {info['fused_variant']}" if info["used_fused"] else "two-pass kernels")
        status = SUCCESS if info["status"] == SUCCESS else MAX_ITERATIONS_EXCEEDED
        return SolveResult(solution=x, status=status, iterations=int(info["iterations"]),
                           convergence=float(info["convergence"]), used_fused=bool(info["used_fused"]),
                           elapsed_ms=float(info["ms"]), comm_ms=float(info["comm_ms"]),
                           fallbacks=int(info["fallbacks"]), fused_variant=int(info["fused_variant"]),
                           nonfinite=bool(info["nonfinite"]), comm_fallbacks=int(info["comm_fallbacks"]),
                           comm=str(info["comm"]))

    def gather_solution(self, x_local: np.ndarray) -> np.ndarray:
        """Full solution vector from the column shards of every rank (identity for a row shard)."""
        if not self.column_shard:
            return x_local
        parts = self.comm.all_gather_object((int(getattr(self.rtm, "col_offset", 0)), np.asarray(x_local)))
        out = np.zeros(int(getattr(self.rtm, "nvoxel_total", self.rtm.nvoxel)), dtype=np.float64)
        for off, xs in parts:
            out[off: off + xs.size] = xs
        return out

    def forward_project(self, x_local) -> np.ndarray:
        """f = A x for this shard (utility / tests)."""
        return self.engine.forward(_host_f64(x_local))
