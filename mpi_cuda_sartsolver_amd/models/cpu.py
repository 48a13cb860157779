"""CPU SART solvers (the ``--use_cpu`` path): fp64 arithmetic over the fp32 RTM shard.

Reference: ``SARTSolverMPI`` / ``LogSARTSolverMPI`` (reference sartsolver.cpp:133-339), with host MPI.
Here the O(P*V) loops run in the native OpenMP kernels (csrc/native/cpu_kernels.cpp) and the
reductions go through the same :class:`Communicator` as the GPU path (``gloo`` process group across
ranks; per iteration one vector and one scalar collective, as the reference).

``semantics="cpu"`` (default) reproduces the reference CPU path exactly: no normalisation, the cold
start back-projects the raw measurement including negative (saturated) pixels, the linear update is
not clamped at 1e-7 and the logarithmic variant uses 1e-100 as clamp and epsilon.
``semantics="gpu"`` evaluates the GPU semantics in fp64 (the oracle of models/reference.py, sharded).
"""
from __future__ import annotations

import time
from typing import Optional

import numpy as np
import torch

from ..ops import native
from ..ops.state import MAX_ITERATIONS_EXCEEDED, SUCCESS
from ..parallel.comm import Communicator, SingleProcessComm
from .sart import SolveResult, SolverParams


class CPUSARTSolver:
    def __init__(self, A_local: np.ndarray, laplacian=None, comm: Optional[Communicator] = None,
                 params: Optional[SolverParams] = None, logarithmic: bool = False, semantics: str = "cpu",
                 allow_zero_tolerance: bool = False):
        self.n = native()
        self.A = np.ascontiguousarray(A_local, dtype=np.float32)
        self.P, self.V = self.A.shape
        self.comm = comm or SingleProcessComm()
        self.params = params or SolverParams()
        self.params.validate(allow_zero_tolerance)
        self.log = bool(logarithmic)
        if semantics not in ("cpu", "gpu"):
            raise ValueError("semantics must be 'cpu' or 'gpu'")
        self.semantics = semantics
        self.L = laplacian if (laplacian is not None and laplacian.nnz > 0 and self.params.beta_laplace > 0) else None
        rho, ell = self.n.cpu_raysums(self.A, self.P, self.V)
        self.rho = self._allreduce(rho)
        self.ell = ell
        p = self.params
        if semantics == "gpu":  # fp32 thresholds on fp32-rounded sums, as the GPU kernels compare
            rho32, ell32 = self.rho.astype(np.float32), ell.astype(np.float32)
            self.dvalid = rho32 > np.float32(p.ray_density_threshold)
            self.rho_s = np.where(self.dvalid, rho32.astype(np.float64), 1.0)
            self.pvalid_len = ell32 > np.float32(p.ray_length_threshold)
            self.inv_len = np.where(self.pvalid_len, 1.0 / np.where(ell32 > 0, ell32, 1.0), 0.0)
        else:
            self.dvalid = self.rho > p.ray_density_threshold
            self.rho_s = np.where(self.dvalid, self.rho, 1.0)
            self.pvalid_len = ell > p.ray_length_threshold
            self.inv_len = np.where(self.pvalid_len, 1.0 / np.where(ell != 0, ell, 1.0), 0.0)

    # ------------------------------------------------------------------------------------------
    def _allreduce(self, arr: np.ndarray, op: str = "sum") -> np.ndarray:
        if self.comm.world_size == 1:
            return arr
        t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float64))
        self.comm.all_reduce_(t, op=op)
        return t.numpy()

    def _penalty(self, x: np.ndarray) -> np.ndarray:
        if self.L is None:
            return 0.0
        return self.params.beta_laplace * self.L.matvec(np.log(x) if self.log else x)

    def _fwd(self, x):
        return self.n.cpu_forward(self.A, self.P, self.V, x)

    def _bwd(self, w):
        return self.n.cpu_backproject(self.A, self.P, self.V, np.ascontiguousarray(w, dtype=np.float64))

    # ------------------------------------------------------------------------------------------
    def solve(self, measurement, solution=None) -> SolveResult:
        t0 = time.perf_counter()
        p = self.params
        g = np.asarray(measurement, dtype=np.float64)
        if g.size != self.P:
            raise ValueError(f"measurement has {g.size} pixels, the local shard has {self.P}")
        if self.semantics == "gpu":
            norm = self.comm.all_reduce_scalar(float(g.max()) if g.size else -np.inf, op="max")
            if not norm > 0:
                norm = 1.0
            gw = (g / norm).astype(np.float32).astype(np.float64)
            eps, clamp = 1e-7, 1e-7
        else:
            norm, gw, eps, clamp = 1.0, g, 1e-100, (1e-100 if self.log else None)
        G = self.comm.all_reduce_scalar(float(np.sum(np.where(g > 0, g * g, 0.0)))) / (norm * norm)
        a = np.where(gw >= 0, self.inv_len, 0.0)
        if solution is None:
            w0 = np.maximum(gw, 0.0) if self.semantics == "gpu" else gw
            x = np.where(self.dvalid, self._allreduce(self._bwd(w0)) / self.rho_s, 0.0)
        else:
            x = np.asarray(solution, dtype=np.float64).copy() / norm
            if x.size != self.V:
                raise ValueError("Solution vector must be empty or contain nvoxel elements.")
        if clamp is not None:
            x = np.maximum(x, clamp)
        O = np.where(self.dvalid, self._allreduce(self._bwd(a * gw)), 0.0) if self.log else None
        f, _ = self._fwd(x)
        conv_prev = 0.0
        conv = 0.0
        status, iters = MAX_ITERATIONS_EXCEEDED, p.max_iterations
        for it in range(p.max_iterations):
            pen = self._penalty(x)
            red = self._allreduce(self._bwd(a * f) if self.log else self._bwd(a * (gw - f)))
            if self.log:
                Fv = np.where(self.dvalid, red[: self.V], 0.0)
                x = x * ((O + eps) / (Fv + eps)) ** p.relaxation * np.exp(-pen)
            else:
                d = np.where(self.dvalid, p.relaxation / self.rho_s * red[: self.V], 0.0) - pen
                x = x + d
                x = np.where(np.signbit(x), 0.0, x) if self.semantics == "cpu" else np.maximum(x, 0.0)
            f, f2 = self._fwd(x)
            F = self.comm.all_reduce_scalar(f2)
            conv = (G - F) / G if G != 0 else 0.0
            if it and abs(conv - conv_prev) < p.conv_tolerance:
                status, iters = SUCCESS, it + 1
                break
            conv_prev = conv
        return SolveResult(solution=x * norm, status=status, iterations=iters, convergence=conv, used_fused=False,
                           elapsed_ms=1e3 * (time.perf_counter() - t0))
