"""CPU SART solvers (the ``--use_cpu`` path): fp64 arithmetic over the fp32 RTM shard.

Reference: ``SARTSolverMPI`` / ``LogSARTSolverMPI`` (reference sartsolver.cpp:133-339), with host MPI.
The solver runs in C++ (csrc/native/cpu_solver.cpp, ``sart::CpuSolver``): the O(P*V) loops are the
OpenMP kernels of csrc/native/cpu_kernels.cpp and the reductions go through the native host
communicator (TCP across ranks, fixed rank order; per iteration one vector and one scalar collective,
as the reference).

``semantics="cpu"`` (default) reproduces the reference CPU path exactly: no normalisation, the cold
start back-projects the raw measurement including negative (saturated) pixels, the linear update is
not clamped at 1e-7 and the logarithmic variant uses 1e-100 as clamp and epsilon.
``semantics="gpu"`` evaluates the GPU semantics in fp64 (the oracle of models/reference.py, sharded).
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from ..ops import native
from ..ops.state import MAX_ITERATIONS_EXCEEDED, SUCCESS
from ..parallel.comm import Communicator, SingleProcessComm, native_host_communicator
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
        p = self.params
        sp = self.n.SolverParams()
        sp.logarithmic = self.log
        sp.ray_density_threshold = float(p.ray_density_threshold)
        sp.ray_length_threshold = float(p.ray_length_threshold)
        sp.conv_tolerance = float(p.conv_tolerance)
        sp.beta_laplace = float(p.beta_laplace)
        sp.relaxation = float(p.relaxation)
        sp.max_iterations = int(p.max_iterations)
        sp.allow_zero_tolerance = bool(allow_zero_tolerance)
        self.host_comm = native_host_communicator(self.comm)
        self.solver = self.n.CpuSolver(self.A, self.P, self.V, self.host_comm, sp, semantics == "gpu")
        self.L = laplacian if (laplacian is not None and laplacian.nnz > 0 and p.beta_laplace > 0) else None
        if self.L is not None:
            if self.L.n != self.V:
                raise ValueError("Laplacian and ray-transfer matrices have different number of voxels.")
            self.solver.set_laplacian(self.L.n, self.L.row_ptr_host, self.L.col_host, self.L.val_host)

    @property
    def rho(self) -> np.ndarray:
        return self.solver.ray_density()

    @property
    def ell(self) -> np.ndarray:
        return self.solver.ray_length()

    def solve(self, measurement, solution=None) -> SolveResult:
        g = np.ascontiguousarray(np.asarray(measurement, dtype=np.float64).ravel())
        if g.size != self.P:
            raise ValueError(f"measurement has {g.size} pixels, the local shard has {self.P}")
        x0 = None
        if solution is not None:
            x0 = np.ascontiguousarray(np.asarray(solution, dtype=np.float64).ravel())
            if x0.size != self.V:
                raise ValueError("Solution vector must be empty or contain nvoxel elements.")
        x, info = self.solver.solve(g, x0)
        status = SUCCESS if info["status"] == SUCCESS else MAX_ITERATIONS_EXCEEDED
        return SolveResult(solution=x, status=status, iterations=int(info["iterations"]),
                           convergence=float(info["convergence"]), used_fused=False, elapsed_ms=float(info["ms"]))
