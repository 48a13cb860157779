"""Multi-frame SART: up to 16 independent frames solved together on the fp32 matrix cores.

The reference solves the time series strictly frame by frame (reference main.cpp:131-140), streaming
the RTM twice per iteration per frame. For throughput on long time series (BASELINE.json config 5),
frames can be batched: the forward and back projections become skinny GEMMs ``A.X`` / ``A^T.W`` with
16 right-hand sides (csrc/kernels/multiframe.hip, ``v_mfma_f32_16x16x4_f32``), reading A once per
iteration for all 16 frames. Every frame keeps its own normalisation, saturation mask, convergence
history and status; frames that converge are frozen while the others continue. Batched frames are
cold-started (no warm start chain between them), like ``--no_guess``.
"""
from __future__ import annotations

import math
from typing import List, Optional

import numpy as np
import torch

from ..ops import hip
from ..ops.state import MAX_ITERATIONS_EXCEEDED, SUCCESS
from ..parallel.comm import Communicator, SingleProcessComm
from .laplacian import LaplacianCSR
from .rtm import DenseRTM
from .sart import SolveResult, SolverParams

NF = 16


class MultiFrameSARTSolver:
    def __init__(self, rtm: DenseRTM, laplacian: Optional[LaplacianCSR] = None, comm: Optional[Communicator] = None,
                 params: Optional[SolverParams] = None, logarithmic: bool = False, batch: int = NF,
                 check_interval: int = 16, allow_zero_tolerance: bool = False):
        self.k = hip()
        self.rtm = rtm
        self.dev = rtm.device
        self.comm = comm or SingleProcessComm()
        self.params = params or SolverParams()
        self.params.validate(allow_zero_tolerance)
        self.log = bool(logarithmic)
        self.batch = max(1, min(int(batch), NF))
        self.check_interval = max(1, int(check_interval))
        self.L = laplacian if (laplacian is not None and laplacian.nnz > 0 and self.params.beta_laplace > 0) else None
        P, Pp, V, ld = rtm.npixel, rtm.nrows_pad, rtm.nvoxel, rtm.ld
        self.P, self.Pp, self.V, self.ld = P, Pp, V, ld
        if Pp % 32:
            raise ValueError("padded rows must be a multiple of 32")
        self.nsf = self.k.mf_forward_num_splits(ld, Pp)
        self.nsb = self.k.mf_backproject_num_splits(ld, P)
        f32 = dict(dtype=torch.float32, device=self.dev)
        self.X = torch.zeros((NF, ld), **f32)
        self.Fs = torch.zeros((self.nsf, Pp, NF), **f32)
        self.W = torch.zeros((Pp, NF), **f32)
        self.part = torch.zeros((self.nsb, ld, NF), **f32)
        self.pen = torch.zeros((NF, ld), **f32)
        self._stream = lambda: torch.cuda.current_stream(self.dev).cuda_stream  # noqa: E731
        self._ray_sums()

    def _ray_sums(self):
        k, s = self.k, self._stream()
        ell = torch.zeros(self.Pp, dtype=torch.float64, device=self.dev)
        k.rowsum_f64(self.rtm.A.data_ptr(), self.ld, self.P, ell.data_ptr(), s)
        ns = k.backproject_num_splits(self.ld, self.Pp)
        part = torch.zeros(ns * self.ld, dtype=torch.float64, device=self.dev)
        k.colsum_f64(self.rtm.A.data_ptr(), self.ld, self.P, ns, part.data_ptr(), s)
        rho = torch.zeros(self.ld, dtype=torch.float64, device=self.dev)
        k.reduce_partials_f64(part.data_ptr(), self.ld, ns, rho.data_ptr(), s)
        self.comm.all_reduce_(rho)
        p = self.params
        rho32 = rho.to(torch.float32)
        ell32 = ell.to(torch.float32)
        valid = rho32 > np.float32(p.ray_density_threshold)
        one = torch.ones_like(rho32)
        safe = torch.where(valid, rho32, one)
        self.dinv = torch.where(valid, one / safe, torch.zeros_like(rho32))
        self.dscale = torch.where(valid, torch.tensor(np.float32(p.relaxation), device=self.dev) / safe,
                                  torch.zeros_like(rho32))
        self.dmask = valid.to(torch.float32)
        lvalid = ell32 > np.float32(p.ray_length_threshold)
        self.inv_len = torch.where(lvalid, 1.0 / torch.where(lvalid, ell32, torch.ones_like(ell32)),
                                   torch.zeros_like(ell32))

    # ------------------------------------------------------------------------------------------
    def _forward(self) -> torch.Tensor:
        self.k.mf_forward(self.rtm.A.data_ptr(), self.ld, self.P, self.Pp, self.X.data_ptr(), self.ld,
                          self.Fs.data_ptr(), self.nsf, self._stream())
        return self.Fs.sum(0) if self.nsf > 1 else self.Fs[0]

    def _backproject(self, W: torch.Tensor) -> torch.Tensor:
        self.W.copy_(W)
        self.k.mf_backproject(self.rtm.A.data_ptr(), self.ld, self.P, self.W.data_ptr(), self.nsb,
                              self.part.data_ptr(), self._stream())
        return self.part.sum(0)  # [ld, NF]

    def _penalty(self) -> Optional[torch.Tensor]:
        if self.L is None:
            return None
        s = self._stream()
        beta = float(np.float32(self.params.beta_laplace))
        for f in range(NF):
            self.k.penalty(self.log, self.L.row_ptr.data_ptr(), self.L.col.data_ptr(), self.L.val.data_ptr(), self.V,
                           beta, self.X[f].data_ptr(), self.pen[f].data_ptr(), 0, s)
        return self.pen

    # ------------------------------------------------------------------------------------------
    def solve_batch(self, measurements) -> List[SolveResult]:
        g_all = np.asarray(measurements, dtype=np.float64)
        if g_all.ndim == 1:
            g_all = g_all[None]
        out: List[SolveResult] = []
        for b0 in range(0, g_all.shape[0], self.batch):
            out.extend(self._solve16(g_all[b0: b0 + self.batch]))
        return out

    def _solve16(self, g_np: np.ndarray) -> List[SolveResult]:
        p = self.params
        B = g_np.shape[0]
        dev = self.dev
        G64 = torch.zeros((self.Pp, NF), dtype=torch.float64, device=dev)
        G64[: self.P, :B] = torch.from_numpy(np.ascontiguousarray(g_np.T)).to(dev)
        gmax = G64[: self.P, :B].max(0).values if self.P else torch.full((B,), -math.inf, device=dev)
        norm = torch.ones(NF, dtype=torch.float64, device=dev)
        norm[:B] = gmax
        self.comm.all_reduce_(norm, op="max")
        norm = torch.where(norm > 0, norm, torch.ones_like(norm))
        gpos = torch.clamp(G64[: self.P], min=0.0)
        Gsq = (gpos * gpos).sum(0)
        self.comm.all_reduce_(Gsq)
        Gsq = Gsq / (norm * norm)
        Gsq = torch.where(Gsq > 0, Gsq, torch.ones_like(Gsq))
        ghat = (G64 / norm).to(torch.float32)  # [Pp, NF]
        a = torch.where(ghat >= 0, self.inv_len[:, None], torch.zeros_like(ghat))
        # cold start x0 = [rho > tau] A^T max(ghat, 0) / rho, clamped at 1e-7
        d0 = self._backproject(torch.clamp(ghat, min=0.0))
        self.comm.all_reduce_(d0)
        X = torch.clamp(d0 * self.dinv[:, None], min=1e-7).T.contiguous()
        X[:, self.V:] = 0
        X[B:] = 0
        self.X.copy_(X)
        O = None
        if self.log:
            O = self._backproject(a * ghat)
            self.comm.all_reduce_(O)
            O = (O * self.dmask[:, None]).T.contiguous()  # [NF, ld]
        done = torch.zeros(NF, dtype=torch.bool, device=dev)
        done[B:] = True
        status = torch.full((NF,), MAX_ITERATIONS_EXCEEDED, dtype=torch.int32, device=dev)
        iters = torch.full((NF,), p.max_iterations, dtype=torch.int32, device=dev)
        conv_prev = torch.zeros(NF, dtype=torch.float64, device=dev)
        conv = torch.zeros(NF, dtype=torch.float64, device=dev)
        eps = 1e-7
        alpha = float(np.float32(p.relaxation))
        buf = torch.zeros(NF * self.ld + NF, dtype=torch.float32, device=dev)
        for s in range(p.max_iterations + 1):
            F = self._forward()  # [Pp, NF], F(x_s)
            F2 = (F.double() ** 2).sum(0)
            W = a * F if self.log else a * (ghat - F)
            D = self._backproject(W).T  # [NF, ld]
            D = D * (self.dmask if self.log else self.dscale)[None, :]
            pen = self._penalty()
            buf[: NF * self.ld].copy_(D.reshape(-1))
            buf[NF * self.ld:] = F2.to(torch.float32)
            self.comm.all_reduce_(buf)
            D = buf[: NF * self.ld].view(NF, self.ld)
            F2 = buf[NF * self.ld:].double()
            if s >= 1:
                conv = (Gsq - F2) / Gsq
                newly = (~done) & (abs(conv - conv_prev) < p.conv_tolerance) if s >= 2 else torch.zeros_like(done)
                status = torch.where(newly, torch.full_like(status, SUCCESS), status)
                iters = torch.where(newly, torch.full_like(iters, s), iters)
                done = done | newly
                conv_prev = torch.where(done & ~newly, conv_prev, conv)
            if s >= p.max_iterations:
                break
            if self.log:
                r = ((O + eps) / (D + eps)) ** alpha
                if pen is not None:
                    r = r * torch.exp(-pen)
                Xn = self.X * r
            else:
                Xn = self.X + D
                if pen is not None:
                    Xn = Xn - pen
                Xn = torch.clamp(Xn, min=0.0)
            self.X.copy_(torch.where(done[:, None], self.X, Xn))
            if (s + 1) % self.check_interval == 0 and bool(done.all()):
                break
        Xh = (self.X[:B, : self.V].double() * norm[:B, None]).cpu().numpy()
        st = status[:B].cpu().numpy()
        it = iters[:B].cpu().numpy()
        cv = conv[:B].cpu().numpy()
        return [SolveResult(solution=Xh[f], status=int(st[f]), iterations=int(it[f]), convergence=float(cv[f]),
                            used_fused=False) for f in range(B)]

    def solve(self, measurement, solution=None) -> SolveResult:
        return self.solve_batch(np.asarray(measurement)[None])[0]
