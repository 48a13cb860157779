"""fp64 SART oracle on the device (torch), for shards too large for the host oracle.

Same GPU semantics as :func:`models.reference.sart_gpu_semantics` (reference sartsolver_cuda.cpp:138-354,
sart_kernels.cu), fixed iteration count, evaluated in fp64 over a device-resident fp32 (or bf16) row shard.
The shard is converted to fp64 one row block at a time, so the oracle needs no fp64 copy of the matrix
(the 275 GB single-GPU shard works). With a communicator the shards of all ranks form one problem: the
voxel-length sums are all-reduced exactly as the engine does (row shards only).

Used by the production-geometry GPU tests and by ``bench.py``'s untimed self-check.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .rtm import DenseRTM


def _all_reduce(t: torch.Tensor, comm, op: str = "sum") -> torch.Tensor:
    if comm is None or comm.world_size == 1:
        return t
    if getattr(comm, "backend", "gloo") == "nccl":
        comm.all_reduce_(t, op=op)
        return t
    c = t.cpu()
    comm.all_reduce_(c, op=op)
    return c.to(t.device)


def sart_oracle_f64(rtm: DenseRTM, g, iterations: int, *, logarithmic: bool = False, comm=None,
                    ray_density_threshold: float = 1e-6, ray_length_threshold: float = 1e-6,
                    relaxation: float = 1.0, x_prev: Optional[np.ndarray] = None,
                    block_bytes: int = 1 << 30, laplacian=None, beta_laplace: float = 0.0) -> np.ndarray:
    """``iterations`` SART updates in fp64 on ``rtm`` (this rank's rows; ``g`` this rank's pixels).
    ``laplacian`` (LaplacianCSR, with ``beta_laplace``): the smoothing penalty beta L x (log mode: beta L log x,
    applied as exp(-pen)), as reference.sart_gpu_semantics. Returns the de-normalised solution (fp64, host), like
    ``SARTSolver.solve``."""
    dev = rtm.device
    P, V = rtm.npixel, rtm.nvoxel
    A = rtm.A
    rb = max(1, min(P, block_bytes // (8 * rtm.ld)))
    blocks = [(r0, min(P, r0 + rb)) for r0 in range(0, P, rb)]
    f64 = torch.float64

    def Ablk(r0, r1):
        return A[r0:r1, :V].to(f64)

    g = torch.as_tensor(np.asarray(g, dtype=np.float64), device=dev)
    gf = torch.where(torch.isfinite(g), g, torch.full_like(g, -1.0))
    mx = torch.max(gf).reshape(1) if P else torch.full((1,), -np.inf, dtype=f64, device=dev)
    norm = float(_all_reduce(mx, comm, "max").item())
    if not norm > 0:
        norm = 1.0
    gs = torch.sum(torch.where(gf > 0, gf * gf, torch.zeros_like(gf))).reshape(1)
    ghat = (gf / norm).to(torch.float32).to(f64)
    rho = torch.zeros(V, dtype=f64, device=dev)
    ell = torch.zeros(P, dtype=f64, device=dev)
    for r0, r1 in blocks:
        a = Ablk(r0, r1)
        rho += a.sum(0)
        ell[r0:r1] = a.sum(1)
    rho = _all_reduce(rho, comm).to(torch.float32)
    ell = ell.to(torch.float32)
    dvalid = rho > ray_density_threshold
    rho64 = torch.where(dvalid, rho.to(f64), torch.ones_like(rho, dtype=f64))
    ellv = ell > ray_length_threshold
    # 1 / len in fp32, as the kernels (k_prep_rows) and the host oracle compute it
    inv_len = torch.where(ellv, 1.0 / torch.where(ellv, ell, torch.ones_like(ell)), torch.zeros_like(ell)).to(f64)
    arow = torch.where(ghat >= 0, inv_len, torch.zeros_like(inv_len))

    def bwd(w):
        d = torch.zeros(V, dtype=f64, device=dev)
        for r0, r1 in blocks:
            d += Ablk(r0, r1).T @ w[r0:r1]
        return _all_reduce(d, comm)

    def sweep(x):
        # one conversion per row block: f_b = A_b x, w_b (pixel-local), acc += A_b^T w_b (the fused order)
        acc = torch.zeros(V, dtype=f64, device=dev)
        for r0, r1 in blocks:
            a = Ablk(r0, r1)
            f = a @ x
            w = arow[r0:r1] * f if logarithmic else arow[r0:r1] * (ghat[r0:r1] - f)
            acc += a.T @ w
        return _all_reduce(acc, comm)

    Lm = None
    if laplacian is not None and beta_laplace > 0 and laplacian.nnz > 0:
        Lm = torch.sparse_csr_tensor(torch.as_tensor(laplacian.row_ptr_host, dtype=torch.int64),
                                     torch.as_tensor(laplacian.col_host, dtype=torch.int64),
                                     torch.as_tensor(np.asarray(laplacian.val_host, dtype=np.float32), dtype=f64),
                                     size=(V, V)).to(dev)

    def penalty(x):
        if Lm is None:
            return None
        return beta_laplace * (Lm @ (torch.log(x) if logarithmic else x).unsqueeze(1)).squeeze(1)

    zero = torch.zeros(V, dtype=f64, device=dev)
    if x_prev is None:
        x = torch.where(dvalid, bwd(torch.clamp(ghat, min=0.0)) / rho64, zero)
    else:
        x = torch.as_tensor(np.asarray(x_prev, dtype=np.float64), device=dev) / norm
    x = torch.clamp(x, min=1e-7)
    O = torch.where(dvalid, bwd(arow * ghat), zero) if logarithmic else None
    eps = 1e-7
    for _ in range(iterations):
        pen = penalty(x)  # (from the iterate before the update, as the kernels)
        if logarithmic:
            Fv = torch.where(dvalid, sweep(x), zero)
            x = x * ((O + eps) / (Fv + eps)) ** relaxation
            if pen is not None:
                x = x * torch.exp(-pen)
        else:
            d = torch.where(dvalid, relaxation / rho64 * sweep(x), zero)
            x = torch.clamp(x + d - (pen if pen is not None else 0.0), min=0.0)
    return (x * norm).cpu().numpy()
