"""fp64 numpy oracles of the two SART semantics of the reference, used by the tests.

* :func:`sart_gpu_semantics` -- the reference GPU path (normalisation by max(g), fp32 thresholds,
  eps = 1e-7 clamp, reference sartsolver_cuda.cpp:138-354 + sart_kernels.cu), evaluated in fp64.
* :func:`sart_cpu_semantics` -- the reference ``--use_cpu`` path (sartsolver.cpp:133-339): no
  normalisation, the cold start uses the raw measurement including negative pixels, no clamp in the
  linear variant, 1e-100 clamp / epsilon in the logarithmic one.

* :func:`sart_fp32_emulation` -- the GPU semantics evaluated in fp32 with numpy/BLAS sums, or in the reference
  kernels' own summation order (``order="reference"``): what an fp32 solver such as the reference's (cuBLAS Sgemv
  + fp32 atomics) produces. Its distance to the fp64 oracle is the inherent fp32 error of a problem; tests bound
  ours by it (tests/test_gpu_realistic.py: the larger of the two orders' errors).

All return (solution fp64, status, iterations) where iterations counts the updates applied.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

SUCCESS, MAX_ITERATIONS_EXCEEDED = 0, -1


def _penalty(L, x, beta, logx):
    if L is None or getattr(L, "nnz", 0) == 0 or beta == 0:
        return np.zeros_like(x)
    return beta * L.matvec(np.log(x) if logx else x)


def sart_gpu_semantics(A, g, L=None, *, logarithmic=False, ray_density_threshold=1e-6, ray_length_threshold=1e-6,
                       conv_tolerance=1e-5, beta_laplace=1e-2, relaxation=1.0, max_iterations=2000,
                       x_prev: Optional[np.ndarray] = None):
    A = np.asarray(A, dtype=np.float32).astype(np.float64)
    g = np.asarray(g, dtype=np.float64)
    norm = g.max()
    if not norm > 0:
        norm = 1.0
    ghat = (g / norm).astype(np.float32).astype(np.float64)
    G = np.sum(np.where(g > 0, g * g, 0.0)) / norm ** 2
    rho = A.sum(axis=0).astype(np.float32)
    ell = A.sum(axis=1).astype(np.float32)
    dvalid = rho > np.float32(ray_density_threshold)
    rho64 = np.where(dvalid, rho.astype(np.float64), 1.0)
    inv_len = np.where(ell > np.float32(ray_length_threshold), 1.0 / np.where(ell > 0, ell, 1.0), 0.0)
    a = np.where(ghat >= 0, inv_len, 0.0)
    if x_prev is None:
        x = np.where(dvalid, A.T @ np.maximum(ghat, 0.0) / rho64, 0.0)
    else:
        x = np.asarray(x_prev, dtype=np.float64) / norm
    x = np.maximum(x, 1e-7)
    eps = 1e-7
    O = np.where(dvalid, A.T @ (a * ghat), 0.0) if logarithmic else None
    f = A @ x
    conv_prev = 0.0
    for it in range(max_iterations):
        if logarithmic:
            pen = _penalty(L, x, beta_laplace, True)
            Fv = np.where(dvalid, A.T @ (a * f), 0.0)
            x = x * ((O + eps) / (Fv + eps)) ** relaxation * np.exp(-pen)
        else:
            pen = _penalty(L, x, beta_laplace, False)
            d = np.where(dvalid, relaxation / rho64 * (A.T @ (a * (ghat - f))), 0.0)
            x = np.maximum(x + d - pen, 0.0)
        f = A @ x
        conv = (G - f @ f) / G
        if it and abs(conv - conv_prev) < conv_tolerance:
            return x * norm, SUCCESS, it + 1
        conv_prev = conv
    return x * norm, MAX_ITERATIONS_EXCEEDED, max_iterations


def sart_cpu_semantics(A, g, L=None, *, logarithmic=False, ray_density_threshold=1e-6, ray_length_threshold=1e-6,
                       conv_tolerance=1e-5, beta_laplace=1e-2, relaxation=1.0, max_iterations=2000,
                       x_prev: Optional[np.ndarray] = None):
    A = np.asarray(A, dtype=np.float32).astype(np.float64)
    g = np.asarray(g, dtype=np.float64)
    rho = A.sum(axis=0)
    ell = A.sum(axis=1)
    dvalid = rho > ray_density_threshold
    rho_s = np.where(dvalid, rho, 1.0)
    pvalid = (ell > ray_length_threshold) & (g >= 0)
    a = np.where(pvalid, 1.0 / np.where(ell != 0, ell, 1.0), 0.0)
    if x_prev is None:
        x = np.where(dvalid, (A.T @ g) / rho_s, 0.0)
    else:
        x = np.asarray(x_prev, dtype=np.float64).copy()
    eps = 1e-100
    if logarithmic:
        x = np.maximum(x, eps)
    G = np.sum(np.where(g > 0, g * g, 0.0))
    f = A @ x
    conv_prev = 0.0
    O = np.where(dvalid, A.T @ (a * g), 0.0) if logarithmic else None
    for it in range(max_iterations):
        if logarithmic:
            pen = _penalty(L, x, beta_laplace, True)
            Fv = np.where(dvalid, A.T @ (a * f), 0.0)
            x = x * ((O + eps) / (Fv + eps)) ** relaxation * np.exp(-pen)
        else:
            pen = _penalty(L, x, beta_laplace, False)
            d = np.where(dvalid, relaxation / rho_s * (A.T @ (a * (g - f))), 0.0) - pen
            x = x + d
            x = np.where(np.signbit(x), 0.0, x)
        f = A @ x
        conv = (G - f @ f) / G
        if it and abs(conv - conv_prev) < conv_tolerance:
            return x, SUCCESS, it + 1
        conv_prev = conv
    return x, MAX_ITERATIONS_EXCEEDED, max_iterations


def _serial_tiles(KN, v, tile=256):
    """fp32 sum_k KN[k, :] v[k] in the reference kernels' order: each output sums its terms serially in fp32
    within tiles of ``tile`` consecutive k (one CUDA thread's loop, sart_kernels.cu:86-104), and the tile partials
    are added in turn (the atomicAdd of each block, :107)."""
    f32 = np.float32
    v = np.asarray(v, dtype=f32)
    out = np.zeros(KN.shape[1], dtype=f32)
    for k0 in range(0, KN.shape[0], tile):
        acc = np.zeros(KN.shape[1], dtype=f32)
        for k in range(k0, min(k0 + tile, KN.shape[0])):
            acc += KN[k] * v[k]
        out += acc
    return out


def sart_fp32_emulation(A, g, L=None, *, logarithmic=False, ray_density_threshold=1e-6, ray_length_threshold=1e-6,
                        beta_laplace=1e-2, relaxation=1.0, max_iterations=10, x_prev: Optional[np.ndarray] = None,
                        order: str = "blas"):
    """Fixed-iteration GPU semantics with fp32 vectors and fp32 matrix products (no convergence test).

    order "blas": numpy/BLAS fp32 products (blocked / pairwise sums); "reference": every product summed in the
    reference CUDA kernels' order (serial fp32 sums over tiles of 256 terms, tile partials added in turn;
    ``_serial_tiles``), the accumulation pattern of the reference's own fp32 GPU solver. The two bracket what an
    fp32 evaluation of the algorithm gives; the tests bound ours by the larger of their errors."""
    f32 = np.float32
    A32 = np.asarray(A, dtype=f32)
    if order == "reference":
        A32T = np.ascontiguousarray(A32.T)

        class _Op:  # M @ v in the reference kernels' order (KN: M transposed, rows = the summed index)
            def __init__(self, KN):
                self.KN = KN

            def __matmul__(self, v):
                return _serial_tiles(self.KN, v)

        Aop, ATop = _Op(A32T), _Op(A32)
    elif order == "blas":
        Aop, ATop = A32, A32.T
    else:
        raise ValueError(f"unknown summation order {order!r}")
    g = np.asarray(g, dtype=np.float64)
    norm = g.max()
    if not norm > 0:
        norm = 1.0
    ghat = (g / norm).astype(f32)
    rho = A32.astype(np.float64).sum(axis=0).astype(f32)
    ell = A32.astype(np.float64).sum(axis=1).astype(f32)
    dvalid = rho > f32(ray_density_threshold)
    rho_s = np.where(dvalid, rho, f32(1))
    inv_len = np.where(ell > f32(ray_length_threshold), f32(1) / np.where(ell > 0, ell, f32(1)), f32(0)).astype(f32)
    a = np.where(ghat >= 0, inv_len, f32(0)).astype(f32)
    scale = np.where(dvalid, f32(relaxation) / rho_s, f32(0)).astype(f32)
    if x_prev is None:
        x = np.where(dvalid, (ATop @ np.maximum(ghat, f32(0))) / rho_s, f32(0)).astype(f32)
    else:
        x = (np.asarray(x_prev, dtype=np.float64) / norm).astype(f32)
    x = np.maximum(x, f32(1e-7))
    eps = f32(1e-7)
    O = np.where(dvalid, ATop @ (a * ghat), f32(0)).astype(f32) if logarithmic else None
    for _ in range(max_iterations):
        f = (Aop @ x).astype(f32)
        if logarithmic:
            pen = _penalty(L, x.astype(np.float64), beta_laplace, True).astype(f32)
            Fv = np.where(dvalid, ATop @ (a * f), f32(0)).astype(f32)
            x = (x * ((O + eps) / (Fv + eps)) ** f32(relaxation) * np.exp(-pen)).astype(f32)
        else:
            pen = _penalty(L, x.astype(np.float64), beta_laplace, False).astype(f32)
            d = (scale * (ATop @ (a * (ghat - f)))).astype(f32)
            x = np.maximum(x + d - pen, f32(0)).astype(f32)
    return x.astype(np.float64) * norm, MAX_ITERATIONS_EXCEEDED, max_iterations
