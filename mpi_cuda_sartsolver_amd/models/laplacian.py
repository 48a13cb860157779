"""Sparse Laplacian regulariser.

The reference stores it as COO with a sorted flat index ``i * nvoxel + j`` and walks it with 64-bit
div/mod and fp32 atomics on the GPU (reference laplacian.cpp:34-91, sart_kernels.cu:179-202). The
sorted flat index is already row-major, so the row pointers follow from a bincount + scan: we keep CSR
(int64 row_ptr, int32 col, fp32 val) on the device and evaluate ``beta * L x`` with one thread per row
and no atomics.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch


class LaplacianCSR:
    def __init__(self, n: int, i, j, val, device: Optional[torch.device] = None):
        i = np.asarray(i, dtype=np.int64)
        j = np.asarray(j, dtype=np.int64)
        val = np.asarray(val, dtype=np.float32)
        if not (i.shape == j.shape == val.shape):
            raise ValueError("i, j and value arrays must have the same length")
        if i.size and (i.min() < 0 or j.min() < 0 or i.max() >= n or j.max() >= n):
            raise ValueError("Laplacian index out of range")
        flat = i * n + j
        order = np.argsort(flat, kind="stable")
        flat = flat[order]
        self.n = int(n)
        self.nnz = int(flat.size)
        rows = flat // n
        cols = (flat % n).astype(np.int32)
        row_ptr = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(np.bincount(rows, minlength=n), out=row_ptr[1:])
        self.row_ptr_host, self.col_host, self.val_host = row_ptr, cols, val[order]
        self.device = device
        if device is not None and device.type == "cuda":
            self.row_ptr = torch.from_numpy(row_ptr).to(device)
            self.col = torch.from_numpy(cols).to(device)
            self.val = torch.from_numpy(self.val_host.copy()).to(device)

    @classmethod
    def from_flat(cls, n: int, flat_index, val, device=None) -> "LaplacianCSR":
        flat = np.asarray(flat_index, dtype=np.int64)
        return cls(n, flat // n, flat % n, val, device=device)

    @classmethod
    def grid_3d(cls, nx: int, ny: int, nz: int, device=None) -> "LaplacianCSR":
        """Standard 7-point graph Laplacian on an nx*ny*nz grid (used for tests and benchmarks)."""
        n = nx * ny * nz
        idx = np.arange(n).reshape(nx, ny, nz)
        rows, cols, vals = [idx.ravel()], [idx.ravel()], []
        deg = np.zeros((nx, ny, nz), dtype=np.float32)
        for axis in range(3):
            a = np.moveaxis(idx, axis, 0)
            lo, hi = a[:-1].ravel(), a[1:].ravel()
            rows += [lo, hi]
            cols += [hi, lo]
            d = np.moveaxis(deg, axis, 0)
            d[:-1] += 1
            d[1:] += 1
        vals = [deg.ravel()] + [-np.ones(r.size, dtype=np.float32) for r in rows[1:]]
        return cls(n, np.concatenate(rows), np.concatenate(cols), np.concatenate(vals), device=device)

    def to_dense(self) -> np.ndarray:
        d = np.zeros((self.n, self.n), dtype=np.float64)
        for r in range(self.n):
            s, e = self.row_ptr_host[r], self.row_ptr_host[r + 1]
            d[r, self.col_host[s:e]] += self.val_host[s:e]
        return d

    def matvec(self, x: np.ndarray) -> np.ndarray:
        out = np.zeros(self.n, dtype=np.float64)
        rows = np.repeat(np.arange(self.n), np.diff(self.row_ptr_host))
        np.add.at(out, rows, self.val_host.astype(np.float64) * x[self.col_host])
        return out
