"""Device-resident dense ray-transfer-matrix shard.

The reference keeps the whole shard in a host ``std::vector<float>`` and copies it to the GPU with one
``cudaMemcpy`` (reference raytransfer.hpp:20, sartsolver_cuda.cpp:104-106); the host copy is never
freed. Here the shard lives only in HBM: it is filled either on the device (synthetic generator) or by
streaming row blocks from HDF5 through a pinned staging buffer (``fill_rows``), so a 275 GB shard
needs no 275 GB of host RAM.

Layout: row-major fp32 (or bf16), ``nrows_pad x ld`` with zero padding. ``ld`` is chosen so the fused
sweep can split the columns into slabs (``choose_ld``); otherwise it is a multiple of 64.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from ..ops import hip
from ..parallel.partition import round_up


@dataclass(frozen=True)
class FusedGeometry:
    K: int        # float4 per lane per row in a slab (slab width 1024*K columns)
    J: int        # column slabs
    I: int        # row groups
    grid: int     # I * J persistent workgroups (<= number of CUs)
    variant: int  # register-ring configuration (csrc/kernels/fused_sweep.hip)
    T: int        # rows per tile
    kw: int = 8   # variant 6 fp32: lane-vectors per lane per row (slab 1024 kw / T columns)
    xl: bool = True  # variant 6: XCD-local row groups (else chip-wide groups of I = CUs // J, granules via memory)


def choose_ld(nvoxel: int, max_waste: float = 0.10, storage: str = "fp32") -> int:
    """Padded row length (native ``sart::choose_ld``, csrc/engine/geometry.cpp: the single source of truth
    for the engine, both drivers and this package): the variant 6 width with the lowest estimated time per
    row, else a multiple of 8192 (variant 3), else the next multiple of 64. fp32 shards also consider slabs of
    7 / 6 KiB columns (kw 7 / 6), bf16 shards keep the 8-KiB slabs of their tiles."""
    return int(hip().choose_ld(int(nvoxel), float(max_waste), storage == "fp32"))


def fused_geometry(ld: int, num_cus: int, variant: int = 6, rows_per_tile: Optional[int] = None,
                   narrow_slabs: bool = True, chip_wide: bool = True) -> Optional[FusedGeometry]:
    """Persistent-grid geometry of the fused sweep (native ``sart::fused_geometry``).

    variant 6 (default): XCD-local row groups (L2 hand-offs); the four compute waves of a workgroup
    cover T rows x (4 / T) sub-slabs of 2048 columns, so a row is split over J = ld * T / 8192
    workgroups and each XCD runs G = (CUs per XCD) // J row groups (T = rows_per_tile or env
    SART_FUSED_T, else the T with the lowest time per row). Rows wider than an XCD's 32 slabs, and widths whose
    J leaves CUs of every XCD idle, use chip-wide row groups instead (T = 1, I = CUs // J, ``xl=False``;
    chip_wide=False excludes them). Variant 3: slabs of 1024*K columns, K chosen for <= 32 slabs (the
    fallback). None: no fused path.
    """
    g = hip().fused_geometry(int(ld), int(num_cus), int(variant), int(rows_per_tile or 0), bool(narrow_slabs),
                             bool(chip_wide))
    if not g.valid():
        return None
    return FusedGeometry(K=g.K, J=g.J, I=g.I, grid=g.grid, variant=g.variant, T=g.T, kw=g.kw, xl=g.xl)


class DenseRTM:
    """Local shard [row_offset, row_offset + npixel) x [col_offset, col_offset + nvoxel) of the RTM on one
    GPU: a row shard (col_offset 0, nvoxel = all voxels; the reference layout) or a column shard (all pixel
    rows of some voxels, ``col_offset`` / ``nvoxel_total`` set)."""

    def __init__(self, npixel: int, nvoxel: int, row_offset: int = 0, device: Optional[torch.device] = None,
                 ld: Optional[int] = None, row_align: int = 64, col_offset: int = 0,
                 nvoxel_total: Optional[int] = None, storage: str = "fp32"):
        if npixel <= 0 or nvoxel <= 0:
            raise ValueError("RTM shard must have npixel > 0 and nvoxel > 0")
        self.npixel = int(npixel)
        self.nvoxel = int(nvoxel)
        self.row_offset = int(row_offset)
        self.col_offset = int(col_offset)
        self.nvoxel_total = int(nvoxel_total) if nvoxel_total is not None else self.nvoxel
        if self.col_offset < 0 or self.col_offset + self.nvoxel > self.nvoxel_total:
            raise ValueError("column shard outside [0, nvoxel_total)")
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.ld = int(ld) if ld is not None else choose_ld(self.nvoxel, storage=storage)
        if self.ld % 64 or self.ld < self.nvoxel:
            raise ValueError("ld must be a multiple of 64 and >= nvoxel")
        self.nrows_pad = round_up(self.npixel, row_align)
        # storage precision: "fp32" (the reference's) or "bf16" (opt-in: half the HBM bytes per sweep and twice
        # the matrix per GPU; the two-pass kernels widen to fp32 in registers, sums stay fp32 / fp64)
        if storage not in ("fp32", "bf16"):
            raise ValueError("storage must be 'fp32' or 'bf16'")
        self.storage = storage
        dt = torch.bfloat16 if storage == "bf16" else torch.float32
        self.A = torch.empty((self.nrows_pad, self.ld), dtype=dt, device=self.device)

    # ------------------------------------------------------------------ construction helpers
    @property
    def nbytes(self) -> int:
        return self.nrows_pad * self.ld * self.A.element_size()

    @property
    def is_bf16(self) -> bool:
        return self.storage == "bf16"

    # rows converted per block when an fp32 source is stored as bf16 (bounds the fp32 scratch to ~256 MiB)
    def _block_rows(self) -> int:
        return max(64, min(self.nrows_pad, (256 << 20) // (4 * self.ld)))

    def _store_rows(self, local_row: int, src) -> None:
        """Store a device fp32 block [n, ld] into rows [local_row, local_row + n) (native RNE conversion for bf16)."""
        n = src.shape[0]
        if not self.is_bf16:
            self.A[local_row: local_row + n].copy_(src)
            return
        src = src.contiguous()
        hip().f32_to_bf16(src.data_ptr(), n * self.ld, self.A[local_row].data_ptr(), self.stream_handle)

    @property
    def stream_handle(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def zero_padding(self) -> None:
        if self.ld > self.nvoxel:
            self.A[:, self.nvoxel:].zero_()
        if self.nrows_pad > self.npixel:
            self.A[self.npixel:].zero_()

    @property
    def is_column_shard(self) -> bool:
        return self.nvoxel < self.nvoxel_total

    @classmethod
    def synthetic(cls, npixel: int, nvoxel: int, row_offset: int = 0, seed: int = 1234, lo: float = 0.0,
                  hi: float = 1.0, device=None, ld=None, col_offset: int = 0,
                  nvoxel_total: Optional[int] = None, storage: str = "fp32") -> "DenseRTM":
        """On-device random dense RTM; element (p, v) depends only on (seed, global p, global v), so row and
        column shards of one global matrix agree bit for bit."""
        m = cls(npixel, nvoxel, row_offset, device=device, ld=ld, col_offset=col_offset, nvoxel_total=nvoxel_total,
                storage=storage)
        if not m.is_bf16:
            hip().synth_matrix(m.A.data_ptr(), m.ld, m.nrows_pad, m.npixel, m.nvoxel, m.row_offset, int(seed),
                               float(lo), float(hi), m.stream_handle, m.col_offset, m.nvoxel_total)
            return m
        # bf16: generate fp32 row blocks of the same global matrix and round them into the shard
        nb = m._block_rows()
        scratch = torch.empty((nb, m.ld), dtype=torch.float32, device=m.device)
        for r0 in range(0, m.nrows_pad, nb):
            n = min(nb, m.nrows_pad - r0)
            valid = max(0, min(n, m.npixel - r0))
            hip().synth_matrix(scratch.data_ptr(), m.ld, n, valid, m.nvoxel, m.row_offset + r0, int(seed),
                               float(lo), float(hi), m.stream_handle, m.col_offset, m.nvoxel_total)
            m._store_rows(r0, scratch[:n])
        torch.cuda.synchronize(m.device)
        return m

    @classmethod
    def from_dense(cls, A_local, row_offset: int = 0, device=None, ld=None, col_offset: int = 0,
                   nvoxel_total: Optional[int] = None, storage: str = "fp32") -> "DenseRTM":
        """Upload a host (numpy / torch) dense block [npixel, nvoxel]."""
        t = torch.as_tensor(A_local, dtype=torch.float32)
        m = cls(t.shape[0], t.shape[1], row_offset, device=device, ld=ld, col_offset=col_offset,
                nvoxel_total=nvoxel_total, storage=storage)
        m.A.zero_()
        m.fill_rows(0, t)
        return m

    def fill_rows(self, local_row: int, block) -> None:
        """Copy a host block of rows [local_row, local_row + len(block)) x [0, nvoxel) into HBM."""
        t = torch.as_tensor(block, dtype=torch.float32)
        n = t.shape[0]
        if not self.is_bf16:
            self.A[local_row: local_row + n, : self.nvoxel].copy_(t, non_blocking=t.is_pinned())
            return
        nb = self._block_rows()
        for r0 in range(0, n, nb):
            k = min(nb, n - r0)
            scratch = torch.zeros((k, self.ld), dtype=torch.float32, device=self.device)
            scratch[:, : self.nvoxel].copy_(t[r0: r0 + k])
            self._store_rows(local_row + r0, scratch)
        torch.cuda.synchronize(self.device)

    def to_bf16(self) -> "DenseRTM":
        """bf16-stored copy of this shard (same geometry), rounded to nearest even by the native kernel."""
        # row_align = nrows_pad reproduces this shard's padded row count
        m = DenseRTM(self.npixel, self.nvoxel, self.row_offset, device=self.device, ld=self.ld,
                     row_align=self.nrows_pad, col_offset=self.col_offset, nvoxel_total=self.nvoxel_total,
                     storage="bf16")
        src = self.A if not self.is_bf16 else self.A.float()
        nb = m._block_rows()
        for r0 in range(0, self.nrows_pad, nb):
            m._store_rows(r0, src[r0: r0 + nb])
        torch.cuda.synchronize(self.device)
        return m

    def to_host(self):
        return self.A[: self.npixel, : self.nvoxel].float().cpu().numpy()


class SparseRTM:
    """Device-resident sparse row shard [row_offset, row_offset + npixel) x nvoxel of the RTM: CSR (forward
    projection, row sums) and CSC (back-projection, column sums) copies of the non-zeros, fp32 values
    (csrc/kernels/sparse.hip). The reference scatters a sparse COO RTM into its dense shard
    (raytransfer.cpp:67-91); a no-reflection RTM of a few MB then streams as many bytes per iteration as a dense
    one. ``SARTSolver`` runs the two-pass sweep on these kernels (the fused sweep is dense-only)."""

    is_bf16 = False
    is_column_shard = False

    def __init__(self, npixel: int, nvoxel: int, row_ptr, col, val, row_offset: int = 0,
                 device: Optional[torch.device] = None):
        import numpy as np

        from ..ops import native

        if npixel <= 0 or nvoxel <= 0:
            raise ValueError("RTM shard must have npixel > 0 and nvoxel > 0")
        self.npixel, self.nvoxel, self.row_offset = int(npixel), int(nvoxel), int(row_offset)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
        ci = np.ascontiguousarray(col, dtype=np.int32)
        vv = np.ascontiguousarray(val, dtype=np.float32)
        if rp.size != self.npixel + 1 or rp[-1] != vv.size or ci.size != vv.size:
            raise ValueError("inconsistent CSR arrays")
        cp, ri, cv = native().csr_transpose(self.npixel, self.nvoxel, rp, ci, vv)
        self.nnz = int(vv.size)
        self.nrows_pad = round_up(self.npixel, 64)
        self.ld = round_up(self.nvoxel, 64)

        def dev(a):  # at least one element: a zero-size tensor has no stable data pointer
            t = torch.from_numpy(a if a.size else np.zeros(1, dtype=a.dtype))
            return t.to(self.device)

        self.row_ptr, self.col, self.val = dev(rp), dev(ci), dev(vv)
        self.col_ptr, self.row, self.cval = dev(cp), dev(ri), dev(cv)

    @property
    def density(self) -> float:
        return self.nnz / float(self.npixel * self.nvoxel)

    @property
    def nbytes(self) -> int:
        return 2 * self.nnz * 8 + (self.npixel + self.nvoxel + 2) * 8

    def pointers(self):
        return (self.row_ptr.data_ptr(), self.col.data_ptr(), self.val.data_ptr(), self.col_ptr.data_ptr(),
                self.row.data_ptr(), self.cval.data_ptr())

    @classmethod
    def from_entries(cls, npixel: int, nvoxel: int, rows, cols, vals, row_offset: int = 0, device=None):
        """From (local row, column, value) entries in any order (a later duplicate wins, zeros are dropped)."""
        import numpy as np

        from ..ops import native

        rp, ci, vv = native().csr_from_entries(int(npixel), int(nvoxel), np.asarray(rows, dtype=np.int64),
                                               np.asarray(cols, dtype=np.int32), np.asarray(vals, dtype=np.float32))
        return cls(npixel, nvoxel, rp, ci, vv, row_offset=row_offset, device=device)

    @classmethod
    def from_dense(cls, A_local, row_offset: int = 0, device=None):
        """The non-zeros of a dense host matrix (numpy, fp32 values)."""
        import numpy as np

        A = np.asarray(A_local, dtype=np.float32)
        r, c = np.nonzero(A)
        return cls.from_entries(A.shape[0], A.shape[1], r, c, A[r, c], row_offset=row_offset, device=device)
