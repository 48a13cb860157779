"""HDF5 inputs and outputs (native C++ module, HDF5 C API).

Mirrors the reference driver's start-up sequence (reference main.cpp:27-59): classify the input
files, check attribute consistency, sort RTM segments per camera, validate frame masks / voxel maps /
RTM-image pairing and compute the total (npixel, nvoxel). Loading differs by design:

* the RTM row shard is streamed from HDF5 in row blocks through two pinned host buffers straight into
  HBM (``load_rtm_shard``); the reference keeps the full shard in host RAM for the whole run and reads
  one row per HDF5 call (reference raytransfer.cpp:92-110, sartsolver_cuda.cpp:104-106);
* the Laplacian becomes a device CSR matrix (reference keeps COO, laplacian.cpp:34-91).
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from ..ops import native


@dataclass
class InputSet:
    rtm_files: dict            # camera -> [segment files] (voxel order)
    image_files: dict          # camera -> image file
    camera_names: list
    npixel: int
    nvoxel: int
    frame_masks: dict          # camera -> int32 mask (flattened, row-major)
    rtm_name: str
    has_sparse: bool = False
    extra: dict = field(default_factory=dict)


def validate_inputs(input_files, rtm_name: str = "with_reflections", wavelength_threshold: float = 50.0) -> InputSet:
    """Same checks, in the same order, as the reference (main.cpp:32-59)."""
    n = native()
    rtm, img = n.categorize_input_files(list(input_files))
    if not rtm:
        raise RuntimeError("No RTM files given.")
    if not img:
        raise RuntimeError("No image files given.")
    n.check_group_attribute_consistency(rtm, "rtm/" + rtm_name, ["wavelength"], False)
    n.check_group_attribute_consistency(rtm, "rtm/voxel_map", ["nx", "ny", "nz"], True)
    sorted_rtm = n.sort_rtm_files(rtm)
    n.check_rtm_frame_consistency(sorted_rtm)
    n.check_rtm_voxel_consistency(sorted_rtm)
    n.check_group_attribute_consistency(img, "image", ["wavelength"], False)
    sorted_img = n.sort_image_files(img)
    n.check_rtm_image_consistency(sorted_rtm, sorted_img, rtm_name, wavelength_threshold)
    npixel, nvoxel = n.get_total_rtm_size(sorted_rtm)
    masks = n.read_rtm_frame_masks(sorted_rtm)
    return InputSet(rtm_files=dict(sorted_rtm), image_files=dict(sorted_img), camera_names=list(sorted_img.keys()),
                    npixel=int(npixel), nvoxel=int(nvoxel), frame_masks=dict(masks), rtm_name=rtm_name,
                    has_sparse=bool(n.rtm_has_sparse(sorted_rtm, rtm_name)))


def read_rtm_rows(inputs: InputSet, row_begin: int, row_end: int, ld: Optional[int] = None, col_begin: int = 0,
                  col_end: Optional[int] = None) -> np.ndarray:
    """Host copy of global RTM rows [row_begin, row_end) x columns [col_begin, col_end) (tests, CPU path)."""
    col_end = inputs.nvoxel if col_end is None else int(col_end)
    ld = ld or (col_end - col_begin)
    out = np.zeros((row_end - row_begin, ld), dtype=np.float32)
    native().RtmReader(inputs.rtm_files, inputs.rtm_name, inputs.nvoxel, col_begin, col_end).read(row_begin, row_end,
                                                                                                  out)
    return out


def rtm_sparse_density(inputs: InputSet) -> float:
    """Stored entries / (npixel x nvoxel) when every RTM dataset is sparse COO, else -1 (the driver's
    ``--rtm_format auto`` test)."""
    return float(native().rtm_sparse_density(inputs.rtm_files, inputs.rtm_name, inputs.npixel, inputs.nvoxel))


def load_rtm_shard_sparse(inputs: InputSet, row_offset: int, npixel_local: int, device):
    """This rank's RTM rows as a device-resident ``SparseRTM`` (CSR + CSC of the non-zeros; COO datasets are read
    directly, dense ones through row blocks): the ``--rtm_format sparse`` shard of the native driver."""
    from ..models.rtm import SparseRTM

    reader = native().RtmReader(inputs.rtm_files, inputs.rtm_name, inputs.nvoxel)
    rp, col, val = reader.read_csr(row_offset, row_offset + npixel_local)
    return SparseRTM(npixel_local, inputs.nvoxel, rp, col, val, row_offset=row_offset, device=device)


def load_rtm_shard(inputs: InputSet, row_offset: int, npixel_local: int, device, ld: Optional[int] = None,
                   block_bytes: int = 256 << 20, col_offset: int = 0, ncols: Optional[int] = None,
                   storage: str = "fp32"):
    """Stream this rank's RTM rows into a device-resident ``DenseRTM``; with ``col_offset`` / ``ncols`` only
    that voxel block of every row is read (column hyperslabs: a column shard reads 1/N of the file).

    Two pinned host buffers alternate: while block k is copied host->HBM (async on the current stream),
    block k+1 is read from HDF5 by a helper thread (the native reader releases the GIL; sparse segments are
    read once per shard). Peak host memory is 2 * block_bytes regardless of the shard size. ``storage``
    "bf16": each block is rounded into the bf16 shard on the device through an fp32 staging block, so peak
    HBM is the bf16 shard plus one block (never the fp32 shard).
    """
    import torch

    from ..models.rtm import DenseRTM

    n = native()
    V = inputs.nvoxel
    nc = V - col_offset if ncols is None else int(ncols)
    reader = n.RtmReader(inputs.rtm_files, inputs.rtm_name, V, col_offset, col_offset + nc)
    rtm = DenseRTM(npixel_local, nc, row_offset, device=device, ld=ld, col_offset=col_offset, nvoxel_total=V,
                   storage=storage)
    rtm.A.zero_()
    rows_per_block = max(1, min(npixel_local, block_bytes // (4 * nc)))
    bufs = [torch.empty((rows_per_block, nc), dtype=torch.float32).pin_memory() for _ in range(2)]
    stage = (torch.zeros((rows_per_block, rtm.ld), dtype=torch.float32, device=device) if rtm.is_bf16 else None)
    events = [None, None]
    stream = torch.cuda.current_stream(device)

    def read_into(buf, r0, r1):
        buf[: r1 - r0].zero_()
        reader.read_ptr(row_offset + r0, row_offset + r1, buf.data_ptr(), nc)

    blocks = [(r, min(npixel_local, r + rows_per_block)) for r in range(0, npixel_local, rows_per_block)]
    if not blocks:
        return rtm
    read_into(bufs[0], *blocks[0])
    for k, (r0, r1) in enumerate(blocks):
        cur = bufs[k % 2]
        reader_thread = None
        if k + 1 < len(blocks):
            nxt = bufs[(k + 1) % 2]
            if events[(k + 1) % 2] is not None:
                events[(k + 1) % 2].synchronize()  # the copy that last used this buffer is done
            reader_thread = threading.Thread(target=read_into, args=(nxt, *blocks[k + 1]))
            reader_thread.start()
        if stage is None:
            rtm.A[r0:r1, :nc].copy_(cur[: r1 - r0], non_blocking=True)
        else:  # stream-ordered: the next block's copy into the staging rows waits for this conversion
            stage[: r1 - r0, :nc].copy_(cur[: r1 - r0], non_blocking=True)
            rtm._store_rows(r0, stage[: r1 - r0])
        ev = torch.cuda.Event()
        ev.record(stream)
        events[k % 2] = ev
        if reader_thread is not None:
            reader_thread.join()
    torch.cuda.synchronize(device)
    return rtm


def load_laplacian(path: str, nvoxel: int, device=None):
    from ..models.laplacian import LaplacianCSR

    i, j, v = native().read_laplacian(path, nvoxel)
    return LaplacianCSR(nvoxel, i, j, v, device=device)


def open_composite_image(inputs: InputSet, time_intervals, npixel_local: int, offset_pixel: int,
                         max_cache_size: int = 100):
    ci = native().CompositeImage(inputs.image_files, inputs.frame_masks, time_intervals, npixel_local, offset_pixel)
    ci.max_cache_size = max_cache_size
    return ci


def read_voxel_grid(inputs: InputSet):
    """Voxel map of the first camera's segments (reference main.cpp:115-125)."""
    g = native().VoxelGrid()
    first = next(iter(inputs.rtm_files.values()))
    g.read(list(first), "rtm/voxel_map")
    return g
