"""Synthetic input cases in the reference HDF5 schema (written by the native module; h5py is absent).

``make_case`` builds a complete multi-camera problem: per camera one or more RTM segment files (dense
or sparse COO), a frame mask, a voxel map, an image time series generated from a known phantom with
``g = A x_true`` (optionally with saturated pixels), and optionally a Laplacian file. The returned
dictionary holds the global dense matrix and phantoms so tests can compare the solver output.

``raytraced=True`` takes the matrix from the ray-traced camera model with wall reflections
(utils/raytrace.py: Siddon path lengths, 1/r^2, specular bounces and a diffuse wall term; >= 90 % zeros in
the direct part, values over > 1e8) on every voxel of ``grid``, and a slowly varying ring phantom per frame.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

from ..ops import native


@dataclass
class Case:
    files: list
    rtm_files: list
    image_files: list
    laplacian_file: str | None
    A: np.ndarray               # global dense RTM in solver order (cameras by name, masked pixels)
    times: dict                 # camera -> frame times
    frames: dict                # camera -> [T, H, W]
    phantoms: np.ndarray        # [T, nvoxel]
    npixel: int
    nvoxel: int
    grid: tuple
    masks: dict = field(default_factory=dict)


def _grid_voxels(nx, ny, nz, nvoxel, rng):
    flat = np.sort(rng.choice(nx * ny * nz, size=nvoxel, replace=False))
    return flat // (ny * nz), (flat // nz) % ny, flat % nz


def make_case(directory: str, cameras=("cam_a", "cam_b"), shapes=((6, 8), (5, 7)), nvoxel=48, grid=(4, 4, 4),
              segments=2, sparse_cameras=(), nframes=4, dt=0.1, time_offsets=None, saturate=0.0,
              laplacian=False, wavelength=656.3, rtm_name="with_reflections", seed=0, coordinate_system="",
              bounds=(), raytraced=False, mask_fraction=0.2, direct_only=False) -> Case:
    os.makedirs(directory, exist_ok=True)
    n = native()
    rng = np.random.default_rng(seed)
    nx, ny, nz = grid
    traced = None
    if raytraced:
        from ..utils.raytrace import Camera, default_cameras, phantom, raytraced_rtm

        nvoxel = nx * ny * nz
        flat = np.arange(nvoxel)
        vi, vj, vk = flat // (ny * nz), (flat // nz) % ny, flat % nz
        base = default_cameras(n=4)
        cams = [Camera(cam, b.position, b.look_at, tuple(sh), b.field_of_view, b.up)
                for cam, sh, b in zip(cameras, shapes, base)]
        A_all, info = raytraced_rtm(grid=grid, cameras=cams, seed=seed)
        if direct_only:  # the no-reflection matrix: the direct line-of-sight part only (~1 % non-zeros)
            A_all = np.asarray(info["direct"], dtype=np.float32)
        traced = {cam: A_all[r0:r1] for cam, (r0, r1) in info["rows"].items()}
        phantoms = np.stack([phantom(grid, t=float(k), seed=seed) for k in range(nframes)])
    else:
        vi, vj, vk = _grid_voxels(nx, ny, nz, nvoxel, rng)
        phantoms = rng.random((nframes, nvoxel)) + 0.1
    seg_edges = np.linspace(0, nvoxel, segments + 1).astype(int)
    time_offsets = time_offsets or [0.0] * len(cameras)
    blocks, files, rtm_files, image_files, masks = [], [], [], [], {}
    times, frames = {}, {}
    for c, (cam, (h, w)) in enumerate(zip(cameras, shapes)):
        mask = (rng.random((h, w)) > mask_fraction).astype(np.uint8)
        mask[0, 0] = 1
        npix = int(mask.sum())
        if traced is not None:
            A_cam = np.ascontiguousarray(traced[cam][mask.ravel() > 0])
        else:
            A_cam = rng.random((npix, nvoxel)).astype(np.float32)
            A_cam[A_cam < 0.3] = 0.0  # some structural zeros
        masks[cam] = mask
        for s in range(segments):
            v0, v1 = seg_edges[s], seg_edges[s + 1]
            path = os.path.join(directory, f"rtm_{cam}_seg{s}.h5")
            kw = dict(path=path, camera_name=cam, wavelength=wavelength, npixel=npix, nvoxel=int(v1 - v0),
                      frame_mask=mask, vi=vi[v0:v1].astype(np.uint64), vj=vj[v0:v1].astype(np.uint64),
                      vk=vk[v0:v1].astype(np.uint64), vvalue=np.arange(v1 - v0, dtype=np.int32), nx=nx, ny=ny,
                      nz=nz, rtm_name=rtm_name, coordinate_system=coordinate_system, bounds=list(bounds))
            block = A_cam[:, v0:v1]
            if cam in sparse_cameras:
                p, v = np.nonzero(block)
                n.write_rtm_file(pixel_index=p.astype(np.uint64), voxel_index=v.astype(np.uint64),
                                 value=block[p, v].astype(np.float32), **kw)
            else:
                n.write_rtm_file(dense=np.ascontiguousarray(block), **kw)
            rtm_files.append(path)
        blocks.append(A_cam)
        # images: frame t = A_cam x_t scattered into the masked pixels, zero elsewhere
        t = time_offsets[c] + dt * np.arange(nframes)
        fr = np.zeros((nframes, h, w))
        for k in range(nframes):
            g = A_cam.astype(np.float64) @ phantoms[k]
            if saturate > 0:
                g[rng.random(npix) < saturate] = -1.0
            img = np.zeros(h * w)
            img[mask.ravel() > 0] = g
            fr[k] = img.reshape(h, w)
        ipath = os.path.join(directory, f"image_{cam}.h5")
        n.write_image_file(ipath, cam, wavelength + 1.0, t, fr)
        image_files.append(ipath)
        times[cam], frames[cam] = t, fr
    order = np.argsort(cameras)
    A = np.concatenate([blocks[o] for o in order], axis=0)
    lap = None
    if laplacian:
        from ..models.laplacian import LaplacianCSR

        # chain Laplacian over the voxel order; the 3-D grid Laplacian for ray-traced cases (every voxel present)
        L = LaplacianCSR.grid_3d(nx, ny, nz) if raytraced else LaplacianCSR.grid_3d(1, 1, nvoxel)
        rows = np.repeat(np.arange(nvoxel), np.diff(L.row_ptr_host))
        lap = os.path.join(directory, "laplacian.h5")
        n.write_laplacian_file(lap, nvoxel, rows.astype(np.uint64), L.col_host.astype(np.uint64), L.val_host)
    files = rtm_files + image_files
    return Case(files=files, rtm_files=rtm_files, image_files=image_files, laplacian_file=lap, A=A, times=times,
                frames=frames, phantoms=phantoms, npixel=A.shape[0], nvoxel=nvoxel, grid=grid, masks=masks)
