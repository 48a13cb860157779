"""Ray-traced synthetic ray-transfer matrices with reflections (test fixtures of realistic structure).

The reference is built for production RTMs of a fusion-device camera system: dense or sparse COO matrices whose
default dataset is ``with_reflections`` (reference arguments.cpp:135-137, raytransfer.cpp:67-110), i.e. the
direct line-of-sight contribution of every pixel plus low-amplitude light reflected by the vessel wall. Such a
matrix has nothing of a uniform random one: each pixel's direct row touches only the O(n) voxels its ray
crosses (>= 90 % exact zeros), entries span many decades (corner-clipping path lengths, the 1/r^2 fall-off,
reflectivities of 1e-2 .. 1e-4 per bounce, a diffuse wall term of ~1e-9), and some pixels / voxels are seen
only through reflections (row and column sums below the solver's thresholds). The reference multiplies the raw
fp32 values with plain FMAs (sart_kernels.cu:63-110), so it assumes nothing about that range; these matrices
are what the numerics tests of every default path run on (tests/test_realistic_rtm.py,
tests/test_gpu_realistic.py).

Model (numpy, sized for tests: P x V up to a few 1e7 elements):

* voxel grid: ``nx x ny x nz`` cells of the unit cube, inside a vessel box ``[-margin, 1 + margin]^3``;
* pinhole cameras on the vessel wall looking at the cube (``field_of_view`` narrower than the cube for some of
  them, so part of the grid is seen only through reflections), ``ss x ss`` sub-rays per pixel;
* direct term: Siddon path length of each sub-ray through each voxel x ``cos^4`` of the pixel's off-axis angle
  x ``(r0 / r)^2`` (r: distance of the crossing from the pinhole, r0: to the grid centre);
* specular reflections: at the wall the ray is mirrored and continues with the face's reflectivity
  (``bounces`` times, 1e-2 .. 1e-4 each), each bounce traced through the grid again;
* diffuse term: where the primary ray hits a "rough" band of one wall face, a Lambertian spot lights every voxel
  with ``diffuse * cos / (pi d^2)`` x the voxel volume (a dense, very small block of rows).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class Camera:
    name: str
    position: tuple
    look_at: tuple
    shape: tuple            # (H, W) pixels
    field_of_view: float    # full angle across the image width, degrees
    up: tuple = (0.0, 0.0, 1.0)


def default_cameras(shape=(32, 32), n=2):
    """Two (or up to four) cameras on different walls; the second has a narrow view (part of the grid unseen)."""
    cams = [
        Camera("cam_a", (1.33, 0.35, 0.62), (0.5, 0.5, 0.5), shape, 84.0),
        Camera("cam_b", (1.30, -0.30, 0.40), (0.5, 0.5, 0.5), shape, 70.0),
        Camera("cam_c", (-0.33, 0.80, 0.55), (0.5, 0.45, 0.5), shape, 55.0, (0.0, 1.0, 1.0)),
        Camera("cam_d", (0.62, 0.55, 1.33), (0.5, 0.5, 0.5), shape, 48.0, (1.0, 0.0, 0.0)),
    ]
    return cams[:n]


def _unit(v):
    v = np.asarray(v, dtype=np.float64)
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def siddon(O, D, n, lo=0.0, hi=1.0):
    """Exact path lengths of rays O + t D (t >= 0, |D| = 1) through the cells of an n = (nx, ny, nz) grid over
    [lo, hi]^3. Returns (ray index, flat cell index i * ny * nz + j * nz + k, length, t at the segment middle)."""
    O = np.asarray(O, dtype=np.float64)
    D = np.asarray(D, dtype=np.float64)
    R = O.shape[0]
    n = np.asarray(n)
    h = (hi - lo) / n
    t_lo = np.full(R, 0.0)
    t_hi = np.full(R, np.inf)
    planes = []
    for a in range(3):
        d = D[:, a]
        nz_ = np.abs(d) > 1e-15
        p = lo + np.arange(n[a] + 1) * h[a]
        with np.errstate(divide="ignore", invalid="ignore"):
            t = (p[None, :] - O[:, a, None]) / np.where(nz_, d, 1.0)[:, None]
        t0 = np.minimum(t[:, 0], t[:, -1])
        t1 = np.maximum(t[:, 0], t[:, -1])
        inside = (O[:, a] > lo) & (O[:, a] < hi)
        t0 = np.where(nz_, t0, np.where(inside, -np.inf, np.inf))
        t1 = np.where(nz_, t1, np.where(inside, np.inf, -np.inf))
        t_lo = np.maximum(t_lo, t0)
        t_hi = np.minimum(t_hi, t1)
        planes.append(np.where(nz_[:, None], t, np.nan))
    hit = t_hi > t_lo
    T = np.concatenate(planes + [t_lo[:, None], t_hi[:, None]], axis=1)
    T = np.where(np.isnan(T), t_hi[:, None], T)
    T = np.clip(T, t_lo[:, None], np.where(hit, t_hi, t_lo)[:, None])
    T.sort(axis=1)
    with np.errstate(invalid="ignore"):  # rays that miss: infinite bounds
        seg = np.diff(T, axis=1)
        mid = 0.5 * (T[:, 1:] + T[:, :-1])
    keep = (seg > 1e-13) & np.isfinite(seg) & hit[:, None]
    ray, col = np.nonzero(keep)
    tm = mid[ray, col]
    pts = O[ray] + tm[:, None] * D[ray]
    idx = np.clip(np.floor((pts - lo) / h).astype(np.int64), 0, n - 1)
    flat = (idx[:, 0] * n[1] + idx[:, 1]) * n[2] + idx[:, 2]
    return ray, flat, seg[ray, col], tm


def _wall_hit(O, D, lo, hi):
    """First exit of rays (inside the box) through the box [lo, hi]^3: t, axis, side (0 = lo face, 1 = hi)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        t = np.where(D > 0, (hi - O) / D, np.where(D < 0, (lo - O) / D, np.inf))
    a = np.argmin(t, axis=1)
    tw = t[np.arange(len(O)), a]
    side = (D[np.arange(len(O)), a] > 0).astype(np.int64)
    return tw, a, side


def pixel_rays(cam: Camera, ss: int = 2):
    """Sub-ray origins / directions of every pixel (row-major), their pixel index and cos^4 weight / ss^2."""
    H, W = cam.shape
    fwd = _unit(np.subtract(cam.look_at, cam.position))
    right = _unit(np.cross(fwd, cam.up))
    up = np.cross(right, fwd)
    half = np.tan(np.radians(cam.field_of_view) / 2)
    u = (np.arange(W * ss) + 0.5) / (W * ss) * 2 - 1
    v = (np.arange(H * ss) + 0.5) / (H * ss) * 2 - 1
    vv, uu = np.meshgrid(v, u, indexing="ij")
    d = fwd[None, None] + half * uu[..., None] * right + half * (H / W) * (-vv)[..., None] * up
    cos = 1.0 / np.linalg.norm(d, axis=-1)
    d = d * cos[..., None]
    pix = (np.arange(H * ss)[:, None] // ss) * W + (np.arange(W * ss)[None, :] // ss)
    O = np.broadcast_to(np.asarray(cam.position, dtype=np.float64), d.shape)
    return O.reshape(-1, 3), d.reshape(-1, 3), pix.ravel(), (cos ** 4).ravel() / ss ** 2


def raytraced_rtm(grid=(16, 16, 16), cameras=None, ss=2, margin=0.35, bounces=3, reflectivity=(1e-5, 3e-3),
                  diffuse=1e-6, rough_patch=(0, 0.0, 0.5), seed=0, dtype=np.float32, keep_direct=True):
    """Dense [sum of camera pixels, nx * ny * nz] RTM in the reference's order (cameras in the given order, pixels
    row-major, voxels by flat grid index i * ny * nz + j * nz + k). Returns (A, info) with info: per-camera row
    ranges, the direct-only matrix (for the sparsity statistics; keep_direct=False: None, for large matrices) and
    the face reflectivities."""
    rng = np.random.default_rng(seed)
    cameras = cameras or default_cameras()
    n = np.asarray(grid)
    V = int(np.prod(n))
    lo_w, hi_w = -margin, 1.0 + margin
    R = np.exp(rng.uniform(np.log(reflectivity[0]), np.log(reflectivity[1]), 6))  # face 2 * axis + side
    centre = np.full(3, 0.5)
    h = 1.0 / n
    cell = np.stack(np.meshgrid(*[(np.arange(k) + 0.5) / k for k in n], indexing="ij"), -1).reshape(-1, 3)
    blocks, direct_blocks, rows = [], [], {}
    p0 = 0
    for cam in cameras:
        H, W = cam.shape
        P = H * W
        Acam = np.zeros(P * V)
        Adir = np.zeros(P * V) if keep_direct else None
        O, D, pix, wt = pixel_rays(cam, ss)
        r0 = np.linalg.norm(centre - np.asarray(cam.position))
        amp = wt.copy()
        cur_O, cur_D = O.copy(), D.copy()
        for b in range(bounces + 1):
            ray, flat, seg, tm = siddon(cur_O, cur_D, n)
            if b == 0:
                r = tm
            else:  # distance of a reflected crossing: along the unfolded path from the pinhole
                r = path_len[ray] + tm
            val = amp[ray] * seg * (r0 / np.maximum(r, 1e-3)) ** 2
            np.add.at(Acam, pix[ray] * V + flat, val)
            if b == 0 and keep_direct:
                np.add.at(Adir, pix[ray] * V + flat, val)
            if b == 0:
                path_len = np.zeros(len(cur_O))
            tw, a, side = _wall_hit(cur_O, cur_D, lo_w, hi_w)
            face = 2 * a + side
            hitp = cur_O + tw[:, None] * cur_D
            if b == 0 and diffuse > 0:  # Lambertian spots on the rough faces: a dense, tiny term
                fa, c0, c1 = rough_patch  # face, and the band c0 <= (next axis coordinate) < c1 on it
                ax2 = (a + 1) % 3
                crd = hitp[np.arange(len(hitp)), ax2]
                rough = (face == fa) & (crd >= c0) & (crd < c1)
                for i in np.nonzero(rough)[0]:
                    nin = np.zeros(3)
                    nin[a[i]] = -1.0 if side[i] else 1.0
                    dv = cell - hitp[i]
                    d2 = np.einsum("ij,ij->i", dv, dv)
                    cosw = np.maximum(dv @ nin, 0.0) / np.sqrt(d2)
                    Acam[pix[i] * V:(pix[i] + 1) * V] += amp[i] * diffuse * cosw / (np.pi * d2) * np.prod(h)
            path_len = path_len + tw
            amp = amp * R[face]
            cur_D = cur_D.copy()
            cur_D[np.arange(len(cur_D)), a] *= -1.0
            cur_O = hitp.copy()  # nudged back inside the vessel
            cur_O[np.arange(len(cur_O)), a] -= 1e-9 * (2 * side - 1)
        blocks.append(Acam.reshape(P, V).astype(dtype))
        del Acam
        if keep_direct:
            direct_blocks.append(Adir.reshape(P, V).astype(dtype))
        rows[cam.name] = (p0, p0 + P)
        p0 += P
    A = np.concatenate(blocks) if len(blocks) > 1 else blocks[0]
    del blocks
    info = dict(rows=rows, direct=np.concatenate(direct_blocks) if keep_direct else None, reflectivity=R,
                grid=tuple(grid), cameras=cameras)
    return A, info


def raytraced_direct_coo(grid=(16, 16, 16), cameras=None, ss=2):
    """The direct line-of-sight part of ``raytraced_rtm`` (the no-reflection RTM: no bounces, no diffuse band) as COO
    triplets (global pixel row, flat voxel, value fp32; one entry per (pixel, voxel), sub-rays summed) without a
    dense matrix, so it scales to 64k x 64k and beyond. Returns (rows, cols, vals, row_ranges)."""
    cameras = cameras or default_cameras()
    n = np.asarray(grid)
    V = int(np.prod(n))
    centre = np.full(3, 0.5)
    out_r, out_c, out_v, rows = [], [], [], {}
    p0 = 0
    for cam in cameras:
        H, W = cam.shape
        O, D, pix, wt = pixel_rays(cam, ss)
        r0 = np.linalg.norm(centre - np.asarray(cam.position))
        ray, flat, seg, tm = siddon(O, D, n)
        val = wt[ray] * seg * (r0 / np.maximum(tm, 1e-3)) ** 2
        key = pix[ray].astype(np.int64) * V + flat
        uk, inv = np.unique(key, return_inverse=True)
        acc = np.zeros(uk.size)
        np.add.at(acc, inv, val)
        out_r.append(uk // V + p0)
        out_c.append(uk % V)
        out_v.append(acc.astype(np.float32))
        rows[cam.name] = (p0, p0 + H * W)
        p0 += H * W
    return (np.concatenate(out_r), np.concatenate(out_c).astype(np.int32), np.concatenate(out_v), rows)


def phantom(grid=(16, 16, 16), t=0.0, seed=0):
    """Smooth emissivity: a tilted ring (torus-like shell) whose peak drifts slowly with t, on a weak background,
    plus a localized blob; values in (0, ~1.1]."""
    rng = np.random.default_rng(seed)
    n = np.asarray(grid)
    c = np.stack(np.meshgrid(*[(np.arange(k) + 0.5) / k for k in n], indexing="ij"), -1).reshape(-1, 3)
    x, y, z = c[:, 0] - 0.5, c[:, 1] - 0.5, c[:, 2] - 0.5
    R0 = 0.28 + 0.02 * np.sin(2 * np.pi * 0.05 * t)
    rr = np.sqrt(x * x + y * y)
    ring = np.exp(-((rr - R0) ** 2 + (z - 0.05 * np.sin(0.3 * t)) ** 2) / (2 * 0.07 ** 2))
    ang = np.arctan2(y, x)
    ring *= 0.75 + 0.25 * np.cos(ang - 0.2 * t)
    bc = np.array([0.15, -0.1, 0.1]) + 0.02 * rng.standard_normal(3)
    blob = 0.6 * np.exp(-np.sum((c - 0.5 - bc) ** 2, axis=1) / (2 * 0.05 ** 2))
    return 0.02 + ring + blob


def rtm_stats(A, direct=None, ray_length_threshold=1e-6, ray_density_threshold=1e-6):
    """Structure figures of an RTM (what tests/test_realistic_rtm.py pins)."""
    A = np.asarray(A, dtype=np.float64)
    nzv = np.abs(A[A != 0])
    out = dict(
        zero_fraction=float(np.mean(A == 0)),
        dynamic_range=float(nzv.max() / nzv.min()) if nzv.size else 0.0,
        rows_below=int(np.sum(A.sum(1) <= ray_length_threshold)),
        cols_below=int(np.sum(A.sum(0) <= ray_density_threshold)),
    )
    if direct is not None:
        out["direct_zero_fraction"] = float(np.mean(np.asarray(direct) == 0))
    return out
