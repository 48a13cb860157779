#!/usr/bin/env python3
"""Sparse RTM path against the dense one on the same ray-traced no-reflection RTM (the reference's "sparse" dataset,
manual.pdf p.3: a few MB instead of tens of GB) at 64k x 64k: two 128 x 256 cameras looking into a 32 x 32 x 64
voxel grid (utils/raytrace.py: Siddon path lengths, cos^4, 1/r^2; built as COO without a dense array).

Runs SARTSolver on a SparseRTM (CSR + CSC kernels, csrc/kernels/sparse.hip) and on the DenseRTM of the same
non-zeros (fused sweep and two-pass kernels), 100 SART iterations per cold-start frame solve (bench.py's unit),
and reports SART it/s, the bytes each path streams per iteration and the agreement of the solutions. One JSON line
per path.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", default="32,32,64")
    ap.add_argument("--shape", default="128,256", help="pixels per camera (H,W); two cameras")
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--no-dense", action="store_true")
    ap.add_argument("--random-density", type=float, default=0.0,
                    help="instead of the ray-traced matrix: uniform random positions at this density, --shape rows x "
                         "--grid voxels (the break-even density of the sparse path against the dense fused sweep)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--frames", default="", help="comma list of multi-frame batch widths to time as well (SpMM)")
    a = ap.parse_args()
    import torch

    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM, SparseRTM
    from mpi_cuda_sartsolver_amd.models.sart import SARTSolver, SolverParams
    from mpi_cuda_sartsolver_amd.utils.raytrace import Camera, default_cameras, phantom, raytraced_direct_coo

    grid = tuple(int(x) for x in a.grid.split(","))
    H, W = (int(x) for x in a.shape.split(","))
    dev = torch.device("cuda", 0)
    t0 = time.perf_counter()
    cams = [Camera(f"cam_{i}", b.position, b.look_at, (H, W), b.field_of_view, b.up)
            for i, b in enumerate(default_cameras(n=2))]
    P, V = 2 * H * W, int(np.prod(grid))
    if a.random_density > 0:
        rng = np.random.default_rng(7)
        nnz = int(a.random_density * P * V)
        flat = np.unique(rng.integers(0, P * V, size=nnz, dtype=np.int64))
        r, c = flat // V, (flat % V).astype(np.int32)
        v = rng.random(flat.size, dtype=np.float32) + 0.01
    else:
        r, c, v, _ = raytraced_direct_coo(grid=grid, cameras=cams)
    sp = SparseRTM.from_entries(P, V, r, c, v, device=dev)
    build_s = time.perf_counter() - t0
    x_true = phantom(grid, t=1.0) if a.random_density <= 0 else np.random.default_rng(1).random(V) + 0.1
    p = SolverParams(max_iterations=a.iters, conv_tolerance=0.0)
    lines = []

    def run(name, solver, g):
        solver.solve(g)  # warm-up
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.steps):
            res = solver.solve(g)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.steps
        rec = dict(path=name, P=P, V=V, nnz=sp.nnz, density=round(sp.density, 6), iters=a.iters,
                   ms_per_solve=round(1e3 * dt, 3), iters_per_s=round(a.iters / dt, 1),
                   used_fused=bool(res.used_fused),
                   rtm=("uniform random positions" if a.random_density > 0 else "ray-traced direct (no reflections)"),
                   grid=list(grid))
        lines.append(rec)
        print(json.dumps(rec), flush=True)
        return res.solution

    s_sp = SARTSolver(sp, None, None, p, allow_zero_tolerance=True)
    g = s_sp.forward_project(x_true)  # f = A x_true on the GPU (the sparse forward)
    x_sp = run("sparse (CSR + CSC)", s_sp, g)
    lines[-1].update(bytes_per_iter=2 * sp.nnz * 8, build_s=round(build_s, 2))
    for nf in [int(t) for t in a.frames.split(",") if t]:
        from mpi_cuda_sartsolver_amd.models.multiframe import MultiFrameSARTSolver

        Xs = np.stack([phantom(grid, t=0.1 * k) for k in range(nf)]) if a.random_density <= 0 else \
            np.random.default_rng(2).random((nf, V)) + 0.1
        Gs = np.stack([s_sp.forward_project(Xs[k]) for k in range(nf)])
        mf = MultiFrameSARTSolver(sp, None, None, p, batch=nf, allow_zero_tolerance=True)
        mf.solve_batch(Gs)  # warm-up
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.steps):
            mf.solve_batch(Gs)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.steps
        rec = dict(path=f"sparse multi-frame x{nf} (SpMM)", P=P, V=V, nnz=sp.nnz, density=round(sp.density, 6),
                   iters=a.iters, frames=nf, ms_per_solve=round(1e3 * dt, 3),
                   frame_iters_per_s=round(nf * a.iters / dt, 1), grid=list(grid))
        lines.append(rec)
        print(json.dumps(rec), flush=True)
        del mf
    if not a.no_dense:
        rt = DenseRTM(P, V, device=dev)
        rt.A.zero_()
        rt.A[torch.from_numpy(r).to(dev), torch.from_numpy(c.astype(np.int64)).to(dev)] = torch.from_numpy(v).to(dev)
        for fused in (True, False):
            s_d = SARTSolver(rt, None, None, p, use_fused=fused, allow_zero_tolerance=True)
            x_d = run("dense fused sweep" if fused else "dense two-pass", s_d, g)
            lines[-1].update(bytes_per_iter=(1 if s_d.use_fused else 2) * rt.nrows_pad * rt.ld * 4,
                             rel_vs_sparse=float(np.linalg.norm(x_d - x_sp) / np.linalg.norm(x_sp)))
            print(json.dumps(lines[-1]), flush=True)
            del s_d
    if a.out:
        with open(a.out, "a") as f:
            for rec in lines:
                f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
