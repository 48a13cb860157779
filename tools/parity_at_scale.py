#!/usr/bin/env python3
"""Parity at a production shape: every default path on the 64k x 64k ray-traced RTM with
reflections (utils/raytrace.py, 32 x 32 x 64 voxels, two 128 x 256 cameras; the matrix of tools/series_native.py)
against the device fp64 oracle after 1 and 20 SART updates, bounded by the fp32 two-pass kernels' error on the same
frame (mpi_cuda_sartsolver_amd/utils/parity.py). Also its no-reflection part held sparse, and (--wide) one chip-wide
width: a 32768-row shard x 327680 voxels (64 x 64 x 80, two 128 x 128 cameras), fused sweep vs two-pass.

    python tools/parity_at_scale.py --out gpurun_out/parity_r6_64k_raytraced.jsonl [--wide]
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
    ap.add_argument("--nvox", type=int, default=65536)
    ap.add_argument("--cam", default="128x256")
    ap.add_argument("--iters", default="1,20")
    ap.add_argument("--no-sparse", action="store_true")
    ap.add_argument("--no-bf16", action="store_true")
    ap.add_argument("--wide", action="store_true", help="also the 32768 x 327680 chip-wide shard (fused vs two-pass)")
    ap.add_argument("--only-wide", action="store_true")
    ap.add_argument("--batches", default="32,64,128")
    ap.add_argument("--variants", default="lin,lin+lap,log,log+lap")
    ap.add_argument("--frames", default="0,1")
    ap.add_argument("--no-single", action="store_true", help="multi-frame paths only (the two-pass yardstick stays)")
    ap.add_argument("--tag", default="")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "parity_at_scale.jsonl"))
    a = ap.parse_args()
    import torch

    from mpi_cuda_sartsolver_amd.models.laplacian import LaplacianCSR
    from mpi_cuda_sartsolver_amd.utils import parity
    from mpi_cuda_sartsolver_amd.utils.raytrace import raytraced_direct_coo

    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    outf = open(a.out, "a")

    def emit(rec):
        line = json.dumps(rec)
        print(line, flush=True)
        outf.write(line + "\n")
        outf.flush()

    dev = torch.device("cuda", 0)
    iters = [int(v) for v in a.iters.split(",")]
    if not a.only_wide:
        t0 = time.perf_counter()
        cam = tuple(int(v) for v in a.cam.split("x"))
        A, X, cams, grid, info, rng = parity.raytraced_problem(a.nvox, cam)
        Ad = torch.from_numpy(A).to(dev)
        G = parity.frames_from(Ad, X, rng)
        del Ad
        torch.cuda.empty_cache()
        L = LaplacianCSR.grid_3d(*grid, device=dev)
        sparse_A = None
        if not a.no_sparse:
            r, c, v, _ = raytraced_direct_coo(grid=grid, cameras=cams)
            sparse_A = np.zeros(A.shape, np.float32)
            sparse_A[r, c] = v
        emit(dict(setup=True, shape=list(A.shape), grid=list(grid), cams=list(cam), seconds=time.perf_counter() - t0,
                  rtm="ray-traced with reflections (utils/raytrace.py)", frames="phantom(t = 0.1 k), 2 % saturated"))
        variants = [("log" in v, "lap" in v) for v in a.variants.split(",")]
        parity.run(A, G, dev, iters=iters, laplacian=L, bf16=not a.no_bf16, sparse_A=sparse_A, emit=emit,
                   batches=tuple(int(b) for b in a.batches.split(",") if b), variants=variants,
                   frames=tuple(int(f) for f in a.frames.split(",")), single=not a.no_single,
                   column_shard=not a.no_single, tag=f"{A.shape[0]}x{A.shape[1]}{a.tag}")
        del A, G, sparse_A
        torch.cuda.empty_cache()
    if a.wide or a.only_wide:
        t0 = time.perf_counter()
        A, X, cams, grid, info, rng = parity.raytraced_problem(327680, (128, 128), nframes=2)
        Ad = torch.from_numpy(A).to(dev)
        G = parity.frames_from(Ad, X, rng)
        del Ad
        torch.cuda.empty_cache()
        emit(dict(setup=True, shape=list(A.shape), grid=list(grid), cams=[128, 128], seconds=time.perf_counter() - t0))
        parity.run(A, G, dev, iters=iters, batches=(), variants=[(False, False), (True, False)], bf16=False,
                   column_shard=False, emit=emit, tag=f"{A.shape[0]}x{A.shape[1]} chip-wide")


if __name__ == "__main__":
    main()
