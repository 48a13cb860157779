#!/usr/bin/env python3
"""Time-series throughput of the multi-frame engine: continuous batching (all frames in one solve_batch call,
finished slots refilled between sweeps) against group-by-group batching (one call per group of nf frames, each
group running as long as its slowest frame), on a series whose frames need different iteration counts.
One JSON line per mode. Usage: series_bench.py [--npix P] [--nvox V] [--frames N] [--batch nf] [--dtype ...]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mpi_cuda_sartsolver_amd.models.multiframe import MultiFrameSARTSolver  # noqa: E402
from mpi_cuda_sartsolver_amd.models.sart import SolverParams  # noqa: E402
from mpi_cuda_sartsolver_amd.utils.synthetic import make_problem  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npix", type=int, default=16384)
    ap.add_argument("--nvox", type=int, default=16384)
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--tol", type=float, default=1e-5)
    ap.add_argument("--max-iter", type=int, default=400)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    prob = make_problem(a.npix, a.nvox, seed=5, device=dev, storage=a.dtype)
    rng = np.random.default_rng(1)
    x_true = prob.x_true.detach().to("cpu", torch.float64).numpy() if hasattr(prob, "x_true") else rng.random(a.nvox)
    # a series with mixed step sizes between frames: small steps converge fast, large ones slowly
    steps = rng.choice([0.002, 0.02, 0.2], size=a.frames)
    X = np.empty((a.frames, a.nvox))
    cur = x_true.copy()
    for f in range(a.frames):
        cur = np.abs(cur * (1.0 + steps[f] * rng.standard_normal(a.nvox)))
        X[f] = cur
    A = prob.rtm.A[: a.npix, : a.nvox].float()
    G = (torch.from_numpy(X).to(dev, torch.float32) @ A.T).double().cpu().numpy()
    p = SolverParams(max_iterations=a.max_iter, conv_tolerance=a.tol)
    s = MultiFrameSARTSolver(prob.rtm, None, None, p, batch=a.batch)
    s.solve_batch(G[: a.batch], x0=None, chain=True)  # warm-up
    torch.cuda.synchronize()
    for mode in ("continuous", "groups"):
        t0 = time.perf_counter()
        if mode == "continuous":
            res = s.solve_batch(G, x0=None, chain=True)
        else:
            res, warm = [], None
            for b0 in range(0, a.frames, s.batch_width):
                r = s.solve_batch(G[b0: b0 + s.batch_width], x0=warm, chain=True)
                res += r
                warm = r[-1].solution
        dt = time.perf_counter() - t0
        its = [r.iterations for r in res]
        print(json.dumps({"mode": mode, "frames": a.frames, "batch": s.batch_width, "dtype": a.dtype,
                          "npix": a.npix, "nvox": a.nvox, "seconds": round(dt, 4), "frames_per_s": round(a.frames / dt, 2),
                          "iterations_mean": float(np.mean(its)), "iterations_max": int(np.max(its)),
                          "converged": int(sum(r.status == 0 for r in res))}), flush=True)


if __name__ == "__main__":
    main()
