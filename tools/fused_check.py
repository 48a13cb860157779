#!/usr/bin/env python3
"""Correctness probe of the fused sweep at large shapes (one GPU): one SART iteration from the cold start with
the fused sweep and with the two-pass kernels, both against the device fp64 oracle (models/oracle.py).
Usage: fused_check.py [--dtype fp32|bf16] [--sched S] PxV [PxV ...]   (one JSON line per shape)"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mpi_cuda_sartsolver_amd.models.oracle import sart_oracle_f64  # noqa: E402
from mpi_cuda_sartsolver_amd.models.sart import SARTSolver, SolverParams  # noqa: E402
from mpi_cuda_sartsolver_amd.utils.synthetic import make_problem  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shapes", nargs="+")
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--iters", type=int, default=1)
    ap.add_argument("--T", type=int, default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    t0 = time.time()

    def progress(msg):  # keeps long shapes visibly alive (stderr lands in the step's log)
        print(f"[{time.time() - t0:7.1f}s] {msg}", file=sys.stderr, flush=True)

    for sh in a.shapes:
        P, V = (int(v) for v in sh.split("x"))
        progress(f"{sh}: building the problem")
        prob = make_problem(P, V, seed=3, device=dev, storage=a.dtype)
        g = prob.measurement.cpu().numpy()
        p = SolverParams(max_iterations=a.iters, conv_tolerance=0.0)
        out = {"P": P, "V": V, "dtype": a.dtype, "iters": a.iters}
        xs = {}
        for fused in (True, False):
            s = SARTSolver(prob.rtm, None, None, p, allow_zero_tolerance=True, use_fused=fused,
                           fused_rows_per_tile=a.T)
            progress(f"{sh}: {'fused' if fused else 'two-pass'} solve")
            r = s.solve(g)
            if fused:
                out.update(geom=[s.geom.variant, s.geom.T, s.geom.J, s.geom.I, s.geom.cpl], kw=s.geom.kw, xl=s.geom.xl,
                           sched=s.k.fused_get_schedule(), fallbacks=r.fallbacks, used_fused=r.used_fused)
                r2 = s.solve(g)
                out["fused_repeat_bitwise"] = bool(np.array_equal(r.solution, r2.solution))
            xs[fused] = r.solution
            del s
            torch.cuda.empty_cache()
        progress(f"{sh}: fp64 oracle")
        x64 = sart_oracle_f64(prob.rtm, g, a.iters)
        n = np.linalg.norm(x64)
        out["rel_fused"] = float(np.linalg.norm(xs[True] - x64) / n)
        out["rel_two_pass"] = float(np.linalg.norm(xs[False] - x64) / n)
        print(json.dumps(out), flush=True)
        del prob
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
