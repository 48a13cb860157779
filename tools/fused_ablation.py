#!/usr/bin/env python3
"""Exchange ablation of the fused sweep on a given shard and storage: the full sweep against the same kernel with
the inter-workgroup exchange disabled (fused_set_debug(1): no granule stores / waits, timing only; the iterates
are garbage). Equal times mean the sweep is bound by streaming A, not by the row-dot hand-off.

    python tools/fused_ablation.py [--dtype bf16] [--iters 10] 65536x262144 ...

One JSON line per (shape, mode): ms per sweep from (solve(iters) - solve(1)) / (iters - 1), effective TB/s.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mpi_cuda_sartsolver_amd.models.sart import SARTSolver, SolverParams  # noqa: E402
from mpi_cuda_sartsolver_amd.ops import hip  # noqa: E402
from mpi_cuda_sartsolver_amd.parallel.comm import SingleProcessComm  # noqa: E402
from mpi_cuda_sartsolver_amd.utils.synthetic import make_problem  # noqa: E402


def solve_ms(solver, g, reps=3):
    best = float("inf")
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        solver.solve(g)
        torch.cuda.synchronize()
        best = min(best, 1e3 * (time.perf_counter() - t0))
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shapes", nargs="*", default=["65536x262144"])
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="bf16")
    ap.add_argument("--iters", type=int, default=11)
    a = ap.parse_args()
    k = hip()
    dev = torch.device("cuda", 0)
    comm = SingleProcessComm()
    for shape in a.shapes:
        P, V = (int(v) for v in shape.split("x"))
        prob = make_problem(P, V, row_offset=0, seed=1, device=dev, storage=a.dtype)
        g = prob.measurement
        mk = lambda n: SARTSolver(prob.rtm, None, comm, SolverParams(max_iterations=n, conv_tolerance=0.0),  # noqa: E731
                                  use_fused=True, check_interval=32, allow_zero_tolerance=True)
        s1, sn = mk(1), mk(a.iters)
        for dbg, mode in ((0, "full"), (1, "no_exchange")):
            k.fused_set_debug(dbg | int(os.environ.get("SART_FUSED_DBG_EXTRA", "0")))
            solve_ms(s1, g, reps=1)  # warm
            t1, tn = solve_ms(s1, g), solve_ms(sn, g)
            ms = (tn - t1) / (a.iters - 1)
            print(json.dumps({"shape": shape, "dtype": a.dtype, "mode": mode, "T": sn.geom.T,
                              "dbg_extra": int(os.environ.get("SART_FUSED_DBG_EXTRA", "0")),
                              "schedule": (int(os.environ.get("SART_BF16_T2_SCHED", "7"))
                                           if a.dtype == "bf16" and sn.geom.T == 2 else sn.k.fused_get_schedule()),
                              "J": sn.geom.J, "I": sn.geom.I,
                              "ms_per_sweep": round(ms, 4), "TBps": round(prob.rtm.nbytes / ms / 1e9, 3)}), flush=True)
        k.fused_set_debug(0)
        del s1, sn, prob
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
