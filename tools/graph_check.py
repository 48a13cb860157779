#!/usr/bin/env python3
"""Eager vs HIP-graph chunk replay: time per SART iteration on small problems, where launch overhead is a
visible share of an iteration (one JSON line per shape and mode)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM  # noqa: E402
from mpi_cuda_sartsolver_amd.models.sart import SARTSolver, SolverParams  # noqa: E402
from mpi_cuda_sartsolver_amd.utils.synthetic import make_problem  # noqa: E402

dev = torch.device("cuda", 0)
for P, V in ((2048, 4096), (8192, 16384), (16384, 65536)):
    prob = make_problem(P, V, seed=3, device=dev)
    for fused in (True, False):
        for graph in (False, True):
            s = SARTSolver(prob.rtm, None, None, SolverParams(max_iterations=400, conv_tolerance=0.0),
                           use_fused=fused, check_interval=32, use_graph=graph, allow_zero_tolerance=True)
            s.solve(prob.measurement)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            reps = 3
            for _ in range(reps):
                r = s.solve(prob.measurement)
            dt = (time.perf_counter() - t0) / reps
            print(json.dumps(dict(P=P, V=V, fused=fused, graph=graph, iterations=r.iterations,
                                  us_per_iter=round(1e6 * dt / r.iterations, 2))), flush=True)
            del s
    del prob
    torch.cuda.empty_cache()
