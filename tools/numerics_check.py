#!/usr/bin/env python3
"""Numerics diagnostic (one GPU): relative distance of the fused sweep, the two-pass kernels and an fp32
numpy emulation (models/reference.sart_fp32_emulation) to the fp64 oracle, per configuration. One JSON line
per configuration. Shows whether a deviation is the inherent fp32 error of the problem or ours."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mpi_cuda_sartsolver_amd.models.reference import sart_fp32_emulation, sart_gpu_semantics  # noqa: E402
from mpi_cuda_sartsolver_amd.models.sart import SARTSolver, SolverParams  # noqa: E402
from mpi_cuda_sartsolver_amd.utils.synthetic import host_problem, make_problem  # noqa: E402


def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def main():
    dev = torch.device("cuda", 0)
    cfgs = [("host", 2048, 4096, 40, False), ("host", 2048, 4096, 40, True), ("host", 1000, 16384, 12, False),
            ("host", 512, 32768, 12, False), ("host", 3000, 16384, 10, False), ("host", 3000, 16384, 10, True),
            ("synth", 1024, 65536, 10, False), ("synth", 512, 131072, 10, False), ("synth", 256, 262144, 10, False),
            ("synth", 512, 100000, 10, False), ("synth", 512, 200000, 10, False), ("synth", 1024, 65536, 3, False),
            ("synth", 1024, 65536, 3, True)]
    for kind, P, V, it, log in cfgs:
        if kind == "host":
            A, g, _ = host_problem(P, V, seed=P + V, saturate_fraction=0.02)
            from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM

            rtm = DenseRTM.from_dense(A, device=dev)
        else:
            prob = make_problem(P, V, seed=P + 5, device=dev, saturate_fraction=0.02)
            rtm = prob.rtm
            A = rtm.to_host()
            g = prob.measurement.cpu().numpy()
        kw = dict(max_iterations=it, conv_tolerance=0.0)
        out = {"kind": kind, "P": P, "V": V, "iters": it, "log": log}
        x64, _, _ = sart_gpu_semantics(A, g, logarithmic=log, **kw)
        x32, _, _ = sart_fp32_emulation(A, g, logarithmic=log, max_iterations=it)
        out["emu_fp32"] = rel(x32, x64)
        for fused in (True, False):
            s = SARTSolver(rtm, None, None, SolverParams(**kw), logarithmic=log, use_fused=fused,
                           allow_zero_tolerance=True)
            r = s.solve(g)
            out["fused" if fused else "two_pass"] = rel(r.solution, x64)
            if fused:
                xf = r.solution
                out["geom"] = [s.geom.variant, s.geom.T, s.geom.J, s.geom.I] if s.use_fused else None
            else:
                out["fused_vs_two_pass"] = rel(xf, r.solution)
            del s
        print(json.dumps(out), flush=True)
        del rtm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
