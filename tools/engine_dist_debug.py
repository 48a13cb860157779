#!/usr/bin/env python3
"""Debug aid: multi-rank engine (row shards) vs one rank holding the whole synthetic problem, step by step."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mpi_cuda_sartsolver_amd.models.sart import SARTSolver, SolverParams  # noqa: E402
from mpi_cuda_sartsolver_amd.parallel.comm import init_distributed  # noqa: E402
from mpi_cuda_sartsolver_amd.parallel.partition import row_partition  # noqa: E402
from mpi_cuda_sartsolver_amd.utils.synthetic import make_problem  # noqa: E402


def main():
    comm = init_distributed(use_gpu=True)
    dev = torch.device("cuda", torch.cuda.current_device())
    P, V = 3000, 4096
    b = row_partition(P, comm.world_size, comm.rank)
    loc = make_problem(b.size, V, row_offset=b.offset, seed=7, device=dev, saturate_fraction=0.02)
    full = make_problem(P, V, row_offset=0, seed=7, device=dev, saturate_fraction=0.0) if comm.rank == 0 else None
    gfull = comm.all_gather_object(loc.measurement.cpu().numpy())
    for it in (1, 2, 5, 30):
        params = SolverParams(max_iterations=it, conv_tolerance=1e-12)
        s = SARTSolver(loc.rtm, None, comm, params, use_fused=False)
        r = s.solve(loc.measurement)
        if comm.rank == 0:
            s1 = SARTSolver(full.rtm, None, None, params, use_fused=False)
            if it == 1:
                rd, rd1 = s.ray_density64, s1.ray_density64
                Ah = full.rtm.A[:P, :V].double().cpu().numpy()
                rdo = Ah.sum(0)
                print("rho multi", rd.min(), rd.max(), "single", rd1.min(), rd1.max(), "oracle", rdo.min(), rdo.max(),
                      flush=True)
                print("ell single vs oracle", np.abs(s1.ray_length64 - Ah.sum(1)).max(), flush=True)
                print("ell multi(rank0) vs oracle", np.abs(s.ray_length64 - Ah[:b.size].sum(1)).max(), flush=True)
            r1 = s1.solve(np.concatenate(gfull))
            print("norms", np.linalg.norm(r.solution), np.linalg.norm(r1.solution), flush=True)
            print(f"it={it} rel={np.linalg.norm(r.solution - r1.solution) / np.linalg.norm(r1.solution):.3e} "
                  f"iters {r.iterations}/{r1.iterations}", flush=True)
    comm.barrier()


if __name__ == "__main__":
    main()
