#!/usr/bin/env python3
"""Multi-rank consistency check of the GPU solver: solve one synthetic global problem on N ranks
(row-sharded) and save rank 0's solution. Compare outputs of different N (tests/test_gpu_distributed.py)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npix", type=int, default=3000)
    ap.add_argument("--nvox", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--tol", type=float, default=1e-6, help="convergence tolerance (0: exactly --iters iterations)")
    ap.add_argument("--logarithmic", action="store_true")
    ap.add_argument("--fused", action="store_true")
    ap.add_argument("--multiframe", action="store_true")
    ap.add_argument("--batch", type=int, default=16, help="multi-frame batch width (16, 32, 64)")
    ap.add_argument("--columns", action="store_true", help="column (voxel) shards instead of row shards")
    ap.add_argument("--save-problem", action="store_true",
                    help="(1 rank) also save the global A and g as <out>.A.npy / <out>.g.npy for host oracles")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import numpy as np
    import torch

    from mpi_cuda_sartsolver_amd.models.laplacian import LaplacianCSR
    from mpi_cuda_sartsolver_amd.models.sart import SARTSolver, SolverParams
    from mpi_cuda_sartsolver_amd.parallel.comm import init_distributed
    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM
    from mpi_cuda_sartsolver_amd.parallel.partition import col_partition, row_partition
    from mpi_cuda_sartsolver_amd.utils.synthetic import make_problem

    comm = init_distributed(use_gpu=True)
    dev = torch.device("cuda", torch.cuda.current_device())
    if a.columns:  # every rank: all pixels (full measurement) and the RTM columns of its voxel block
        cb = col_partition(a.nvox, comm.world_size, comm.rank)
        prob = make_problem(a.npix, a.nvox, seed=7, device=dev, saturate_fraction=0.02)
        prob.rtm = DenseRTM.synthetic(a.npix, cb.size, 0, seed=7, device=dev, col_offset=cb.offset,
                                      nvoxel_total=a.nvox)
    else:
        b = row_partition(a.npix, comm.world_size, comm.rank)
        prob = make_problem(b.size, a.nvox, row_offset=b.offset, seed=7, device=dev, saturate_fraction=0.02)
    L = LaplacianCSR.grid_3d(16, 16, 16, device=dev) if a.nvox == 4096 else None
    if a.save_problem and comm.world_size == 1:  # the global problem (a 1-rank shard holds all of it)
        np.save(a.out + ".A.npy", prob.rtm.to_host())
        np.save(a.out + ".g.npy", prob.measurement.cpu().numpy())
    params = SolverParams(max_iterations=a.iters, conv_tolerance=a.tol, beta_laplace=1e-3)
    if a.multiframe:
        from mpi_cuda_sartsolver_amd.models.multiframe import MultiFrameSARTSolver

        s = MultiFrameSARTSolver(prob.rtm, L, comm, params, logarithmic=a.logarithmic, batch=a.batch,
                                 allow_zero_tolerance=a.tol == 0)
        g = prob.measurement.cpu().numpy()
        res = s.solve_batch(np.stack([g, 0.5 * g, 2.0 * g]))
        x = np.stack([r.solution for r in res])
        meta = [dict(status=r.status, iterations=r.iterations, comm=r.comm or s.native_comm.backend,
                     comm_fallbacks=r.comm_fallbacks) for r in res]
        meta[0]["ranks"] = comm.all_gather_object(dict(comm=res[0].comm, comm_fallbacks=res[0].comm_fallbacks))
    else:
        s = SARTSolver(prob.rtm, L, comm, params, logarithmic=a.logarithmic, use_fused=a.fused,
                       partition="cols" if a.columns else None, time_collectives=True,
                       allow_zero_tolerance=a.tol == 0)
        r = s.solve(prob.measurement)
        r2 = s.solve(prob.measurement, solution=r.solution)  # warm start path
        x = np.stack([s.gather_solution(r.solution), s.gather_solution(r2.solution)])
        meta = [dict(status=r.status, iterations=r.iterations, fused=r.used_fused, comm=r.comm or s.native_comm.backend,
                     comm_ms=r.comm_ms, fallbacks=r.fallbacks, comm_fallbacks=r.comm_fallbacks, variant=r.fused_variant,
                     describe=s.native_comm.describe),
                dict(status=r2.status, iterations=r2.iterations, fallbacks=r2.fallbacks, comm=r2.comm,
                     comm_fallbacks=r2.comm_fallbacks)]
        # every rank's fallback history: a persistent-sweep timeout must be handled identically everywhere
        g = s.geom
        meta[0]["ranks"] = comm.all_gather_object(dict(
            fallbacks=r.fallbacks, variant=r.fused_variant, fused=r.used_fused, shared=s.shared_device,
            comm=r.comm, comm_fallbacks=r.comm_fallbacks, comm2=r2.comm, fallbacks2=r2.fallbacks,
            comm_fallbacks2=r2.comm_fallbacks, plan_cus=s.plan_cus, ranks_per_device=s.ranks_per_device,
            grid=(dict(J=g.J, I=g.I, T=g.T, kw=g.kw, workgroups=g.grid) if g is not None else None)))
        if not a.columns:  # the replicated solution must be bitwise identical on every rank
            xs = comm.all_gather_object(x)
            meta[0]["x_bitwise_equal"] = all(np.array_equal(xs[0], xi) for xi in xs)

    if comm.rank == 0:
        np.save(a.out + ".npy", x)
        with open(a.out + ".json", "w") as f:
            json.dump(meta, f)
    comm.barrier()


if __name__ == "__main__":
    main()
