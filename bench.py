#!/usr/bin/env python3
"""Headline benchmark: SART iterations/s and GFLOPS on a dense synthetic RTM (BASELINE.json).

    python bench.py [--gpus N --steps K --warmup W]           # N == 1
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

One *step* = one frame solve with a cold start and exactly ``--iters`` SART iterations (100 by
default, BASELINE config "64k x 64k fp32 RTM on 1 MI355X, 100 SART iterations"). Scaling is weak:
every GPU holds a ``--npix x --nvox`` fp32 row shard (default 65536 x 65536 = 17.2 GB), so the RTM
is (65536*N) x 65536 at N GPUs. ``value`` is the whole-job GFLOPS with the repo convention of
4*P*V flop per SART iteration; ``iters_per_s`` is the node-wide iteration rate.
The timed region contains the complete solves (setup, every iteration, solution download).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "SART iterations/sec (whole node) on dense RTM; GFLOPS at 1/2/4/8 MI355X"


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--npix", type=int, default=65536, help="pixel rows per GPU (weak scaling)")
    ap.add_argument("--nvox", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=100, help="SART iterations per frame solve")
    ap.add_argument("--variant", choices=["linear", "log"], default="linear")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    ap.add_argument("--no-fused", action="store_true", help="use the two-pass kernels instead of the fused sweep")
    ap.add_argument("--seed", type=int, default=1234)
    args = ap.parse_args()

    import torch

    from mpi_cuda_sartsolver_amd.models.sart import SARTSolver, SolverParams
    from mpi_cuda_sartsolver_amd.parallel.comm import init_distributed
    from mpi_cuda_sartsolver_amd.parallel.partition import row_partition
    from mpi_cuda_sartsolver_amd.utils.synthetic import make_problem

    comm = init_distributed(use_gpu=True)
    n = comm.world_size
    if n != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {n}; using {n}", file=sys.stderr)
    dev = torch.device("cuda", torch.cuda.current_device())

    npix_total = args.npix * n if args.scaling == "weak" else args.npix
    blk = row_partition(npix_total, n, comm.rank)
    prob = make_problem(blk.size, args.nvox, row_offset=blk.offset, seed=args.seed, device=dev)
    params = SolverParams(max_iterations=args.iters, conv_tolerance=0.0)  # fixed iteration count
    solver = SARTSolver(prob.rtm, None, comm, params, logarithmic=args.variant == "log",
                        use_fused=not args.no_fused, check_interval=32, allow_zero_tolerance=True)
    g = prob.measurement

    for _ in range(args.warmup):
        solver.solve(g)
    torch.cuda.synchronize()
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    iters = 0
    res = None
    for _ in range(args.steps):
        res = solver.solve(g)
        iters += res.iterations
    torch.cuda.synchronize()
    comm.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    elapsed = comm.all_reduce_scalar(elapsed, op="max")

    iters_per_s = iters / elapsed
    flop_per_iter = 4.0 * npix_total * args.nvox
    gflops = flop_per_iter * iters_per_s / 1e9
    bytes_per_iter = prob.rtm.nbytes * (1 if solver.use_fused else 2)
    out = {
        "metric": METRIC,
        "value": round(gflops, 2),
        "unit": "GFLOPS",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (on-device random dense RTM, random phantom; no HDF5)",
        "iters_per_s": round(iters_per_s, 3),
        "sart_iterations_per_step": args.iters,
        "status_last": res.status if res else None,
        "fused_sweep": solver.use_fused,
        "fused_variant": solver.geom.variant if solver.use_fused else None,
        "fused_rows_per_tile": solver.geom.T if solver.use_fused else None,
        "fused_schedule": solver.k.fused_get_schedule() if solver.use_fused else None,
        "effective_hbm_TBps_per_gpu": round(bytes_per_iter * iters_per_s / 1e12, 3),
        "config": {
            "model": f"SART-{args.variant} dense RTM",
            "npixel_total": npix_total,
            "nvoxel": args.nvox,
            "global_batch": 1,
            "seq_len": args.nvox,
            "parallelism": f"row-shard dp{n}" if n > 1 else "single",
            "rtm_GB_per_gpu": round(prob.rtm.nbytes / 1e9, 2),
        },
    }
    if comm.rank == 0:
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
