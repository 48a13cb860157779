"""``sartsolver`` command-line driver.

Same CLI, input validation, frame loop, output file and console output as the reference binary
(reference main.cpp:25-151), re-organised for MI355X:

* one process per GPU launched by ``torchrun`` (``python -m torch.distributed.run --nproc-per-node 8
  -m mpi_cuda_sartsolver_amd ...``) instead of ``mpirun``; rank -> GPU = LOCAL_RANK;
* every rank loads only its pixel rows, streamed from HDF5 straight into HBM; with
  ``--parallel_read`` all ranks read at once, otherwise they take turns (reference main.cpp:78-86);
* the next composite frame is read on a helper thread while the current one is solved;
* fatal errors tear the process group down instead of leaving peers blocked in a collective.

Extensions: ``--resume``, ``--batch_frames N`` (multi-frame MFMA solver), ``--two_pass``,
``--partition_voxels`` (voxel-column shards), ``--rtm_bf16`` (bf16-stored RTM), ``--profile FILE`` (JSON lines
per frame).
"""
from __future__ import annotations

import concurrent.futures as cf
import json
import os
import sys
import time


def _fail(msg: str, comm=None) -> None:
    from .parallel.comm import abort_all

    if comm is not None and comm.world_size > 1:
        abort_all(msg, 1)
    print(msg, file=sys.stderr, flush=True)
    raise SystemExit(1)


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    from .ops import native

    n = native()
    try:
        cfg = n.parse_arguments(argv)
    except RuntimeError as exc:
        _fail(str(exc))
    if cfg.help:
        print(n.usage())
        return 0
    try:
        intervals = n.parse_time_intervals(cfg.time_range)
    except RuntimeError as exc:
        _fail(str(exc))
    return run(cfg, intervals)


def run(cfg, intervals) -> int:
    import numpy as np
    import torch

    from .io import hdf5
    from .models.sart import SolverParams
    from .ops import native

    n = native()
    from .parallel.comm import init_distributed
    from .parallel.partition import col_partition, row_partition

    # ---- metadata validation (every rank, before the process group exists: reference main.cpp:27-59)
    try:
        inputs = hdf5.validate_inputs(cfg.input_files, cfg.raytransfer_name, cfg.wavelength_threshold)
    except RuntimeError as exc:
        _fail(str(exc))

    use_gpu = not cfg.use_cpu
    if use_gpu and not torch.cuda.is_available():
        _fail("No GPU available: run with --use_cpu or on an MI355X node.")
    comm = init_distributed(use_gpu=use_gpu)
    rank, world = comm.rank, comm.world_size
    cols = bool(getattr(cfg, "partition_voxels", False)) and use_gpu
    try:
        if cols:  # voxel-column shards: every rank holds all pixels of its voxel block
            vblock = col_partition(inputs.nvoxel, world, rank)
            if vblock.size == 0:
                raise RuntimeError(f"rank {rank} owns no voxels: use at most {inputs.nvoxel} ranks")
            block = row_partition(inputs.npixel, 1, 0)
        else:
            block = row_partition(inputs.npixel, world, rank)
            if block.size == 0:
                raise RuntimeError(f"rank {rank} owns no pixels: use at most {inputs.npixel} ranks")
        image = hdf5.open_composite_image(inputs, intervals, block.size, block.offset, cfg.max_cached_frames)
        params = SolverParams(ray_density_threshold=cfg.ray_density_threshold,
                              ray_length_threshold=cfg.ray_length_threshold, conv_tolerance=cfg.conv_tolerance,
                              beta_laplace=cfg.beta_laplace, relaxation=cfg.relaxation,
                              max_iterations=cfg.max_iterations)
        device = torch.device("cuda", torch.cuda.current_device()) if use_gpu else None
        laplacian = hdf5.load_laplacian(cfg.laplacian_file, inputs.nvoxel, device) if cfg.laplacian_file else None

        def load():
            if cols:
                return hdf5.load_rtm_shard(inputs, 0, inputs.npixel, device, col_offset=vblock.offset,
                                           ncols=vblock.size)
            if use_gpu:
                # --rtm_bf16: each streamed block is rounded into the bf16 shard (native RNE conversion)
                return hdf5.load_rtm_shard(inputs, block.offset, block.size, device,
                                           storage="bf16" if getattr(cfg, "rtm_bf16", False) else "fp32")
            return hdf5.read_rtm_rows(inputs, block.offset, block.stop)

        if cfg.parallel_read or world == 1:
            shard = load()
        else:
            shard = None
            for r in range(world):
                if r == rank:
                    shard = load()
                comm.barrier()

        if use_gpu:
            if cfg.batch_frames > 1:
                from .models.multiframe import MultiFrameSARTSolver

                solver = MultiFrameSARTSolver(shard, laplacian, comm, params, logarithmic=cfg.logarithmic,
                                              batch=cfg.batch_frames)
            else:
                from .models.sart import SARTSolver
                from .ops import hip

                solver = SARTSolver(shard, laplacian, comm, params, logarithmic=cfg.logarithmic,
                                    use_fused=not cfg.two_pass, fused_min_bytes=hip().fused_min_bytes_from_env(),
                                    partition="cols" if cols else None, time_collectives=bool(cfg.profile_file))
        else:
            from .models.cpu import CPUSARTSolver

            solver = CPUSARTSolver(shard, laplacian, comm, params, logarithmic=cfg.logarithmic)

        writer = voxelgrid = None
        skip_until = -float("inf")
        warm = None
        if rank == 0:
            append = False
            if cfg.resume and os.path.exists(cfg.output_file):
                stored_t, last_x, _ = n.read_solution_file(cfg.output_file)
                if len(stored_t):
                    append = True
                    skip_until = float(stored_t[-1])
                    warm = np.asarray(last_x)
            writer = n.SolutionWriter(cfg.output_file, inputs.camera_names, inputs.nvoxel,
                                      cfg.max_cached_solutions, append)
            voxelgrid = hdf5.read_voxel_grid(inputs)
            for wmsg in voxelgrid.warnings:
                print("warning:", wmsg, file=sys.stderr)
        skip_until = comm.broadcast_object(skip_until)
        warm = comm.broadcast_object(warm if not cfg.no_guess else None)
        if cols and warm is not None:
            warm = np.asarray(warm)[vblock.offset: vblock.stop]  # this rank's voxels
        profile = open(cfg.profile_file, "w") if (cfg.profile_file and rank == 0) else None

        solution = warm
        pool = cf.ThreadPoolExecutor(1)
        nframes = image.nframe
        frames = (i for i in range(nframes) if image.frame_time(i) > skip_until + 1e-12)
        if cfg.batch_frames > 1 and use_gpu:
            _run_batched(cfg, solver, image, frames, pool, writer, profile, rank, solution)
        else:
            idx = next(frames, None)
            fut = pool.submit(image.frame, idx) if idx is not None else None
            while fut is not None:
                frame = fut.result()
                cur = idx
                idx = next(frames, None)
                fut = pool.submit(image.frame, idx) if idx is not None else None  # prefetch
                t0 = time.perf_counter()
                res = solver.solve(frame, None if (cfg.no_guess or solution is None) else solution)
                solution = res.solution
                x_full = solver.gather_solution(res.solution) if cols else res.solution  # collective
                if rank == 0:
                    writer.add(x_full, int(res.status), image.frame_time(cur), list(image.camera_frame_time(cur)),
                               int(res.iterations))
                    ms = 1e3 * (time.perf_counter() - t0)
                    print(f"Processed in: {ms} ms", flush=True)
                    if profile:
                        profile.write(json.dumps({"frame": cur, "time": image.frame_time(cur), "status": res.status,
                                                  "iterations": res.iterations, "convergence": res.convergence,
                                                  "ms": ms, "solve_ms": getattr(res, "elapsed_ms", ms),
                                                  "comm_ms": getattr(res, "comm_ms", -1.0),
                                                  "fused": bool(getattr(res, "used_fused", False)),
                                                  "ranks": comm.world_size,
                                                  "device_comm": getattr(getattr(solver, "native_comm", None),
                                                                         "describe", "none"),
                                                  "driver": "python"}) + "\n")
                if cfg.no_guess or (getattr(res, "nonfinite", False) and not np.all(np.isfinite(solution))):
                    solution = None  # cold start after a frame whose iterate stayed non-finite
        pool.shutdown()
        if rank == 0:
            writer.flush()
            if not (cfg.resume and skip_until > -float("inf")):
                voxelgrid.write(cfg.output_file, "voxel_map")
            if profile:
                profile.close()
        comm.barrier()
    except SystemExit:
        raise
    except Exception as exc:  # any rank: report and take the whole job down
        import traceback

        traceback.print_exc()
        _fail(f"rank {rank}: {type(exc).__name__}: {exc}", comm)
    finally:
        try:
            import torch.distributed as dist

            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:
            pass
    return 0


def _run_batched(cfg, solver, image, frames, pool, writer, profile, rank, warm=None) -> None:
    """--batch_frames N: N slots on the matrix cores with continuous batching (a finished frame's slot takes the
    next frame between two sweeps), frames read in windows of 4 N. Without --no_guess the frames form a
    warm-started time series (a window's first N frames start from the previous window's last solution or the
    resumed one, later frames from the latest finished frame); with --no_guess every frame cold-starts
    (reference main.cpp:127-139)."""
    import numpy as np

    idxs = list(frames)
    warm = None if cfg.no_guess else warm
    window = 4 * cfg.batch_frames
    for b0 in range(0, len(idxs), window):
        chunk = idxs[b0: b0 + window]
        batch = np.stack(list(pool.map(image.frame, chunk)))
        t0 = time.perf_counter()
        results = solver.solve_batch(batch, x0=warm, chain=not cfg.no_guess)
        first_warm = idxs[b0 - 1] if (b0 > 0 and warm is not None) else -1  # the window's x0, as a frame
        last = results[-1].solution
        warm = None if (cfg.no_guess or not np.all(np.isfinite(last))) else last
        ms = 1e3 * (time.perf_counter() - t0)
        if rank == 0:
            for i, res in zip(chunk, results):
                writer.add(res.solution, int(res.status), image.frame_time(i), list(image.camera_frame_time(i)),
                           int(res.iterations))
                print(f"Processed in: {ms / len(chunk)} ms", flush=True)
                if profile:
                    wf = chunk[res.warm_from] if res.warm_from >= 0 else first_warm
                    profile.write(json.dumps({"frame": i, "time": image.frame_time(i), "status": res.status,
                                              "iterations": res.iterations, "ms": ms / len(chunk),
                                              "batch": cfg.batch_frames, "warm_from": wf if not cfg.no_guess else -1})
                                  + "\n")


if __name__ == "__main__":
    sys.exit(main())
