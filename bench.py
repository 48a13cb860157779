#!/usr/bin/env python3
"""Headline benchmark: SART iterations/s and GFLOPS on a dense synthetic RTM (BASELINE.json).

    python bench.py [--gpus N --steps K --warmup W]           # N ranks (self-launched when N > 1)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

One *step* = one frame solve with a cold start and exactly ``--iters`` SART iterations (100 by
default, BASELINE config "64k x 64k fp32 RTM on 1 MI355X, 100 SART iterations"). Scaling is weak:
every GPU holds a ``--npix x --nvox`` fp32 row shard (default 65536 x 65536 = 17.2 GB), so the RTM
is (65536*N) x 65536 at N GPUs. ``value`` is the whole-job GFLOPS with the repo convention of
4*P*V flop per SART iteration; ``iters_per_s`` is the node-wide iteration rate.
The timed region contains the complete solves (setup, every iteration, solution download).

Launching: ``--gpus N`` with N > 1 and no launcher environment (WORLD_SIZE / MPI rank variables) starts
``torch.distributed.run --nproc-per-node N`` as a child process before any GPU call and passes its JSON
line and exit code through, like the reference's ``mpirun -np N`` (reference main.cpp:63-68). Under a
launcher, a world size different from ``--gpus`` is an error (exit 1). A per-rank watchdog exits non-zero
when a stage (setup, self-check, warmup, timed steps) makes no progress for ``--watchdog`` seconds.
Before timing, a one-iteration self-check compares the fused sweep and the two-pass kernels on the same shard
with the device fp64 oracle (``selfcheck`` in the JSON line).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "SART iterations/sec (whole node) on dense RTM; GFLOPS at 1/2/4/8 MI355X"

# BASELINE.json configs as weak-scaling presets (rows per GPU): at N = 8 GPUs "512kx256k" is the
# 524288 x 262144 RTM (68.7 GB per GPU) and "2tb" is 1966080 x 262144 fp32 = 2.06 TB (258 GB per GPU)
# with the Laplacian and a 64-frame batch; "256k" fills one GPU with a 262144 x 262144 shard (275 GB).
PRESETS = {
    "64k": dict(npix=65536, nvox=65536, iters=100),
    "256k": dict(npix=262144, nvox=262144, iters=20),
    "512kx256k": dict(npix=65536, nvox=262144, iters=100),
    "2tb": dict(npix=245760, nvox=262144, iters=20, frames=64, laplacian=True),
}


def shared_gpu_env(ranks: int, ndev: int) -> dict:
    """Environment of a rehearsal with more ranks than GPUs (--share-gpus)."""
    # RCCL refuses two ranks on one device: gloo host collectives under the one-shot P2P all-reduce (auto-selected
    # against the staged base), and the fused sweep on each rank's share of the CUs
    env = dict(SART_DIST_BACKEND="gloo", SART_P2P_WRAP_STAGED="1", SART_FUSED_SHARED="1")
    # Hardware queues: the GPU maps 24 compute queues (KFD num_cp_queues); 8 ranks x HIP's default 4 = 32
    # over-subscribe it and the scheduler time-slices the processes, so every P2P all-reduce waits out a time slice
    # for a descheduled peer (10.3 ms per call, 83.7 it/s; with 1 queue per rank 111 us, 172.4 it/s:
    # profiles/bench_r4_n8_rehearsal_one_gpu_q{4,1}.json). One rank per GPU is unaffected. The cap is a ceiling on
    # whatever the environment sets (the GPU boxes export HIP's default, 4).
    per_gpu = -(-ranks // max(ndev, 1))
    have = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
    env["GPU_MAX_HW_QUEUES"] = str(max(1, min(have, 12 // per_gpu)))
    return env


def grid_dims(n: int) -> tuple[int, int, int]:
    """nx * ny * nz == n with the factors as close to a cube as possible (synthetic voxel grid)."""
    best = (n, 1, 1)
    for nx in range(1, int(round(n ** (1 / 3))) + 2):
        if n % nx:
            continue
        m = n // nx
        for ny in range(nx, int(m ** 0.5) + 1):
            if m % ny == 0:
                cand = tuple(sorted((nx, ny, m // ny), reverse=True))
                if max(cand) < max(best):
                    best = cand
    return best


LAUNCHER_VARS = ("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE")


def launched_world() -> int | None:
    """World size set by a launcher (torchrun, mpirun), None when this process was started directly."""
    for v in LAUNCHER_VARS:
        if os.environ.get(v):
            return int(os.environ[v])
    return None


def free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpu_count() -> int:
    """GPUs this process may use, counted without initialising HIP (a launcher must start from a process that has
    not touched the GPU): HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES, else the GPU nodes
    of the KFD topology (nodes with SIMDs), else torch's count."""
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        e = os.environ.get(v)
        if e is not None:
            return len([t for t in e.split(",") if t.strip() != ""])
    nodes = "/sys/class/kfd/kfd/topology/nodes"
    try:
        n = 0
        for d in os.listdir(nodes):
            try:
                with open(os.path.join(nodes, d, "properties")) as f:
                    props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
                n += int(props.get("simd_count", "0")) > 0
            except (OSError, ValueError):
                pass
        if n:
            return n
    except OSError:
        pass
    import torch

    return torch.cuda.device_count()


def self_launch(n: int, argv: list[str], env_extra: dict) -> int:
    """Start N ranks of this script under torch.distributed.run (one rank per GPU) and return their exit
    code; rank 0's JSON line reaches our stdout unchanged. No GPU call happens in this process."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__), *argv]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", **env_extra)
    return subprocess.run(cmd, env=env).returncode


class Watchdog:
    """Per-rank progress watchdog: exits the process (code 3) when no stage completes for `limit` seconds,
    so a hang (e.g. in a collective or a communicator self-test) cannot hold the GPUs until an outer timeout."""

    def __init__(self, limit: float, rank: int):
        import threading

        self.limit, self.rank = float(limit), rank
        self.stage, self.t = "start", time.monotonic()
        if self.limit > 0:
            threading.Thread(target=self._run, daemon=True).start()

    def kick(self, stage: str) -> None:
        self.stage, self.t = stage, time.monotonic()

    def _run(self) -> None:
        while True:
            time.sleep(min(5.0, self.limit / 4))
            if time.monotonic() - self.t > self.limit:
                print(f"bench watchdog: rank {self.rank} made no progress for {self.limit:.0f} s in stage "
                      f"'{self.stage}'; exiting", file=sys.stderr, flush=True)
                os._exit(3)


def _split_a_dtype(solver) -> str:
    """The operand pieces the split-A multi-frame projections ran with (MultiFrameSARTSolver.forward_split /
    backproject_split): f16 pairs are ~2^-22 per product (not fp32-exact: 2^-24), bf16 pairs 2^-17, bf16 triples
    fp32-exact."""
    desc = {"f16x2": "f16 MFMA on two f16 pieces of A (scaled per %s) and of the fp32 operand (3 products, ~2^-22 "
                     "per product)",
            "bf16x2": "bf16 MFMA on hi + lo bf16 pieces of A and of the fp32 operand (3 products, ~2^-17 per product)",
            "bf16x3": "bf16 MFMA on hi + mid + lo bf16 pieces of A and W (6 products, fp32-exact)"}
    fwd = desc.get(solver.forward_split, solver.forward_split)
    bwd = desc.get(solver.backproject_split, solver.backproject_split)
    return ("fp32 RTM; forward: " + (fwd % "row" if "%s" in fwd else fwd) + "; back-projection: "
            + (bwd % "column" if "%s" in bwd else bwd) + "; fp32 accumulation")


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); > 1 self-launches under torchrun")
    ap.add_argument("--share-gpus", action="store_true",
                    help="rehearsal: allow more ranks than visible GPUs (ranks share devices, gloo host "
                         "collectives, two-pass kernels)")
    ap.add_argument("--watchdog", type=float, default=600.0,
                    help="seconds without progress after which a rank exits non-zero (0: off)")
    ap.add_argument("--no-selfcheck", action="store_true", help="skip the untimed fused-vs-two-pass check")
    ap.add_argument("--launch-check", action="store_true",
                    help="launch and rendezvous only (no GPU work): prints the JSON line with value null")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--npix", type=int, default=65536, help="pixel rows per GPU (weak scaling)")
    ap.add_argument("--nvox", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=100, help="SART iterations per frame solve")
    ap.add_argument("--ld", type=int, default=None,
                    help="padded row length of the shard (default: choose_ld; geometry A/B runs with SART_FUSED_KW)")
    ap.add_argument("--variant", choices=["linear", "log"], default="linear")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    ap.add_argument("--no-fused", action="store_true", help="use the two-pass kernels instead of the fused sweep")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--mf-split-a", choices=["auto", "on", "off"], default="auto",
                    help="multi-frame fp32 shards: split A in registers into two f16 pieces (scaled per row for the "
                         "forward, per column for the back-projection) for the 16-bit matrix cores (auto: from 32 "
                         "frames on) or fp32 MFMA")
    ap.add_argument("--frames", type=int, default=1,
                    help="frames per step; > 1 solves them together with the multi-frame MFMA engine (up to 128 per "
                         "batch on bf16 storage and on split-A fp32 shards; 64 on the fp32 MFMA path and the "
                         "six-product bf16 back-projection)")
    ap.add_argument("--partition", choices=["rows", "cols"], default="rows",
                    help="rows: the reference's pixel shards (default); cols: voxel shards, each GPU holds all "
                         "pixels of --nvox voxels (two-pass kernels, all-reduce of A.x)")
    ap.add_argument("--laplacian", action="store_true",
                    help="add the 7-point grid Laplacian regulariser (beta 1e-2, the reference default)")
    ap.add_argument("--rtm-dtype", choices=["fp32", "bf16"], default="fp32",
                    help="RTM storage precision; bf16 is opt-in (half the bytes per sweep; fp32 products and sums in "
                         "the single-frame kernels, bf16 MFMA with hi+lo split X / W and fp32 accumulation with "
                         "--frames); the BASELINE headline is fp32")
    ap.add_argument("--config", choices=sorted(PRESETS), default=None,
                    help="BASELINE.json configuration preset (sets npix / nvox / iters / frames / laplacian)")
    args = ap.parse_args()
    if args.config:  # the preset's values, except flags given explicitly (e.g. --config 2tb --frames 128)
        given = {a.split("=")[0] for a in sys.argv[1:] if a.startswith("--")}
        for k, v in PRESETS[args.config].items():
            if "--" + k.replace("_", "-") not in given:
                setattr(args, k, v)
    if args.rtm_dtype == "bf16" and args.partition == "cols":
        ap.error("--rtm-dtype bf16 runs row shards")
    if args.partition == "cols" and args.frames > 1:
        ap.error("--partition cols solves single frames (the multi-frame engine uses row shards)")

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    world = launched_world()
    if world is None and args.gpus > 1:
        env_extra = {}
        if not args.launch_check:
            ndev = visible_gpu_count()
            if ndev < args.gpus and not args.share_gpus:
                print(f"bench: --gpus {args.gpus} but only {ndev} GPU(s) visible (--share-gpus to rehearse "
                      "on fewer devices)", file=sys.stderr)
                return 1
            if ndev < args.gpus:
                env_extra.update(shared_gpu_env(args.gpus, ndev))
        return self_launch(args.gpus, sys.argv[1:], env_extra)
    if (world or 1) != args.gpus:
        print(f"bench: --gpus {args.gpus} but the launcher started {world or 1} rank(s)", file=sys.stderr)
        return 1
    if world and world > 1 and args.share_gpus and not args.launch_check:
        ndev = visible_gpu_count()
        if ndev < world:  # an external launcher (torchrun) with ranks sharing GPUs: the same set-up, before HIP starts
            os.environ.update(shared_gpu_env(world, ndev))
    # A device all-reduce that waits this long for a peer gives up; the engine then re-solves the frame on the base
    # communicator (RCCL), so a stalled P2P path costs one timeout instead of the watchdog's limit.
    os.environ.setdefault("SART_P2P_TIMEOUT_S", "30")

    import torch

    from mpi_cuda_sartsolver_amd.parallel.comm import init_distributed

    if args.launch_check:  # CPU rehearsal of the launch path: rendezvous, barrier, max-reduction, JSON line
        comm = init_distributed(use_gpu=False)
        wd = Watchdog(args.watchdog, comm.rank)
        comm.barrier()
        wd.kick("barrier")
        t = comm.all_reduce_scalar(float(comm.rank), op="max")
        if comm.rank == 0:
            print(json.dumps({"metric": METRIC, "value": None, "unit": "GFLOPS", "n_gpus": comm.world_size,
                              "steps": args.steps, "warmup": args.warmup, "launch_check": True,
                              "max_rank": int(t)}), flush=True)
        return 0

    from mpi_cuda_sartsolver_amd.models.sart import SARTSolver, SolverParams
    from mpi_cuda_sartsolver_amd.parallel.partition import row_partition
    from mpi_cuda_sartsolver_amd.utils.synthetic import make_problem

    t_setup = time.perf_counter()
    comm = init_distributed(use_gpu=True)
    n = comm.world_size
    wd = Watchdog(args.watchdog, comm.rank)
    dev = torch.device("cuda", torch.cuda.current_device())

    cols = args.partition == "cols"
    nvox_total = args.nvox
    if cols:  # voxel shards: every GPU holds all --npix pixels of its block of voxels
        from mpi_cuda_sartsolver_amd.parallel.partition import col_partition
        from mpi_cuda_sartsolver_amd.utils.synthetic import make_column_problem

        npix_total = args.npix
        nvox_total = args.nvox * n if args.scaling == "weak" else args.nvox
        cb = col_partition(nvox_total, n, comm.rank)
        prob = make_column_problem(npix_total, cb.size, cb.offset, nvox_total, comm, seed=args.seed, device=dev)
    else:
        npix_total = args.npix * n if args.scaling == "weak" else args.npix
        blk = row_partition(npix_total, n, comm.rank)
        prob = make_problem(blk.size, args.nvox, row_offset=blk.offset, seed=args.seed, device=dev,
                            storage=args.rtm_dtype, ld=args.ld)
    params = SolverParams(max_iterations=args.iters, conv_tolerance=0.0)  # fixed iteration count
    lap = None
    if args.laplacian:
        from mpi_cuda_sartsolver_amd.models.laplacian import LaplacianCSR

        lap = LaplacianCSR.grid_3d(*grid_dims(nvox_total))
    if args.frames > 1:
        import numpy as np

        from mpi_cuda_sartsolver_amd.models.multiframe import MultiFrameSARTSolver

        solver = MultiFrameSARTSolver(prob.rtm, lap, comm, params, logarithmic=args.variant == "log",
                                      batch=min(128, args.frames), check_interval=32, allow_zero_tolerance=True,
                                      split_a={"auto": None, "on": True, "off": False}[args.mf_split_a])
        g1 = prob.measurement.cpu().numpy()
        g = np.stack([g1 * (1.0 + 0.05 * f) for f in range(args.frames)])  # distinct frames of one problem

        class _Batch:  # one step = all frames
            def __init__(self, s):
                self.s = s

            def solve(self, gb):
                rs = self.s.solve_batch(gb)
                r = rs[-1]
                r.iterations = sum(x.iterations for x in rs)
                return r

        runner = _Batch(solver)
    else:
        # The engine itself decides whether ranks share a GPU (PCI bus id on every rank) and then runs the
        # two-pass kernels: the fused sweep is a persistent grid that needs its device to itself.
        # time_collectives (N > 1): timing events around each per-iteration all-reduce (GPU-side only)
        solver = SARTSolver(prob.rtm, lap, comm, params, logarithmic=args.variant == "log",
                            use_fused=not args.no_fused, check_interval=32, allow_zero_tolerance=True,
                            partition=args.partition, time_collectives=n > 1)
        g = prob.measurement
        runner = solver
    multi = args.frames > 1
    startup = {"setup_s": round(time.perf_counter() - t_setup, 2)}  # process group, shard, engine, comm self-tests
    if n > 1:  # of which the device communicator's own start-up (p2p: IPC mapping, self-test, size probes)
        startup["comm_setup_s"] = round(float(solver.native_comm.setup_seconds), 2)
    wd.kick("setup")

    class _Counts:  # recoveries over the WHOLE run (self-check, warm-up and timed steps), not the timed steps only
        def __init__(self):
            self.comm = self.fused = 0

        def add(self, r):
            self.comm += int(getattr(r, "comm_fallbacks", 0))
            self.fused += int(getattr(r, "fallbacks", 0))

    counts = _Counts()
    selfcheck = None
    if not multi and solver.use_fused and not args.no_selfcheck:
        # Untimed: ONE iteration from the cold start (x1 = x0 + d(x0): every part of the sweep runs once) with
        # the fused sweep and with the two-pass kernels on this very shard and grid, both against the device fp64
        # oracle (models/oracle.py, all ranks). At x0 the residual is large, so the comparison measures the
        # kernels (a wrong index or hand-off shows as O(1)) rather than the fp32 drift of later iterations on
        # an ill-conditioned dense random matrix (1e-3 .. 1e-1 after a few iterations at these sizes).
        import numpy as np

        from mpi_cuda_sartsolver_amd.models.oracle import sart_oracle_f64

        t_check = time.perf_counter()
        p1 = SolverParams(max_iterations=1, conv_tolerance=0.0)
        kw = dict(logarithmic=args.variant == "log", allow_zero_tolerance=True, partition=args.partition)
        gh = g.cpu().numpy() if hasattr(g, "cpu") else np.asarray(g)
        rf = SARTSolver(prob.rtm, None, comm, p1, use_fused=True, **kw).solve(gh)
        r2 = SARTSolver(prob.rtm, None, comm, p1, use_fused=False, **kw).solve(gh)
        counts.add(rf)
        counts.add(r2)
        xf, x2 = rf.solution, r2.solution
        x64 = sart_oracle_f64(prob.rtm, gh, 1, logarithmic=args.variant == "log", comm=comm)
        nrm = max(float(np.linalg.norm(x64)), 1e-300)
        ef = comm.all_reduce_scalar(float(np.linalg.norm(xf - x64)) / nrm, op="max")
        e2 = comm.all_reduce_scalar(float(np.linalg.norm(x2 - x64)) / nrm, op="max")
        selfcheck = {"iterations": 1, "rel_fused_vs_f64": ef, "rel_two_pass_vs_f64": e2}
        torch.cuda.empty_cache()
        startup["selfcheck_s"] = round(time.perf_counter() - t_check, 2)
        # the same bounds as the GPU tests: fp32 shards fused <= 1.25x the two-pass error (tests/test_gpu_solver.py);
        # bf16 shards 1.5x (tests/test_gpu_bf16.py: the fused row dots take x as a hi + lo bf16 pair; wide rows of a
        # 32768-row shard measure 1.14-1.27x, profiles/bf16_r4_widths_cw_vs_xl.jsonl)
        bound = 1.5 if args.rtm_dtype == "bf16" else 1.25
        selfcheck["bound"] = bound
        if not ef <= max(bound * e2, 1e-5):
            print(f"bench: fused sweep self-check failed: {selfcheck}", file=sys.stderr, flush=True)
            return 2
        wd.kick("selfcheck")

    for i in range(args.warmup):
        counts.add(runner.solve(g))
        wd.kick(f"warmup {i}")
    torch.cuda.synchronize()
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    iters = 0
    comm_ms = 0.0
    comm_fallbacks = 0
    res = None
    for i in range(args.steps):
        res = runner.solve(g)
        iters += res.iterations
        comm_ms += max(getattr(res, "comm_ms", -1.0), 0.0)
        comm_fallbacks += int(getattr(res, "comm_fallbacks", 0))
        counts.add(res)
        wd.kick(f"step {i}")
    torch.cuda.synchronize()
    comm.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    elapsed = comm.all_reduce_scalar(elapsed, op="max")

    iters_per_s = iters / elapsed
    flop_per_iter = 4.0 * npix_total * nvox_total
    gflops = flop_per_iter * iters_per_s / 1e9
    use_fused = (not multi) and solver.use_fused
    # bytes of A per SART iteration of ONE frame: fused 1 read, two-pass 2 reads, multi-frame 2 reads per batch
    bytes_per_iter = prob.rtm.nbytes * (2.0 / min(solver.batch_width, args.frames) if multi else (1 if use_fused else 2))
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
        "dtype": (_split_a_dtype(solver) if multi and solver.split_a else "fp32") if args.rtm_dtype == "fp32" else (
            "bf16 RTM storage, bf16 MFMA with hi+lo bf16 split of X / W, fp32 accumulation" if multi
            else "bf16 RTM storage; fused row dots on bf16 dot2 with hi+lo split x, fp32 sums"
            if solver.use_fused else "bf16 RTM storage, fp32 compute"),
        "data": "synthetic (on-device random dense RTM, random phantom; no HDF5)",
        "iters_per_s": round(iters_per_s, 3),
        "sart_iterations_per_step": args.iters,
        "status_last": res.status if res else None,
        "fused_sweep": use_fused,
        "fused_variant": solver.geom.variant if use_fused else None,
        "fused_rows_per_tile": solver.geom.T if use_fused else None,
        # the pipeline schedule the sweep kernel actually ran (T, kw and chip-wide groups pick it; the global knob
        # fused_get_schedule() is only the default), recorded by the launcher of the last sweep
        "fused_schedule": solver.k.fused_last_schedule() if use_fused else None,
        "fused_grid": ({"J": solver.geom.J, "I": solver.geom.I, "workgroups": solver.geom.grid,
                        "ld": solver.ld, "kw": solver.geom.kw, "xcd_local": solver.geom.xl} if use_fused else None),
        "selfcheck": selfcheck,
        "shared_gpus": bool(getattr(solver, "shared_device", False)) if not multi else None,
        "fused_plan_cus": solver.plan_cus if use_fused else None,
        "startup": startup,
        "frames_per_step": args.frames,
        # multi-frame operand pieces that ran (f16x2 / bf16x2 / bf16x3 / fp32 / bf16-storage)
        "mf_split": ({"forward": solver.forward_split, "backproject": solver.backproject_split} if multi else None),
        # per-iteration device all-reduce: RCCL, or the one-shot P2P kernel when it beat RCCL at start-up
        "allreduce": (solver.native_comm.describe if n > 1 else "none (1 rank)"),
        # frames re-solved after a device all-reduce timeout / a persistent-sweep timeout, over the whole run
        # (self-check + warm-up + timed steps) and within the timed steps alone
        "allreduce_fallbacks": counts.comm,
        "allreduce_fallbacks_timed": comm_fallbacks,
        "fused_fallbacks": counts.fused,
        # rank 0's GPU time inside the all-reduces per SART iteration (includes waiting for slower ranks)
        "allreduce_us_per_iter": (round(1e3 * comm_ms / max(iters, 1), 2) if n > 1 and not multi else None),
        "effective_hbm_TBps_per_gpu": round(bytes_per_iter * iters_per_s / 1e12, 3),
        "config": {
            "model": f"SART-{args.variant} dense RTM" + (" + Laplacian" if lap is not None else "")
                     + (" multi-frame (MFMA)" if multi else ""),
            "preset": args.config,
            "npixel_total": npix_total,
            "nvoxel": nvox_total,
            "global_batch": args.frames,
            "seq_len": nvox_total,
            "parallelism": (f"{'col' if cols else 'row'}-shard dp{n}" if n > 1 else "single"),
            "partition": args.partition,
            "rtm_GB_per_gpu": round(prob.rtm.nbytes / 1e9, 2),
            "rtm_storage": args.rtm_dtype,
        },
    }
    if comm.rank == 0:
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
