"""``sartsolver`` command-line driver: ``python -m mpi_cuda_sartsolver_amd [options] input_files...``.

A thin launcher of the native driver (csrc/driver/sartsolver_main.cpp, built into
``mpi_cuda_sartsolver_amd/_lib/sartsolver``), so the frame loop -- input validation, row / column shards,
streamed HDF5 -> HBM loads, frame prefetch, warm starts, ``--batch_frames``, ``--resume``, ``--profile`` -- exists
once (reference main.cpp:25-151). The executable runs as a child process with this process's arguments and
environment and its exit code is returned; this process touches no GPU.

Ranks: one process per GPU, started by ``torchrun`` (``python -m torch.distributed.run --nproc-per-node 8 -m
mpi_cuda_sartsolver_amd ...``: every rank's child reads RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR /
MASTER_PORT) or by ``mpiexec`` (PMI_* / OMPI_* variables; the launcher's file descriptors stay open for the
child, so PMI reaches it), like the reference's ``mpirun`` (reference main.cpp:63-68). The Python solver API
(``models.sart.SARTSolver``, ``models.multiframe.MultiFrameSARTSolver``, ``models.cpu.CPUSARTSolver``) drives the
same native engines for programmatic use.
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path


def driver_binary() -> Path:
    """The native driver executable built in-tree by ``mpi_cuda_sartsolver_amd._build``."""
    return Path(__file__).resolve().parent / "_lib" / "sartsolver"


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    binary = driver_binary()
    if not os.access(binary, os.X_OK):
        print(f"sartsolver: the native driver is not built ({binary}); run python -m mpi_cuda_sartsolver_amd._build",
              file=sys.stderr, flush=True)
        return 1
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (P2P all-reduce, RCCL) on this platform
    sys.stdout.flush()
    sys.stderr.flush()
    return subprocess.run([str(binary), *argv], env=env, close_fds=False).returncode


if __name__ == "__main__":
    sys.exit(main())
