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

Signals: launchers stop their workers with SIGTERM (torchrun, mpiexec) or SIGINT / SIGHUP. This process forwards
each of them to the driver and waits for it, so the driver never outlives its launcher holding a GPU or blocked
in a collective; the driver also asks the kernel for SIGTERM should this process die without forwarding
(``SART_PARENT_PID``, PR_SET_PDEATHSIG in sartsolver_main.cpp).
"""
from __future__ import annotations

import os
import signal
import subprocess
import threading
import sys
from pathlib import Path

FORWARDED = (signal.SIGTERM, signal.SIGINT, signal.SIGHUP)


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
    env["SART_PARENT_PID"] = str(os.getpid())  # the driver exits if this process is already gone at its start
    sys.stdout.flush()
    sys.stderr.flush()
    proc = subprocess.Popen([str(binary), *argv], env=env, close_fds=False)
    received: list[int] = []

    def forward(signum, _frame):
        received.append(signum)
        try:
            proc.send_signal(signum)
        except ProcessLookupError:
            pass

    # signal handlers can only be installed from the main thread: elsewhere (main() called from a worker thread)
    # the driver is simply waited for; any failure while setting up kills and reaps the child instead of leaving it
    previous = {}
    try:
        if threading.current_thread() is threading.main_thread():
            for s in FORWARDED:
                previous[s] = signal.signal(s, forward)
        while True:
            try:
                rc = proc.wait()
                break
            except InterruptedError:  # pragma: no cover - PEP 475 retries wait() itself
                continue
    except BaseException:
        if proc.poll() is None:
            proc.kill()
        proc.wait()
        raise
    finally:
        for s, h in previous.items():
            signal.signal(s, h)
    if rc < 0 and received:  # killed by the forwarded signal: report it like a shell does
        return 128 - rc
    return rc


if __name__ == "__main__":
    sys.exit(main())
