"""Communicators for the per-iteration reductions.

The reference reduces the voxel correction through host memory with CUDA-unaware MPI: D2H copy,
``MPI_Allreduce``, H2D copy, plus a second scalar ``MPI_Allreduce`` every iteration
(reference sartsolver_cuda.cpp:242-255). Here one collective per iteration runs on device buffers:

* :class:`TorchDistComm` -- ``torch.distributed`` process group for the Python layer's host-side collectives
  (scalars, barriers, object exchange; gloo by default). The per-iteration device collectives belong to the
  native engine's communicator (:func:`native_communicator`): RCCL over xGMI (``device_backend == "rccl"``,
  one process per GPU), brought up once per process by the engine -- or staged through host memory
  (``"staged"``: several ranks sharing one GPU in the tests, or every rank after a failed RCCL bring-up).
* :class:`SingleProcessComm` -- world size 1, every collective is the identity.

The scalar ``||A x||^2`` rides in the same buffer as the correction vector (one collective, not two).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist


class Communicator:
    rank: int = 0
    world_size: int = 1

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:  # in place
        raise NotImplementedError

    def all_reduce_scalar(self, v: float, op: str = "sum") -> float:
        raise NotImplementedError

    def barrier(self) -> None:
        pass

    def broadcast_object(self, obj, src: int = 0):
        return obj

    def all_gather_object(self, obj) -> list:
        return [obj]

    @property
    def is_root(self) -> bool:
        return self.rank == 0


class SingleProcessComm(Communicator):
    def all_reduce_(self, t, op="sum"):
        return t

    def all_reduce_scalar(self, v, op="sum"):
        return float(v)


_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}


class TorchDistComm(Communicator):
    """Wraps an initialised torch.distributed process group."""

    def __init__(self, group: Optional[dist.ProcessGroup] = None, device: Optional[torch.device] = None,
                 device_backend: Optional[str] = None):
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialised")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        # the native engine's device collectives: "rccl" or "staged" (default: follow the process group)
        self.device_backend = device_backend or ("rccl" if self.backend == "nccl" else "staged")
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu")
        self.device = device

    def all_reduce_(self, t, op="sum"):
        if self.world_size > 1:
            dist.all_reduce(t, op=_OPS[op], group=self.group)
        return t

    def all_reduce_scalar(self, v, op="sum"):
        if self.world_size == 1:
            return float(v)
        dev = self.device if self.backend == "nccl" else torch.device("cpu")
        t = torch.tensor([float(v)], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=_OPS[op], group=self.group)
        return float(t.item())

    def barrier(self):
        if self.world_size > 1:
            if self.backend == "nccl" and self.device is not None and self.device.type == "cuda":
                dist.barrier(group=self.group, device_ids=[self.device.index])
            else:
                dist.barrier(group=self.group)

    def broadcast_object(self, obj, src=0):
        if self.world_size == 1:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=src, group=self.group)
        return lst[0]

    def all_gather_object(self, obj):
        if self.world_size == 1:
            return [obj]
        out = [None] * self.world_size
        dist.all_gather_object(out, obj, group=self.group)
        return out


def env_world() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from torchrun / MPI-style environment variables."""
    rank = int(os.environ.get("RANK", os.environ.get("OMPI_COMM_WORLD_RANK", os.environ.get("PMI_RANK", "0"))))
    world = int(os.environ.get("WORLD_SIZE", os.environ.get("OMPI_COMM_WORLD_SIZE", os.environ.get("PMI_SIZE", "1"))))
    local = int(os.environ.get("LOCAL_RANK", os.environ.get("OMPI_COMM_WORLD_LOCAL_RANK", str(rank))))
    return rank, world, local


def init_distributed(use_gpu: bool = True, timeout_s: float = 1800.0) -> Communicator:
    """One process per GPU (torchrun). Rank -> GPU is LOCAL_RANK (reference: rank % device_count,
    sartsolver_cuda.cpp:96-98). World size 1 needs no process group at all."""
    import datetime

    rank, world, local = env_world()
    gpu = use_gpu and torch.cuda.is_available()
    if gpu:
        ndev = torch.cuda.device_count()
        torch.cuda.set_device(local % ndev)
    if world == 1:
        return SingleProcessComm()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    # Device collectives: the engine's own RCCL communicator (one per process, brought up by the engine; a failed
    # bring-up on any rank leaves every rank on staged collectives + P2P, csrc/engine/comm.cpp make_rccl_comm).
    # SART_DIST_BACKEND=gloo / tcp: staged from the start (several ranks sharing ONE GPU in the tests: RCCL refuses
    # two ranks on one device). The process group only carries the Python layer's host-side collectives, over gloo,
    # so RCCL is not brought up a second time by torch; SART_DIST_BACKEND=nccl puts the group on RCCL as well.
    env = os.environ.get("SART_DIST_BACKEND", "")
    device_backend = "staged" if (not gpu or env in ("gloo", "tcp")) else "rccl"
    backend = "nccl" if (gpu and env == "nccl") else "gloo"
    if not dist.is_initialized():
        kwargs = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kwargs["device_id"] = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group(**kwargs)
    dev = torch.device("cuda", torch.cuda.current_device()) if gpu else None
    return TorchDistComm(device=dev, device_backend=device_backend)


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("", 0))
        return s.getsockname()[1]


def native_communicator(comm: Optional[Communicator], device: int = 0):
    """The native engine's communicator (csrc/engine/comm.hpp) for a Python communicator, created once
    per process group and cached on it:

    * world size 1 -> ``LocalComm``;
    * ``device_backend == "rccl"`` -> the engine's own RCCL communicator over xGMI (unique id handed out through
      the process group) with a TCP side channel for host scalars; if RCCL fails to come up on any rank, every
      rank gets the staged communicator instead (``describe`` says so);
    * ``"staged"`` -> staged communicator (device buffers staged through the TCP host communicator,
      reductions in fixed rank order), e.g. several ranks sharing one GPU in tests;
    * both wrapped in the one-shot P2P all-reduce (csrc/kernels/p2p_allreduce.hip) per ``SART_P2P``:
      ``auto`` (default; RCCL groups only: used when faster than RCCL at the engine's message size),
      ``1`` (forced, also over gloo), ``0`` (off). ``native.describe`` says what was chosen and why.
    """
    from ..ops import hip

    k = hip()
    if comm is None or comm.world_size == 1:
        return k.local_comm()
    cached = getattr(comm, "_native_comm", None)
    if cached is not None:
        return cached
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = comm.broadcast_object(_free_port() if comm.rank == 0 else None, src=0)
    p2p = os.environ.get("SART_P2P", "auto")
    device_backend = getattr(comm, "device_backend", "rccl" if getattr(comm, "backend", "gloo") == "nccl" else "staged")
    if device_backend == "rccl":
        uid = comm.broadcast_object(k.rccl_unique_id() if comm.rank == 0 else None, src=0)
        native = k.rccl_comm(device, uid, comm.rank, comm.world_size, host, int(port))
        if p2p not in ("0", "off"):  # one-shot P2P all-reduce over xGMI (self-tested, timed against RCCL)
            native = k.p2p_comm(device, native)
    else:
        native = k.staged_comm(comm.rank, comm.world_size, host, int(port))
        # several ranks sharing one GPU (tests): exercise the P2P kernel path (SART_P2P_WRAP_STAGED=1 also
        # runs the auto selection against the staged base)
        if p2p in ("1", "on") or os.environ.get("SART_P2P_WRAP_STAGED") == "1":
            native = k.p2p_comm(device, native)
    comm._native_comm = native
    return native


def native_host_communicator(comm: Optional[Communicator]):
    """Host-only collectives for the native CPU solver (csrc/native/host_comm.hpp): local for one rank,
    TCP (fixed rank order) otherwise. Cached on the process group."""
    from ..ops import native

    n = native()
    if comm is None or comm.world_size == 1:
        return n.local_host_comm()
    cached = getattr(comm, "_native_host_comm", None)
    if cached is not None:
        return cached
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = comm.broadcast_object(_free_port() if comm.rank == 0 else None, src=0)
    hc = n.tcp_host_comm(comm.rank, comm.world_size, host, int(port))
    comm._native_host_comm = hc
    return hc


def abort_all(msg: str, code: int = 1) -> None:
    """Fatal error in a multi-rank run: tear the group down instead of a bare exit that leaves the
    peers blocked in a collective (reference exits per rank: sartsolver_cuda.cpp:45-75)."""
    import sys

    print(msg, file=sys.stderr, flush=True)
    try:
        if dist.is_initialized():
            dist.destroy_process_group()
    finally:
        os._exit(code)
