"""Native engine pieces that run without a GPU: the TCP communicator (csrc/engine/comm.cpp) across
processes, and the C++ fused-sweep geometry against the Python one (models/rtm.py)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _tcp_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    from mpi_cuda_sartsolver_amd.ops import hip

    if rank % 2:  # the device communicator's host side (staged) and the native host communicator interoperate
        k = hip()
        c = k.staged_comm(rank, world, "127.0.0.1", port, 60.0)
    else:
        from mpi_cuda_sartsolver_amd.ops import native

        k = native()
        c = k.tcp_host_comm(rank, world, "127.0.0.1", port, 60.0)
    v = np.arange(5, dtype=np.float64) * (rank + 1) + 0.1 * rank
    s = c.all_reduce_host(v, k.ReduceOp.SUM)
    m = c.all_reduce_host(np.array([float(rank), -float(rank)]), k.ReduceOp.MAX)
    b = c.broadcast_bytes(b"hello from 1" if rank == 1 else b"", 12, 1)
    c.barrier()
    q.put((rank, s.tolist(), m.tolist(), b))


@pytest.mark.parametrize("world", [2, 3])
def test_tcp_comm_collectives(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_tcp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    expect = sum(np.arange(5) * (r + 1) + 0.1 * r for r in range(world))
    for rank, s, m, b in out:
        np.testing.assert_array_equal(s, out[0][1])  # bitwise identical on every rank
        np.testing.assert_allclose(s, expect, rtol=1e-15)
        assert m == [world - 1.0, 0.0]
        assert b == b"hello from 1"
