#!/usr/bin/env python3
"""Device all-reduce equivalence check (SURVEY §7.4 tests/comm): run under torchrun with N ranks; every
rank reduces rank-dependent fp32 data of many sizes through the engine's native communicator and compares
the result BITWISE with the rank-order sum ((v0 + v1) + v2) + ... (sum) or the maximum, which is what the
one-shot P2P kernel computes on every rank. Rank 0 writes a JSON summary (--out)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--sizes", default="1,3,4,7,1023,1024,1025,4096,65537,300001,524288,600000")
    ap.add_argument("--time-n", type=int, default=65537)
    a = ap.parse_args()
    import torch

    from mpi_cuda_sartsolver_amd.ops import hip
    from mpi_cuda_sartsolver_amd.parallel.comm import init_distributed, native_communicator

    comm = init_distributed(use_gpu=True)
    dev = torch.device("cuda", torch.cuda.current_device())
    k = native_communicator(comm, dev.index)
    ops = hip().ReduceOp
    stream = torch.cuda.current_stream().cuda_stream
    W, R = comm.world_size, comm.rank
    results = []
    cases = [(int(s), op, 0) for s in a.sizes.split(",") for op in ("sum", "max")]
    cases += [(n, "sum", 1) for n in (5, 4097)]  # buffer offset by one element: not 16-B aligned
    # announce the message sizes like an engine does (SART_P2P=auto times P2P against the base at exactly these)
    t_prep = time.perf_counter()
    k.prepare(sorted({n for n, _, _ in cases} | {a.time_n}))
    prepare_s = time.perf_counter() - t_prep
    for n, op, off in cases:
        data = [torch.randn(n, generator=torch.Generator().manual_seed(1000 * r + n), dtype=torch.float32)
                for r in range(W)]
        want = data[0].clone()
        for r in range(1, W):
            want = want + data[r] if op == "sum" else torch.maximum(want, data[r])
        store = torch.zeros(n + off, device=dev)
        buf = store[off:]
        buf.copy_(data[R].to(dev))
        torch.cuda.synchronize()
        k.all_reduce_device(buf.data_ptr(), n, False, ops.SUM if op == "sum" else ops.MAX, stream)
        torch.cuda.synchronize()
        got = buf.cpu()
        results.append(dict(n=n, op=op, offset=off, exact=bool(torch.equal(got, want)),
                            close=bool(torch.allclose(got, want, rtol=1e-5, atol=1e-5))))
    k.check()
    # latency at the engine's message size (64k voxels + the piggy-backed scalar)
    buf = torch.zeros(a.time_n, device=dev)
    for _ in range(5):
        k.all_reduce_device(buf.data_ptr(), a.time_n, False, ops.SUM, stream)
    torch.cuda.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    reps = 50
    for _ in range(reps):
        k.all_reduce_device(buf.data_ptr(), a.time_n, False, ops.SUM, stream)
    torch.cuda.synchronize()
    us = 1e6 * (time.perf_counter() - t0) / reps
    if R == 0:
        with open(a.out, "w") as f:
            json.dump(dict(world=W, backend=k.backend, describe=k.describe, results=results, us_per_call=us,
                           setup_s=k.setup_seconds, prepare_s=prepare_s), f)
    comm.barrier()


if __name__ == "__main__":
    main()
