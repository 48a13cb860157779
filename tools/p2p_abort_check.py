#!/usr/bin/env python3
"""Failure propagation of the P2P all-reduce: two ranks on one GPU; rank 1 aborts its
communicator after a few all-reduces and exits, rank 0 enters the next all-reduce and must fail fast (the
abort word that rank 1 wrote into rank 0's memory ends the poll) instead of waiting for SART_P2P_TIMEOUT_S.

    python tools/p2p_abort_check.py --out result.json      # launches both ranks itself
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(out):
    import torch

    from mpi_cuda_sartsolver_amd.ops import hip
    from mpi_cuda_sartsolver_amd.parallel.comm import init_distributed, native_communicator

    comm = init_distributed(use_gpu=True)
    dev = torch.device("cuda", torch.cuda.current_device())
    k = native_communicator(comm, dev.index)
    stream = torch.cuda.current_stream().cuda_stream
    buf = torch.ones(65537, device=dev)
    for _ in range(3):
        k.all_reduce_device(buf.data_ptr(), buf.numel(), False, hip().ReduceOp.SUM, stream)
    torch.cuda.synchronize()
    k.check()
    ok = bool(torch.all(buf == 8.0).item())  # 1 -> 2 -> 4 -> 8 with two ranks
    if comm.rank == 1:
        k.abort()
        time.sleep(10.0)  # keep the exported buffers alive while rank 0 still pushes into them
        os._exit(3)
    time.sleep(1.0)  # rank 1 is gone (or going) when rank 0 enters the next all-reduce
    t0 = time.perf_counter()
    k.all_reduce_device(buf.data_ptr(), buf.numel(), False, hip().ReduceOp.SUM, stream)
    torch.cuda.synchronize()
    err = ""
    try:
        k.check()
    except RuntimeError as e:
        err = str(e)
    res = dict(backend=k.backend, first_ok=ok, error=err, seconds=time.perf_counter() - t0,
               nan=bool(torch.isnan(buf).any().item()))
    with open(out, "w") as f:
        json.dump(res, f)
    os._exit(0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--worker", action="store_true")
    a = ap.parse_args()
    if a.worker:
        worker(a.out)
        return
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), SART_DIST_BACKEND="gloo", SART_P2P="1", SART_P2P_TIMEOUT_S="120",
                   HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONPATH=ROOT)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "--worker", "--out", a.out],
                                      env=env))
    codes = [p.wait(timeout=300) for p in procs]
    print(json.dumps(dict(exit_codes=codes)))
    sys.exit(0 if codes == [0, 3] else 1)


if __name__ == "__main__":
    main()
