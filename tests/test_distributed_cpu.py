"""Multi-process tests over torch.distributed/gloo (world size 2 and 3) -- the decomposition, the
reductions and the CLI are exercised exactly as on GPUs, with CPU ranks (rendezvous on 127.0.0.1)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir, log, lap):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    from mpi_cuda_sartsolver_amd.models.cpu import CPUSARTSolver
    from mpi_cuda_sartsolver_amd.models.laplacian import LaplacianCSR
    from mpi_cuda_sartsolver_amd.models.sart import SolverParams
    from mpi_cuda_sartsolver_amd.ops import native
    from mpi_cuda_sartsolver_amd.parallel.comm import init_distributed
    from mpi_cuda_sartsolver_amd.parallel.partition import row_partition
    from mpi_cuda_sartsolver_amd.utils.synthetic import host_problem

    native().cpu_set_num_threads(2)
    comm = init_distributed(use_gpu=False)
    A, g, _ = host_problem(301, 125, seed=5, saturate_fraction=0.03)
    b = row_partition(A.shape[0], world, rank)
    L = LaplacianCSR.grid_3d(5, 5, 5) if lap else None
    for semantics in ("cpu", "gpu"):
        s = CPUSARTSolver(A[b.offset:b.stop], L, comm, SolverParams(max_iterations=80, conv_tolerance=1e-8,
                                                                    beta_laplace=1e-3),
                          logarithmic=log, semantics=semantics)
        r = s.solve(g[b.offset:b.stop])
        if rank == 0:
            np.save(os.path.join(out_dir, f"x_{semantics}_{world}.npy"), r.solution)
            with open(os.path.join(out_dir, f"meta_{semantics}_{world}.json"), "w") as f:
                json.dump({"status": r.status, "iterations": r.iterations}, f)
    import torch.distributed as dist

    dist.destroy_process_group()


@pytest.mark.parametrize("log,lap", [(False, False), (True, True)])
def test_cpu_solver_rank_invariance(tmp_path, log, lap):
    for world in (1, 2, 3):
        if world == 1:
            _worker_single(str(tmp_path), log, lap)
        else:
            mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), log, lap), nprocs=world,
                               join=True, start_method="spawn")
    for sem in ("cpu", "gpu"):
        x1 = np.load(tmp_path / f"x_{sem}_1.npy")
        m1 = json.loads((tmp_path / f"meta_{sem}_1.json").read_text())
        for world in (2, 3):
            xw = np.load(tmp_path / f"x_{sem}_{world}.npy")
            mw = json.loads((tmp_path / f"meta_{sem}_{world}.json").read_text())
            np.testing.assert_allclose(xw, x1, rtol=1e-8, atol=1e-12)
            assert abs(mw["iterations"] - m1["iterations"]) <= 1 and mw["status"] == m1["status"]


def _worker_single(out_dir, log, lap):
    from mpi_cuda_sartsolver_amd.models.cpu import CPUSARTSolver
    from mpi_cuda_sartsolver_amd.models.laplacian import LaplacianCSR
    from mpi_cuda_sartsolver_amd.models.sart import SolverParams
    from mpi_cuda_sartsolver_amd.utils.synthetic import host_problem

    A, g, _ = host_problem(301, 125, seed=5, saturate_fraction=0.03)
    L = LaplacianCSR.grid_3d(5, 5, 5) if lap else None
    for semantics in ("cpu", "gpu"):
        s = CPUSARTSolver(A, L, None, SolverParams(max_iterations=80, conv_tolerance=1e-8, beta_laplace=1e-3),
                          logarithmic=log, semantics=semantics)
        r = s.solve(g)
        np.save(os.path.join(out_dir, f"x_{semantics}_1.npy"), r.solution)
        with open(os.path.join(out_dir, f"meta_{semantics}_1.json"), "w") as f:
            json.dump({"status": r.status, "iterations": r.iterations}, f)


def _run_cli(args, nproc, cwd, port):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", HSA_ENABLE_IPC_MODE_LEGACY="0")
    if nproc == 1:
        cmd = [sys.executable, "-m", "mpi_cuda_sartsolver_amd", *args]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "mpi_cuda_sartsolver_amd", *args]
    res = subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stdout + res.stderr
    return res.stdout


def test_cli_cpu_two_ranks_equals_one(tmp_path):
    from mpi_cuda_sartsolver_amd.io.fixtures import make_case
    from mpi_cuda_sartsolver_amd.ops import native

    case = make_case(str(tmp_path / "case"), sparse_cameras=("cam_b",), laplacian=True, nframes=3)
    base = ["--use_cpu", "-m", "150", "-c", "1e-7", "-l", case.laplacian_file, "-b", "1e-3"]
    out1 = _run_cli(base + ["-o", str(tmp_path / "o1.h5"), *case.files], 1, str(tmp_path), 0)
    out2 = _run_cli(base + ["-o", str(tmp_path / "o2.h5"), *case.files], 2, str(tmp_path), _free_port())
    assert out1.count("Processed in:") == 3 and out2.count("Processed in:") == 3
    n = native()
    t1, x1, s1 = n.read_solution_file(str(tmp_path / "o1.h5"))
    t2, x2, s2 = n.read_solution_file(str(tmp_path / "o2.h5"))
    np.testing.assert_array_equal(t1, t2)
    np.testing.assert_array_equal(s1, s2)
    np.testing.assert_allclose(x2, x1, rtol=1e-8)
