"""MPI host collectives against both MPI ABIs (csrc/native/host_comm_mpi.cpp).

The reference's deployment stack is Open MPI 4.1.0 (reference README.md:42-44); MPICH-family launches are
covered end to end by tests/test_native_driver.py (mpiexec). Open MPI is not installed here, so a fake
libmpi of each ABI (tests/fake_mpi/fake_mpi.c: one process posing as rank 0 of 2, the peer adding 1 to SUM
and 100 to MAX elements, every handle checked) verifies that the right handles, MPI_IN_PLACE value,
datatype and operation reach the library."""
import json
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "fake_mpi", "fake_mpi.c")

PROBE = r"""
import json, numpy as np
from mpi_cuda_sartsolver_amd.ops import native
n = native()
c = n.mpi_host_comm()
d = c.all_reduce_host(np.array([1.0, 2.0]), n.ReduceOp.SUM)
m = c.all_reduce_host(np.array([5.0, 200.0]), n.ReduceOp.MAX)
f = c.all_reduce_host_f32(np.array([0.5, 3.0], dtype=np.float32), n.ReduceOp.SUM)
b = c.broadcast_bytes(b"abc", 3, 0)
c.barrier()
print(json.dumps(dict(rank=c.rank, size=c.size, backend=c.backend, version=n.mpi_library_version(),
                      d=d.tolist(), m=m.tolist(), f=f.tolist(), b=b.decode())))
"""


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
@pytest.mark.parametrize("abi", ["openmpi", "mpich"])
def test_mpi_host_comm_abi(tmp_path, abi):
    lib = tmp_path / f"libfake_{abi}.so"
    flags = ["-DOMPI_ABI"] if abi == "openmpi" else []
    subprocess.run(["gcc", "-shared", "-fPIC", "-O1", *flags, "-o", str(lib), SRC], check=True)
    env = dict(os.environ, PYTHONPATH=ROOT, SART_MPI_LIB=str(lib))
    r = subprocess.run([sys.executable, "-c", PROBE], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert (out["rank"], out["size"]) == (0, 2)
    assert out["backend"] == ("mpi(openmpi)" if abi == "openmpi" else "mpi")
    assert ("Open MPI" in out["version"]) == (abi == "openmpi")
    assert out["d"] == [2.0, 3.0] and out["m"] == [100.0, 200.0] and out["f"] == [1.5, 4.0]
    assert out["b"] == "abc"


def test_launcher_detection():
    probe = "from mpi_cuda_sartsolver_amd.ops import native; print(native().mpi_launch_detected())"
    base = {k: v for k, v in os.environ.items() if k not in ("RANK", "PMI_SIZE", "OMPI_COMM_WORLD_SIZE",
                                                               "SART_HOST_COMM")}
    for extra, expect in (({"OMPI_COMM_WORLD_SIZE": "4"}, "True"), ({"PMI_SIZE": "2"}, "True"),
                          ({"OMPI_COMM_WORLD_SIZE": "4", "RANK": "0"}, "False"), ({}, "False")):
        env = dict(base, PYTHONPATH=ROOT, **extra)
        r = subprocess.run([sys.executable, "-c", probe], env=env, capture_output=True, text=True, timeout=60)
        assert r.stdout.strip() == expect, (extra, r.stdout, r.stderr)


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_mpi_world_must_match_launcher(tmp_path):
    """A libmpi of the other family initialises as a singleton (every process rank 0 of 1) instead of joining the
    launcher's world: the world size is checked against OMPI_COMM_WORLD_SIZE / PMI_SIZE and a mismatch is an error
    naming SART_MPI_LIB (the fake library reports a world of 2)."""
    lib = tmp_path / "libfake_openmpi.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-O1", "-DOMPI_ABI", "-o", str(lib), SRC], check=True)
    base = {k: v for k, v in os.environ.items() if k not in ("RANK", "PMI_SIZE", "OMPI_COMM_WORLD_SIZE")}
    probe = "from mpi_cuda_sartsolver_amd.ops import native; c = native().mpi_host_comm(); print(c.size)"
    for extra, ok in (({"OMPI_COMM_WORLD_SIZE": "2"}, True), ({"OMPI_COMM_WORLD_SIZE": "4"}, False),
                      ({"PMI_SIZE": "3"}, False)):
        env = dict(base, PYTHONPATH=ROOT, SART_MPI_LIB=str(lib), **extra)
        r = subprocess.run([sys.executable, "-c", probe], env=env, capture_output=True, text=True, timeout=120)
        if ok:
            assert r.returncode == 0 and r.stdout.strip() == "2", r.stderr[-2000:]
        else:
            assert r.returncode != 0 and "SART_MPI_LIB" in r.stderr, (extra, r.stderr[-2000:])
