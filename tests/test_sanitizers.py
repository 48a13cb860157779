"""Host runtime under AddressSanitizer + UndefinedBehaviorSanitizer (csrc/tests/host_selftest.cpp)."""
import os
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
NATIVE = ROOT / "csrc" / "native"


def test_host_runtime_asan_ubsan(tmp_path):
    from mpi_cuda_sartsolver_amd import _build

    if not _build.hdf5_available():
        pytest.skip("HDF5 not available")
    exe = tmp_path / "host_selftest"
    srcs = [ROOT / "csrc" / "tests" / "host_selftest.cpp"] + [
        NATIVE / f for f in ("config.cpp", "cpu_kernels.cpp", "cpu_solver.cpp", "fixtures.cpp", "frames.cpp", "h5.cpp",
                             "host_comm.cpp", "host_comm_mpi.cpp", "inputs.cpp", "solver_params.cpp",
                             "sparse_csr.cpp")]
    hdf5 = _build.HDF5_PREFIX
    libdir = tmp_path / "hdf5"
    libdir.mkdir()
    for so in (hdf5 / "lib").glob("libhdf5.so.*"):
        if so.name.count(".") == 2:
            (libdir / so.name).symlink_to(so)
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-fopenmp", "-DSART_HAVE_HDF5=1", f"-isystem{hdf5 / 'include'}",
           *map(str, srcs), str(hdf5 / "lib" / "libhdf5.so"), "-ldl", f"-Wl,-rpath,{libdir}", "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    # verify_asan_link_order=0: the environment may preload libraries ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               OMP_NUM_THREADS="2", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-6000:]
    assert "host selftest OK" in r.stdout
