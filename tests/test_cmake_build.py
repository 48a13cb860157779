"""The CMake build (CMakeLists.txt, alternative to mpi_cuda_sartsolver_amd/_build.py) configures, compiles
every source for gfx950 and links the native driver (compile and link only: no GPU needed)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("cmake") is None or not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs cmake and ROCm")
def test_cmake_builds_sartsolver(tmp_path):
    b = tmp_path / "cmake"
    gen = ["-G", "Ninja"] if shutil.which("ninja") else []
    r = subprocess.run(["cmake", "-S", ROOT, "-B", str(b), *gen, "-DCMAKE_HIP_ARCHITECTURES=gfx950",
                        "-DCMAKE_BUILD_TYPE=Release"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    r = subprocess.run(["cmake", "--build", str(b), "-j8", "--target", "sartsolver"], capture_output=True,
                       text=True, timeout=1200)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    exe = b / "sartsolver"
    assert exe.exists()
    r = subprocess.run([str(exe), "--help"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "input_files" in r.stdout
