#!/usr/bin/env python3
"""Compile-time A/B variants of the HIP module without touching the product build: one kernel source rebuilt with
extra -D flags, linked with the other objects of build/hip into ab/<name>/ (a copy of the package's Python files and
bench.py beside the variant _sart_hip), so `python ab/<name>/bench.py ...` runs the variant on the GPU box.

    python tools/ab_build.py fflush4 -DSART_MF_FLUSH=4 [--src multiframe_bf16.hip]
"""
import argparse
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--src", default="multiframe_bf16.hip")
    a, a.flags = ap.parse_known_args()  # the -D flags
    from mpi_cuda_sartsolver_amd import _build as b

    b.build_hip(verbose=False)  # the product objects first
    objdir = b.BUILDDIR / "hip"
    dst = ROOT / "ab" / a.name
    if dst.exists():
        shutil.rmtree(dst)
    pkg = dst / "mpi_cuda_sartsolver_amd"
    shutil.copytree(ROOT / "mpi_cuda_sartsolver_amd", pkg,
                    ignore=shutil.ignore_patterns("*.so", "*.objs", "__pycache__", "sartsolver", "hdf5"))
    shutil.copy2(ROOT / "bench.py", dst / "bench.py")
    shutil.copytree(ROOT / "tools", dst / "tools", ignore=shutil.ignore_patterns("__pycache__"))
    src = b.CSRC / "kernels" / a.src
    obj = dst / (src.stem + ".o")
    flags = ["-O3", "-std=c++20", "-fPIC", f"--offload-arch={b.ARCH}", "-Wall", "-Wno-unused-function", "-x", "hip",
             "-munsafe-fp-atomics", *a.flags]
    subprocess.run([b._hipcc(), *flags, "-c", str(src), "-o", str(obj)], check=True)
    objs = [str(obj) if o.name == src.stem + ".o" else str(o) for o in sorted(objdir.glob("*.o"))]
    out = pkg / "_lib" / ("_sart_hip" + b._ext_suffix())
    subprocess.run([b._hipcc(), "-shared", "-fPIC", f"--offload-arch={b.ARCH}", *objs, f"-L{b.ROCM / 'lib'}",
                    "-lrccl", "-lrocprofiler-sdk-roctx", "-o", str(out)], check=True)
    obj.unlink()
    print(out)


if __name__ == "__main__":
    main()
