"""In-tree build of the native extension modules.

* ``_sart_hip``    -- hand-written gfx950 HIP kernels (csrc/kernels/*.hip) + pybind11 glue, built with
                      ``hipcc --offload-arch=gfx950``. Links only against the HIP runtime.
* ``_sart_native`` -- host C++17 runtime: CLI/config parser, time intervals, HDF5 I/O (C API of the
                      HDF5 1.10 library under /opt/conda), composite-image streamer, solution writer,
                      voxel grids and the fp64 multithreaded CPU solver kernels.

Both land in ``mpi_cuda_sartsolver_amd/_lib`` so they travel with the repository snapshot to the GPU
box (the reference builds one binary with GNU make, reference Makefile:47-96).
Objects are cached under ``build/`` keyed by a hash of the source, the shared headers and the flags.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import json
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
LIBDIR = Path(__file__).resolve().parent / "_lib"
# SART_BUILD_DEBUG=1: kernels and engine with -O1 -g (device line info for rocprofv3 / printf debugging, with
# HIP_LAUNCH_BLOCKING=1 AMD_SERIALIZE_KERNEL=3 at run time), objects under build-debug/. The
# modules land in the same _lib/ as the optimised build: rebuild without the variable afterwards.
DEBUG = os.environ.get("SART_BUILD_DEBUG") == "1"
BUILDDIR = ROOT / ("build-debug" if DEBUG else "build")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("SART_OFFLOAD_ARCH", "gfx950")

HDF5_PREFIX = Path(os.environ.get("SART_HDF5_PREFIX", "/opt/conda"))


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _py_includes() -> list[str]:
    import pybind11

    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm is required to build the gfx950 kernels)")


def _digest(paths: list[Path], flags: list[str]) -> str:
    h = hashlib.sha256()
    for p in paths:
        h.update(p.read_bytes())
    h.update("\0".join(flags).encode())
    return h.hexdigest()[:24]


def _compile_many(jobs: list[tuple[list[str], Path, str]], verbose: bool) -> None:
    """jobs: (command, object path, digest). Skips objects whose digest stamp matches."""
    todo = []
    for cmd, obj, dig in jobs:
        stamp = obj.with_suffix(obj.suffix + ".stamp")
        if obj.exists() and stamp.exists() and stamp.read_text() == dig:
            continue
        todo.append((cmd, obj, dig, stamp))
    if not todo:
        return

    def run(job):
        cmd, obj, dig, stamp = job
        if verbose:
            print("[build]", " ".join(cmd[:2]), obj.name, flush=True)
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"compile failed for {obj.name}:\n{' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
        stamp.write_text(dig)

    workers = min(len(todo), max(1, min(8, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(workers) as ex:
        for f in [ex.submit(run, j) for j in todo]:
            f.result()


def _link(cmd: list[str], out: Path, objs: list[Path], verbose: bool) -> None:
    # relink when an object is newer than the output or the output came from another object set (the debug
    # build writes the same modules from build-debug/)
    newest = max(o.stat().st_mtime for o in objs)
    stamp = out.with_name(out.name + ".objs")
    key = "\n".join(str(o) for o in objs)
    if out.exists() and out.stat().st_mtime >= newest and stamp.exists() and stamp.read_text() == key:
        return
    if verbose:
        print("[link]", out.name, flush=True)
    tmp = out.with_name(out.name + ".tmp")
    res = subprocess.run(cmd[:-1] + [str(tmp)], capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"link failed for {out.name}:\n{' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    os.replace(tmp, out)
    stamp.write_text(key)


def build_hip(verbose: bool = True) -> Path:
    hipcc = _hipcc()
    objdir = BUILDDIR / "hip"
    objdir.mkdir(parents=True, exist_ok=True)
    LIBDIR.mkdir(parents=True, exist_ok=True)
    headers = (sorted((CSRC / "kernels").glob("*.hpp")) + sorted((CSRC / "engine").glob("*.hpp")) +
               sorted((CSRC / "native").glob("*.hpp")))
    common = ["-O1" if DEBUG else "-O3", "-std=c++20", "-fPIC", f"--offload-arch={ARCH}", "-Wall",
              "-Wno-unused-function"] + (["-g", "-DSART_DEBUG=1"] if DEBUG else [])
    jobs = []
    objs = []
    for src in sorted((CSRC / "kernels").glob("*.hip")):
        flags = common + ["-x", "hip", "-munsafe-fp-atomics"]
        obj = objdir / (src.stem + ".o")
        jobs.append(([hipcc, *flags, "-c", str(src), "-o", str(obj)], obj, _digest([src, *headers], flags)))
        objs.append(obj)
    # native engine (host C++ on the HIP runtime + RCCL): csrc/engine
    eflags = ["-O0" if DEBUG else "-O2", "-std=c++17", "-fPIC", "-Wall", "-D__HIP_PLATFORM_AMD__",
              f"-I{ROCM / 'include'}"] + (["-g"] if DEBUG else [])
    for src in sorted((CSRC / "engine").glob("*.cpp")) + [CSRC / "native" / "host_comm.cpp",
                                                          CSRC / "native" / "host_comm_mpi.cpp",
                                                          CSRC / "native" / "solver_params.cpp"]:
        obj = objdir / ("engine_" + src.stem + ".o")
        jobs.append(([hipcc, *eflags, "-c", str(src), "-o", str(obj)], obj, _digest([src, *headers], eflags)))
        objs.append(obj)
    bind = CSRC / "bindings" / "hip_module.cpp"
    bflags = ["-O2", "-std=c++17", "-fPIC", *[f"-I{p}" for p in _py_includes()], "-D__HIP_PLATFORM_AMD__"]
    bobj = objdir / "hip_module.o"
    jobs.append(([hipcc, *bflags, "-c", str(bind), "-o", str(bobj)], bobj, _digest([bind, *headers], bflags)))
    objs.append(bobj)
    _compile_many(jobs, verbose)
    out = LIBDIR / ("_sart_hip" + _ext_suffix())
    _link([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), f"-L{ROCM / 'lib'}", "-lrccl",
           "-lrocprofiler-sdk-roctx", "-o", str(out)], out, objs, verbose)
    return out


def hdf5_available() -> bool:
    return (HDF5_PREFIX / "include" / "hdf5.h").exists() and (HDF5_PREFIX / "lib" / "libhdf5.so").exists()


def build_native(verbose: bool = True) -> Path:
    cxx = os.environ.get("CXX", shutil.which("g++") or "g++")
    objdir = BUILDDIR / "native"
    objdir.mkdir(parents=True, exist_ok=True)
    LIBDIR.mkdir(parents=True, exist_ok=True)
    srcdir = CSRC / "native"
    headers = sorted(srcdir.glob("*.hpp"))
    flags = ["-O3", "-std=c++17", "-fPIC", "-fopenmp", "-ffp-contract=off", "-Wall", "-Wno-sign-compare",
             *[f"-I{p}" for p in _py_includes()], f"-I{srcdir}"]
    libs = ["-fopenmp"]
    if hdf5_available():
        flags += ["-DSART_HAVE_HDF5=1", f"-isystem{HDF5_PREFIX / 'include'}"]
        # no rpath into /opt/conda/lib: it would also redirect libstdc++ to conda's older copy. The
        # loader (ops.native) preloads libhdf5 by absolute path instead.
        libs += [f"-L{HDF5_PREFIX / 'lib'}", "-lhdf5"]
    jobs, objs = [], []
    for src in sorted(srcdir.glob("*.cpp")) + [CSRC / "bindings" / "native_module.cpp"]:
        obj = objdir / (src.stem + ".o")
        jobs.append(([cxx, *flags, "-c", str(src), "-o", str(obj)], obj, _digest([src, *headers], flags)))
        objs.append(obj)
    _compile_many(jobs, verbose)
    out = LIBDIR / ("_sart_native" + _ext_suffix())
    _link([cxx, "-shared", "-fPIC", *map(str, objs), *libs, "-o", str(out)], out, objs, verbose)
    return out


def build_driver(verbose: bool = True) -> Path:
    """Native ``sartsolver`` executable (csrc/driver): the GPU kernels and engine objects of build_hip,
    the host runtime objects of build_native (g++/OpenMP) and the driver, linked with hipcc against
    the HIP runtime, RCCL, HDF5 and libgomp. HDF5 is found through a private RUNPATH directory that
    holds only libhdf5 (conda's libstdc++ must not shadow the system one)."""
    if not hdf5_available():
        raise RuntimeError("the native driver needs HDF5 (SART_HDF5_PREFIX)")
    build_native(verbose)
    build_hip(verbose)
    hipcc = _hipcc()
    objdir = BUILDDIR / "driver"
    objdir.mkdir(parents=True, exist_ok=True)
    headers = (sorted((CSRC / "kernels").glob("*.hpp")) + sorted((CSRC / "engine").glob("*.hpp")) +
               sorted((CSRC / "native").glob("*.hpp")))
    src = CSRC / "driver" / "sartsolver_main.cpp"
    dflags = ["-O2", "-std=c++17", "-Wall", "-D__HIP_PLATFORM_AMD__", "-DSART_HAVE_HDF5=1",
              f"-isystem{HDF5_PREFIX / 'include'}", f"-I{ROCM / 'include'}"]
    dobj = objdir / "sartsolver_main.o"
    _compile_many([([hipcc, *dflags, "-c", str(src), "-o", str(dobj)], dobj, _digest([src, *headers], dflags))],
                  verbose)
    hip_objs = [o for o in sorted((BUILDDIR / "hip").glob("*.o")) if o.name != "hip_module.o"]
    native_objs = [o for o in sorted((BUILDDIR / "native").glob("*.o"))
                   if o.name not in ("native_module.o", "host_comm.o", "host_comm_mpi.o", "solver_params.o")]
    objs = [dobj, *hip_objs, *native_objs]
    libdir = LIBDIR / "hdf5"  # private RUNPATH entry: only libhdf5
    libdir.mkdir(parents=True, exist_ok=True)
    for so in HDF5_PREFIX.joinpath("lib").glob("libhdf5.so.*"):
        if so.name.count(".") == 2:  # libhdf5.so.<soversion>
            link = libdir / so.name
            if not link.exists():
                link.symlink_to(so)
    out = LIBDIR / "sartsolver"
    # libhdf5 by path, not -L: a -L/opt/conda/lib would also resolve libstdc++ to conda's older copy
    _link([hipcc, f"--offload-arch={ARCH}", *map(str, objs), f"-L{ROCM / 'lib'}", "-lrccl",
           "-lrocprofiler-sdk-roctx", str(HDF5_PREFIX / "lib" / "libhdf5.so"), "-lgomp", "-lpthread", "-ldl",
           "-Wl,-rpath,$ORIGIN/hdf5", f"-Wl,-rpath,{ROCM / 'lib'}", "-o", str(out)], out, objs, verbose)
    return out


def build_all(verbose: bool = True) -> list[Path]:
    outs = [build_native(verbose)]
    outs.append(build_hip(verbose))
    if hdf5_available():
        outs.append(build_driver(verbose))
    return outs


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    {"hip": build_hip, "native": build_native, "driver": build_driver, "all": build_all}[what]()
    print(json.dumps({"ok": True}))
