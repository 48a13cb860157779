"""Loaders for the native extension modules.

``hip()``    -> the gfx950 HIP kernel module (``_sart_hip``); raises if it is missing -- there is no
               silent eager/PyTorch fallback for any hot op.
``native()`` -> the host C++ runtime module (``_sart_native``: CLI, HDF5 I/O, CPU solver kernels).

``torch`` is imported before ``_sart_hip``: PyTorch-ROCm ships its own ``libamdhip64.so.7``; importing
it first makes the dynamic loader bind our module to that same HIP runtime instance (identical
SONAME), so torch stream handles and allocations are valid in our launches.
"""
from __future__ import annotations

import importlib
import os

_HIP = None
_NATIVE = None


class NativeExtensionMissing(RuntimeError):
    pass


def _import(name: str):
    try:
        return importlib.import_module(f"mpi_cuda_sartsolver_amd._lib.{name}")
    except ImportError as exc:  # pragma: no cover - exercised only on broken installs
        raise NativeExtensionMissing(
            f"native module {name} is not built or not importable ({exc}); "
            "build it with `python -m mpi_cuda_sartsolver_amd._build` (hipcc --offload-arch=gfx950)"
        ) from exc


def hip():
    """Return the HIP kernel module, building it on first use if SART_AUTOBUILD=1."""
    global _HIP
    if _HIP is None:
        import torch  # noqa: F401  (bind to torch's HIP runtime first, see module docstring)

        try:
            _HIP = _import("_sart_hip")
        except NativeExtensionMissing:
            if os.environ.get("SART_AUTOBUILD", "0") == "1":
                from .. import _build

                _build.build_hip(verbose=False)
                _HIP = _import("_sart_hip")
            else:
                raise
    return _HIP


def _preload_hdf5() -> None:
    """Load the HDF5 C library by absolute path (RTLD_GLOBAL) so _sart_native resolves it without an
    rpath into /opt/conda/lib (which would also pull conda's older libstdc++)."""
    import ctypes

    prefix = os.environ.get("SART_HDF5_PREFIX", "/opt/conda")
    for name in ("libhdf5.so", "libhdf5.so.103"):
        path = os.path.join(prefix, "lib", name)
        if os.path.exists(path):
            try:
                ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
                return
            except OSError:
                pass


def native():
    global _NATIVE
    if _NATIVE is None:
        _preload_hdf5()
        try:
            _NATIVE = _import("_sart_native")
        except NativeExtensionMissing:
            if os.environ.get("SART_AUTOBUILD", "0") == "1":
                from .. import _build

                _build.build_native(verbose=False)
                _NATIVE = _import("_sart_native")
            else:
                raise
    return _NATIVE


def hip_available() -> bool:
    try:
        hip()
        return True
    except NativeExtensionMissing:
        return False
