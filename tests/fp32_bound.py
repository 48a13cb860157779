"""The fp32-emulation bound shared by the solver tests (not a test module).

A result of ours after ``iterations`` SART updates is compared with the fp64 oracle of the reference GPU semantics
run for the same number of updates (``sart_gpu_semantics``, conv_tolerance 0) and must be no further from it than
an fp32 evaluation of the same algorithm is (``sart_fp32_emulation``): the larger error of the BLAS summation order
and of the reference kernels' own serial-tile order (summation order alone moves an fp32 evaluation's error by
~10 %, and a pure fp32 kernel lands anywhere in that spread)."""
import numpy as np

ORDERS = ("blas", "reference")


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a) - b) / np.linalg.norm(b))


def fp32_errors(x, A, g, L=None, *, log=False, iterations, beta_laplace=1e-2, x_prev=None, orders=ORDERS):
    from mpi_cuda_sartsolver_amd.models.reference import sart_fp32_emulation, sart_gpu_semantics

    kw = dict(logarithmic=log, max_iterations=int(iterations), beta_laplace=beta_laplace, x_prev=x_prev)
    x64, _, _ = sart_gpu_semantics(A, g, L, conv_tolerance=0.0, **kw)
    e32 = max(rel(sart_fp32_emulation(A, g, L, order=o, **kw)[0], x64) for o in orders)
    return rel(x, x64), e32


def check_fp32_bound(x, A, g, L=None, *, factor=1.0, slack=1e-7, **kw):
    e, e32 = fp32_errors(x, A, g, L, **kw)
    assert e <= factor * e32 + slack, f"rel {e:.3e} vs fp32 emulation {e32:.3e}"
    return e, e32
