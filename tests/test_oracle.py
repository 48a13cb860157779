"""The device fp64 oracle (models/oracle.py) equals the host fp64 oracle (models/reference.py); runs on the
CPU device here, on the GPU in the production-geometry tests and bench.py's self-check."""
import numpy as np
import pytest
import torch

from mpi_cuda_sartsolver_amd.models.oracle import sart_oracle_f64
from mpi_cuda_sartsolver_amd.models.reference import sart_fp32_emulation, sart_gpu_semantics
from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM
from mpi_cuda_sartsolver_amd.utils.synthetic import host_problem


@pytest.mark.parametrize("log", [False, True])
@pytest.mark.parametrize("warm", [False, True])
def test_device_oracle_matches_host_oracle(log, warm):
    A, g, x = host_problem(300, 700, seed=3, saturate_fraction=0.05)
    g = g.copy()
    g[7] = np.nan  # masked like a saturated pixel in both
    ref_g = g.copy()
    ref_g[7] = -1.0
    rtm = DenseRTM.from_dense(A, device=torch.device("cpu"))
    x0 = x * g[np.isfinite(g)].max() if warm else None
    xo = sart_oracle_f64(rtm, g, 7, logarithmic=log, x_prev=x0, block_bytes=64 * rtm.ld * 8)  # several blocks
    xr, _, _ = sart_gpu_semantics(A, ref_g, logarithmic=log, x_prev=x0, max_iterations=7, conv_tolerance=0.0)
    assert np.linalg.norm(xo - xr) / np.linalg.norm(xr) < 1e-12


def test_fp32_emulation_is_close_but_not_exact():
    A, g, _ = host_problem(200, 500, seed=4)
    xr, _, _ = sart_gpu_semantics(A, g, max_iterations=10, conv_tolerance=0.0)
    x32, st, it = sart_fp32_emulation(A, g, max_iterations=10)
    e = np.linalg.norm(x32 - xr) / np.linalg.norm(xr)
    assert 0 < e < 1e-2 and st == -1 and it == 10
