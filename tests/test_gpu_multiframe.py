"""Multi-frame MFMA solver vs the per-frame fp64 oracle of the GPU semantics."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("log", [False, True])
@pytest.mark.parametrize("nframes,batch", [(1, 16), (5, 16), (16, 16), (19, 16), (27, 32), (40, 64)])
def test_multiframe_vs_oracle(log, nframes, batch):
    from mpi_cuda_sartsolver_amd.models.laplacian import LaplacianCSR
    from mpi_cuda_sartsolver_amd.models.multiframe import MultiFrameSARTSolver
    from mpi_cuda_sartsolver_amd.models.reference import sart_gpu_semantics
    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM
    from mpi_cuda_sartsolver_amd.models.sart import SolverParams

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(nframes)
    P, V = 700, 1000
    A = rng.random((P, V), dtype=np.float32)
    X = rng.random((nframes, V)) + 0.05
    G = X @ A.T.astype(np.float64)
    G[rng.random(G.shape) < 0.03] = -1.0
    L = LaplacianCSR.grid_3d(10, 10, 10, device=dev)
    kw = dict(max_iterations=40, conv_tolerance=1e-4, beta_laplace=1e-3)
    s = MultiFrameSARTSolver(DenseRTM.from_dense(A, device=dev), L, None, SolverParams(**kw), logarithmic=log,
                             batch=batch)
    assert s.batch_width == batch
    res = s.solve_batch(G)
    assert len(res) == nframes
    for f in range(nframes):
        x, st, it = sart_gpu_semantics(A, G[f], L, logarithmic=log, **kw)
        assert res[f].status == st
        assert abs(res[f].iterations - it) <= 2
        assert np.linalg.norm(res[f].solution - x) / np.linalg.norm(x) < 3e-3
