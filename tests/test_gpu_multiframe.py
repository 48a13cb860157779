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


@pytest.mark.parametrize("log", [False, True])
def test_multiframe_warm_chain(log):
    """Time-series warm start: batch 0 starts from x0, batch k + 1 from batch k's last solution; each frame
    matches the oracle warm-started from the same vector."""
    from mpi_cuda_sartsolver_amd.models.laplacian import LaplacianCSR
    from mpi_cuda_sartsolver_amd.models.multiframe import MultiFrameSARTSolver
    from mpi_cuda_sartsolver_amd.models.reference import sart_gpu_semantics
    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM
    from mpi_cuda_sartsolver_amd.models.sart import SolverParams

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(77)
    P, V, nframes, batch = 600, 1000, 40, 16
    A = rng.random((P, V), dtype=np.float32)
    base = rng.random(V) + 0.1
    X = base[None] * (1.0 + 0.02 * rng.random((nframes, V)))  # a slowly varying series
    G = X @ A.T.astype(np.float64)
    L = LaplacianCSR.grid_3d(10, 10, 10, device=dev)
    kw = dict(max_iterations=60, conv_tolerance=1e-5, beta_laplace=1e-3)
    s = MultiFrameSARTSolver(DenseRTM.from_dense(A, device=dev), L, None, SolverParams(**kw), logarithmic=log,
                             batch=batch)
    x0 = base * 1.5
    res = s.solve_batch(G, x0=x0, chain=True)
    prev = x0
    for b0 in range(0, nframes, batch):
        b1 = min(nframes, b0 + batch)
        for f in range(b0, b1):
            x, st, it = sart_gpu_semantics(A, G[f], L, logarithmic=log, x_prev=prev, **kw)
            assert res[f].status == st and abs(res[f].iterations - it) <= 2, (f, res[f].iterations, it)
            assert np.linalg.norm(res[f].solution - x) / np.linalg.norm(x) < 3e-3
        prev = res[b1 - 1].solution
    # without chain, a later batch cold-starts even when x0 is given
    cold = s.solve_batch(G[:20], x0=None)
    x, st, it = sart_gpu_semantics(A, G[17], L, logarithmic=log, **kw)
    assert cold[17].status == st and np.linalg.norm(cold[17].solution - x) / np.linalg.norm(x) < 3e-3
