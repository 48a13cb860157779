"""The ray-traced RTM generator (utils/raytrace.py) and the CPU paths on its matrices (no GPU needed).

Pins the structure the GPU numerics tests rely on (tests/test_gpu_realistic.py): >= 90 % exact zeros in the
direct line-of-sight part, values over >= 1e8, rows and columns below the solver thresholds; checks Siddon's path
lengths against geometry; and runs the native fp64 CPU solver (--use_cpu semantics and GPU semantics) and the CLI
on HDF5 files of the model (dense + sparse COO) against the numpy oracles.
"""
import numpy as np
import pytest

from mpi_cuda_sartsolver_amd.utils.raytrace import phantom, raytraced_rtm, rtm_stats, siddon


@pytest.fixture(scope="module")
def rtm():
    return raytraced_rtm(grid=(16, 16, 16))


def test_structure(rtm):
    A, info = rtm
    assert A.shape == (2048, 4096) and A.dtype == np.float32
    st = rtm_stats(A, info["direct"])
    assert st["direct_zero_fraction"] >= 0.9
    assert st["zero_fraction"] >= 0.75  # the diffuse band makes some rows dense (tiny values)
    assert st["dynamic_range"] >= 1e8
    assert st["rows_below"] > 0 and st["cols_below"] > 0
    assert np.all(A >= 0) and np.all(np.isfinite(A))
    # voxels seen only through reflections: column sums far below the directly seen ones, above the threshold
    rho = A.astype(np.float64).sum(0)
    seen = rho[rho > 1e-6]
    assert seen.min() < 1e-2 * np.median(seen)


def test_siddon_lengths():
    """A ray along x through the middle of a 4 x 4 x 4 grid crosses 4 cells of length 1/4; a diagonal ray through
    the unit cube has total length sqrt(3); a ray missing the cube crosses nothing."""
    O = np.array([[-1.0, 0.6, 0.3], [-1.0, -1.0, -1.0], [-1.0, 2.0, 0.5]])
    D = np.array([[1.0, 0.0, 0.0], np.ones(3) / np.sqrt(3), [1.0, 0.0, 0.0]])
    ray, flat, seg, _ = siddon(O, D, (4, 4, 4))
    r0 = ray == 0
    np.testing.assert_allclose(seg[r0], 0.25)
    np.testing.assert_array_equal(np.sort(flat[r0]), [i * 16 + 2 * 4 + 1 for i in range(4)])
    np.testing.assert_allclose(seg[ray == 1].sum(), np.sqrt(3.0))
    assert not np.any(ray == 2)


def test_deterministic(rtm):
    A, _ = rtm
    B, _ = raytraced_rtm(grid=(16, 16, 16))
    assert np.array_equal(A, B)
    x0, x1 = phantom(t=0.0), phantom(t=1.0)
    assert x0.shape == (4096,) and np.all(x0 > 0)
    assert 0 < np.linalg.norm(x1 - x0) / np.linalg.norm(x0) < 0.2  # a slowly varying series


@pytest.mark.parametrize("log", [False, True])
@pytest.mark.parametrize("semantics", ["cpu", "gpu"])
def test_cpu_solver_on_realistic(rtm, log, semantics):
    from mpi_cuda_sartsolver_amd.models.cpu import CPUSARTSolver
    from mpi_cuda_sartsolver_amd.models.laplacian import LaplacianCSR
    from mpi_cuda_sartsolver_amd.models.reference import sart_cpu_semantics, sart_gpu_semantics
    from mpi_cuda_sartsolver_amd.models.sart import SolverParams

    A, _ = rtm
    g = A.astype(np.float64) @ phantom(t=2.0)
    g[::97] = -1.0
    L = LaplacianCSR.grid_3d(16, 16, 16)
    kw = dict(max_iterations=25, conv_tolerance=1e-9, beta_laplace=1e-3)
    r = CPUSARTSolver(A, L, params=SolverParams(**kw), logarithmic=log, semantics=semantics).solve(g)
    oracle = sart_cpu_semantics if semantics == "cpu" else sart_gpu_semantics
    x, st, it = oracle(A, g, L, logarithmic=log, **kw)
    assert (r.status, r.iterations) == (st, it)
    assert np.linalg.norm(r.solution - x) / np.linalg.norm(x) < 1e-9


def test_cli_cpu_on_realistic_hdf5(tmp_path, capfd):
    """--use_cpu on HDF5 files of the ray-traced model (cam_a dense, cam_b sparse COO, two voxel segments each):
    the written solutions equal the reference CPU semantics frame by frame (warm-started chain)."""
    from mpi_cuda_sartsolver_amd import cli
    from mpi_cuda_sartsolver_amd.io.fixtures import make_case
    from mpi_cuda_sartsolver_amd.models.reference import sart_cpu_semantics
    from mpi_cuda_sartsolver_amd.ops import native

    case = make_case(str(tmp_path / "c"), shapes=((16, 16), (16, 16)), grid=(8, 8, 8), raytraced=True,
                     sparse_cameras=("cam_b",), nframes=3, saturate=0.02)
    assert case.nvoxel == 512 and case.A.shape[1] == 512
    assert np.mean(case.A == 0) > 0.5
    out = str(tmp_path / "out.h5")
    assert cli.main(["--use_cpu", "-m", "30", "-c", "1e-9", "-o", out] + case.files) == 0
    assert capfd.readouterr().out.count("Processed in:") == 3
    frames = [np.concatenate([case.frames[c][k].ravel()[case.masks[c].ravel() > 0] for c in sorted(case.masks)])
              for k in range(3)]
    prev = None
    xs = []
    for g in frames:
        x, _, _ = sart_cpu_semantics(case.A, g, None, max_iterations=30, conv_tolerance=1e-9, x_prev=prev)
        xs.append(x)
        prev = x
    _, last, _ = native().read_solution_file(out)
    np.testing.assert_allclose(last, xs[-1], rtol=1e-9, atol=1e-15 * np.abs(xs[-1]).max())


def test_direct_coo_matches_dense_direct_part():
    """raytraced_direct_coo (the no-reflection matrix without a dense array) equals the direct part of
    raytraced_rtm entry for entry."""
    from mpi_cuda_sartsolver_amd.utils.raytrace import raytraced_direct_coo

    A, info = raytraced_rtm(grid=(8, 8, 8))
    r, c, v, rows = raytraced_direct_coo(grid=(8, 8, 8))
    D = np.zeros(A.shape, np.float32)
    D[r, c] = v
    np.testing.assert_array_equal(D, info["direct"])
    assert rows == info["rows"] and v.dtype == np.float32 and np.all(v > 0)
