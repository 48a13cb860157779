"""Parity at a mid-size production-like shape (mpi_cuda_sartsolver_amd/utils/parity.py): a 16384-pixel x 16384-voxel
ray-traced RTM with reflections (two 64 x 128 cameras, 16 x 32 x 32 voxels; 1 GiB fp32) -- a different fused-sweep
geometry and 16k-term sums, where tests/test_gpu_realistic.py holds 2048 x 4096. The fused sweep, the two-pass kernels
and the 64-frame split-A engine (f16 pairs) after 20 SART updates against the device fp64 oracle, each bounded by the
fp32 two-pass kernels' error on the same frame times the documented factor (parity.FACTORS); the 64k x 64k version
of the same comparison is tools/parity_at_scale.py (profiles/parity_r6_64k_raytraced.jsonl)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def problem():
    from mpi_cuda_sartsolver_amd.utils import parity

    dev = torch.device("cuda", 0)
    A, X, cams, grid, info, rng = parity.raytraced_problem(16384, (64, 128), nframes=64)
    G = parity.frames_from(torch.from_numpy(A).to(dev), X, rng)
    return A, G, grid, dev


@pytest.mark.parametrize("log", [False, True])
def test_paths_at_16k(problem, log):
    from mpi_cuda_sartsolver_amd.models.laplacian import LaplacianCSR
    from mpi_cuda_sartsolver_amd.utils import parity

    A, G, grid, dev = problem
    assert A.shape == (16384, 16384)
    recs = parity.run(A, G, dev, iters=(20,), frames=(0,), batches=(64,), variants=[(log, False), (log, True)],
                      laplacian=LaplacianCSR.grid_3d(*grid, device=dev), bf16=False, column_shard=not log,
                      emit=lambda r: None, tag="16k")
    paths = {r["path"] for r in recs}
    assert {"two_pass", "fused", "multiframe64"} <= paths
    bad = [(r["path"], r["laplacian"], r["err"], r["err_two_pass"], r["ratio"]) for r in recs if not r["ok"]]
    assert not bad, bad
    assert all(np.isfinite(r["err"]) and r["err"] < 1e-2 for r in recs)
