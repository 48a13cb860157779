"""Sparse RTM path, host side (no GPU): CSR construction from (row, col, value) entries with the dense scatter's
semantics, the CSC transpose, and RtmReader::read_csr on HDF5 fixtures (dense, sparse COO and mixed cameras, voxel
segments, row windows across cameras) against the dense reader's matrix. The device kernels are in
tests/test_gpu_sparse.py."""
import numpy as np
import pytest

from mpi_cuda_sartsolver_amd.ops import native


def _dense(nrows, ncols, rp, ci, vv):
    A = np.zeros((nrows, ncols), np.float32)
    for r in range(nrows):
        A[r, ci[rp[r]:rp[r + 1]]] = vv[rp[r]:rp[r + 1]]
    return A


def test_csr_from_entries_semantics():
    n = native()
    rows = np.array([2, 0, 2, 1, 0, 2, 0], np.int64)
    cols = np.array([3, 1, 0, 2, 1, 3, 0], np.int32)
    vals = np.array([1.0, 2.0, 3.0, 0.0, 5.0, 7.0, -1.0], np.float32)
    rp, ci, vv = n.csr_from_entries(3, 4, rows, cols, vals)
    # row 0: (1) 2.0 then 5.0 -> the later 5.0 wins, (0) -1.0; row 1: an explicit zero is dropped; row 2: (3) 1.0
    # then 7.0 -> 7.0, (0) 3.0; columns ascending within a row
    assert rp.tolist() == [0, 2, 2, 4]
    assert ci.tolist() == [0, 1, 0, 3]
    assert vv.tolist() == [-1.0, 5.0, 3.0, 7.0]
    with pytest.raises(ValueError):
        n.csr_from_entries(3, 4, np.array([3], np.int64), np.array([0], np.int32), np.array([1.0], np.float32))


@pytest.mark.parametrize("shape,density", [((1, 1), 1.0), ((37, 129), 0.05), ((200, 300), 0.3), ((64, 64), 0.0)])
def test_csr_transpose(shape, density):
    n = native()
    rng = np.random.default_rng(shape[0])
    A = np.where(rng.random(shape) < density, rng.random(shape), 0.0).astype(np.float32)
    r, c = np.nonzero(A)
    perm = rng.permutation(r.size)
    rp, ci, vv = n.csr_from_entries(shape[0], shape[1], r[perm], c[perm], A[r, c][perm])
    np.testing.assert_array_equal(_dense(shape[0], shape[1], rp, ci, vv), A)
    cp, ri, cv = n.csr_transpose(shape[0], shape[1], rp, ci, vv)
    np.testing.assert_array_equal(_dense(shape[1], shape[0], cp, ri, cv), A.T)
    for k in range(shape[1]):  # rows ascending within every column
        assert np.all(np.diff(ri[cp[k]:cp[k + 1]]) > 0)


@pytest.mark.parametrize("sparse_cameras", [(), ("cam_b",), ("cam_a", "cam_b")])
def test_read_rtm_csr_matches_dense_reader(tmp_path, sparse_cameras):
    from mpi_cuda_sartsolver_amd.io.fixtures import make_case

    case = make_case(str(tmp_path / "c"), shapes=((6, 8), (5, 7)), nvoxel=48, segments=2, raytraced=False,
                     sparse_cameras=sparse_cameras, nframes=1, seed=3)
    P, V = case.A.shape
    n = native()
    for r0, r1 in [(0, P), (3, P - 2), (P // 2, P // 2 + 1)]:
        rp, ci, vv, ncols = n.read_rtm_csr(case.files, row_begin=r0, row_end=r1)
        assert ncols == V
        np.testing.assert_array_equal(_dense(r1 - r0, V, rp, ci, vv), case.A[r0:r1].astype(np.float32))


def test_read_rtm_csr_raytraced(tmp_path):
    """A ray-traced matrix (mostly zeros, values over many decades): the CSR holds exactly its non-zeros."""
    from mpi_cuda_sartsolver_amd.io.fixtures import make_case

    case = make_case(str(tmp_path / "c"), shapes=((8, 8), (8, 8)), grid=(6, 6, 6), raytraced=True,
                     sparse_cameras=("cam_a",), nframes=1)
    P, V = case.A.shape
    rp, ci, vv, _ = native().read_rtm_csr(case.files, row_begin=0, row_end=P)
    assert vv.size == np.count_nonzero(case.A)
    np.testing.assert_array_equal(_dense(P, V, rp, ci, vv), case.A.astype(np.float32))
