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


@pytest.mark.parametrize("shape,density", [((1, 1), 1.0), ((37, 129), 0.05), ((200, 300), 0.3), ((64, 64), 0.0),
                                           ((1500, 2000), 0.4)])  # (1.2M non-zeros: the multi-threaded transpose)
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


@pytest.mark.parametrize("fmt", ["auto", "sparse"])
def test_cli_cpu_sparse_matches_dense(tmp_path, capfd, fmt):
    """--use_cpu on sparse COO files of the no-reflection ray-traced model: the CPU solver on the CSR / CSC shard
    (auto picks it at ~1 % non-zeros) gives the dense CPU solver's solutions to fp64 rounding, and the reference CPU
    semantics' oracle chain."""
    from mpi_cuda_sartsolver_amd import cli
    from mpi_cuda_sartsolver_amd.io.fixtures import make_case
    from mpi_cuda_sartsolver_amd.models.reference import sart_cpu_semantics

    case = make_case(str(tmp_path / "c"), shapes=((16, 16), (16, 16)), grid=(8, 8, 8), raytraced=True,
                     direct_only=True, sparse_cameras=("cam_a", "cam_b"), nframes=3, saturate=0.02)
    assert np.count_nonzero(case.A) / case.A.size < 0.1
    outs = {}
    for name, extra in (("sparse", ["--rtm_format", fmt]), ("dense", ["--rtm_format", "dense"])):
        out = str(tmp_path / f"{name}.h5")
        assert cli.main(["--use_cpu", "-m", "30", "-c", "1e-9", "-o", out] + extra + case.files) == 0
        outs[name] = native().read_dataset_f64(out, "solution/value")
    assert capfd.readouterr().out.count("Processed in:") == 6
    np.testing.assert_allclose(outs["sparse"], outs["dense"], rtol=1e-11, atol=1e-14 * np.abs(outs["dense"]).max())
    frames = [np.concatenate([case.frames[c][k].ravel()[case.masks[c].ravel() > 0] for c in sorted(case.masks)])
              for k in range(3)]
    prev = None
    for k, g in enumerate(frames):
        x, _, _ = sart_cpu_semantics(case.A, g, None, max_iterations=30, conv_tolerance=1e-9, x_prev=prev)
        np.testing.assert_allclose(outs["sparse"][k], x, rtol=1e-9, atol=1e-15 * np.abs(x).max())
        prev = x


def test_python_sparse_loader_host_side(tmp_path):
    """io.hdf5: the stored-entry density (the driver's --rtm_format auto test: -1 when a dataset is dense) and the
    reader's CSR of a row window."""
    from mpi_cuda_sartsolver_amd.io.fixtures import make_case
    from mpi_cuda_sartsolver_amd.io.hdf5 import rtm_sparse_density, validate_inputs

    case = make_case(str(tmp_path / "c"), shapes=((8, 8), (8, 8)), grid=(6, 6, 6), raytraced=True, direct_only=True,
                     sparse_cameras=("cam_a", "cam_b"), nframes=1)
    inp = validate_inputs(case.files)
    d = rtm_sparse_density(inp)
    assert d == pytest.approx(np.count_nonzero(case.A) / case.A.size)
    mixed = make_case(str(tmp_path / "m"), sparse_cameras=("cam_b",), nframes=1)
    assert rtm_sparse_density(validate_inputs(mixed.files)) == -1.0
    rp, ci, vv = native().RtmReader(inp.rtm_files, inp.rtm_name, inp.nvoxel).read_csr(5, 70)
    np.testing.assert_array_equal(_dense(65, inp.nvoxel, rp, ci, vv), case.A[5:70].astype(np.float32))


@pytest.mark.parametrize("ptr,col,msg", [
    ([0, 1, 2, 2], [0, 7], "outside"),          # column index past ncols
    ([0, 1, 2, 2], [0, -1], "outside"),         # negative column index
    ([0, 2, 1, 2], [0, 1], "decreases"),        # row pointer not monotone
])
def test_sparse_rtm_rejects_malformed_csr(ptr, col, msg):
    """A malformed user CSR is rejected before anything indexes with it (csr_transpose validates): a bad
    column index would write outside the host transpose and make the device gathers read outside x."""
    import torch

    from mpi_cuda_sartsolver_amd.models.rtm import SparseRTM

    with pytest.raises(ValueError, match=msg):
        SparseRTM(3, 4, np.array(ptr), np.array(col), np.ones(len(col), np.float32), device=torch.device("cpu"))
    with pytest.raises(ValueError, match=msg):
        native().csr_transpose(3, 4, np.array(ptr, np.int64), np.array(col, np.int32), np.ones(len(col), np.float32))


@pytest.mark.parametrize("chunk", ["", "3"])
def test_read_rtm_csr_streams_coo_with_duplicates(tmp_path, monkeypatch, chunk):
    """RtmReader::read_csr streams the COO arrays in hyperslab chunks (SART_COO_CHUNK; 3 entries here: every row's
    entries split across chunks) with a count and a fill pass: unsorted pixel order, an entry repeated at the same
    (row, col) (the LAST one wins, as the dense scatter leaves it), exact zeros dropped, row windows -- equal to the
    dense reader's matrix of the same file."""
    if chunk:
        monkeypatch.setenv("SART_COO_CHUNK", chunk)
    n = native()
    rng = np.random.default_rng(5)
    h, w, V = 4, 4, 10
    P = h * w
    m = 60
    pix = rng.integers(0, P, m).astype(np.uint64)
    vox = rng.integers(0, V, m).astype(np.uint64)
    val = (rng.random(m) + 0.5).astype(np.float32)
    val[::7] = 0.0  # exact zeros (some of them the last of a repeated entry)
    pix[5], vox[5], pix[40], vox[40] = 3, 2, 3, 2  # a repeated (row, col): the later value must win
    val[5], val[40] = 9.0, 4.0
    expected = np.zeros((P, V), np.float32)
    for p, v, x in zip(pix, vox, val):
        expected[p, v] = x
    rtm, img = str(tmp_path / "rtm.h5"), str(tmp_path / "img.h5")
    flat = np.arange(V)
    n.write_rtm_file(path=rtm, camera_name="cam", wavelength=656.3, npixel=P, nvoxel=V,
                     frame_mask=np.ones((h, w), np.uint8), vi=flat.astype(np.uint64), vj=np.zeros(V, np.uint64),
                     vk=np.zeros(V, np.uint64), vvalue=np.arange(V, dtype=np.int32), nx=V, ny=1, nz=1,
                     rtm_name="with_reflections", coordinate_system="", bounds=[], pixel_index=pix, voxel_index=vox,
                     value=val)
    n.write_image_file(img, "cam", 657.3, np.array([0.0]), np.ones((1, h, w)))
    for r0, r1 in [(0, P), (3, 11), (7, 8)]:
        rp, ci, vv, ncols = n.read_rtm_csr([rtm, img], row_begin=r0, row_end=r1)
        assert ncols == V and np.all(vv != 0)
        for r in range(r1 - r0):
            assert np.all(np.diff(ci[rp[r]:rp[r + 1]]) > 0)  # ascending, unique columns per row
        np.testing.assert_array_equal(_dense(r1 - r0, V, rp, ci, vv), expected[r0:r1])
    assert expected[3, 2] == 4.0
