"""Numerics of the gfx950 HIP kernels against plain fp64 PyTorch/numpy references."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def k():
    from mpi_cuda_sartsolver_amd.ops import hip

    return hip()


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda", 0)


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


def _rtm(dev, P, V, seed=0, ld=None):
    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM

    rng = np.random.default_rng(seed)
    A = rng.random((P, V), dtype=np.float32)
    return A, DenseRTM.from_dense(A, device=dev, ld=ld)


def test_native_arch(k):
    assert k.arch() == "gfx950"
    info = k.device_info(0)
    assert "gfx950" in info["gcnArchName"]
    assert k.state_nbytes() == 128


@pytest.mark.parametrize("P,V", [(1000, 3000), (64, 64), (2048, 4096), (777, 1025)])
@pytest.mark.parametrize("epi", [0, 1, 2])
def test_forward_epilogues(k, dev, P, V, epi):
    A, m = _rtm(dev, P, V, seed=P + V)
    rng = np.random.default_rng(1)
    x = rng.random(V).astype(np.float32)
    gh = (rng.random(P) - 0.1).astype(np.float32)
    a = rng.random(P).astype(np.float32)
    xd = torch.zeros(m.ld, device=dev)
    xd[:V] = torch.from_numpy(x)
    ghd = torch.zeros(m.nrows_pad, device=dev)
    ghd[:P] = torch.from_numpy(gh)
    ad = torch.zeros(m.nrows_pad, device=dev)
    ad[:P] = torch.from_numpy(a)
    f = torch.zeros(m.nrows_pad, device=dev)
    w = torch.zeros(m.nrows_pad, device=dev)
    nb = k.forward_num_blocks(m.nrows_pad)
    Fp = torch.zeros(nb, dtype=torch.float64, device=dev)
    k.forward(epi, m.A.data_ptr(), m.ld, P, m.nrows_pad, xd.data_ptr(), ghd.data_ptr(), ad.data_ptr(), f.data_ptr(),
              w.data_ptr(), Fp.data_ptr(), 0, _stream(dev))
    torch.cuda.synchronize()
    fref = A.astype(np.float64) @ x.astype(np.float64)
    fg = f[:P].cpu().numpy().astype(np.float64)
    np.testing.assert_allclose(fg, fref, rtol=2e-5, atol=1e-4)
    assert np.isclose(Fp.sum().item(), np.sum(fg * fg), rtol=1e-9)
    if epi == 1:
        np.testing.assert_allclose(w[:P].cpu().numpy(), a * (gh - fg), rtol=1e-5, atol=1e-4)
    if epi == 2:
        np.testing.assert_allclose(w[:P].cpu().numpy(), a * fg, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("P,V", [(1000, 3000), (64, 64), (4096, 1024), (333, 2111)])
def test_backproject_deterministic(k, dev, P, V):
    A, m = _rtm(dev, P, V, seed=3)
    rng = np.random.default_rng(2)
    w = (rng.random(P) - 0.5).astype(np.float32)
    wd = torch.zeros(m.nrows_pad, device=dev)
    wd[:P] = torch.from_numpy(w)
    ns = k.backproject_num_splits(m.ld, P)
    part = torch.zeros(ns * m.ld, device=dev)
    out = torch.zeros(m.ld, device=dev)
    scale = torch.ones(m.ld, device=dev)
    outs = []
    for _ in range(2):
        k.backproject(m.A.data_ptr(), m.ld, P, wd.data_ptr(), ns, part.data_ptr(), 0, _stream(dev))
        k.reduce_partials(part.data_ptr(), m.ld, ns, scale.data_ptr(), out.data_ptr(), 0, 0, 0, 0, _stream(dev))
        outs.append(out.clone())
    torch.cuda.synchronize()
    ref = A.astype(np.float64).T @ w.astype(np.float64)
    np.testing.assert_allclose(outs[0][:V].cpu().numpy(), ref, rtol=1e-4, atol=2e-4)
    assert torch.equal(outs[0], outs[1]), "back-projection must be bitwise reproducible"
    assert torch.count_nonzero(outs[0][V:]) == 0


def test_ray_sums_f64(k, dev):
    A, m = _rtm(dev, 1500, 2500, seed=9)
    ell = torch.zeros(m.nrows_pad, dtype=torch.float64, device=dev)
    k.rowsum_f64(m.A.data_ptr(), m.ld, m.npixel, ell.data_ptr(), _stream(dev))
    ns = k.backproject_num_splits(m.ld, m.npixel)
    part = torch.zeros(ns * m.ld, dtype=torch.float64, device=dev)
    k.colsum_f64(m.A.data_ptr(), m.ld, m.npixel, ns, part.data_ptr(), _stream(dev))
    rho = torch.zeros(m.ld, dtype=torch.float64, device=dev)
    k.reduce_partials_f64(part.data_ptr(), m.ld, ns, rho.data_ptr(), _stream(dev))
    torch.cuda.synchronize()
    A64 = A.astype(np.float64)
    np.testing.assert_allclose(ell[:1500].cpu().numpy(), A64.sum(1), rtol=1e-12)
    np.testing.assert_allclose(rho[:2500].cpu().numpy(), A64.sum(0), rtol=1e-12)


def test_synthetic_shard_invariance(k, dev):
    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM

    full = DenseRTM.synthetic(300, 1000, 0, seed=5, device=dev)
    top = DenseRTM.synthetic(120, 1000, 0, seed=5, device=dev)
    bot = DenseRTM.synthetic(180, 1000, 120, seed=5, device=dev)
    torch.cuda.synchronize()
    assert torch.equal(full.A[:120, :1000], top.A[:120, :1000])
    assert torch.equal(full.A[120:300, :1000], bot.A[:180, :1000])
    assert torch.count_nonzero(full.A[:, 1000:]) == 0
    assert torch.count_nonzero(full.A[300:]) == 0
    a = full.A[:300, :1000]
    assert 0.0 <= a.min().item() and a.max().item() < 1.0
    assert abs(a.mean().item() - 0.5) < 0.01


@pytest.mark.parametrize("rows", [2, 4])  # 16-row tiles per wave of the MFMA forward kernel
@pytest.mark.parametrize("nf", [16, 32, 64])
@pytest.mark.parametrize("P,V", [(512, 1024), (1000, 2048), (64, 1024), (2048, 4096), (1000, 1088)])
def test_multiframe_mfma(k, dev, P, V, nf, rows):
    k.mf_set_rows(rows)
    k.mf_set_vox(rows // 2)  # 64-voxel tiles per wave of the back-projection: 1 or 2
    try:
        _check_multiframe_mfma(k, dev, P, V, nf)
    finally:
        k.mf_set_rows(0)
        k.mf_set_vox(0)


def _check_multiframe_mfma(k, dev, P, V, nf):
    A, m = _rtm(dev, P, V, seed=11)
    rng = np.random.default_rng(4)
    X = rng.random((nf, V)).astype(np.float32)  # frame-major
    Xd = torch.zeros((nf, m.ld), device=dev)
    Xd[:, :V] = torch.from_numpy(X)
    nsf = 3 if m.ld > 1024 else 1  # ragged splits exercise the 4-float4 tail loop
    Fo3 = torch.zeros((nsf, m.nrows_pad, nf), device=dev)
    k.mf_forward(m.A.data_ptr(), m.ld, P, m.nrows_pad, Xd.data_ptr(), m.ld, Fo3.data_ptr(), nsf, _stream(dev), nf)
    Fo = Fo3.sum(0)
    W = (rng.random((P, nf)) - 0.5).astype(np.float32)
    Wd = torch.zeros((m.nrows_pad, nf), device=dev)
    # back-projection operand layout [rows][16][nf / 16]: frame 16 j + i at position i * (nf / 16) + j
    Wd[:P] = torch.from_numpy(np.ascontiguousarray(W.reshape(P, nf // 16, 16).transpose(0, 2, 1).reshape(P, nf)))
    ns = 3
    part = torch.zeros((ns, m.ld, nf), device=dev)
    k.mf_backproject(m.A.data_ptr(), m.ld, P, Wd.data_ptr(), ns, part.data_ptr(), _stream(dev), nf)
    torch.cuda.synchronize()
    A64 = A.astype(np.float64)
    np.testing.assert_allclose(Fo[:P].cpu().numpy(), A64 @ X.T.astype(np.float64), rtol=2e-5, atol=2e-4)
    bp = part.sum(0)[:V].cpu().numpy()
    np.testing.assert_allclose(bp, A64.T @ W.astype(np.float64), rtol=1e-4, atol=5e-4)
