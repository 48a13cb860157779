"""bf16-stored RTM in the multi-frame engine: the bf16 MFMA projections (csrc/kernels/multiframe_bf16.hip) with
hi + lo bf16 split operands, against fp64 references of the same bf16-rounded matrix, and the whole batched
solver against the per-frame fp64 oracle of the GPU semantics."""
import numpy as np
import pytest
from fp32_bound import check_fp32_bound

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


def _bf16_rtm(dev, P, V, seed):
    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM

    rng = np.random.default_rng(seed)
    A = rng.random((P, V), dtype=np.float32)
    m = DenseRTM.from_dense(A, device=dev, storage="bf16")
    Ab = m.A[:P, :V].float().cpu().numpy().astype(np.float64)  # the matrix the kernels see
    return m, Ab


def test_split_planes(k, dev):
    """hi = rne(x), lo = x - hi rounded stochastically: hi + lo reproduces x to 2^-16 relative, without bias over
    equal values; W planes are frame-major."""
    rng = np.random.default_rng(5)
    x = torch.from_numpy((rng.standard_normal(4096) * 10.0 ** rng.uniform(-6, 6, 4096)).astype(np.float32)).to(dev)
    hi = torch.empty(4096, dtype=torch.bfloat16, device=dev)
    lo = torch.empty_like(hi)
    k.mf_split_x(x.data_ptr(), 4096, hi.data_ptr(), lo.data_ptr(), _stream(dev))
    torch.cuda.synchronize()
    assert torch.equal(hi, x.bfloat16())
    rec = hi.double() + lo.double()
    assert ((rec - x.double()).abs() <= 2.0 ** -16 * x.double().abs()).all()
    # 4096 copies of one value: round-to-nearest lo would repeat one error 4096 times; the stochastic lo's
    # errors average out (mean relative error << the 2^-18 bound of a single element)
    same = torch.full((4096,), 1.2345678, dtype=torch.float32, device=dev)
    k.mf_split_x(same.data_ptr(), 4096, hi.data_ptr(), lo.data_ptr(), _stream(dev))
    torch.cuda.synchronize()
    err = (hi.double() + lo.double() - same.double()).mean().item() / 1.2345678
    assert abs(err) < 2.0 ** -22, err

    # the split-A k order: position 8 g + j of every 32-block holds element 4 g + j (j < 4) or 16 + 4 g + j - 4
    hp, lp = torch.empty_like(hi), torch.empty_like(lo)
    k.mf_split_x(x.data_ptr(), 4096, hi.data_ptr(), lo.data_ptr(), _stream(dev))
    k.mf_split_x(x.data_ptr(), 4096, hp.data_ptr(), lp.data_ptr(), _stream(dev), True)
    torch.cuda.synchronize()
    src = np.array([32 * b + (4 * (p // 8) + p % 8 if p % 8 < 4 else 16 + 4 * (p // 8) + p % 8 - 4)
                    for b in range(128) for p in range(32)])
    assert torch.equal(hp.cpu(), hi.cpu()[src]) and torch.equal(lp.cpu(), lo.cpu()[src])

    nf, rows, ldw = 32, 192, 160
    W = torch.from_numpy(rng.random((rows, nf)).astype(np.float32)).to(dev)  # [rows][16][nf / 16] layout
    wh = torch.zeros((nf, ldw), dtype=torch.bfloat16, device=dev)
    wl = torch.zeros_like(wh)
    k.mf_split_w(W.data_ptr(), rows, nf, ldw, wh.data_ptr(), wl.data_ptr(), _stream(dev))
    torch.cuda.synchronize()
    ng = nf // 16
    for f in (0, 5, 16, 31):
        slot = (f % 16) * ng + f // 16
        assert torch.equal(wh[f], W[:ldw, slot].bfloat16())
        np.testing.assert_allclose((wh[f].double() + wl[f].double()).cpu().numpy(), W[:ldw, slot].double().cpu().numpy(),
                                   rtol=2.0 ** -16)


# (SART_MF_B16_FWD, SART_MF_B16_VT) tiles: register-operand and LDS-shared variants of both kernels
@pytest.mark.parametrize("fwd,bwd", [("", ""), ("4,1", "1,reg"), ("8,1", "2,reg"), ("4,2,lds", "1,lds"),
                                     ("8,1,lds", "2,lds"), ("2,2,lds", "2,lds"), ("4,2,lds,as", "2,lds"),
                                     ("2,2,lds,as", "1,lds")])
@pytest.mark.parametrize("nf", [16, 32, 64, 128])  # 128: one tiling whatever the knobs say
@pytest.mark.parametrize("P,V", [(512, 1024), (1000, 2048), (64, 1024), (2048, 4096), (1000, 1088)])
def test_bf16_mfma_projections(k, dev, P, V, nf, fwd, bwd, monkeypatch):
    if fwd:
        monkeypatch.setenv("SART_MF_B16_FWD", fwd)
    if bwd:
        monkeypatch.setenv("SART_MF_B16_VT", bwd)
    m, Ab = _bf16_rtm(dev, P, V, seed=P + V)
    rng = np.random.default_rng(nf)
    X = rng.random((nf, V)).astype(np.float32)
    Xd = torch.zeros((nf, m.ld), device=dev)
    Xd[:, :V] = torch.from_numpy(X)
    Xh = torch.empty((nf, m.ld), dtype=torch.bfloat16, device=dev)
    Xl = torch.empty_like(Xh)
    k.mf_split_x(Xd.data_ptr(), nf * m.ld, Xh.data_ptr(), Xl.data_ptr(), _stream(dev))
    nsf = 3 if m.ld > 1024 else 1  # ragged column splits
    Fo3 = torch.zeros((nsf, m.nrows_pad, nf), device=dev)
    k.mf_forward_b16(m.A.data_ptr(), m.ld, P, m.nrows_pad, Xh.data_ptr(), Xl.data_ptr(), Fo3.data_ptr(), nsf,
                     _stream(dev), nf)
    W = (rng.random((P, nf)) - 0.5).astype(np.float32)
    Wd = torch.zeros((m.nrows_pad, nf), device=dev)
    Wd[:P] = torch.from_numpy(np.ascontiguousarray(W.reshape(P, nf // 16, 16).transpose(0, 2, 1).reshape(P, nf)))
    Wh = torch.zeros((nf, m.nrows_pad), dtype=torch.bfloat16, device=dev)
    Wl = torch.zeros_like(Wh)
    k.mf_split_w(Wd.data_ptr(), m.nrows_pad, nf, m.nrows_pad, Wh.data_ptr(), Wl.data_ptr(), _stream(dev))
    ns = 3
    part = torch.zeros((ns, m.ld, nf), device=dev)
    # two voxel chunks (the engine's overlapped all-reduce pipeline) written into one partial buffer
    vmid = (m.ld // 2) // 128 * 128  # aligned to either voxel tile (64 or 128 voxels per wave)
    for v0, v1 in ((0, vmid), (vmid, m.ld)):
        k.mf_backproject_b16(m.A.data_ptr(), m.ld, P, Wh.data_ptr(), Wl.data_ptr(), m.nrows_pad, ns, part.data_ptr(),
                             _stream(dev), nf, v0, v1)
    torch.cuda.synchronize()
    F_ref = Ab @ X.T.astype(np.float64)
    F = Fo3.sum(0)[:P].double().cpu().numpy()
    assert np.linalg.norm(F - F_ref) / np.linalg.norm(F_ref) < 2e-6
    np.testing.assert_allclose(F, F_ref, rtol=2e-5, atol=2e-4)
    B_ref = Ab.T @ W.astype(np.float64)
    B = part.sum(0)[:V].double().cpu().numpy()
    assert np.linalg.norm(B - B_ref) / np.linalg.norm(B_ref) < 2e-5
    np.testing.assert_allclose(B, B_ref, rtol=1e-4, atol=5e-4)


@pytest.mark.parametrize("log", [False, True])
@pytest.mark.parametrize("nframes,batch", [(5, 16), (27, 32), (40, 64), (140, 128)])
def test_multiframe_bf16_vs_oracle(log, nframes, batch):
    """The batched solver on a bf16-stored shard follows the fp64 oracle run on the same bf16-rounded matrix."""
    from mpi_cuda_sartsolver_amd.models.laplacian import LaplacianCSR
    from mpi_cuda_sartsolver_amd.models.multiframe import MultiFrameSARTSolver
    from mpi_cuda_sartsolver_amd.models.reference import sart_gpu_semantics
    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM
    from mpi_cuda_sartsolver_amd.models.sart import SolverParams

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(nframes + 100)
    P, V = 700, 1000
    A = rng.random((P, V), dtype=np.float32)
    rtm = DenseRTM.from_dense(A, device=dev, storage="bf16")
    Ab = rtm.A[:P, :V].float().cpu().numpy()
    X = rng.random((nframes, V)) + 0.05
    G = X @ Ab.T.astype(np.float64)
    G[rng.random(G.shape) < 0.03] = -1.0
    L = LaplacianCSR.grid_3d(10, 10, 10, device=dev)
    kw = dict(max_iterations=40, conv_tolerance=1e-4, beta_laplace=1e-3)
    s = MultiFrameSARTSolver(rtm, L, None, SolverParams(**kw), logarithmic=log, batch=batch)
    assert s.batch_width == batch
    res = s.solve_batch(G)
    for f in range(nframes):
        x, st, it = sart_gpu_semantics(Ab, G[f], L, logarithmic=log, **kw)
        assert res[f].status == st
        assert abs(res[f].iterations - it) <= 2
    for f in sorted({0, nframes // 2, nframes - 1}):  # the rounded matrix is exact in the operand: fp32 bound
        check_fp32_bound(res[f].solution, Ab, G[f], L, log=log, iterations=res[f].iterations, beta_laplace=1e-3)


def test_multiframe_bf16_matches_fp32_engine_on_rounded_matrix():
    """Same bf16-rounded matrix stored as fp32 (fp32 MFMA engine) and as bf16 (bf16 MFMA engine): the two
    batched solves agree far inside the oracle tolerance."""
    from mpi_cuda_sartsolver_amd.models.multiframe import MultiFrameSARTSolver
    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM
    from mpi_cuda_sartsolver_amd.models.sart import SolverParams

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(9)
    P, V, nframes = 2048, 4096, 16
    A = rng.random((P, V), dtype=np.float32)
    rb = DenseRTM.from_dense(A, device=dev, storage="bf16")
    Ab = rb.A[:P, :V].float().cpu().numpy()
    rf = DenseRTM.from_dense(Ab, device=dev)
    G = (rng.random((nframes, V)) + 0.1) @ Ab.T.astype(np.float64)
    kw = dict(max_iterations=30, conv_tolerance=0.0)
    xs = []
    for rtm in (rf, rb):
        s = MultiFrameSARTSolver(rtm, None, None, SolverParams(**kw), batch=16, allow_zero_tolerance=True)
        xs.append(np.stack([r.solution for r in s.solve_batch(G)]))
    rel = np.linalg.norm(xs[1] - xs[0]) / np.linalg.norm(xs[0])
    assert rel < 1e-3, rel  # fp32 summation-order noise over 30 iterations (measured 2.6e-4)


# ------------------------------------------------------------------ split-A: fp32 A on the bf16 matrix cores
@pytest.mark.parametrize("fwd,vt,depth", [("", "", ""), ("2,1", "1", "3"), ("2,2", "2", "2"), ("4,2", "2", "3"),
                                           ("4,1,as", "1", "2"), ("2,2,as", "1", "3"), ("2,1,as", "2", "2")])
@pytest.mark.parametrize("nf", [16, 32, 64])
@pytest.mark.parametrize("P,V", [(512, 1024), (1000, 2048), (64, 1024), (2048, 4096), (1000, 1088)])
def test_split_a_projections(k, dev, P, V, nf, fwd, vt, depth, monkeypatch):
    """fp32 A split in registers into bf16 pieces (forward: hi + lo, three products; back-projection: hi + mid +
    lo, six products) against fp64 products of the fp32 matrix: fp32 MFMA accuracy, unlike bf16 storage (whose
    tests compare against the rounded matrix)."""
    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM

    for name, val in (("SART_MF_X3_FWD", fwd), ("SART_MF_X3_VT", vt), ("SART_MF_X3_DEPTH", depth)):
        if val:
            monkeypatch.setenv(name, val)
    rng = np.random.default_rng(P * 7 + V)
    A = rng.random((P, V), dtype=np.float32)
    m = DenseRTM.from_dense(A, device=dev)
    Ad = A.astype(np.float64)
    X = rng.random((nf, V)).astype(np.float32)
    Xd = torch.zeros((nf, m.ld), device=dev)
    Xd[:, :V] = torch.from_numpy(X)
    Xh = torch.empty((nf, m.ld), dtype=torch.bfloat16, device=dev)
    Xl = torch.empty_like(Xh)
    k.mf_split_x(Xd.data_ptr(), nf * m.ld, Xh.data_ptr(), Xl.data_ptr(), _stream(dev), True)  # the x3 k order
    nsf = 3 if m.ld > 1024 else 1
    Fo3 = torch.zeros((nsf, m.nrows_pad, nf), device=dev)
    k.mf_forward_x3(m.A.data_ptr(), m.ld, P, m.nrows_pad, Xh.data_ptr(), Xl.data_ptr(), Fo3.data_ptr(), nsf,
                    _stream(dev), nf)
    W = (rng.random((P, nf)) - 0.5).astype(np.float32)
    Wd = torch.zeros((m.nrows_pad, nf), device=dev)
    Wd[:P] = torch.from_numpy(np.ascontiguousarray(W.reshape(P, nf // 16, 16).transpose(0, 2, 1).reshape(P, nf)))
    Wh = torch.zeros((2, nf, m.nrows_pad), dtype=torch.bfloat16, device=dev)  # hi, mid
    Wl = torch.zeros((nf, m.nrows_pad), dtype=torch.bfloat16, device=dev)
    k.mf_split_w(Wd.data_ptr(), m.nrows_pad, nf, m.nrows_pad, Wh.data_ptr(), Wl.data_ptr(), _stream(dev), True)
    ns = 3
    part = torch.zeros((ns, m.ld, nf), device=dev)
    align = k.mf_backproject_b16_vox_align(m.ld, True)
    vmid = (m.ld // 2) // align * align
    chunks = ((0, vmid), (vmid, m.ld)) if vmid > 0 else ((0, m.ld),)
    for v0, v1 in chunks:
        k.mf_backproject_x3(m.A.data_ptr(), m.ld, P, Wh.data_ptr(), Wl.data_ptr(), m.nrows_pad, ns, part.data_ptr(),
                            _stream(dev), nf, v0, v1)
    torch.cuda.synchronize()
    F_ref = Ad @ X.T.astype(np.float64)
    F = Fo3.sum(0)[:P].double().cpu().numpy()
    assert np.linalg.norm(F - F_ref) / np.linalg.norm(F_ref) < 2e-6
    np.testing.assert_allclose(F, F_ref, rtol=2e-5, atol=2e-4)
    B_ref = Ad.T @ W.astype(np.float64)
    B = part.sum(0)[:V].double().cpu().numpy()
    # signed weights cancel in A^T W: three-piece A and W keep the error at fp32 level (measured ~2e-7)
    assert np.linalg.norm(B - B_ref) / np.linalg.norm(B_ref) < 1e-6
    np.testing.assert_allclose(B, B_ref, rtol=1e-4, atol=5e-5)


@pytest.mark.parametrize("batch", [32, 64])
@pytest.mark.parametrize("iters", [1, 20])
def test_split_a_engine_matches_fp32_mfma(batch, iters):
    """The same fp32 shard through fp32 MFMA and through split-A (f16 pairs) on the 16-bit matrix cores, both
    against the fp64 oracle at the fp32-emulation bound (after 1 iteration: the kernels; after 20: the fp32 drift of
    an ill-conditioned dense random matrix). The split-A engine is the default from 32 frames on."""
    from mpi_cuda_sartsolver_amd.models.multiframe import MultiFrameSARTSolver
    from mpi_cuda_sartsolver_amd.models.reference import sart_gpu_semantics
    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM
    from mpi_cuda_sartsolver_amd.models.sart import SolverParams

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(batch + iters)
    P, V, nframes = 1024, 2048, batch
    A = rng.random((P, V), dtype=np.float32)
    rf = DenseRTM.from_dense(A, device=dev)
    G = (rng.random((nframes, V)) + 0.1) @ A.T.astype(np.float64)
    kw = dict(max_iterations=iters, conv_tolerance=0.0)
    xs = {}
    for split in (False, True):
        s = MultiFrameSARTSolver(rf, None, None, SolverParams(**kw), batch=batch, allow_zero_tolerance=True,
                                 split_a=split)
        assert s.split_a == split
        xs[split] = np.stack([r.solution for r in s.solve_batch(G)])
    assert MultiFrameSARTSolver(rf, None, None, SolverParams(**kw), batch=batch, allow_zero_tolerance=True).split_a
    assert not MultiFrameSARTSolver(rf, None, None, SolverParams(**kw), batch=16, allow_zero_tolerance=True).split_a
    frames = (0, 1, nframes // 2, nframes - 1)
    ref = np.stack([sart_gpu_semantics(A, G[f], None, logarithmic=False, **kw)[0]
                    for f in frames])
    err = {k: np.linalg.norm(v[list(frames)] - ref) / np.linalg.norm(ref) for k, v in xs.items()}
    print("rel vs fp64 oracle: fp32 MFMA %.3g, split-A %.3g" % (err[False], err[True]))
    for split in (False, True):  # both engines at the fp32-emulation bound, frame by frame
        for f in frames:
            check_fp32_bound(xs[split][f], A, G[f], None, iterations=iters, beta_laplace=0.0)


# ------------------------------------------------------------------ blocked X planes ([ld / 32][nf][32])
@pytest.mark.parametrize("storage,fwd", [("fp32", ""), ("fp32", "2,2"), ("fp32", "4,1,as"), ("bf16", ""),
                                         ("bf16", "4,1"), ("bf16", "8,1,lds"), ("bf16", "2,2,lds,as")])
@pytest.mark.parametrize("nf", [16, 32, 64])
@pytest.mark.parametrize("P,V", [(512, 1024), (1000, 2048), (1000, 1088)])
def test_forward_blocked_x_planes_bitwise(k, dev, P, V, nf, storage, fwd, monkeypatch):
    """The forwards read blocked X planes (launch_mf_split_x with ld) at the same k order and MFMA sequence as
    frame-major ones: identical sums bit for bit, over ragged column splits and every forward tile."""
    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM

    a32 = storage == "fp32"
    if fwd:
        monkeypatch.setenv("SART_MF_X3_FWD" if a32 else "SART_MF_B16_FWD", fwd)
    rng = np.random.default_rng(P + V + nf)
    m = DenseRTM.from_dense(rng.random((P, V), dtype=np.float32), device=dev, storage=storage)
    Xd = torch.zeros((nf, m.ld), device=dev)
    Xd[:, :V] = torch.from_numpy(rng.random((nf, V)).astype(np.float32))
    nsf = 3 if m.ld > 1024 else 1
    fwd_op = k.mf_forward_x3 if a32 else k.mf_forward_b16
    outs = []
    for blk in (False, True):
        Xh = torch.empty((nf, m.ld), dtype=torch.bfloat16, device=dev)
        Xl = torch.empty_like(Xh)
        k.mf_split_x(Xd.data_ptr(), nf * m.ld, Xh.data_ptr(), Xl.data_ptr(), _stream(dev), a32, m.ld if blk else 0)
        if blk:  # element (f, c) of the blocked plane sits at (c / 32, f, c % 32)
            perm = Xh.view(m.ld // 32, nf, 32).permute(1, 0, 2).reshape(nf, m.ld)
            torch.testing.assert_close(perm, outs[0][1], rtol=0, atol=0)
        Fo = torch.zeros((nsf, m.nrows_pad, nf), device=dev)
        fwd_op(m.A.data_ptr(), m.ld, P, m.nrows_pad, Xh.data_ptr(), Xl.data_ptr(), Fo.data_ptr(), nsf, _stream(dev),
               nf, blk)
        torch.cuda.synchronize()
        outs.append((Fo, Xh))
    assert torch.equal(outs[0][0], outs[1][0])


# ------------------------------------------------------------------ split-A back-projection on f16 pairs
@pytest.mark.parametrize("ascale,wscale", [(1.0, 1.0), (1e-7, 1.0), (3e4, 1e-6), (1.0, 1e5)])
@pytest.mark.parametrize("nf", [16, 32, 64])
@pytest.mark.parametrize("P,V", [(512, 1024), (1000, 2048), (2048, 4096), (1000, 1088)])
def test_split_a_backprojection_f16_pairs(k, dev, P, V, nf, ascale, wscale):
    """fp32 A and W each held as two f16 pieces of a power-of-two-scaled value (|x s - x1 - x2| <= ~2^-22 |x s|; A
    scaled per voxel column, W per frame), three products, fp32 accumulation, the inverse scales applied in the
    epilogue: against fp64 products of the fp32 operands, also for matrices and weights far from 1 (the scales keep
    both pieces normal), frames of different magnitude (per-frame scales) and columns of different magnitude
    (per-column scales: columns spanning 1e-9 .. 1, the range a single shard-wide scale could not hold)."""
    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM

    rng = np.random.default_rng(P * 3 + V + nf)
    A = (rng.random((P, V), dtype=np.float32) * np.float32(ascale)).astype(np.float32)
    A *= np.logspace(-9, 0, V)[rng.permutation(V)].astype(np.float32)[None, :]  # columns over nine decades
    m = DenseRTM.from_dense(A, device=dev)
    W = ((rng.random((P, nf)) - 0.5) * wscale * np.logspace(0, 3, nf)[None, :]).astype(np.float32)
    Wd = torch.zeros((m.nrows_pad, nf), device=dev)
    Wd[:P] = torch.from_numpy(np.ascontiguousarray(W.reshape(P, nf // 16, 16).transpose(0, 2, 1).reshape(P, nf)))
    scratch = torch.zeros(max(nf, m.ld), dtype=torch.int32, device=dev)
    csc = torch.zeros(2 * m.ld, device=dev)
    k.mf_col_scales(m.A.data_ptr(), m.ld, m.nrows_pad, scratch.data_ptr(), csc.data_ptr(), _stream(dev))
    torch.cuda.synchronize()
    cmax = np.abs(A).max(0)
    sc = csc[:V].double().cpu().numpy()
    assert np.all((2.0 ** 13 <= cmax * sc) & (cmax * sc < 2.0 ** 14)), "per-column scaled maxima in [2^13, 2^14)"
    assert np.array_equal(csc[m.ld:m.ld + V].double().cpu().numpy() * sc, np.ones(V))
    w16 = torch.zeros((2, nf, m.nrows_pad), dtype=torch.int16, device=dev)
    inv = torch.zeros(nf, device=dev)
    k.mf_split_w16(Wd.data_ptr(), m.nrows_pad, nf, m.nrows_pad, w16[0].data_ptr(), w16[1].data_ptr(),
                   scratch.data_ptr(), 1.0, inv.data_ptr(), _stream(dev))
    ns = 3
    part = torch.zeros((ns, m.ld, nf), device=dev)
    vmid = (m.ld // 2) // 64 * 64
    for v0, v1 in ((0, vmid), (vmid, m.ld)):
        k.mf_backproject_h16(m.A.data_ptr(), m.ld, P, w16[0].data_ptr(), w16[1].data_ptr(), m.nrows_pad, ns,
                             part.data_ptr(), _stream(dev), nf, v0, v1, csc.data_ptr(), inv.data_ptr())
    torch.cuda.synchronize()
    B_ref = A.astype(np.float64).T @ W.astype(np.float64)
    B = part.sum(0)[:V].double().cpu().numpy()
    # per frame (frames span three decades): the six-product bf16 split measures ~2e-7 (test_split_a_projections)
    for f in range(nf):
        rel = np.linalg.norm(B[:, f] - B_ref[:, f]) / np.linalg.norm(B_ref[:, f])
        assert rel < 1e-6, (f, rel)
    # per voxel, relative to the column's own scale sum_p |A[p][v]| |W[p][f]| (also the 1e-9 columns)
    bscale = np.abs(A.astype(np.float64)).T @ np.abs(W.astype(np.float64))
    assert np.all(np.abs(B - B_ref) <= (8 * 2.0 ** -22 + 2.0 ** -24 * np.sqrt(P)) * bscale)


# ------------------------------------------------------------------ 128 frames (split-A: 8 MFMA column groups)
@pytest.mark.parametrize("fwd", ["", "2,2,as"])
@pytest.mark.parametrize("P,V", [(512, 1024), (1000, 2048), (64, 1024), (2048, 4096), (1000, 1088)])
def test_split_a_128_frames(k, dev, P, V, fwd, monkeypatch):
    """The 128-frame split-A kernels (forward: hi + lo bf16, three products; back-projection: f16 pairs) against
    fp64 products of the fp32 operands, with the forward's blocked and frame-major X planes bitwise equal."""
    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM

    if fwd:
        monkeypatch.setenv("SART_MF_X3_FWD", fwd)
    nf = 128
    rng = np.random.default_rng(P * 5 + V)
    A = rng.random((P, V), dtype=np.float32)
    m = DenseRTM.from_dense(A, device=dev)
    Ad = A.astype(np.float64)
    X = rng.random((nf, V)).astype(np.float32)
    Xd = torch.zeros((nf, m.ld), device=dev)
    Xd[:, :V] = torch.from_numpy(X)
    nsf = 3 if m.ld > 1024 else 1
    outs = []
    for blk in (False, True):
        Xh = torch.empty((nf, m.ld), dtype=torch.bfloat16, device=dev)
        Xl = torch.empty_like(Xh)
        k.mf_split_x(Xd.data_ptr(), nf * m.ld, Xh.data_ptr(), Xl.data_ptr(), _stream(dev), True, m.ld if blk else 0)
        Fo = torch.zeros((nsf, m.nrows_pad, nf), device=dev)
        k.mf_forward_x3(m.A.data_ptr(), m.ld, P, m.nrows_pad, Xh.data_ptr(), Xl.data_ptr(), Fo.data_ptr(), nsf,
                        _stream(dev), nf, blk)
        torch.cuda.synchronize()
        outs.append(Fo)
    assert torch.equal(outs[0], outs[1])
    F_ref = Ad @ X.T.astype(np.float64)
    F = outs[1].sum(0)[:P].double().cpu().numpy()
    assert np.linalg.norm(F - F_ref) / np.linalg.norm(F_ref) < 2e-6
    np.testing.assert_allclose(F, F_ref, rtol=2e-5, atol=2e-4)
    W = ((rng.random((P, nf)) - 0.5) * np.logspace(0, 3, nf)[None, :]).astype(np.float32)
    Wd = torch.zeros((m.nrows_pad, nf), device=dev)
    Wd[:P] = torch.from_numpy(np.ascontiguousarray(W.reshape(P, nf // 16, 16).transpose(0, 2, 1).reshape(P, nf)))
    scratch = torch.zeros(max(nf, m.ld), dtype=torch.int32, device=dev)
    csc = torch.zeros(2 * m.ld, device=dev)
    k.mf_col_scales(m.A.data_ptr(), m.ld, m.nrows_pad, scratch.data_ptr(), csc.data_ptr(), _stream(dev))
    w16 = torch.zeros((2, nf, m.nrows_pad), dtype=torch.int16, device=dev)
    inv = torch.zeros(nf, device=dev)
    k.mf_split_w16(Wd.data_ptr(), m.nrows_pad, nf, m.nrows_pad, w16[0].data_ptr(), w16[1].data_ptr(),
                   scratch.data_ptr(), 1.0, inv.data_ptr(), _stream(dev))
    ns = 3
    part = torch.zeros((ns, m.ld, nf), device=dev)
    vmid = (m.ld // 2) // 64 * 64
    for v0, v1 in ((0, vmid), (vmid, m.ld)):
        k.mf_backproject_h16(m.A.data_ptr(), m.ld, P, w16[0].data_ptr(), w16[1].data_ptr(), m.nrows_pad, ns,
                             part.data_ptr(), _stream(dev), nf, v0, v1, csc.data_ptr(), inv.data_ptr())
    torch.cuda.synchronize()
    B_ref = Ad.T @ W.astype(np.float64)
    B = part.sum(0)[:V].double().cpu().numpy()
    for f in range(nf):
        rel = np.linalg.norm(B[:, f] - B_ref[:, f]) / np.linalg.norm(B_ref[:, f])
        assert rel < 1e-6, (f, rel)


@pytest.mark.parametrize("log", [False, True])
def test_split_a_engine_128_frames_vs_oracle(log):
    """A 128-frame batch (8 column groups) through the split-A engine with continuous batching (150 frames: 22
    slots refilled) against the fp64 oracle per frame; the fp32 MFMA path (split-A off) takes 64-frame batches."""
    from mpi_cuda_sartsolver_amd.models.laplacian import LaplacianCSR
    from mpi_cuda_sartsolver_amd.models.multiframe import MultiFrameSARTSolver
    from mpi_cuda_sartsolver_amd.models.reference import sart_gpu_semantics
    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM
    from mpi_cuda_sartsolver_amd.models.sart import SolverParams

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(128)
    P, V, nframes = 700, 1000, 150
    A = rng.random((P, V), dtype=np.float32)
    X = rng.random((nframes, V)) + 0.05
    G = X @ A.T.astype(np.float64)
    G[rng.random(G.shape) < 0.03] = -1.0
    L = LaplacianCSR.grid_3d(10, 10, 10, device=dev)
    kw = dict(max_iterations=30, conv_tolerance=1e-4, beta_laplace=1e-3)
    s = MultiFrameSARTSolver(DenseRTM.from_dense(A, device=dev), L, None, SolverParams(**kw), logarithmic=log,
                             batch=128)
    assert s.batch_width == 128 and s.split_a
    res = s.solve_batch(G)
    for f in list(range(0, nframes, 7)) + [127, 128, nframes - 1]:
        x, st, it = sart_gpu_semantics(A, G[f], L, logarithmic=log, **kw)
        assert res[f].status == st and abs(res[f].iterations - it) <= 2, (f, res[f].iterations, it)
    for f in (0, 64, 127, 128, nframes - 1):
        check_fp32_bound(res[f].solution, A, G[f], L, log=log, iterations=res[f].iterations, beta_laplace=1e-3)
    sf = MultiFrameSARTSolver(DenseRTM.from_dense(A, device=dev), None, None, SolverParams(**kw), batch=128,
                              split_a=False)
    assert sf.batch_width == 64
