"""Multi-frame MFMA solver vs the per-frame fp64 oracle of the GPU semantics: statuses and iteration counts of the
tolerance-stopped runs, and solutions at the fp32-emulation bound (tests/fp32_bound.py: no further from the oracle,
after the frame's own update count, than an fp32 evaluation of the same chain)."""
import numpy as np
import pytest
from fp32_bound import check_fp32_bound

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
    for f in sorted({0, nframes // 2, nframes - 1}):
        check_fp32_bound(res[f].solution, A, G[f], L, log=log, iterations=res[f].iterations, beta_laplace=1e-3)


@pytest.mark.parametrize("log", [False, True])
def test_multiframe_warm_chain(log):
    """Time series with device-side refill: the first frames start from x0, every later frame from the current
    iterate of the newest frame in flight (with >= src_age updates) or finished (warm_from, with warm_iter updates),
    rescaled to its own normalisation. Each frame matches the oracle started from its recorded start value; each start value is the
    source's iterate (bitwise when the source had finished, at the oracle's fp32 drift when it was in flight).
    Frames converge after different iteration counts, so slots are refilled at different sweeps."""
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
    # a varying series: some frames close to their predecessor, some far (different iteration counts)
    X = base[None] * (1.0 + rng.choice([0.01, 0.3], size=(nframes, 1)) * rng.random((nframes, V)))
    G = X @ A.T.astype(np.float64)
    L = LaplacianCSR.grid_3d(10, 10, 10, device=dev)
    kw = dict(max_iterations=60, conv_tolerance=1e-5, beta_laplace=1e-3)
    s = MultiFrameSARTSolver(DenseRTM.from_dense(A, device=dev), L, None, SolverParams(**kw), logarithmic=log,
                             batch=batch)
    x0 = base * 1.5
    res = s.solve_batch(G, x0=x0, chain=True, record_starts=True)
    starts, stats = s.starts, s.series_stats
    cap = stats["admit_cap"]
    assert 1 <= cap < batch and stats["frames"] == nframes and 0 < stats["slot_util"] <= 1.0
    assert all(res[f].warm_from == -1 for f in range(cap))
    # until a frame in flight has src_age updates the new frames start from x0 too; every later one is chained
    assert all(res[f].warm_from < f for f in range(nframes))
    first = min(f for f in range(nframes) if res[f].warm_from >= 0)
    assert first <= cap * (stats["src_age"] + 1) and all(res[f].warm_from >= 0 for f in range(first, nframes))
    assert len({res[f].iterations for f in range(nframes)}) > 1  # slots really refill at different sweeps
    assert any(res[f].warm_live for f in range(nframes))  # sources in flight
    norm = G.max(axis=1)
    for f in range(nframes):
        wf, wi = res[f].warm_from, res[f].warm_iter
        if wf < 0:
            src = x0
        elif not res[f].warm_live:  # the source had finished: its solution, rescaled (bitwise)
            assert wi == res[wf].iterations
            src = res[wf].solution
        else:  # in flight: the oracle's iterate of the source after wi updates from its own recorded start,
            # extrapolated along its last update in linear mode (x + c (x - x_prev), MfQueue::src_extrap)
            def it(n):
                return sart_gpu_semantics(A, G[wf], L, logarithmic=log, x_prev=starts[wf],
                                          **dict(kw, max_iterations=n, conv_tolerance=0.0))[0]
            src = it(wi)
            c = 0.0 if log else stats["src_extrap"]
            if c:
                src = src + c * (src - it(wi - 1))
            assert wi >= stats["src_age"]
        want = np.maximum((src / norm[f]).astype(np.float32), np.float32(1e-7))
        got = (starts[f] / norm[f]).astype(np.float32)
        if wf < 0 or not res[f].warm_live:
            np.testing.assert_array_equal(got, want)
        else:
            assert np.linalg.norm(got - want) <= 1e-3 * np.linalg.norm(want), f
        x, st, it = sart_gpu_semantics(A, G[f], L, logarithmic=log, x_prev=starts[f], **kw)
        assert res[f].status == st and abs(res[f].iterations - it) <= 2, (f, res[f].iterations, it)
        if f % 7 == 0 or f == nframes - 1:
            check_fp32_bound(res[f].solution, A, G[f], L, log=log, iterations=res[f].iterations, beta_laplace=1e-3,
                             x_prev=starts[f])
    # without chain, every frame after the first batch cold-starts even when x0 is given
    cold = s.solve_batch(G[:20], x0=x0)
    assert all(r.warm_from == -1 for r in cold)
    x, st, it = sart_gpu_semantics(A, G[17], L, logarithmic=log, **kw)
    assert cold[17].status == st
    check_fp32_bound(cold[17].solution, A, G[17], L, log=log, iterations=cold[17].iterations, beta_laplace=1e-3)
    x, st, it = sart_gpu_semantics(A, G[3], L, logarithmic=log, x_prev=x0, **kw)  # the first batch: from x0
    assert cold[3].status == st and abs(cold[3].iterations - it) <= 2


def test_multiframe_series_iterations_near_sequential():
    """A slowly drifting series (the ray-traced phantom's regime): the pipelined chain keeps the warm start's
    iteration savings -- mean iterations per frame within 2x of the frame-by-frame chain's -- and the slots stay
    busy (the plan admits in the sweep a frame finishes)."""
    from mpi_cuda_sartsolver_amd.models.multiframe import MultiFrameSARTSolver
    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM
    from mpi_cuda_sartsolver_amd.models.sart import SARTSolver, SolverParams

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(3)
    P, V, nframes = 1500, 1200, 96
    A = rng.random((P, V), dtype=np.float32)
    b = rng.random(V) + 0.5
    ph = 2 * np.pi * rng.random(V)
    X = np.stack([b * (1 + 0.05 * np.sin(2 * np.pi * t / 200.0 + ph)) for t in range(nframes)])
    G = X @ A.T.astype(np.float64)
    kw = dict(max_iterations=400, conv_tolerance=1e-7)
    rtm = DenseRTM.from_dense(A, device=dev)
    seq = SARTSolver(rtm, None, None, SolverParams(**kw))
    its, prev = [], None
    for f in range(nframes):
        r = seq.solve(G[f], prev)
        its.append(r.iterations)
        prev = r.solution
    mf = MultiFrameSARTSolver(rtm, None, None, SolverParams(**kw), batch=32)
    res = mf.solve_batch(G, chain=True)
    mean_b, mean_s = np.mean([r.iterations for r in res]), np.mean(its[1:])
    assert all(r.status == 0 for r in res)
    assert mean_b <= 2.0 * mean_s + 1.0, (mean_b, mean_s, mf.series_stats)
    # (96 frames of ~4 sweeps each: admission ramp and drain are a large share of so short a series)
    assert mf.series_stats["slot_util"] > 0.3, mf.series_stats


def test_multiframe_drift_starts(monkeypatch):
    """SART_MF_DRIFT=1 (MfQueue::drift): on a linearly drifting series a chained frame's start adds the frame gap to
    its source times the per-frame change between the two newest finished solutions. Every frame still solves to
    the oracle from its recorded start, and the starts land nearer the frames' own solutions than without the drift."""
    from mpi_cuda_sartsolver_amd.models.multiframe import MultiFrameSARTSolver
    from mpi_cuda_sartsolver_amd.models.reference import sart_gpu_semantics
    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM
    from mpi_cuda_sartsolver_amd.models.sart import SolverParams

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(11)
    P, V, nframes = 800, 1000, 64
    A = rng.random((P, V), dtype=np.float32)
    b, d = rng.random(V) + 0.5, 0.01 * (rng.random(V) - 0.5)
    X = np.stack([b + t * d for t in range(nframes)])
    G = X @ A.T.astype(np.float64)
    kw = dict(max_iterations=300, conv_tolerance=1e-5)  # (the reference default; fp32 sums stall near 1e-7)
    rtm = DenseRTM.from_dense(A, device=dev)
    out = {}
    for drift in ("0", "1"):
        monkeypatch.setenv("SART_MF_DRIFT", drift)
        s = MultiFrameSARTSolver(rtm, None, None, SolverParams(**kw), batch=16)
        res = s.solve_batch(G, chain=True, record_starts=True)
        assert s.series_stats["drift"] == float(drift)
        assert all(r.status == 0 for r in res)
        out[drift] = (res, s.starts.copy())
    res, starts = out["1"]
    chained = [f for f in range(nframes) if res[f].warm_from >= 0]
    assert len(chained) > nframes // 2
    for f in chained[::7]:
        x, st, it = sart_gpu_semantics(A, G[f], None, x_prev=starts[f], **kw)
        assert res[f].status == st and abs(res[f].iterations - it) <= 2, (f, res[f].iterations, it)
    late = range(nframes // 2, nframes)  # (xlast and xlast2 both exist by then)
    dist = {k: np.mean([np.linalg.norm(v[1][f] - v[0][f].solution) / np.linalg.norm(v[0][f].solution) for f in late])
            for k, v in out.items()}
    assert any(not np.array_equal(out["0"][1][f], starts[f]) for f in late)
    assert dist["1"] < dist["0"], dist


@pytest.mark.parametrize("log", [False, True])
def test_multiframe_nonfinite_slot_is_rolled_back_and_refilled(monkeypatch, log):
    """A NaN injected into slot 0's iterate after sweep 5 (SART_FAULT_NAN) stops that frame at the next sweep:
    it returns its last finite iterate (5 updates, flagged non-finite) while the other frames continue, and the
    slot takes the next frame of the queue, which solves normally."""
    from mpi_cuda_sartsolver_amd.models.multiframe import MultiFrameSARTSolver
    from mpi_cuda_sartsolver_amd.models.reference import sart_gpu_semantics
    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM
    from mpi_cuda_sartsolver_amd.models.sart import SolverParams

    monkeypatch.setenv("SART_FAULT_NAN", "5")
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    P, V, nframes = 500, 800, 20
    A = rng.random((P, V), dtype=np.float32)
    G = (rng.random((nframes, V)) + 0.05) @ A.T.astype(np.float64)
    kw = dict(max_iterations=30, conv_tolerance=0.0)  # every frame runs 30 sweeps: slot 0 is live at sweep 5
    s = MultiFrameSARTSolver(DenseRTM.from_dense(A, device=dev), None, None, SolverParams(**kw), logarithmic=log,
                             batch=16, allow_zero_tolerance=True)
    res = s.solve_batch(G)
    assert res[0].nonfinite and res[0].iterations == 5 and np.all(np.isfinite(res[0].solution))
    check_fp32_bound(res[0].solution, A, G[0], None, log=log, iterations=5)
    for f in range(1, nframes):
        assert not res[f].nonfinite
        x, st, it = sart_gpu_semantics(A, G[f], None, logarithmic=log, **kw)
        assert res[f].status == st and abs(res[f].iterations - it) <= 2, (f, res[f].iterations, it)
    for f in (1, 16, nframes - 1):  # frame 16: the refill of the rolled-back slot
        check_fp32_bound(res[f].solution, A, G[f], None, log=log, iterations=res[f].iterations)


@pytest.mark.parametrize("log", [False, True])
@pytest.mark.parametrize("tol", [0.0, 1e-4])
def test_final_sweep_skips_backprojection_bitwise(monkeypatch, log, tol):
    """The batch's final sweep (every running frame decided at max_iter) runs the forward and the decision only;
    its back-projection and update would be discarded. Solutions, iteration counts, statuses and convergence
    values equal those of SART_MF_LAST_BWD=1 (the full final sweep) bit for bit, with slots refilled across chunk
    boundaries (40 frames through 16 slots, chunks of 5 sweeps)."""
    from mpi_cuda_sartsolver_amd.models.laplacian import LaplacianCSR
    from mpi_cuda_sartsolver_amd.models.multiframe import MultiFrameSARTSolver
    from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM
    from mpi_cuda_sartsolver_amd.models.sart import SolverParams

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(11)
    P, V, nframes = 600, 1000, 40
    A = rng.random((P, V), dtype=np.float32)
    G = (rng.random((nframes, V)) + 0.05) @ A.T.astype(np.float64)
    L = LaplacianCSR.grid_3d(10, 10, 10, device=dev)
    rtm = DenseRTM.from_dense(A, device=dev)
    out = {}
    for full in ("1", "0"):
        monkeypatch.setenv("SART_MF_LAST_BWD", full)
        s = MultiFrameSARTSolver(rtm, L, None, SolverParams(max_iterations=12, conv_tolerance=tol, beta_laplace=1e-3),
                                 logarithmic=log, batch=16, check_interval=5, allow_zero_tolerance=True)
        out[full] = s.solve_batch(G)
        del s
    for a, b in zip(out["1"], out["0"]):
        assert (a.status, a.iterations, a.convergence, a.nonfinite) == (b.status, b.iterations, b.convergence,
                                                                        b.nonfinite)
        assert np.array_equal(a.solution, b.solution)
    if tol == 0.0:  # fixed iteration count: every frame reaches the final-sweep decision
        assert all(r.iterations == 12 for r in out["0"])
