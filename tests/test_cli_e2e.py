"""End-to-end CLI runs on generated HDF5 cases: output file vs the fp64 oracle frame by frame. ``cli.main`` runs the
native driver as a child process, so its console output is captured at the file-descriptor level (capfd)."""
import math
import os

import numpy as np
import pytest

from mpi_cuda_sartsolver_amd import cli
from mpi_cuda_sartsolver_amd.io.fixtures import make_case
from mpi_cuda_sartsolver_amd.models.laplacian import LaplacianCSR
from mpi_cuda_sartsolver_amd.models.reference import sart_cpu_semantics, sart_gpu_semantics
from mpi_cuda_sartsolver_amd.ops import native


def _frames(case):
    """Composite frames of a fixture case (cameras share the time grid): masked pixels in name order."""
    nf = len(next(iter(case.times.values())))
    return [np.concatenate([case.frames[c][k].ravel()[case.masks[c].ravel() > 0] for c in sorted(case.masks)])
            for k in range(nf)]


def _laplacian(case):
    if not case.laplacian_file:
        return None
    i, j, v = native().read_laplacian(case.laplacian_file, case.nvoxel)
    return LaplacianCSR(case.nvoxel, i, j, v)


def _expected(case, oracle, warm=True, **kw):
    xs, sts, its = [], [], []
    prev = None
    for g in _frames(case):
        x, st, it = oracle(case.A, g, _laplacian(case), x_prev=prev if warm else None, **kw)
        xs.append(x), sts.append(st), its.append(it)
        prev = x
    return np.array(xs), np.array(sts), its


def chain_errors(case, out, *, log=False, warm=True, warm_from=None, warm_iter=None, warm_live=None, extrap=0.0,
                 beta_laplace=1e-3, A=None, orders=("blas",)):
    """Every frame of a CLI output file against the fp64 oracle of the reference GPU semantics, run for the frame's
    own recorded number of SART updates (solution/iterations) and warm-started like the run (warm: from frame k - 1;
    warm_from: from the listed frame, -1 cold) from the oracle's own solutions -- or, with warm_iter (the pipelined
    chain of --batch_frames), from the listed frame's oracle iterate after that many updates (extrapolated along its
    last update, x + extrap (x - x_prev), as the engine does for a source still in flight); next to it the fp32
    emulation of the same chain (its inherent fp32 error; the largest over the summation ``orders``, see
    sart_fp32_emulation). Returns (ours, fp32) relative errors per frame."""
    from mpi_cuda_sartsolver_amd.models.reference import sart_fp32_emulation

    n = native()
    X = n.read_dataset_f64(out, "solution/value")
    its = n.read_dataset_f64(out, "solution/iterations").astype(int)
    A = case.A if A is None else A
    L = _laplacian(case)
    kw = dict(logarithmic=log, beta_laplace=beta_laplace)
    e_ours, e_32 = [], []
    frames = _frames(case)
    s64, s32 = {}, {o: {} for o in orders}
    p64, p32 = {}, {o: {} for o in orders}  # each frame's start value (x_prev), for the iterates of in-flight sources

    def start(k, src):
        if src < 0:
            return None, {o: None for o in orders}
        n_it = None if warm_iter is None else int(warm_iter[k])
        if n_it is None or n_it < 0 or not (warm_live[k] if warm_live is not None else n_it < int(its[src])):
            return s64[src], {o: s32[o][src] for o in orders}
        def at(fn, n, x_prev, **k2):
            return fn(A, frames[src], L, max_iterations=n, x_prev=x_prev, **k2, **kw)[0]

        def ext(fn, x_prev, **k2):
            x = at(fn, n_it, x_prev, **k2)
            return x + extrap * (x - at(fn, n_it - 1, x_prev, **k2)) if extrap else x

        return (ext(sart_gpu_semantics, p64[src], conv_tolerance=0.0),
                {o: ext(sart_fp32_emulation, p32[o][src], order=o) for o in orders})

    for k, g in enumerate(frames):
        src = (warm_from[k] if warm_from is not None else (k - 1 if warm else -1))
        st64, st32 = start(k, src)
        p64[k] = st64
        x64, _, _ = sart_gpu_semantics(A, g, L, conv_tolerance=0.0, max_iterations=int(its[k]), x_prev=st64, **kw)
        nrm = np.linalg.norm(x64)
        e_ours.append(np.linalg.norm(X[k] - x64) / nrm)
        e = 0.0
        for o in orders:
            p32[o][k] = st32[o]
            x32, _, _ = sart_fp32_emulation(A, g, L, max_iterations=int(its[k]), x_prev=st32[o], order=o, **kw)
            e = max(e, np.linalg.norm(x32 - x64) / nrm)
            s32[o][k] = x32
        e_32.append(e)
        s64[k] = x64
    return np.array(e_ours), np.array(e_32)


# CLI runs are bounded like the solver tests (tests/test_gpu_solver.py): every frame within the fp32 emulation's error
# of the same chain (fixed update counts), so a 2x numerical regression of the end-to-end HDF5 path fails.
CLI_FP32_FACTOR = 1.0


def _read_all(path):
    import subprocess

    # read the whole value dataset through the native reader of the last row + the solution times
    n = native()
    t, last, st = n.read_solution_file(path)
    dump = subprocess.run(["/opt/conda/bin/h5dump", "-d", "/solution/value", "-y", "-w", "0", path],
                          capture_output=True, text=True)
    return t, last, st, dump.stdout


@pytest.mark.parametrize("log", [False, True])
@pytest.mark.parametrize("no_guess", [False, True])
def test_cli_cpu_matches_reference_cpu_semantics(tmp_path, capfd, log, no_guess):
    case = make_case(str(tmp_path / "c"), sparse_cameras=("cam_a",), laplacian=True, nframes=3, saturate=0.05)
    out = str(tmp_path / "out.h5")
    argv = ["--use_cpu", "-m", "120", "-c", "1e-6", "-l", case.laplacian_file, "-b", "1e-3", "-o", out]
    argv += (["-L"] if log else []) + (["--no_guess"] if no_guess else []) + case.files
    assert cli.main(argv) == 0
    assert capfd.readouterr().out.count("Processed in:") == 3
    xs, sts, its = _expected(case, sart_cpu_semantics, warm=not no_guess, logarithmic=log, max_iterations=120,
                             conv_tolerance=1e-6, beta_laplace=1e-3)
    t, last, st, _ = _read_all(out)
    np.testing.assert_allclose(t, next(iter(case.times.values())), atol=1e-12)
    np.testing.assert_array_equal(st, sts)
    np.testing.assert_allclose(last, xs[-1], rtol=1e-7, atol=1e-12 * np.abs(xs[-1]).max())


def test_cli_time_range_and_resume(tmp_path, capfd):
    case = make_case(str(tmp_path / "c"), nframes=6, dt=0.1)
    out = str(tmp_path / "out.h5")
    base = ["--use_cpu", "-m", "50", "-o", out]
    assert cli.main(base + ["-t", "0:0.25"] + case.files) == 0
    t, _, _ = native().read_solution_file(out)
    np.testing.assert_allclose(t, [0.0, 0.1, 0.2], atol=1e-12)
    capfd.readouterr()
    assert cli.main(base + ["--resume"] + case.files) == 0
    assert capfd.readouterr().out.count("Processed in:") == 3  # only the frames after t = 0.2
    t, last, _ = native().read_solution_file(out)
    np.testing.assert_allclose(t, 0.1 * np.arange(6), atol=1e-12)
    xs, _, _ = _expected(case, sart_cpu_semantics, max_iterations=50, conv_tolerance=1e-5, beta_laplace=2e-2)
    np.testing.assert_allclose(last, xs[-1], rtol=1e-7)


def test_cli_errors(tmp_path, capfd):
    case = make_case(str(tmp_path / "c"), nframes=2)
    assert cli.main(["--use_cpu", "-R", "3"] + case.files) == 1
    assert "relaxation" in capfd.readouterr().err
    assert cli.main(["--use_cpu", "-t", "100:200"] + case.files) == 1
    assert "No composite images" in capfd.readouterr().err
    assert cli.main(["--help"]) == 0
    assert "Usage: sartsolver" in capfd.readouterr().out


@pytest.mark.gpu
@pytest.mark.parametrize("log", [False, True])
@pytest.mark.parametrize("extra", [[], ["--two_pass"], ["--batch_frames", "4"]])
def test_cli_gpu_matches_gpu_semantics(tmp_path, capfd, log, extra):
    case = make_case(str(tmp_path / "c"), sparse_cameras=("cam_b",), laplacian=True, nframes=4, saturate=0.05,
                     nvoxel=2048, grid=(16, 16, 16), shapes=((24, 32), (20, 30)))
    out = str(tmp_path / "out.h5")
    argv = ["-m", "60", "-c", "1e-6", "-l", case.laplacian_file, "-b", "1e-3", "-o", out] + (["-L"] if log else [])
    batched = "--batch_frames" in extra
    argv += extra + (["--no_guess"] if batched else []) + case.files
    assert cli.main(argv) == 0
    xs, sts, its = _expected(case, sart_gpu_semantics, warm=not batched, logarithmic=log, max_iterations=60,
                             conv_tolerance=1e-6, beta_laplace=1e-3)
    t, last, st = native().read_solution_file(out)
    assert len(t) == 4
    np.testing.assert_array_equal(st, sts)  # same status per frame as the oracle's tolerance-stopped chain
    # every frame vs the oracle run for OUR recorded update counts, bounded by the fp32 emulation of that chain
    e, e32 = chain_errors(case, out, log=log, warm=not batched)
    assert np.all(e <= CLI_FP32_FACTOR * e32 + 1e-6), (e, e32)


@pytest.mark.gpu
@pytest.mark.parametrize("log", [False, True])
def test_cli_batched_time_series_warm_start(tmp_path, capfd, log):
    """--batch_frames keeps a warm-started time series (reference main.cpp:127-139) at MFMA throughput with
    device-side refill: 16 slots, the sweep in which a frame finishes admits the next one, which starts from the
    current iterate of the newest frame in flight (reported as warm_from / warm_iter in --profile; the first frame
    is solved alone, cold, by the single-frame engine). 3 cameras, 64 frames: the same status for every frame as the sequential
    warm-start series, every frame equal to the oracle of its own pipelined chain, and no more than twice the
    sequential chain's mean iterations per frame."""
    import json
    import time

    case = make_case(str(tmp_path / "c"), cameras=("cam_a", "cam_b", "cam_c"), shapes=((12, 16), (10, 14), (9, 12)),
                     laplacian=True, nframes=64, saturate=0.02, nvoxel=1024, grid=(16, 8, 8), seed=11)
    kw = ["-m", "400", "-c", "1e-4", "-l", case.laplacian_file, "-b", "1e-3"] + (["-L"] if log else [])
    okw = dict(logarithmic=log, max_iterations=400, conv_tolerance=1e-4, beta_laplace=1e-3)
    xs, sts, its = _expected(case, sart_gpu_semantics, warm=True, **okw)
    frames, L = _frames(case), _laplacian(case)
    walls = {}
    for mode, extra in (("batched", ["--batch_frames", "16"]), ("sequential", [])):
        out, prof = str(tmp_path / f"{mode}.h5"), str(tmp_path / f"{mode}.jsonl")
        t0 = time.perf_counter()
        assert cli.main(kw + extra + ["--profile", prof, "-o", out] + case.files) == 0
        walls[mode] = time.perf_counter() - t0
        assert capfd.readouterr().out.count("Processed in:") == 64
        t, last, st = native().read_solution_file(out)
        assert len(t) == 64
        np.testing.assert_array_equal(st, sts)  # same status per frame as the sequential warm-start series
        lines = [json.loads(ln) for ln in open(prof)]
        recs = [r for r in lines if "frame" in r]  # (first line: the RTM load; batched: a series summary last)
        walls[mode + "_iters"] = float(np.mean([r["iterations"] for r in recs]))
        if mode == "batched":
            # the batched chain's own oracle: each frame starts from its reported source iterate (the
            # underdetermined problem's tolerance-stopped answer depends on the initial guess)
            series = [r for r in lines if r.get("series")][0]
            cap = series["admit_cap"]
            nlead = sum(1 for r in recs if r.get("lead"))  # the lead frame: single-frame engine
            assert nlead == 1 and series["frames"] == 64 - nlead and 0 < series["slot_util"] <= 1.0
            wf = {r["frame"]: r["warm_from"] for r in recs}
            wi = {r["frame"]: r["warm_iter"] for r in recs}
            wl = {r["frame"]: r.get("warm_live", 0) for r in recs}
            # frame 0: the lead frame (single-frame engine, cold); every later frame chained to an earlier one
            assert wf[0] == -1 and all(0 <= wf[i] < i for i in range(1, 64)) and cap >= 1
            e, e32 = chain_errors(case, out, log=log, warm_from=[wf[i] for i in range(64)],
                                  warm_iter=[wi[i] for i in range(64)], warm_live=[wl[i] for i in range(64)],
                                  extrap=0.0 if log else series["src_extrap"])
        else:  # the sequential chain
            e, e32 = chain_errors(case, out, log=log, warm=True)
        # every frame within the fp32 emulation's error of the same chain (update counts as recorded)
        assert np.all(e <= CLI_FP32_FACTOR * e32 + 1e-6), (mode, e, e32)
        # the frames after the first (batched: the lead frame runs on the single-frame engine in both modes); not
        # compared: 1024 voxels x 530 pixels make both engines launch-bound (throughput: profiles/series_r6_*.jsonl)
        walls[mode + "_solve_ms"] = series["series_ms"] if mode == "batched" else sum(r["ms"] for r in recs[1:])
    # the pipelined chain keeps the warm start's iteration savings (round 5: the stale window start tripled them)
    assert walls["batched_iters"] <= 2.0 * walls["sequential_iters"] + 1.0, walls
