"""Multi-rank GPU solver path (row shards + collectives) on one GPU: ranks share cuda:0 and reduce over
gloo (SART_DIST_BACKEND=gloo); production runs one rank per GPU over RCCL with the same code."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(nproc, out, extra, script="dist_check.py", timeout=600, **env_extra):
    env = dict(os.environ, PYTHONPATH=ROOT, SART_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.update(env_extra)
    if nproc > 2:  # N ranks x queues within the 24 the GPU maps (a ceiling on the box's default 4, as bench.py)
        have = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
        env["GPU_MAX_HW_QUEUES"] = str(max(1, min(have, 12 // nproc)))
    path = os.path.join(ROOT, "tools", script)
    if nproc == 1:
        cmd = [sys.executable, path, "--out", out, *extra]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), path, "--out", out, *extra]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    if script != "dist_check.py":
        return json.load(open(out))
    return np.load(out + ".npy"), json.load(open(out + ".json"))


def _laplacian(nvox):
    from mpi_cuda_sartsolver_amd.models.laplacian import LaplacianCSR

    return LaplacianCSR.grid_3d(16, 16, 16) if nvox == 4096 else None  # as tools/dist_check.py


def _oracle_rel(tmp_path, xs, extra, iters):
    """Rel. errors of the solutions xs (frame 0) against the fp64 oracle of the 1-rank problem (saved by
    dist_check --save-problem), and the fp32 emulation's error on the same problem (the inherent fp32 error)."""
    from mpi_cuda_sartsolver_amd.models.reference import sart_fp32_emulation, sart_gpu_semantics

    A = np.load(str(tmp_path / "r1.A.npy"))
    g = np.load(str(tmp_path / "r1.g.npy"))
    L = _laplacian(A.shape[1])
    kw = dict(max_iterations=iters, beta_laplace=1e-3, logarithmic="--logarithmic" in extra)
    x64, _, _ = sart_gpu_semantics(A, g, L, conv_tolerance=0.0, **kw)
    x32, _, _ = sart_fp32_emulation(A, g, L, **kw)
    rel = lambda a: float(np.linalg.norm(a - x64) / np.linalg.norm(x64))  # noqa: E731
    return [rel(x) for x in xs], rel(x32)


# Multi-rank solutions are fp32 evaluations in another summation order (row blocks per rank, the all-reduce): every
# one must stay within the fp32 emulation's distance of the fp64 oracle (single-GPU kernels: 0.42-0.63x of it).
RANK_FACTOR = 1.0


@pytest.mark.parametrize("extra", [[], ["--logarithmic"], ["--multiframe"], ["--multiframe", "--logarithmic"],
                                   ["--columns"], ["--columns", "--logarithmic"]])
def test_gpu_solver_rank_invariance(tmp_path, extra):
    fixed = extra + ["--tol", "0", "--iters", "20"]
    x1, m1 = _run(1, str(tmp_path / "r1"), fixed + ["--save-problem"])
    x2, m2 = _run(2, str(tmp_path / "r2"), fixed)
    x3, m3 = _run(3, str(tmp_path / "r3"), fixed)
    (e1, e2, e3), e32 = _oracle_rel(tmp_path, [x1[0], x2[0], x3[0]], extra, 20)
    assert max(e1, e2, e3) <= RANK_FACTOR * e32 + 1e-7, (e1, e2, e3, e32)
    for m in (m2, m3):
        for a, b in zip(m, m1):
            assert a["status"] == b["status"] and a["iterations"] == b["iterations"]
    if "--multiframe" in extra:
        return
    # with the convergence test: the same statuses and (within 3) iteration counts at every rank count
    c1 = _run(1, str(tmp_path / "c1"), extra)[1]
    c3 = _run(3, str(tmp_path / "c3"), extra)[1]
    for a, b in zip(c3, c1):
        assert a["status"] == b["status"] and abs(a["iterations"] - b["iterations"]) <= 3


@pytest.mark.parametrize("log", [False, True])
def test_column_shard_matches_row_shard(tmp_path, log):
    """The voxel-sharded layout (all-reduce of A.x per sweep) solves the same problem as the reference's
    pixel-sharded layout (all-reduce of the correction)."""
    extra = ["--logarithmic"] if log else []
    fixed = extra + ["--tol", "0", "--iters", "20"]
    xr, mr = _run(1, str(tmp_path / "r1"), fixed + ["--save-problem"])
    xc, mc = _run(2, str(tmp_path / "cols"), fixed + ["--columns"])
    (er, ec), e32 = _oracle_rel(tmp_path, [xr[0], xc[0]], extra, 20)
    assert max(er, ec) <= RANK_FACTOR * e32 + 1e-7, (er, ec, e32)
    for a, b in zip(mc, mr):
        assert a["status"] == b["status"] and a["iterations"] == b["iterations"]


@pytest.mark.parametrize("nproc,blocks", [(2, 0), (3, 0), (4, 0), (8, 0), (2, 1024)])
def test_p2p_allreduce_bitwise(tmp_path, nproc, blocks):
    """One-shot P2P all-reduce (csrc/kernels/p2p_allreduce.hip) through IPC-mapped buffers of several
    processes on one GPU: bitwise equal to the rank-order sum / maximum at every size, both call parities;
    vectors above SART_P2P_MAX_BYTES go through the base communicator. 8 processes is the production rank count
    (one per GPU of a node); sharing one GPU they run with 32 / 8 = 4 workgroups per call, and the start-up
    (IPC mapping + self-test) stays under 10 s. blocks 1024: the launch shape of one rank per GPU (up to
    kP2pMaxBlocks = 1024 workgroups per call: 65 at the headline's 65538 floats, 512 at the 2 MiB cap) on the
    shared GPU (SART_P2P_BLOCKS)."""
    env = dict(SART_P2P="1", SART_P2P_TIMEOUT_S="30")
    if blocks:
        env["SART_P2P_BLOCKS"] = str(blocks)
    res = _run(nproc, str(tmp_path / "comm.json"), [], script="comm_check.py", **env)
    assert res["backend"] == "p2p", res["describe"]
    assert res["setup_s"] < 10.0, res["describe"]
    if nproc > 1:
        assert f"{nproc} ranks/GPU, {blocks or 32 // nproc} blocks" in res["describe"], res["describe"]
    for r in res["results"]:
        if r["n"] * 4 <= 2 * 1024 * 1024:
            assert r["exact"], r
        else:  # staged fallback: fp64 host reduction, rounded once
            assert r["close"], r


def test_p2p_auto_selection(tmp_path):
    """SART_P2P=auto times the P2P kernel against the base communicator at exactly the message sizes announced
    (Communicator::prepare, as the engines do) on rank 0 and serves the sizes at which P2P won (here against the
    host-staged base); a size between two probed ones follows the next larger probed size."""
    res = _run(2, str(tmp_path / "comm.json"), ["--sizes", "1,4097,65537,524288"], script="comm_check.py",
               SART_P2P="auto", SART_P2P_WRAP_STAGED="1")
    assert res["backend"] == "p2p" and res["describe"].startswith("p2p at floats"), res["describe"]
    assert "4097" in res["describe"].split("(rank 0")[0], res["describe"]
    assert all(r["exact"] for r in res["results"] if r["n"] <= 4097)
    assert res["prepare_s"] < 10.0, res


@pytest.mark.parametrize("extra", [[], ["--logarithmic"], ["--multiframe"],
                                   ["--multiframe", "--npix", "1024", "--nvox", "65536", "--iters", "12"]])
def test_gpu_solver_rank_invariance_p2p(tmp_path, extra):
    """(The last case has 4 MB of corrections per sweep: the multi-frame engine reduces them in 4 voxel chunks
    on its comm stream, overlapped with the back-projection of the following chunks.)"""
    iters = 12 if "--iters" in extra else 20
    fixed = [e for e in extra] + ["--tol", "0"] + ([] if "--iters" in extra else ["--iters", "20"])
    x1, m1 = _run(1, str(tmp_path / "r1"), fixed + ["--save-problem"])
    xs = []
    for n in (2, 3):
        x, m = _run(n, str(tmp_path / f"p{n}"), fixed, SART_P2P="1")
        assert m[0]["comm"] == "p2p"
        if "--multiframe" not in extra:
            assert m[0]["comm_ms"] > 0  # time_collectives: events around every per-sweep all-reduce
            assert m[0]["x_bitwise_equal"]
        for a, b in zip(m, m1):
            assert a["status"] == b["status"] and a["iterations"] == b["iterations"]
        xs.append(x[0])
    errs, e32 = _oracle_rel(tmp_path, [x1[0]] + xs, extra, iters)
    assert max(errs) <= RANK_FACTOR * e32 + 1e-7, (errs, e32)


@pytest.mark.parametrize("extra", [["--npix", "2048", "--nvox", "65536"],
                                   ["--multiframe", "--batch", "32", "--npix", "1024", "--nvox", "65536"]])
def test_p2p_production_launch_shape(tmp_path, extra):
    """The P2P all-reduce at the launch shape of one rank per GPU (SART_P2P_BLOCKS=1024, as on the 8-GPU node:
    65 workgroups for the single-frame 65538-float vector, 512 for a multi-frame chunk of 16384 voxels x 32 frames =
    the 2 MiB cap) with two ranks on the two-pass kernels: bitwise-equal replicated solutions, the same statuses and
    iteration counts as one rank, and the fp32-emulation bound."""
    fixed = extra + ["--tol", "0", "--iters", "12"]
    x1, m1 = _run(1, str(tmp_path / "r1"), fixed + ["--save-problem"])
    x, m = _run(2, str(tmp_path / "p2"), fixed, timeout=240, SART_P2P="1", SART_P2P_BLOCKS="1024",
                SART_P2P_TIMEOUT_S="30")
    assert m[0]["comm"] == "p2p"
    if "--multiframe" not in extra:
        assert m[0]["x_bitwise_equal"] and "1024 blocks" in m[0]["describe"], m[0]
    for a, b in zip(m, m1):
        assert a["status"] == b["status"] and a["iterations"] == b["iterations"]
    errs, e32 = _oracle_rel(tmp_path, [x1[0], x[0]], extra, 12)
    assert max(errs) <= RANK_FACTOR * e32 + 1e-7, (errs, e32)


@pytest.mark.parametrize("fault_rank", ["", "1", "skip"])
def test_rccl_init_failure_degrades_to_staged(tmp_path, fault_rank):
    """A failed RCCL bring-up (SART_FAULT_RCCL_INIT: on every rank, or reported by rank 1 only after the collective
    init; "skip": rank 1 never enters the init, SART_FAULT_RCCL_INIT_SKIP, so rank 0 waits in its non-blocking init
    until SART_RCCL_INIT_TIMEOUT_S and aborts it) is agreed on over the host communicator: every rank continues on
    staged collectives wrapped by the P2P all-reduce instead of failing (or hanging) the run, ``describe`` names the
    failure, and a 2-rank solve matches the 1-rank one at the fp32-emulation bound within the deadline + 30 s.
    (Without SART_DIST_BACKEND the ranks ask for RCCL, as on the node.)"""
    import time

    fixed = ["--tol", "0", "--iters", "12"]
    x1, m1 = _run(1, str(tmp_path / "r1"), fixed + ["--save-problem"])
    env = dict(SART_DIST_BACKEND="", SART_FAULT_RCCL_INIT="1", SART_P2P="1", SART_P2P_TIMEOUT_S="30")
    if fault_rank == "skip":
        env = dict(SART_DIST_BACKEND="", SART_FAULT_RCCL_INIT_SKIP="1", SART_RCCL_INIT_TIMEOUT_S="10", SART_P2P="1",
                   SART_P2P_TIMEOUT_S="30")
    elif fault_rank:
        env["SART_FAULT_RANK"] = fault_rank
    t0 = time.perf_counter()
    x, m = _run(2, str(tmp_path / "f2"), fixed, timeout=240, **env)
    if fault_rank == "skip":
        assert time.perf_counter() - t0 < 10 + 30 + 60, "the init deadline did not bound the bring-up"
    d = m[0]["describe"]
    assert m[0]["comm"] == "p2p" and "RCCL init failed" in d and "staged" in d, d
    assert m[0]["x_bitwise_equal"]
    for a, b in zip(m, m1):
        assert a["status"] == b["status"] and a["iterations"] == b["iterations"]
    errs, e32 = _oracle_rel(tmp_path, [x1[0], x[0]], [], 12)
    assert max(errs) <= RANK_FACTOR * e32 + 1e-7, (errs, e32)


def test_p2p_peer_abort_fails_fast(tmp_path):
    """A rank that aborts writes the abort word of every peer: a peer waiting in the P2P all-reduce stops
    within seconds (NaN output, check() raises) instead of polling until SART_P2P_TIMEOUT_S (120 s here)."""
    out = str(tmp_path / "abort.json")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "p2p_abort_check.py"), "--out", out],
                       capture_output=True, text=True, timeout=400, env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.load(open(out))
    assert res["backend"] == "p2p" and res["first_ok"]
    assert "aborted" in res["error"] and res["nan"] and res["seconds"] < 30, res


def test_shared_device_detected_from_identity(tmp_path):
    """Ranks on one physical GPU are detected from the device identity (boot id + host + PCI bus id, not
    LOCAL_WORLD_SIZE, which only torchrun sets) on every rank, and use the two-pass kernels when the fused sweep is
    requested without SART_FUSED_SHARED=1."""
    x, m = _run(2, str(tmp_path / "s2"), ["--fused"], LOCAL_WORLD_SIZE="1")
    assert all(r["shared"] and not r["fused"] and r["ranks_per_device"] == 2 for r in m[0]["ranks"]), m[0]["ranks"]


FUSED_SHAPE = ["--fused", "--npix", "8192", "--nvox", "32768", "--iters", "20", "--tol", "0"]


@pytest.mark.parametrize("nproc", [2, 4])
def test_fused_sweep_on_shared_gpu(tmp_path, nproc):
    """The production multi-rank path on ONE GPU: 2 / 4 ranks, each running the fused sweep (variant 6) on its own
    share of the CUs (SART_FUSED_SHARED=1: persistent grids planned for 256 / N CUs, side by side), with the
    one-shot P2P all-reduce of the corrections every sweep (32 / N workgroups per call, so the spinning all-reduce
    workgroups of the ranks ahead leave the CUs a lagging rank's sweep needs). Every rank reports fused, no
    fallback and comm p2p; the replicated x is bitwise identical on every rank; the 1-rank and the N-rank
    solutions are within the fp32 emulation's error of the fp64 oracle (reference loop:
    sartsolver_cuda.cpp:231-262)."""
    x1, m1 = _run(1, str(tmp_path / "r1"), FUSED_SHAPE + ["--save-problem"])
    assert m1[0]["fused"] and m1[0]["ranks"][0]["plan_cus"] >= 128
    xn, mn = _run(nproc, str(tmp_path / f"p{nproc}"), FUSED_SHAPE, SART_FUSED_SHARED="1", SART_P2P="1")
    ranks = mn[0]["ranks"]
    for r in ranks:
        assert r["fused"] and r["variant"] == 6 and r["fallbacks"] == 0 and r["fallbacks2"] == 0, ranks
        assert r["comm"] == "p2p" and r["comm_fallbacks"] == 0 and r["ranks_per_device"] == nproc, ranks
        assert r["plan_cus"] * nproc <= m1[0]["ranks"][0]["plan_cus"], ranks
        assert r["grid"]["workgroups"] <= r["plan_cus"], ranks
    assert mn[0]["x_bitwise_equal"]
    for a, b in zip(mn, m1):
        assert a["status"] == b["status"] == -1 and a["iterations"] == b["iterations"] == 20
    (e1, e2), e32 = _oracle_rel(tmp_path, [x1[0], xn[0]], [], 20)
    assert max(e1, e2) <= RANK_FACTOR * e32 + 1e-7, (e1, e2, e32)


@pytest.mark.parametrize("shape", [["--tol", "0"], ["--tol", "1e-5", "--logarithmic"], FUSED_SHAPE,
                                   FUSED_SHAPE + ["--logarithmic"], ["--npix", "4096", "--nvox", "65536"]])
def test_p2p_fused_reduce_is_bitwise(tmp_path, shape):
    """At N > 1 the P2P kernel forms the per-sweep vector from the partial rows itself (one launch instead of
    k_reduce_partials + the all-reduce) and, by default, also decides and updates x (one launch instead of three:
    every workgroup takes ||A x||^2 from the tail slots of all ranks). x, status and iterations are bitwise those of
    the three-launch path (SART_P2P_FUSED_REDUCE=0) and of the two-launch one (SART_P2P_FUSED_UPDATE=0), on the
    two-pass and the fused sweep, with and without the convergence test (the last case: 65 workgroups)."""
    env = dict(SART_P2P="1", SART_FUSED_SHARED="1")
    runs = {}
    for tag, extra in (("three", dict(SART_P2P_FUSED_REDUCE="0")), ("two", dict(SART_P2P_FUSED_UPDATE="0")),
                       ("one", {})):
        runs[tag] = _run(2, str(tmp_path / tag), shape, **env, **extra)
    for x, m in runs.values():
        assert m[0]["comm"] == "p2p" and m[0]["x_bitwise_equal"]
    xa, ma = runs["three"]
    for tag in ("two", "one"):
        xb, mb = runs[tag]
        for a, b in zip(ma, mb):
            assert a["status"] == b["status"] and a["iterations"] == b["iterations"], (tag, a, b)
        assert np.array_equal(xa, xb), tag


@pytest.mark.parametrize("fused", [False, True])
def test_p2p_timeout_degrades_to_base_on_every_rank(tmp_path, fused):
    """A P2P all-reduce that times out on some rank mid-solve (SART_FAULT_P2P: rank 1 never raises its flags in
    its 3rd call, so rank 0 waits SART_P2P_TIMEOUT_S) is agreed on after the solve: EVERY rank switches to the
    base communicator (staged here, RCCL in production) and re-solves the frame; the result matches the 1-rank
    solve and later frames stay on the base path. A stall costs about one timeout, not one per queued sweep."""
    import time

    extra = FUSED_SHAPE if fused else ["--iters", "20", "--tol", "0"]
    x1, m1 = _run(1, str(tmp_path / "r1"), extra + ["--save-problem"])
    env = dict(SART_P2P="1", SART_FAULT_P2P="3", SART_FAULT_RANK="1", SART_P2P_TIMEOUT_S="4")
    if fused:
        env["SART_FUSED_SHARED"] = "1"
    t0 = time.monotonic()
    x, m = _run(2, str(tmp_path / "f2"), extra, **env)
    wall = time.monotonic() - t0
    ranks = m[0]["ranks"]
    for r in ranks:
        assert r["comm_fallbacks"] == 1 and r["comm"] == "staged", ranks
        assert r["comm_fallbacks2"] == 0 and r["comm2"] == "staged", ranks
        assert r["fused"] == fused and r["fallbacks"] == 0, ranks
    assert m[0]["x_bitwise_equal"]
    assert wall < 120, wall
    (e1, e2), e32 = _oracle_rel(tmp_path, [x1[0], x[0]], [], 20)
    assert max(e1, e2) <= RANK_FACTOR * e32 + 1e-7, (e1, e2, e32)


def test_p2p_timeout_degrades_multiframe(tmp_path):
    """The multi-frame engine's chunked all-reduce on its comm stream: a P2P stall on rank 1 (SART_FAULT_P2P) is
    agreed on after the batch, every rank re-solves the batch on the staged base, and every frame matches the 1-rank
    batch within the fp32 emulation's error of the oracle."""
    extra = ["--multiframe", "--iters", "20", "--tol", "0"]
    x1, m1 = _run(1, str(tmp_path / "r1"), extra + ["--save-problem"])
    x, m = _run(2, str(tmp_path / "f2"), extra, SART_P2P="1", SART_FAULT_P2P="4", SART_FAULT_RANK="1",
                SART_P2P_TIMEOUT_S="4")
    for r in m[0]["ranks"]:
        assert r["comm"] == "staged" and r["comm_fallbacks"] == 1, m[0]["ranks"]
    assert all(f["comm"] == "staged" for f in m)
    (e1, e2), e32 = _oracle_rel(tmp_path, [x1[0], x[0]], extra, 20)
    assert max(e1, e2) <= RANK_FACTOR * e32 + 1e-7, (e1, e2, e32)


@pytest.mark.parametrize("nproc", [2, 3])
def test_fused_timeout_on_one_rank_falls_back_on_all(tmp_path, nproc):
    """A persistent-sweep timeout reported by ONE rank (device-side fault injection on rank 1) reaches every
    rank through the error word of the per-sweep all-reduce: all ranks stop the frame at the same sweep,
    fall back together (v6 -> v3 ...), re-solve, and the result matches the 1-rank solve. A rank-local
    decision would leave the peers blocked in the next collective (round-1 advisor finding)."""
    x1, m1 = _run(1, str(tmp_path / "r1"), ["--fused"])
    assert m1[0]["fused"] and m1[0]["fallbacks"] == 0
    x, m = _run(nproc, str(tmp_path / f"f{nproc}"), ["--fused"], SART_FUSED_SHARED="1", SART_FAULT_INJECT="1",
                SART_FAULT_RANK="1")
    ranks = m[0]["ranks"]
    assert len(ranks) == nproc
    assert ranks[0]["fallbacks"] >= 1, ranks
    assert all((r["fallbacks"], r["variant"], r["fused"]) == (ranks[0]["fallbacks"], ranks[0]["variant"],
                                                              ranks[0]["fused"]) for r in ranks), ranks
    assert np.linalg.norm(x - x1) / np.linalg.norm(x1) < 2e-3
    for a, b in zip(m, m1):
        assert a["status"] == b["status"] and abs(a["iterations"] - b["iterations"]) <= 3
