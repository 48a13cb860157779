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


def _run(nproc, out, extra, script="dist_check.py", **env_extra):
    env = dict(os.environ, PYTHONPATH=ROOT, SART_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", **env_extra)
    path = os.path.join(ROOT, "tools", script)
    if nproc == 1:
        cmd = [sys.executable, path, "--out", out, *extra]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), path, "--out", out, *extra]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    if script != "dist_check.py":
        return json.load(open(out))
    return np.load(out + ".npy"), json.load(open(out + ".json"))


@pytest.mark.parametrize("extra", [[], ["--logarithmic"], ["--multiframe"], ["--multiframe", "--logarithmic"],
                                   ["--columns"], ["--columns", "--logarithmic"]])
def test_gpu_solver_rank_invariance(tmp_path, extra):
    x1, m1 = _run(1, str(tmp_path / "r1"), extra)
    x2, m2 = _run(2, str(tmp_path / "r2"), extra)
    x3, m3 = _run(3, str(tmp_path / "r3"), extra)
    for x, m in ((x2, m2), (x3, m3)):
        assert np.linalg.norm(x - x1) / np.linalg.norm(x1) < 2e-3
        for a, b in zip(m, m1):
            assert a["status"] == b["status"] and abs(a["iterations"] - b["iterations"]) <= 3


@pytest.mark.parametrize("log", [False, True])
def test_column_shard_matches_row_shard(tmp_path, log):
    """The voxel-sharded layout (all-reduce of A.x per sweep) solves the same problem as the reference's
    pixel-sharded layout (all-reduce of the correction)."""
    extra = ["--logarithmic"] if log else []
    xr, mr = _run(1, str(tmp_path / "rows"), extra)
    xc, mc = _run(2, str(tmp_path / "cols"), extra + ["--columns"])
    assert np.linalg.norm(xc - xr) / np.linalg.norm(xr) < 2e-3
    for a, b in zip(mc, mr):
        assert a["status"] == b["status"] and abs(a["iterations"] - b["iterations"]) <= 3


@pytest.mark.parametrize("nproc", [2, 3])
def test_p2p_allreduce_bitwise(tmp_path, nproc):
    """One-shot P2P all-reduce (csrc/kernels/p2p_allreduce.hip) through IPC-mapped buffers of several
    processes on one GPU: bitwise equal to the rank-order sum / maximum at every size, both call parities;
    vectors above SART_P2P_MAX_BYTES go through the base communicator."""
    res = _run(nproc, str(tmp_path / "comm.json"), [], script="comm_check.py", SART_P2P="1")
    assert res["backend"] == "p2p", res["describe"]
    for r in res["results"]:
        if r["n"] * 4 <= 2 * 1024 * 1024:
            assert r["exact"], r
        else:  # staged fallback: fp64 host reduction, rounded once
            assert r["close"], r


def test_p2p_auto_selection(tmp_path):
    """SART_P2P=auto times the P2P kernel against the base communicator at 4k .. 512k floats on rank 0 and
    serves vectors up to the largest size at which P2P won (here against the host-staged base)."""
    res = _run(2, str(tmp_path / "comm.json"), ["--sizes", "1,4097,65537,524288"], script="comm_check.py",
               SART_P2P="auto", SART_P2P_WRAP_STAGED="1")
    assert res["backend"] == "p2p" and res["describe"].startswith("p2p up to"), res["describe"]
    assert all(r["exact"] for r in res["results"] if r["n"] <= 4097)


@pytest.mark.parametrize("extra", [[], ["--logarithmic"], ["--multiframe"],
                                   ["--multiframe", "--npix", "1024", "--nvox", "65536", "--iters", "12"]])
def test_gpu_solver_rank_invariance_p2p(tmp_path, extra):
    """(The last case has 4 MB of corrections per sweep: the multi-frame engine reduces them in 4 voxel chunks
    on its comm stream, overlapped with the back-projection of the following chunks.)"""
    x1, m1 = _run(1, str(tmp_path / "r1"), extra)
    # different row partitions sum in different orders: fp32 drift grows with the width (3e-3 measured at
    # 65536 voxels x 12 iterations; profiles/numerics_r2.jsonl)
    tol = 6e-3 if "65536" in extra else 2e-3
    for n in (2, 3):
        x, m = _run(n, str(tmp_path / f"p{n}"), extra, SART_P2P="1")
        assert m[0]["comm"] == "p2p"
        if "--multiframe" not in extra:
            assert m[0]["comm_ms"] > 0  # time_collectives: events around every per-sweep all-reduce
        assert np.linalg.norm(x - x1) / np.linalg.norm(x1) < tol
        for a, b in zip(m, m1):
            assert a["status"] == b["status"] and abs(a["iterations"] - b["iterations"]) <= 3


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
    """Ranks on one physical GPU are detected from the PCI bus id (not LOCAL_WORLD_SIZE, which only torchrun
    sets) on every rank, and use the two-pass kernels even when the fused sweep is requested."""
    x, m = _run(2, str(tmp_path / "s2"), ["--fused"], LOCAL_WORLD_SIZE="1")
    assert all(r["shared"] and not r["fused"] for r in m[0]["ranks"]), m[0]["ranks"]


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
