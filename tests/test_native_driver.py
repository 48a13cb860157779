"""The native ``sartsolver`` executable (csrc/driver/sartsolver_main.cpp) against the fp64 oracle, and the Python
entry point ``python -m mpi_cuda_sartsolver_amd`` (a launcher of that executable, cli.py): same arguments, same
output file bit for bit, multi-rank runs under torchrun (--no-python for the executable itself) and mpiexec."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from mpi_cuda_sartsolver_amd.io.fixtures import make_case
from mpi_cuda_sartsolver_amd.ops import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "mpi_cuda_sartsolver_amd", "_lib", "sartsolver")


@pytest.fixture(scope="module")
def binary():
    from mpi_cuda_sartsolver_amd import _build

    if not _build.hdf5_available():
        pytest.skip("HDF5 not available")
    _build.build_driver(verbose=False)
    return BIN


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env():
    return dict(os.environ, OMP_NUM_THREADS="2", HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONPATH=ROOT)


def _run_native(binary, args, nproc=1, cwd=None):
    if nproc == 1:
        cmd = [binary, *args]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), "--no-python", binary, *args]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=_env(), cwd=cwd)


def _run_python(args, cwd=None):
    cmd = [sys.executable, "-m", "mpi_cuda_sartsolver_amd", *args]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=_env(), cwd=cwd)


def _case(tmp_path, **kw):
    opts = dict(sparse_cameras=("cam_b",), laplacian=True, nframes=3, saturate=0.05)
    opts.update(kw)
    return make_case(str(tmp_path / "case"), **opts)


@pytest.mark.parametrize("log", [False, True])
def test_native_cpu_module_entry_point_forwards(tmp_path, binary, log):
    """python -m mpi_cuda_sartsolver_amd launches the same executable (cli.py): arguments and output forwarded, the
    file bit for bit (the CPU solver's parity with the reference CPU semantics: test_cli_e2e)."""
    case = _case(tmp_path)
    base = ["--use_cpu", "-m", "80", "-c", "1e-7", "-l", case.laplacian_file, "-b", "1e-3"] + (["-L"] if log else [])
    r1 = _run_native(binary, base + ["-o", str(tmp_path / "n.h5"), *case.files])
    assert r1.returncode == 0, r1.stdout + r1.stderr
    assert r1.stdout.count("Processed in:") == 3
    r2 = _run_python(base + ["-o", str(tmp_path / "p.h5"), *case.files])
    assert r2.returncode == 0, r2.stdout + r2.stderr
    n = native()
    t1, x1, s1 = n.read_solution_file(str(tmp_path / "n.h5"))
    t2, x2, s2 = n.read_solution_file(str(tmp_path / "p.h5"))
    np.testing.assert_array_equal(t1, t2)
    np.testing.assert_array_equal(s1, s2)
    np.testing.assert_array_equal(x1, x2)  # same C++ solver, same thread count: bitwise


def test_native_cpu_ranks_invariance_and_resume(tmp_path, binary):
    case = _case(tmp_path, nframes=4, dt=0.1)
    base = ["--use_cpu", "-m", "60", "-c", "1e-7", "-l", case.laplacian_file, "-b", "1e-3"]
    one = str(tmp_path / "one.h5")
    r = _run_native(binary, base + ["-o", one, *case.files])
    assert r.returncode == 0, r.stderr
    two = str(tmp_path / "two.h5")
    r = _run_native(binary, base + ["-o", two, *case.files], nproc=2)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    n = native()
    t1, x1, s1 = n.read_solution_file(one)
    t2, x2, s2 = n.read_solution_file(two)
    np.testing.assert_array_equal(t1, t2)
    np.testing.assert_array_equal(s1, s2)
    np.testing.assert_allclose(x2, x1, rtol=1e-8)
    # resume: the first two frames, then the rest appended
    part = str(tmp_path / "part.h5")
    r = _run_native(binary, base + ["-t", "0:0.15", "-o", part, *case.files])
    assert r.returncode == 0, r.stderr
    r = _run_native(binary, base + ["--resume", "-o", part, *case.files])
    assert r.returncode == 0, r.stderr
    assert r.stdout.count("Processed in:") == 2
    t3, x3, _ = n.read_solution_file(part)
    np.testing.assert_allclose(t3, t1, atol=1e-12)
    np.testing.assert_allclose(x3, x1, rtol=1e-10)


MPIEXEC = "/opt/conda/bin/mpiexec"


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="MPICH mpiexec not installed")
@pytest.mark.parametrize("nproc", [2, 3])
def test_native_cpu_under_mpiexec(tmp_path, binary, nproc):
    """The reference's own launch (mpiexec, host MPI collectives on MPI_COMM_WORLD): the MPI host
    communicator (host_comm_mpi.cpp, libmpi loaded at run time) gives the single-rank solution."""
    case = _case(tmp_path)
    base = ["--use_cpu", "-m", "60", "-c", "1e-7", "-l", case.laplacian_file, "-b", "1e-3"]
    one = str(tmp_path / "one.h5")
    r = _run_native(binary, base + ["-o", one, *case.files])
    assert r.returncode == 0, r.stderr
    out, prof = str(tmp_path / "mpi.h5"), str(tmp_path / "mpi.jsonl")
    env = {k: v for k, v in _env().items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([MPIEXEC, "-n", str(nproc), binary, *base, "--profile", prof, "-o", out, *case.files],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.count("Processed in:") == 3  # rank 0 only
    import json

    lines = [json.loads(s) for s in open(prof)]
    assert lines and all(d["comm"] == "mpi" and d["ranks"] == nproc for d in lines)
    n = native()
    t1, x1, s1 = n.read_solution_file(one)
    t2, x2, s2 = n.read_solution_file(out)
    np.testing.assert_array_equal(t1, t2)
    np.testing.assert_array_equal(s1, s2)
    np.testing.assert_allclose(x2, x1, rtol=1e-8, atol=1e-12)


def test_native_cli_errors(tmp_path, binary):
    case = _case(tmp_path, nframes=1)
    r = _run_native(binary, ["--use_cpu", "-R", "3", *case.files])
    assert r.returncode == 1 and "relaxation" in r.stderr
    r = _run_native(binary, ["--use_cpu", "-t", "100:200", *case.files])
    assert r.returncode == 1 and "No composite images" in r.stderr
    r = _run_native(binary, ["--use_cpu", case.files[0]])
    assert r.returncode == 1
    r = _run_native(binary, ["--help"])
    assert r.returncode == 0 and "Usage: sartsolver" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("log", [False, True])
@pytest.mark.parametrize("extra", [[], ["--batch_frames", "2", "--no_guess"]])
def test_native_gpu_vs_oracle_and_module_entry_point(tmp_path, binary, log, extra):
    """The native driver on the GPU: every frame within the fp32 emulation's error of the fp64 oracle chain run for
    the recorded update counts (test_cli_e2e.chain_errors: an independent parity check of the frame loop, warm
    starts and output); --profile's first line reports the HDF5 -> HBM load, the others the solves. Then the module
    entry point (python -m mpi_cuda_sartsolver_amd, cli.py) must forward the arguments and exit code to the same
    executable: bitwise the same file."""
    from test_cli_e2e import CLI_FP32_FACTOR, chain_errors

    case = make_case(str(tmp_path / "c"), sparse_cameras=("cam_b",), laplacian=True, nframes=3, saturate=0.05,
                     nvoxel=2048, grid=(16, 16, 16), shapes=((24, 32), (20, 30)))
    base = ["-m", "60", "-c", "1e-6", "-l", case.laplacian_file, "-b", "1e-3"] + (["-L"] if log else []) + extra
    prof = str(tmp_path / "n.jsonl")
    r1 = _run_native(binary, base + ["--profile", prof, "-o", str(tmp_path / "n.h5"), *case.files])
    assert r1.returncode == 0, r1.stdout + r1.stderr
    recs = [json.loads(line) for line in open(prof)]
    load = recs[0]
    assert load.get("load") and load["rtm_GB"] > 0 and load["load_s"] > 0 and load["rank0"]["blocks"] >= 1, load
    assert load["sparse"] is True  # cam_b is a sparse COO file
    for rec in recs[1:]:  # bytes of the fp32 shard: 4 per element, one (fused) or two reads per sweep
        assert "load" not in rec
        if "rtm_GBps" in rec:  # (batched frames report per-frame times only)
            assert abs(rec["rtm_GBps"] / rec["gflops"] - (1 if rec["fused"] else 2)) < 1e-4, rec  # 6 printed digits
    e, e32 = chain_errors(case, str(tmp_path / "n.h5"), log=log, warm="--no_guess" not in extra)
    assert np.all(e <= CLI_FP32_FACTOR * e32 + 1e-6), (e, e32)
    r2 = _run_python(base + ["-o", str(tmp_path / "p.h5"), *case.files])
    assert r2.returncode == 0, r2.stdout + r2.stderr
    n = native()
    t1, x1, s1 = n.read_solution_file(str(tmp_path / "n.h5"))
    t2, x2, s2 = n.read_solution_file(str(tmp_path / "p.h5"))
    np.testing.assert_array_equal(t1, t2)
    np.testing.assert_array_equal(s1, s2)
    np.testing.assert_array_equal(x1, x2)  # the same executable behind both entry points: bitwise


@pytest.mark.gpu
@pytest.mark.parametrize("p2p", ["0", "1"])
def test_native_gpu_two_ranks_one_device(tmp_path, binary, p2p):
    """Two ranks on the box's single GPU, staged (TCP) reductions or the one-shot P2P all-reduce through
    IPC-mapped buffers: equals the one-rank run; --profile reports the GPU time in the all-reduces."""
    case = make_case(str(tmp_path / "c"), laplacian=True, nframes=2, nvoxel=2048, grid=(16, 16, 16),
                     shapes=((24, 32), (20, 30)))
    base = ["-m", "40", "-c", "1e-6", "-l", case.laplacian_file, "-b", "1e-3", "--two_pass"]
    r = _run_native(binary, base + ["-o", str(tmp_path / "one.h5"), *case.files])
    assert r.returncode == 0, r.stderr
    saved = {k: os.environ.get(k) for k in ("SART_DIST_BACKEND", "SART_P2P")}
    os.environ["SART_DIST_BACKEND"] = "tcp"
    os.environ["SART_P2P"] = p2p
    prof = str(tmp_path / "prof.jsonl")
    try:
        r = _run_native(binary, base + ["--profile", prof, "-o", str(tmp_path / "two.h5"), *case.files], nproc=2)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    import json

    lines = [json.loads(x) for x in open(prof)]
    assert lines[0]["load"] and lines[0]["ranks"] == 2  # the HDF5 -> HBM load of both ranks
    lines = lines[1:]
    assert len(lines) == 2 and all(d["ranks"] == 2 and d["comm_ms"] >= 0 and d["sweeps"] >= 1 for d in lines)
    assert lines[0]["device_comm"].startswith("p2p" if p2p == "1" else "staged"), lines[0]["device_comm"]
    n = native()
    _, x1, s1 = n.read_solution_file(str(tmp_path / "one.h5"))
    _, x2, s2 = n.read_solution_file(str(tmp_path / "two.h5"))
    np.testing.assert_array_equal(s1, s2)
    assert np.linalg.norm(x2 - x1) / np.linalg.norm(x1) < 2e-3


@pytest.mark.gpu
@pytest.mark.parametrize("log", [False, True])
def test_partition_voxels_cli(tmp_path, binary, log):
    """--partition_voxels (voxel-column shards, all-reduce of A x): 1 and 2 ranks of the native driver and
    2 ranks of the Python driver agree with the pixel-row run (Laplacian, warm starts, sparse camera)."""
    case = make_case(str(tmp_path / "c"), sparse_cameras=("cam_b",), laplacian=True, nframes=2, nvoxel=2048,
                     grid=(16, 16, 16), shapes=((24, 32), (20, 30)))
    base = ["-m", "40", "-c", "1e-6", "-l", case.laplacian_file, "-b", "1e-3", "--two_pass"] + (["-L"] if log else [])
    r = _run_native(binary, base + ["-o", str(tmp_path / "rows.h5"), *case.files])
    assert r.returncode == 0, r.stderr
    outs = {}
    env_backend = os.environ.get("SART_DIST_BACKEND")
    os.environ["SART_DIST_BACKEND"] = "tcp"
    try:
        for name, nproc, runner in (("v1", 1, "native"), ("v2", 2, "native"), ("p2", 2, "python")):
            out = str(tmp_path / f"{name}.h5")
            args = base + ["--partition_voxels", "-o", out, *case.files]
            if runner == "native":
                r = _run_native(binary, args, nproc=nproc)
            else:
                os.environ["SART_DIST_BACKEND"] = "gloo"
                cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
                       "--master-addr", "127.0.0.1", "--master-port", str(_port()), "-m", "mpi_cuda_sartsolver_amd",
                       *args]
                r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=_env())
            assert r.returncode == 0, name + r.stdout[-2000:] + r.stderr[-4000:]
            outs[name] = out
    finally:
        if env_backend is None:
            os.environ.pop("SART_DIST_BACKEND", None)
        else:
            os.environ["SART_DIST_BACKEND"] = env_backend
    n = native()
    t0, x0, s0 = n.read_solution_file(str(tmp_path / "rows.h5"))
    for name, out in outs.items():
        t, x, s = n.read_solution_file(out)
        np.testing.assert_array_equal(t, t0)
        np.testing.assert_array_equal(s, s0)
        assert np.linalg.norm(x - x0) / np.linalg.norm(x0) < 2e-3, name


@pytest.mark.gpu
@pytest.mark.parametrize("log", [False, True])
@pytest.mark.parametrize("two_pass", [False, True])
def test_rtm_bf16_cli(tmp_path, binary, log, two_pass):
    """--rtm_bf16: the native driver (HDF5 blocks rounded into a bf16 shard on the device) and the Python
    driver (DenseRTM.to_bf16) run the same engine bit for bit, and match the fp64 oracle of the reference GPU
    semantics on the bf16-rounded matrix."""
    import torch

    from mpi_cuda_sartsolver_amd.models.reference import sart_gpu_semantics

    case = make_case(str(tmp_path / "c"), sparse_cameras=("cam_b",), laplacian=False, nframes=2, saturate=0.05,
                     nvoxel=2048, grid=(16, 16, 8), shapes=((24, 32), (20, 30)))
    base = ["-m", "40", "-c", "1e-9", "--rtm_bf16"] + (["-L"] if log else []) + (["--two_pass"] if two_pass else [])
    prof = str(tmp_path / "n.jsonl")
    r1 = _run_native(binary, base + ["--profile", prof, "-o", str(tmp_path / "n.h5"), *case.files])
    assert r1.returncode == 0, r1.stdout + r1.stderr
    for line in open(prof):  # bytes of the bf16 shard: 2 per element, one (fused) or two reads per sweep
        rec = json.loads(line)
        if rec.get("load"):
            continue
        reads = 1 if rec["fused"] else 2
        assert abs(rec["rtm_GBps"] / rec["gflops"] - reads * 2 / 4) < 1e-4, rec  # (6 printed digits)
    r2 = _run_python(base + ["-o", str(tmp_path / "p.h5"), *case.files])
    assert r2.returncode == 0, r2.stdout + r2.stderr
    n = native()
    t1, x1, s1 = n.read_solution_file(str(tmp_path / "n.h5"))
    t2, x2, s2 = n.read_solution_file(str(tmp_path / "p.h5"))
    np.testing.assert_array_equal(s1, s2)
    np.testing.assert_array_equal(x1, x2)
    Ar = torch.from_numpy(np.ascontiguousarray(case.A, dtype=np.float32)).to(torch.bfloat16).float().numpy()
    prev = None
    for k in range(2):
        g = np.concatenate([case.frames[c][k].ravel()[case.masks[c].ravel() > 0] for c in sorted(case.masks)])
        prev, _, _ = sart_gpu_semantics(Ar, g, None, logarithmic=log, max_iterations=40, conv_tolerance=1e-9,
                                        x_prev=prev)
    assert np.linalg.norm(x1 - prev) / np.linalg.norm(prev) < 1.5e-2


def test_partition_voxels_rejects_cpu_and_batches(tmp_path, binary):
    case = _case(tmp_path, nframes=1)
    r = _run_native(binary, ["--use_cpu", "--partition_voxels", *case.files])
    assert r.returncode == 1 and "partition_voxels" in r.stderr
    r = _run_native(binary, ["--batch_frames", "4", "--partition_voxels", *case.files])
    assert r.returncode == 1 and "partition_voxels" in r.stderr


@pytest.mark.parametrize("sig", ["SIGTERM", "SIGKILL"])
def test_module_entry_point_does_not_orphan_the_driver(tmp_path, binary, sig):
    """torchrun / mpiexec stop workers with SIGTERM: cli.py forwards it to the native driver and waits (exit code
    128 + 15); a parent killed outright (SIGKILL) takes the driver with it (PR_SET_PDEATHSIG from SART_PARENT_PID).
    Either way no driver outlives its launcher holding a GPU or sitting in a collective."""
    import signal
    import time

    import psutil

    case = _case(tmp_path, nframes=1)
    # rank 0 of a 2-rank world whose peer never comes: the driver blocks in the host rendezvous, like a rank whose
    # peer has already failed
    env = dict(_env(), RANK="0", WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    args = ["--use_cpu", "-o", str(tmp_path / "o.h5"), *case.files]
    p = subprocess.Popen([sys.executable, "-m", "mpi_cuda_sartsolver_amd", *args], env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    try:
        child = None
        for _ in range(300):  # the driver starts within seconds (python import + exec)
            kids = psutil.Process(p.pid).children()
            if kids:
                child = kids[0]
                break
            time.sleep(0.1)
        assert child is not None and child.exe().endswith("sartsolver"), "driver not started"
        time.sleep(1.0)  # inside the rendezvous
        assert p.poll() is None and child.is_running()
        p.send_signal(getattr(signal, sig))
        rc = p.wait(timeout=60)
        if sig == "SIGTERM":
            assert rc == 128 + signal.SIGTERM, rc  # forwarded, the driver's death reported like a shell does
        gone, alive = psutil.wait_procs([child], timeout=30)
        assert not alive, f"driver {child.pid} outlived its parent after {sig}"
    finally:
        if p.poll() is None:
            p.kill()
            p.wait()


@pytest.mark.gpu
@pytest.mark.parametrize("p2p", ["0", "1"])
@pytest.mark.parametrize("batch", [[], ["--batch_frames", "16"]], ids=["frame", "batch16"])
def test_native_sparse_two_ranks_one_device(tmp_path, binary, p2p, batch):
    """The sparse RTM path (--rtm_format sparse) on two ranks of the box's single GPU (row shards of the CSR, the
    per-iteration all-reduce staged or P2P) against the one-rank sparse run and the dense run of the same files;
    frame by frame and as a batch (the multi-frame engine's SpMM, its chunked all-reduce of the back-projection)."""
    case = make_case(str(tmp_path / "c"), sparse_cameras=("cam_a", "cam_b"), laplacian=True, nframes=2,
                     grid=(12, 12, 12), shapes=((24, 32), (20, 30)), raytraced=True)
    base = ["-m", "40", "-c", "1e-6", "-l", case.laplacian_file, "-b", "1e-3"] + batch
    r = _run_native(binary, base + ["--rtm_format", "sparse", "-o", str(tmp_path / "one.h5"), *case.files])
    assert r.returncode == 0, r.stderr
    assert "sparse: " in r.stdout
    r = _run_native(binary, base + ["--rtm_format", "dense", "-o", str(tmp_path / "dense.h5"), *case.files])
    assert r.returncode == 0, r.stderr
    saved = {k: os.environ.get(k) for k in ("SART_DIST_BACKEND", "SART_P2P")}
    os.environ["SART_DIST_BACKEND"] = "tcp"
    os.environ["SART_P2P"] = p2p
    prof = str(tmp_path / "prof.jsonl")
    try:
        r = _run_native(binary, base + ["--rtm_format", "sparse", "--profile", prof, "-o", str(tmp_path / "two.h5"),
                                        *case.files], nproc=2)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    import json

    load = json.loads(open(prof).readline())
    assert load["rtm_format"] == "sparse" and load["nnz"] > 0 and load["ranks"] == 2
    n = native()
    _, x1, s1 = n.read_solution_file(str(tmp_path / "one.h5"))
    _, x2, s2 = n.read_solution_file(str(tmp_path / "two.h5"))
    _, xd, sd = n.read_solution_file(str(tmp_path / "dense.h5"))
    np.testing.assert_array_equal(s1, s2)
    assert np.linalg.norm(x2 - x1) / np.linalg.norm(x1) < 2e-3
    assert np.linalg.norm(xd - x1) / np.linalg.norm(x1) < 2e-3


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--two_pass", "-L"], ["--rtm_format", "sparse"]])
def test_warm_start_on_device_is_bitwise(tmp_path, binary, extra):
    """Frames 1.. start from the previous solution still on the device (rescaled there) instead of a host round trip
    (SART_WARM_ON_DEVICE=0): the same start values, so the whole series is bitwise equal."""
    case = make_case(str(tmp_path / "c"), sparse_cameras=("cam_a", "cam_b"), laplacian=True, nframes=4,
                     grid=(12, 12, 12), shapes=((24, 32), (20, 30)), raytraced=True)
    base = ["-m", "30", "-c", "1e-6", "-l", case.laplacian_file, "-b", "1e-3"] + extra
    r = _run_native(binary, base + ["-o", str(tmp_path / "dev.h5"), *case.files])
    assert r.returncode == 0, r.stderr
    saved = os.environ.get("SART_WARM_ON_DEVICE")
    os.environ["SART_WARM_ON_DEVICE"] = "0"
    try:
        r = _run_native(binary, base + ["-o", str(tmp_path / "host.h5"), *case.files])
    finally:
        if saved is None:
            os.environ.pop("SART_WARM_ON_DEVICE", None)
        else:
            os.environ["SART_WARM_ON_DEVICE"] = saved
    assert r.returncode == 0, r.stderr
    n = native()
    X1 = n.read_dataset_f64(str(tmp_path / "dev.h5"), "solution/value")
    X2 = n.read_dataset_f64(str(tmp_path / "host.h5"), "solution/value")
    assert X1.shape[0] == 4
    np.testing.assert_array_equal(X1, X2)
