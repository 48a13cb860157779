"""bench.py launch contract on the CPU (gloo): ``--gpus N`` self-launches N ranks, a world size that differs
from ``--gpus`` is an error, and too few devices is an error unless ranks may share them (rehearsal).
The reference launches its ranks through mpirun (reference main.cpp:63-68)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE")}
    env.update(PYTHONPATH=ROOT, **extra)
    return env


def test_self_launch_reports_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--steps", "2", "--warmup", "1", "--launch-check"],
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 3 and out["launch_check"] and out["max_rank"] == 2
    assert out["steps"] == 2 and out["warmup"] == 1


def test_world_size_mismatch_is_an_error():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--launch-check"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 1 and "launcher started 2 rank" in r.stderr


def test_too_few_devices_is_an_error():
    # no GPU in this container: 2 ranks need 2 devices unless --share-gpus
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=_env(), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 1 and "GPU(s) visible" in r.stderr
