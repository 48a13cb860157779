#!/usr/bin/env python3
"""BASELINE config 1: 2048 x 4096, one frame, the CPU path (``sartsolver --use_cpu``), MPI = 1 / 2 / 4.

Writes a dense 2048 x 4096 case in the reference HDF5 schema (io/fixtures.py: two 32 x 32 cameras, all pixels
unmasked, 16^3 voxels in two segments per camera), runs the native driver on it and reads the driver's own
"Processed in: <ms> ms" line (the reference's timing instrument, reference main.cpp:127-140). Runs: a fixed 100
iterations (-c 1e-30: the convergence test never fires) and the reference default stopping rule (-m 2000 -c 1e-5);
MPI = 1 directly, MPI = 2 / 4 under mpiexec (MPICH, /opt/conda/bin) with the CPUs split between the ranks.
With --gpu the same case also runs through the GPU path (fused sweep) for comparison. One JSON line per run.
"""
import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="1,2,4")
    ap.add_argument("--gpu", action="store_true", help="also run the GPU path on the same case")
    ap.add_argument("--raytraced", action="store_true", help="the ray-traced RTM with reflections instead")
    ap.add_argument("--out", default=None, help="append JSON lines here")
    a = ap.parse_args()
    from mpi_cuda_sartsolver_amd.io.fixtures import make_case

    binary = os.path.join(ROOT, "mpi_cuda_sartsolver_amd", "_lib", "sartsolver")
    ncpu = len(os.sched_getaffinity(0))
    ncpu = min(ncpu, int(os.environ.get("OMP_NUM_THREADS", ncpu) or ncpu))
    tmp = tempfile.mkdtemp(prefix="cfg1_")
    t0 = time.perf_counter()
    case = make_case(os.path.join(tmp, "case"), shapes=((32, 32), (32, 32)), nvoxel=4096, grid=(16, 16, 16),
                     nframes=1, mask_fraction=0.0, raytraced=a.raytraced, seed=5)
    assert case.A.shape == (2048, 4096), case.A.shape
    make_s = time.perf_counter() - t0
    P, V = case.A.shape
    lines = []

    def run(tag, argv, nranks=1, threads=ncpu):
        env = dict(os.environ, OMP_NUM_THREADS=str(max(1, threads)), HSA_ENABLE_IPC_MODE_LEGACY="0")
        out = os.path.join(tmp, f"{tag}.h5")
        cmd = [binary, *argv, "-o", out, *case.files]
        if nranks > 1:
            mpiexec = shutil.which("mpiexec") or "/opt/conda/bin/mpiexec"
            cmd = [mpiexec, "-n", str(nranks), *cmd]
        t = time.perf_counter()
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
        wall = time.perf_counter() - t
        if r.returncode != 0:
            raise RuntimeError(f"{tag}: rc {r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}")
        ms = [float(m) for m in re.findall(r"Processed in:\s*([0-9.eE+-]+)\s*ms", r.stdout)]
        from mpi_cuda_sartsolver_amd.ops import native

        its = int(native().read_dataset_f64(out, "solution/iterations")[0])
        rec = dict(config="2048x4096 1 frame (BASELINE config 1)", run=tag, path="cpu" if "--use_cpu" in argv else "gpu",
                   mpi_ranks=nranks, omp_threads_per_rank=threads, iterations=its, processed_ms=ms[0],
                   iters_per_s=round(its / (ms[0] / 1e3), 2),
                   gflops=round(4.0 * P * V * its / (ms[0] / 1e3) / 1e9, 2), wall_s=round(wall, 3),
                   rtm="ray-traced with reflections" if a.raytraced else "dense random (fixtures.make_case)",
                   fixture_s=round(make_s, 2))
        print(json.dumps(rec), flush=True)
        lines.append(rec)

    for n in [int(x) for x in a.ranks.split(",")]:
        run(f"cpu_fixed100_mpi{n}", ["--use_cpu", "-m", "100", "-c", "1e-30"], n, ncpu // n)
        run(f"cpu_default_mpi{n}", ["--use_cpu", "-m", "2000", "-c", "1e-5"], n, ncpu // n)
    if a.gpu:
        run("gpu_fixed100", ["-m", "100", "-c", "1e-30"])
        run("gpu_default", ["-m", "2000", "-c", "1e-5"])
    if a.out:
        with open(a.out, "a") as f:
            for rec in lines:
                f.write(json.dumps(rec) + "\n")
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
