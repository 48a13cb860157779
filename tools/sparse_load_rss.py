#!/usr/bin/env python3
"""Host memory of the sparse RTM load: a COO RTM file of --nnz entries (default 100M: 2 GB of
pixel / voxel indices and values) loaded by the native driver with --rtm_format sparse on 1 and 4 ranks (ranks in
parallel, --parallel_read), one frame, 2 SART updates. Reports, from the driver's --profile load line, every rank's
peak RSS growth over the load (rss_growth_MB_max) next to the largest shard's CSR + CSC bytes (shard_MB_max): the
streamed reader (RtmReader::read_csr: count + fill passes over hyperslab chunks, no whole-array read or sort) keeps
the growth at the CSR + CSC the shard needs anyway, and the load rate.

    python tools/sparse_load_rss.py --out gpurun_out/sparse_load_rss.jsonl [--nnz 100000000] [--ranks 1,4]
"""
import argparse
import json
import os
import shutil
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nnz", type=int, default=100_000_000)
    ap.add_argument("--h", type=int, default=256)
    ap.add_argument("--w", type=int, default=256)
    ap.add_argument("--nvox", type=int, default=262144)
    ap.add_argument("--ranks", default="1,4")
    ap.add_argument("--cpu", action="store_true", help="--use_cpu (a rehearsal of the script without a GPU)")
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp") + "/sart_sparse_rss")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "sparse_load_rss.jsonl"))
    a = ap.parse_args()
    from mpi_cuda_sartsolver_amd.ops import native

    n = native()
    os.makedirs(a.dir, exist_ok=True)
    t0 = time.perf_counter()
    P, V = a.h * a.w, a.nvox
    rng = np.random.default_rng(1)
    # unique (pixel, voxel) pairs in shuffled order (the file order of a ray tracer's output is arbitrary)
    flat = np.unique(rng.integers(0, P * V, int(a.nnz * 1.02), dtype=np.int64))[: a.nnz]
    rng.shuffle(flat)
    pix, vox = (flat // V).astype(np.uint64), (flat % V).astype(np.uint64)
    del flat
    val = (rng.random(pix.size, dtype=np.float32) + 0.01).astype(np.float32)
    rtm, img = os.path.join(a.dir, "rtm.h5"), os.path.join(a.dir, "img.h5")
    ix = np.arange(V, dtype=np.uint64)
    n.write_rtm_file(path=rtm, camera_name="cam", wavelength=656.3, npixel=P, nvoxel=V,
                     frame_mask=np.ones((a.h, a.w), np.uint8), vi=ix, vj=np.zeros(V, np.uint64),
                     vk=np.zeros(V, np.uint64), vvalue=np.arange(V, dtype=np.int32), nx=V, ny=1, nz=1,
                     rtm_name="with_reflections", coordinate_system="", bounds=[], pixel_index=pix, voxel_index=vox,
                     value=val)
    nnz = int(val.size)
    del pix, vox, val
    n.write_image_file(img, "cam", 657.3, np.array([0.0]), np.ones((1, a.h, a.w)))
    write_s = time.perf_counter() - t0
    binary = os.path.join(ROOT, "mpi_cuda_sartsolver_amd", "_lib", "sartsolver")
    outf = open(a.out, "a")
    for nr in [int(v) for v in a.ranks.split(",")]:
        prof = os.path.join(a.dir, f"prof{nr}.jsonl")
        argv = [binary] + (["--use_cpu"] if a.cpu else []) + ["--rtm_format", "sparse", "-m", "2", "--parallel_read", "--profile", prof,
                "-o", os.path.join(a.dir, f"o{nr}.h5"), rtm, img]
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", SART_DIST_BACKEND="tcp", MASTER_ADDR="127.0.0.1",
                   SART_COMM_PORT=str(free_port()), WORLD_SIZE=str(nr))
        t = time.perf_counter()
        procs = [subprocess.Popen(argv, env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), stdout=subprocess.PIPE,
                                  stderr=subprocess.PIPE, text=True) for r in range(nr)]
        outs = [p.communicate(timeout=900) for p in procs]
        wall = time.perf_counter() - t
        for line in outs[0][1].splitlines():  # SART_LOAD_TRACE=1: the reader's pass times (rank 0)
            if line.startswith("read_csr"):
                print(line, flush=True)
        rc = [p.returncode for p in procs]
        if any(rc):
            raise SystemExit(f"ranks={nr}: rc {rc}\n{outs[0][1][-3000:]}")
        load = json.loads(open(prof).readline())
        rec = dict(nnz=nnz, npixel=P, nvoxel=V, file_GB=nnz * 20 / 1e9, write_s=round(write_s, 1), ranks=nr,
                   process_wall_s=round(wall, 2), load_s=load["load_s"], rss_growth_MB_max=load["rss_growth_MB_max"],
                   shard_MB_max=load["shard_MB_max"],
                   growth_over_shard=load["rss_growth_MB_max"] / load["shard_MB_max"] if load["shard_MB_max"] else None,
                   load_Mnnz_per_s=nnz / 1e6 / load["load_s"] if load["load_s"] else None,
                   rank0=load.get("rank0"), reader="RtmReader::read_csr (streamed COO, count + fill passes)")
        line = json.dumps(rec)
        print(line, flush=True)
        outf.write(line + "\n")
        outf.flush()
    shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
