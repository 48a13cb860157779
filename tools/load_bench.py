#!/usr/bin/env python3
"""HDF5 -> HBM load path of the native driver (reference raytransfer.cpp:92-110 reads a dense RTM one
row hyperslab at a time into host memory and copies the whole shard afterwards).

Writes multi-GB synthetic RTM fixtures with the native streaming writer (dense fp32 [npixel, nvoxel], and a sparse
COO file), drops them from the page cache (fdatasync + POSIX_FADV_DONTNEED), and runs ``sartsolver --profile`` for
two iterations on each, so the first profile line holds the load of the device shard: wall time, the reader's summed
HDF5 time, the summed GPU time of the host -> HBM copies, the time the copy loop waited for the reader and for a
staging buffer, and the resident-set growth. Cases:

* dense, cold cache, blocked reads (the default: 256 MiB staging blocks, <= 64 MiB hyperslabs, two pinned buffers)
* dense, cold cache, one row per hyperslab (SART_RTM_ROWS_PER_READ=1: the reference's read pattern, same pipeline)
* dense, warm cache (the file in the page cache: the pipeline without the storage device)
* sparse COO, cold cache

One JSON line per case to --out (and stdout).
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp") + "/sart_load_bench")
    ap.add_argument("--gb", type=float, default=8.6, help="dense fixture size (GB, nvoxel fixed at --nvox)")
    ap.add_argument("--nvox", type=int, default=65536)
    ap.add_argument("--sparse-nnz", type=int, default=256, help="nonzeros per pixel of the sparse fixture")
    ap.add_argument("--cases", default="dense,dense_row,dense_warm,sparse")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "load_bench.jsonl"))
    ap.add_argument("--keep", action="store_true")
    a = ap.parse_args()
    from mpi_cuda_sartsolver_amd.ops import native

    n = native()
    binary = os.path.join(ROOT, "mpi_cuda_sartsolver_amd", "_lib", "sartsolver")
    os.makedirs(a.dir, exist_ok=True)
    free = shutil.disk_usage(a.dir).free
    w = 128
    npix = int(a.gb * 1e9 / (4 * a.nvox))
    npix = max(w, npix // w * w)
    if npix * a.nvox * 4 > 0.8 * free:  # stay inside the scratch disk
        npix = max(w, int(0.8 * free / (4 * a.nvox)) // w * w)
    h = npix // w
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    outf = open(a.out, "a")

    def emit(rec):
        line = json.dumps(rec)
        print(line, flush=True)
        outf.write(line + "\n")
        outf.flush()

    img = os.path.join(a.dir, "image.h5")
    import numpy as np

    n.write_image_file(img, "cam_s", 657.0, np.array([0.0]), np.ones((1, h, w)))
    files = {}

    def fixture(kind):
        if kind in files:
            return files[kind]
        path = os.path.join(a.dir, f"rtm_{kind}.h5")
        t0 = time.perf_counter()
        nbytes = n.write_synthetic_rtm_file(path, "cam_s", 656.3, h, w, a.nvox, seed=7,
                                            nnz_per_row=a.sparse_nnz if kind == "sparse" else 0, drop_cache=True)
        dt = time.perf_counter() - t0
        emit({"fixture": kind, "path": path, "npixel": npix, "nvoxel": a.nvox, "value_GB": nbytes / 1e9,
              "file_GB": os.path.getsize(path) / 1e9, "write_s": round(dt, 2), "disk_free_GB": free / 1e9})
        files[kind] = path
        return path

    env0 = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for case in a.cases.split(","):
        kind = "sparse" if case.startswith("sparse") else "dense"
        path = fixture(kind)
        env = dict(env0)
        if case == "dense_row":
            env["SART_RTM_ROWS_PER_READ"] = "1"
        if case == "dense_small":  # 64 MiB blocks (128 MiB of pinned staging): what the RSS growth scales with
            env["SART_RTM_BLOCK_MB"] = "64"
        if case == "dense_warm":  # read once to pull the file into the page cache
            with open(path, "rb") as f:
                while f.read(64 << 20):
                    pass
        else:
            n.drop_file_cache(path)
        prof = os.path.join(a.dir, f"prof_{case}.jsonl")
        sol = os.path.join(a.dir, f"sol_{case}.h5")
        t0 = time.perf_counter()
        r = subprocess.run([binary, "-m", "2", "--profile", prof, "-o", sol, path, img], env=env,
                           capture_output=True, text=True, timeout=900)
        wall = time.perf_counter() - t0
        if r.returncode != 0:
            emit({"case": case, "error": r.returncode, "stderr": r.stderr[-2000:]})
            return 1
        recs = [json.loads(x) for x in open(prof)]
        load = recs[0]
        rec = {"case": case, "process_wall_s": round(wall, 2), **load}
        # a working double buffer: load_s ~ setup_s + max(read_s, h2d_s) + one block's copy
        blk = load["h2d_s"] / max(1, load["rank0"]["blocks"])
        rec["overlap"] = {
            "max_read_h2d_s": round(max(load["read_s"], load["h2d_s"]), 3),
            "sum_read_h2d_s": round(load["read_s"] + load["h2d_s"], 3),
            "setup_plus_max_plus_block_s": round(load.get("setup_s", 0.0) + max(load["read_s"], load["h2d_s"]) + blk, 3),
        }
        rec["solve"] = {k: recs[1].get(k) for k in ("iterations", "solve_ms", "fused", "rtm_GBps")} if len(recs) > 1 else None
        emit(rec)
        for p in (prof, sol):
            if os.path.exists(p):
                os.remove(p)
    if not a.keep:
        shutil.rmtree(a.dir, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
